"""A/B of the sharded pivot forms at world size 1 on one shape (default: the 8-GPU per-rank
shape of 16384^2, 2049 x 16384): update kernel average and whole-pivot time per form.
usage: python tools/fold_ab.py [rows] [cols] [K]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]
for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29561"), ("RANK", "0"),
             ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
    os.environ.setdefault(k, v)
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from simplex_mi355x import _lib, lp  # noqa: E402
from simplex_mi355x.sharded import HipShardBackend, RcclComm  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 2049
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    n, m = R - 1, C - 1
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    L = _lib.load()
    T = lp.dense_tableau("uniform", 0, n, m)
    off = 1 << 62
    forms = (("fused+fold", True, 0, False), ("fused", True, off, False),
             ("unfused", False, off, False), ("overlap-events", True, off, "events"),
             ("overlap-values", True, off, "values"))
    only = os.environ.get("FORMS")
    for name, fused, fold, overlap in forms:
        if only and name not in only.split(","):
            continue
        L.smx_tune_fold(fold)
        be = HipShardBackend(T, n, m, m, 0, 1, device="cuda:0", fused=fused, overlap=overlap)
        comm = RcclComm()
        be.run_native(10, comm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        upd, tot = be.run_native_timed(K, comm)
        wall = time.perf_counter() - t0
        st = be.state()
        print(json.dumps({"form": name, "rows": R, "cols": C, "K": K,
                          "update_us": float(np.mean(upd)) * 1e3,
                          "pivot_us": wall / K * 1e6, "valid": st["npivots"] == K + 10}),
              flush=True)
        comm.close()
        del be
        torch.cuda.empty_cache()
    L.smx_tune_fold(off)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
