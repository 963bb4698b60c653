"""Native RCCL shard driver, 1-rank job: trajectory and table vs the C oracle (bit for bit).
Run as a subprocess by tests/test_gpu_sharded.py (it initialises torch.distributed)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]
for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29541"), ("RANK", "0"),
             ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
    os.environ.setdefault(k, v)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import c_oracle  # noqa: E402
from simplex_mi355x import lp  # noqa: E402
from simplex_mi355x.sharded import HipShardBackend, RcclComm, ShardedSolver  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
ok = True
cases = (("uniform", 1023, 777, 120), ("mixed", 600, 500, 150),
         ("degenerate", 300, 300, 100), ("uniform", 40, 30, 400),
         ("mixed", 4095, 4095, 40))
modes = (("overlap", True, True), ("fused", True, False), ("unfused", False, False))
for (mode, fused, overlap), (kind, n, m, k) in [(md, c) for md in modes for c in cases]:
    T = lp.dense_tableau(kind, 5, n, m)
    be = HipShardBackend(T, n, m, m, 0, 1, device="cuda:0", fused=fused, overlap=overlap)
    comm = RcclComm()
    st = ShardedSolver(be, comm=comm).run(k)
    Tref, s_ref, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    got = be.local_table()
    same = (st["npivots"] == done and np.array_equal(be.log(0, done), log)
            and np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
            and (not st["term"] or st["status"] == s_ref))
    print(mode, kind, n, m, "pivots", st["npivots"], done,
          "ok" if same else "MISMATCH", flush=True)
    ok &= same
    comm.close()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
