"""Pivots/s and update-kernel GB/s across tableau sizes on one MI355X (BASELINE configs 2-4).
Graph path: k pivots captured once as a hipGraph and replayed; eager path: smx_run_timed with
HIP events around every update kernel.  usage: python tools/sweep_sizes.py > out.jsonl"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simplex_mi355x import lp  # noqa: E402
from simplex_mi355x.device import DeviceTableau  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1024,2048,4096,8192,16384").split(",")]
    for S in sizes:
        n = m = S - 1
        T = lp.dense_tableau("uniform", 0, n, m)
        dev = DeviceTableau(T, n, m, m)
        k = 200 if S <= 8192 else 100
        chunk = 50
        dev.run(chunk, graph=True)            # capture + warm
        dev.sync_state()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k // chunk):
            dev.run(chunk, graph=True)
        torch.cuda.synchronize()
        tg = time.perf_counter() - t0
        st = dev.sync_state()
        ok_graph = int(st["npivots"]) == chunk + k and not st["term"]
        upd, dev_ms = dev.run_timed(k)
        torch.cuda.synchronize()
        st = dev.sync_state()
        ok_eager = int(st["npivots"]) == chunk + 2 * k and not st["term"]
        bytes_pp = 16.0 * S * S
        rec = {"size": S, "pivots_graph": k, "graph_pivots_per_s": k / tg,
               "graph_us_per_pivot": tg / k * 1e6, "eager_device_us_per_pivot": dev_ms / k * 1e3,
               "update_kernel_us": float(np.mean(upd)) * 1e3,
               "update_gbs": bytes_pp / (float(np.mean(upd)) * 1e-3) / 1e9,
               "whole_pivot_gbs_graph": bytes_pp / (tg / k) / 1e9,
               "valid": bool(ok_graph and ok_eager)}
        print(json.dumps(rec), flush=True)
        dev.close()
        del dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
