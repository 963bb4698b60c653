import os, sys, time, json
sys.path[:0] = ["/root/repo", "/root/repo/simplex-method-solver_amd"]
import numpy as np, torch
from simplex_mi355x import _lib, lp
from simplex_mi355x.device import DeviceTableau
n = m = 16383
T = lp.dense_tableau("uniform", 0, n, m)
dev = DeviceTableau(T, n, m, m)
P = dev.block_plan()[1]
_lib.check(_lib.load().smx_timer_reserve(64), "reserve")
res = {"eager": [], "graph": []}
for rep in range(4):
    for mode in ("eager", "graph"):
        dev.upload(T)
        dev.run(5, graph=True); dev.sync_state()
        if mode == "graph":
            dev.prepare(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "eager":
            dev.run_block_timed(20, P)
        else:
            dev.run(20, graph=True)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e3)
        dev.sync_state()
print(json.dumps({k: [round(x, 3) for x in v] for k, v in res.items()}))
