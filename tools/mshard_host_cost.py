"""Host enqueue vs device time per pivot of the single-process multi-device drop-in
(``SimplexMethod(..., devices=[...])`` -> ``MultiTableau.run`` -> ``smx_mshard_run``; the
reference caller's shape, main.py:313, scaled to the north-star table).

  python tools/mshard_host_cost.py [--size 16384] [--ranks 1,2,4,8] [--k 48] [--pivots 8]

Every rank lives on cuda:0 (a one-GPU box: the copy exchange).  Per rank count one JSON line:
``host_us_per_pivot`` = wall time of the ``run(k)`` call itself (it returns once every launch of
every rank is enqueued) / k; ``device_us_per_pivot`` = wall time until every stream drained / k
(all ranks share one GPU here, so this is the SUM of the ranks' device work; on N GPUs each
device carries ~1/N of it: ``device_us_per_pivot_per_gpu``).  The host is on the critical path
of an N-GPU run when host_us_per_pivot exceeds device_us_per_pivot_per_gpu.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--k", type=int, default=48)
    ap.add_argument("--pivots", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--exchange", default=None, help="copy (default on one device) or rccl "
                    "(one host thread per device; one rank per device, so world 1 here)")
    ap.add_argument("--forms", default="eager,graph",
                    help="eager (smx_mshard_run) and / or graph (smx_mshard_graph_create: copy "
                         "exchange on one device, one replay per chain)")
    a = ap.parse_args()
    import torch
    from simplex_mi355x import lp
    from simplex_mi355x.multi import MultiTableau
    n = m = a.size - 1
    T = lp.dense_tableau("uniform", 0, n, m)
    for world in (int(x) for x in a.ranks.split(",")):
        mt = MultiTableau(T, n, m, m, ["cuda:0"] * world, pivots=a.pivots, exchange=a.exchange,
                          graph_chain="graph" in a.forms)
        mt.run(a.pivots, graph=False)   # warm-up: prime, first kernels
        mt.sync_state()
        logs = {}
        forms = [f == "graph" for f in a.forms.split(",") if f == "eager" or mt.graph_chain]
        for graph in forms:
            host, wall = [], []
            for rep in range(a.reps + (1 if graph else 0)):   # graph: the first run captures
                mt.upload(T)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                mt.run(a.k, graph=graph)
                t1 = time.perf_counter()
                st = mt.sync_state()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                assert int(st["npivots"]) == a.k, st
                if graph and rep == 0:
                    continue
                host.append((t1 - t0) / a.k * 1e6)
                wall.append((t2 - t0) / a.k * 1e6)
            logs[graph] = mt.read_log(0, a.k).tolist()
            if len(logs) == 2:   # the graph replays exactly the eager chain's pivots
                assert logs[True] == logs[False]
            dev = min(wall)
            print(json.dumps({"size": a.size, "ranks": world, "exchange": mt.exchange,
                              "form": "graph" if graph else "eager",
                              "pivots_per_sweep": a.pivots, "k": a.k,
                              "host_us_per_pivot": round(min(host), 2),
                              "device_us_per_pivot": round(dev, 2),
                              "device_us_per_pivot_per_gpu": round(dev / world, 2),
                              "host_bound_on_n_gpus": min(host) > dev / world}), flush=True)
        mt.close()
        del mt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
