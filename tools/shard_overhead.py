"""Where do the sharded path's per-pivot microseconds go?  1-rank RCCL job on one GPU.
(a) host enqueue time vs wall time for K eager pivots; (b) the same K pivots captured once in a
torch.cuda.CUDAGraph (kernels + the RCCL all-gather) and replayed."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))
for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517"), ("RANK", "0"),
             ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
    os.environ.setdefault(k, v)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from simplex_mi355x import lp  # noqa: E402
from simplex_mi355x.sharded import HipShardBackend, ShardedSolver  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
S = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
n = m = S - 1
T = lp.dense_tableau("uniform", 0, n, m)
be = HipShardBackend(T, n, m, m, 0, 1, device="cuda:0")
sol = ShardedSolver(be)
sol.run(20)
K = 200
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    sol.pivot()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"eager: host enqueue {(t1 - t0) / K * 1e6:.1f} us/pivot, wall {(t2 - t0) / K * 1e6:.1f} us/pivot")
st = be.state()
print("state", st)
# graph capture of G pivots (parity must be even to replay: G even)
G = 20
try:
    g = torch.cuda.CUDAGraph()
    d = be.dev
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=d.stream):
        for _ in range(G):
            sol.pivot()
    d.step -= G          # capture does not execute; the host counter advanced anyway
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K // G):
        g.replay()
        d.step += G
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    st2 = be.state()
    print(f"graph: wall {(t2 - t0) / K * 1e6:.1f} us/pivot; pivots {st2['npivots'] - st['npivots']} (expect {K})")
except Exception as exc:  # report, do not hide
    print("graph capture failed:", type(exc).__name__, exc)
dist.destroy_process_group()
