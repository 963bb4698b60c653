"""Stage timing of the Info-object batch API on 20 000 UI-shaped LPs (no profiler)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402
from bench_batch import make  # noqa: E402
from simplex_mi355x import batch  # noqa: E402

probs = make(20000)
batch.solve_batch(probs[:2000], max_pivots=64, history=True)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    idx = [k for k, (c, f) in enumerate(probs) if batch._eligible(c, f)]
    tabs, dims = batch.pack([probs[k] for k in idx])
    t1 = time.perf_counter()
    out = batch.solve_batch_arrays(tabs, dims, 64, True)
    t2 = time.perf_counter()
    for q, k in enumerate(idx):
        batch._assemble(probs[k], dims[q], out["final"][q], out["rc"][q], out["xv"][q],
                        out["snaps"][out["snap_off"][q]:out["snap_off"][q + 1]],
                        int(out["status"][q]), int(out["npivots"][q]), 64)
    t3 = time.perf_counter()
    t4 = time.perf_counter()
    batch.solve_batch(probs, max_pivots=64, history=True)
    t5 = time.perf_counter()
    n = len(probs)
    print(f"pack {1e6*(t1-t0)/n:.1f} us/LP, device+copies {1e6*(t2-t1)/n:.1f} us/LP, "
          f"assemble {1e6*(t3-t2)/n:.1f} us/LP, solve_batch {n/(t5-t4):.0f} LPs/s", flush=True)
