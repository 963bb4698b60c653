"""cProfile of the Info-object batch API (solve_batch, history=True) on 20 000 UI-shaped LPs."""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402
from bench_batch import make  # noqa: E402
from simplex_mi355x.batch import solve_batch  # noqa: E402

probs = make(20000)
solve_batch(probs[:2000], max_pivots=64, history=True)   # warm
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
solve_batch(probs, max_pivots=64, history=True)
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
