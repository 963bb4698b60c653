"""Driver for rocprofv3 counter passes on the block sweep (k_blk_sweep<P>) of a seeded N x N LP.

  python tools/sweep_pmc.py [--size 16384] [--pivots 8] [--k 32] [--reps 2]

Uploads the LP, runs `reps` timed block chains of k pivots from the same start (HIP events around
every sweep), prints one JSON line per rep.  Small and deterministic so every `--pmc` pass sees
the same dispatches (tools/pmc_sweep.sh).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--pivots", type=int, default=8)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau
    _lib.tune_resident(-1)
    n = m = a.size - 1
    T = lp.dense_tableau("uniform", 0, n, m)
    dev = DeviceTableau(T, n, m, m, block=a.pivots)
    for rep in range(a.reps):
        dev.upload(T)
        sw, tot = dev.run_block_timed(a.k, a.pivots)
        ctl = dev.sync_state()
        print(json.dumps({"rep": rep, "size": a.size, "pivots": a.pivots, "k": a.k,
                          "npivots": int(ctl["npivots"]), "sweep_us": [float(x) * 1e3 for x in sw],
                          "sweep_us_mean": float(np.mean(sw)) * 1e3,
                          "sweep_gbs": 16.0 * a.size * a.size / (float(np.mean(sw)) * 1e-3) / 1e9,
                          "total_ms": tot}), flush=True)


if __name__ == "__main__":
    main()
