"""Per-pivot time of block pivots (smx_block_*: P pivots per HBM sweep) vs the fused one-pivot
chain, on seeded uniform LPs, by tableau size and pivots per sweep.

  python tools/block_bench.py [--sizes 4096,8192,16384] [--pivots 1,2,3,4,6,8] [--k 48]
      [--planner 0,1] [--form 0]

One JSON line per (size, path): us per pivot from HIP events on the solver stream around one
graph replay of k pivots (after a warm-up replay), the average sweep time of a timed run
(smx_block_run_timed) and the planner's share, and whether the trajectory equals the fused
chain's (pivot log and final table bits).
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
    ap.add_argument("--sizes", default="4096,8192,16384")
    ap.add_argument("--pivots", default="1,2,3,4,5,6,8")
    ap.add_argument("--k", type=int, default=48)
    ap.add_argument("--bpc", type=int, default=0, help="blocks per CU of the sweep (0: library)")
    ap.add_argument("--form", default="0", help="smx_tune_block_form settings to compare, e.g. 4,5")
    ap.add_argument("--planner", default="0",
                    help="smx_tune_block_planner settings to compare (0 the window planner, persistent where "
                         "eligible, 2 its launch form, 1 the "
                         "register-form chains), e.g. 0,1")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau
    _lib.tune_resident(-1)
    if a.bpc:
        _lib.check(_lib.load().smx_tune_set(-2, a.bpc), "smx_tune_set")
    for N in (int(x) for x in a.sizes.split(",")):
        n = m = N - 1
        T = lp.dense_tableau("uniform", a.seed, n, m)
        dev = DeviceTableau(T, n, m, m, block=0)
        k = a.k
        ref_log = ref_tab = None
        runs = [(0, 0, 0)] + [(int(x), int(f), int(pl)) for x in a.pivots.split(",")
                              for f in a.form.split(",") for pl in a.planner.split(",")]
        for P, form, planner in runs:
            _lib.tune_block_form(form)
            _lib.tune_block_planner(planner, 0)
            dev.close()   # captured graphs bake in the layout: capture afresh for every run
            dev.block = P
            dev.upload(T)
            dev.step = 0
            dev.prepare(k)
            dev.run(k)
            dev.sync_state()
            dev.upload(T)
            dev.step = 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(dev.stream)
            dev.run(k)
            e1.record(dev.stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            ctl = dev.sync_state()
            log = dev.read_log(0, int(ctl["npivots"]))
            tab = dev.download().view(np.int64)
            row = {"size": N, "path": "fused" if P == 0 else f"block{P}", "planner": planner,
                   "form": form, "k": k,
                   "bpc": a.bpc,
                   "us_per_pivot": ms * 1e3 / k, "pivots_s": k / ms * 1e3,
                   "npivots": int(ctl["npivots"])}
            if P == 0:
                ref_log, ref_tab = log, tab
            else:
                row["same_as_fused"] = bool(np.array_equal(log, ref_log) and
                                            np.array_equal(tab, ref_tab))
                for _ in range(2):   # an untimed eager run first
                    dev.upload(T)
                    dev.step = 0
                    sw, tot = dev.run_block_timed(k, P)
                ctl = dev.sync_state()
                row["eager_same_as_fused"] = bool(
                    np.array_equal(dev.read_log(0, int(ctl["npivots"])), ref_log) and
                    np.array_equal(dev.download().view(np.int64), ref_tab))
                row["sweep_us"] = float(np.mean(sw)) * 1e3
                row["sweep_gbs"] = 16.0 * N * N / (float(np.mean(sw)) * 1e-3) / 1e9
                row["eager_us_per_pivot"] = tot * 1e3 / k
                row["planner_us_per_block"] = (tot - float(np.sum(sw))) * 1e3 / len(sw)
            print(json.dumps(row), flush=True)
        dev.close()
        del dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
