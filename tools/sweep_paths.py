"""Which path the block sweep's units take, sweep by sweep, along a long trajectory.

  SMX_LIB=libsmx_diag.so python tools/sweep_paths.py [--size 16384 | --rows R --cols C]
      [--kind uniform] [--pivots 20] [--warmup 5] [--k 200] [--idle 0] [--bpc 0] [--form 0]

One JSON line per block of `pivots` pivots: the sweep's HIP-event time, and -- with the
diagnostic build (`make -C simplex-method-solver_amd/csrc diag`, loaded through SMX_LIB) -- the
number of (row, 128-column chunk) units per path of blk_sweep_body_flag (smx_block.hpp kPc*:
fast / zero-extended / window-tracked / window failed -> exact / exact directly, plus why units
missed the fast path).  `--idle S` sleeps S seconds before every block (a sweep that is fast after
a pause but slow back to back is the clock, not the data).  A last line sums the run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]

PATHS = ["fast", "zero", "window", "window_fail", "exact", "chunk_not_free", "chunk_not_zok",
         "row_flag0", "row_flag3", "x_fail", "chunk_e", "chunk_p", "clk_cycles", "clk_ticks"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pivots", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=200)
    ap.add_argument("--idle", type=float, default=0.0)
    ap.add_argument("--bpc", type=int, default=0, help="sweep blocks per CU (0: library)")
    ap.add_argument("--form", type=int, default=0, help="smx_tune_block_form (0: library)")
    a = ap.parse_args()
    import ctypes

    import numpy as np
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau
    L = _lib.load()
    _lib.tune_resident(-1)
    if a.bpc:
        _lib.check(L.smx_tune_set(-2, a.bpc), "smx_tune_set")
    _lib.tune_block_form(a.form)
    R = a.rows or a.size
    C = a.cols or a.size
    n, m = R - 1, C - 1
    T = lp.dense_tableau(a.kind, a.seed, n, m)
    dev = DeviceTableau(T, n, m, m, block=a.pivots, log_cap=max(1 << 16, a.warmup + a.k + 64))
    del T
    cnt = (ctypes.c_int64 * len(PATHS))()
    diag = L.smx_diag_path_counts(cnt, len(PATHS), 1) > 0
    if a.warmup:
        dev.run_block_timed(a.warmup, a.pivots)
        dev.sync_state()
    if diag:
        L.smx_diag_path_counts(cnt, len(PATHS), 1)
    _lib.check(L.smx_timer_reserve(8), "smx_timer_reserve")
    tot_counts = np.zeros(len(PATHS), dtype=np.int64)
    sweeps = []
    done = 0
    t_start = time.perf_counter()
    while done < a.k:
        if a.idle:
            time.sleep(a.idle)
        P = min(a.pivots, a.k - done)
        sw, tot = dev.run_block_timed(P, P)
        ctl = dev.sync_state()
        rec = {"block": len(sweeps), "pivot0": a.warmup + done, "pivots": P,
               "sweep_ms": round(float(sw[0]), 4), "device_ms": round(tot, 4),
               "t_s": round(time.perf_counter() - t_start, 3)}
        if diag:
            L.smx_diag_path_counts(cnt, len(PATHS), 1)
            c = np.frombuffer(cnt, dtype=np.int64).copy()
            tot_counts += c
            units = int(c[0] + c[1] + c[2] + c[3] + c[4])
            rec["units"] = units
            rec["paths"] = {k: int(v) for k, v in zip(PATHS[:12], c[:12]) if v}
            if c[13]:   # shader clock over the sweep bodies (s_memtime / s_memrealtime at 100 MHz)
                rec["clock_ghz"] = round(float(c[12]) / float(c[13]) * 0.1, 4)
        sweeps.append(rec)
        print(json.dumps(rec), flush=True)
        done += P
        if ctl["term"]:
            break
    ms = [s["sweep_ms"] for s in sweeps if s["pivots"] == a.pivots]
    summ = {"summary": True, "rows": R, "cols": C, "kind": a.kind, "seed": a.seed,
            "pivots": a.pivots, "warmup": a.warmup, "k": done, "idle_s": a.idle,
            "bpc": a.bpc, "form": a.form, "diag": diag,
            "mean_sweep_ms": float(np.mean(ms)) if ms else None,
            "first_sweep_ms": ms[0] if ms else None, "last_sweep_ms": ms[-1] if ms else None}
    if diag:
        units = int(tot_counts[:5].sum())
        summ["units"] = units
        summ["path_share"] = {k: round(int(v) / units, 5) for k, v in zip(PATHS[:12],
                                                                          tot_counts[:12])
                              if v and units}
        if tot_counts[13]:
            summ["clock_ghz"] = round(float(tot_counts[12]) / float(tot_counts[13]) * 0.1, 4)
    print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
