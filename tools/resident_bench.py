"""Per-pivot time of the on-chip resident loop (smx_resident_run) vs the fused launch chain
(hipGraph replay) on seeded uniform LPs, by tableau size and workgroup count.

  python tools/resident_bench.py [--sizes 256,512,1024,2048] [--wgs 0,64,128,256] [--k 400]
                                 [--trace]

Prints one JSON line per (size, path): us per pivot from HIP events on the solver stream around
one run of k pivots (after a warm-up run), and whether the trajectory stayed valid (k pivots).
--trace adds the anatomy of steps 100..163 from s_memrealtime stamps (smx_resident_trace):
medians over workgroups and steps of each phase (A record, B publish, C poll+decide, D row
fetch, E update, gap to the next step) and the spread of the publish times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]


def timed(dev, k, reps=3):
    import torch
    best = None
    for _ in range(reps):
        dev.upload(dev._host)
        dev.run(8)
        dev.sync_state()
        dev.prepare(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(dev.stream)
        dev.run(k)
        e1.record(dev.stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        ctl = dev.sync_state()
        ok = int(ctl["npivots"]) == k + 8 and not ctl["term"]
        best = ms if best is None or ms < best else best
    return best * 1e3 / k, ok


def anatomy(dev, k, G):
    import numpy as np
    import torch
    from simplex_mi355x import _lib
    L = _lib.load()
    tr = torch.zeros(64 * G * 8, dtype=torch.int64, device=dev.device)
    L.smx_resident_trace(tr.data_ptr(), 100)
    try:
        timed(dev, k, reps=1)
    finally:
        L.smx_resident_trace(None, 0)
    t = tr.cpu().numpy().reshape(64, G, 8).astype(np.float64) * 0.01   # 100 MHz ticks -> us
    ph = {"A_record": t[:, :, 1] - t[:, :, 0], "B_publish": t[:, :, 2] - t[:, :, 1],
          "C_poll_decide": t[:, :, 3] - t[:, :, 2], "D_row": t[:, :, 4] - t[:, :, 3],
          "E_update": t[:, :, 5] - t[:, :, 4], "gap_next": t[1:, :, 0] - t[:-1, :, 5],
          "step": t[1:, :, 0] - t[:-1, :, 0]}
    out = {key: float(np.median(v)) for key, v in ph.items()}
    pub = t[:, :, 2]
    out["publish_spread"] = float(np.median(pub.max(axis=1) - pub.min(axis=1)))
    out["last_publish_to_decided"] = float(np.median(t[:, :, 3].min(axis=1) - pub.max(axis=1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,512,1024,2048")
    ap.add_argument("--wgs", default="0,32,64,128,256")
    ap.add_argument("--k", type=int, default=400)
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--overlap", default="1", help="smx_tune_resident_overlap settings, e.g. 0,1")
    ap.add_argument("--seeds", default="0")
    a = ap.parse_args()
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau
    for size, seed in [(int(x), int(sd)) for x in a.sizes.split(",") for sd in a.seeds.split(",")]:
        n = m = size - 1
        T = lp.dense_tableau(a.kind, seed, n, m)
        dev = DeviceTableau(T, n, m, m, log_cap=1 << 16)
        dev._host = T
        dev.resident = False
        us, ok = timed(dev, a.k)
        print(json.dumps({"size": size, "seed": seed, "mode": "chain", "us_per_pivot": us,
                          "valid": ok}), flush=True)
        dev.resident = None
        for wg, ovl in [(int(x), int(o)) for x in a.wgs.split(",") for o in a.overlap.split(",")]:
            _lib.tune_resident(wg)
            _lib.tune_resident_overlap(ovl)
            plan = dev.resident_plan()
            if plan is None:
                continue
            us, ok = timed(dev, a.k)
            rec = {"size": size, "seed": seed, "mode": "resident", "overlap": ovl,
                   "wg": plan[1][0], "rows_per_wg": plan[1][1],
                   "ept": plan[1][2], "lds": plan[1][3], "us_per_pivot": us, "valid": ok}
            if a.trace and a.k >= 170:
                rec["anatomy_us"] = anatomy(dev, a.k, plan[1][0])
            print(json.dumps(rec), flush=True)
        _lib.tune_resident(0)
        _lib.tune_resident_overlap(2)
        dev.close()


if __name__ == "__main__":
    main()
