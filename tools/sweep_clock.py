"""Shader clock of the block sweep from a rocprofv3 GRBM pass (tools/gpu_round.sh clock20 /
clock200: --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_BUSY_CYCLES) into
profiles/sweep_clock.json, which bench.py reads for two_term.valu_frac_at_clock.

GRBM_GUI_ACTIVE is summed over the 8 XCDs (rocprofv3 reports the sum); one XCD's busy cycles over
the dispatch's duration is the clock it ran at:  clock_ghz = GRBM_GUI_ACTIVE / 8 / duration_ns.

usage: python tools/sweep_clock.py COUNTER_CSV WORKLOAD [--kernel k_blk_sweep<20] [--first]
  WORKLOAD e.g. 16384x16384/k_blk_sweep<20>; --first takes the first matching dispatch only (the
  driver's timed sweep in a bench20 pass), else the median over all of them.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "sweep_clock.json")


def dispatch_clocks(path, needle):
    per = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if needle not in r["Kernel_Name"]:
                continue
            d = per.setdefault(int(r["Dispatch_Id"]), {})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = []
    for k in sorted(per):
        d = per[k]
        if "GRBM_GUI_ACTIVE" in d and d["ns"] > 0:
            out.append({"dispatch": k, "ns": d["ns"], "clock_ghz": d["GRBM_GUI_ACTIVE"] / 8 / d["ns"],
                        "valu": d.get("SQ_INSTS_VALU")})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("workload")
    ap.add_argument("--kernel", default="k_blk_sweep<20")
    ap.add_argument("--first", action="store_true")
    a = ap.parse_args()
    ds = dispatch_clocks(a.csv, a.kernel)
    if not ds:
        raise SystemExit(f"no {a.kernel} dispatch with GRBM_GUI_ACTIVE in {a.csv}")
    pick = ds[:1] if a.first else ds
    ghz = statistics.median(d["clock_ghz"] for d in pick)
    rec = {"clock_ghz": round(ghz, 4), "dispatches": len(pick),
           "clock_range_ghz": [round(min(d["clock_ghz"] for d in ds), 4),
                               round(max(d["clock_ghz"] for d in ds), 4)],
           "source": os.path.relpath(a.csv, REPO) + (" (first dispatch)" if a.first else
                                                      " (median over dispatches)")}
    db = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            db = json.load(fh)
    db[a.workload] = rec
    with open(OUT, "w") as fh:
        json.dump(db, fh, indent=1)
        fh.write("\n")
    print(a.workload, rec)


if __name__ == "__main__":
    main()
