"""Per-dispatch means of rocprofv3 --pmc counters for the kernels whose name matches a pattern.

  python tools/pmc_summary.py PATTERN run_counter_collection.csv [...] [--json OUT]

Each CSV is one pass (tools/pmc_sweep.sh); rows are (dispatch, counter) pairs.  Prints one line
per counter: mean value per dispatch over the matching dispatches, and the dispatch count."""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict


def summarize(pattern: str, paths: list[str]) -> dict:
    rx = re.compile(pattern)
    vals: dict[str, list[float]] = defaultdict(list)
    names = set()
    for p in paths:
        with open(p) as fh:
            for row in csv.DictReader(fh):
                if not rx.search(row["Kernel_Name"]):
                    continue
                names.add(row["Kernel_Name"])
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {"kernels": sorted(names),
            "counters": {k: {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
                         for k, v in sorted(vals.items())}}


if __name__ == "__main__":
    args = sys.argv[1:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        del args[i:i + 2]
    res = summarize(args[0], args[1:])
    for k, v in res["counters"].items():
        print(f"{k:28s} {v['mean_per_dispatch']:.6g}  ({v['dispatches']} dispatches)")
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
