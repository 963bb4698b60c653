"""Timeline of a rocprofv3 kernel trace: per-kernel-name counts, mean durations and the mean gap
between consecutive dispatches of the sweep kernel (what the per-pivot critical path adds).
usage: python tools/trace_gaps.py run_kernel_trace.csv [name_substring_of_sweep]"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_update"
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = defaultdict(list)
    for s, e, n in rows:
        per[n[:60]].append((e - s) / 1e3)
    for n, d in sorted(per.items(), key=lambda x: -sum(x[1])):
        print(f"{len(d):6d} x {statistics.mean(d):9.2f} us  {n}")
    sw = [(s, e) for s, e, n in rows if key in n]
    gaps = [(sw[i + 1][0] - sw[i][1]) / 1e3 for i in range(len(sw) - 1)]
    if gaps:
        print(f"sweep-to-sweep gap: mean {statistics.mean(gaps):.2f} us, "
              f"median {statistics.median(gaps):.2f} us over {len(gaps)}")
    # what runs inside the gap after each sweep (first 3 examples, late in the run)
    for i in range(len(sw) - 5, len(sw) - 2):
        s0, e0 = sw[i]
        s1 = sw[i + 1][0]
        inside = [(round((s - e0) / 1e3, 1), round((e - s) / 1e3, 1), n[:40])
                  for s, e, n in rows if e0 - 200_000 <= s <= s1 and key not in n]
        print("after sweep", i, "gap", round((s1 - e0) / 1e3, 1), "us:", inside)


if __name__ == "__main__":
    main()
