"""Kernel stats from a rocprofv3 rocpd database (the default output format when
--output-format csv is not given) in the layout of rocprofv3's kernel_stats.csv
(Name, Calls, TotalDurationNs, AverageNs).  usage: python tools/rocpd_stats.py run_results.db > out.csv"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    # top_kernels durations are in microseconds
    for name, calls, tot_us, avg_us, pct in con.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(tot_us * 1e3), round(avg_us * 1e3, 1), pct])


if __name__ == "__main__":
    main()
