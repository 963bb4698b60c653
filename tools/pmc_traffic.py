"""Derive HBM bytes per launch of the update kernel from two rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_KEY [OUT_JSON] [KERNEL_SUBSTRING]

Each pass is `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (separate runs: on gfx950 the two
do not fit one pass).  Both counters are in KiB.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.  The Infinity Cache is counted, not
excluded, which does not matter at 16384^2 (2 x 2 GiB ping-pong >> 256 MiB).
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter, needle="k_update"):
    vals = []
    for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and needle in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, key = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else None
    needle = sys.argv[5] if len(sys.argv) > 5 else "k_update"
    f = per_dispatch(fdir, "FETCH_SIZE", needle)
    w = per_dispatch(wdir, "WRITE_SIZE", needle)
    fetch_kib = statistics.median(f)
    write_kib = statistics.median(w)
    rec = {
        "kernel": needle,
        "dispatches": [len(f), len(w)],
        "fetch_size_kib_median": fetch_kib,
        "write_size_kib_median": write_kib,
        "read_bytes_corrected": 2.0 * fetch_kib * 1024.0,
        "write_bytes": write_kib * 1024.0,
        "bytes_per_launch": 2.0 * fetch_kib * 1024.0 + write_kib * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> B",
    }
    print(json.dumps(rec, indent=1))
    if out:
        data = {}
        if os.path.exists(out):
            with open(out) as fh:
                data = json.load(fh)
        data[key] = rec
        with open(out, "w") as fh:
            json.dump(data, fh, indent=1)


if __name__ == "__main__":
    main()
