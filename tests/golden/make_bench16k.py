"""Generate ``tests/golden/bench16k.json``: the bench line's own workload (16384 x 16384 uniform
random LP, seed 0; BASELINE config 4 at one GPU) run through the C oracle, so ``bench.py`` can
check its trajectory and final table after the timed region and print ``"parity": true/false``
in the line.  Runs in the build container (two 2 GiB buffers)::

    python tests/golden/make_bench16k.py [--pivots 220] [--threads 8]

Records: every pivot ``(r, c)`` of get_solution's loop (simplex.py:184-198) up to ``--pivots``,
and the SHA-256 of the table (rows[:n, :m+1] in C order, then f-row[:m]; the hash of
``make_config5.table_sha256``) after 25 pivots (the driver's ``--warmup 5 --steps 20``) and
after 220 (the default ``--warmup 20 --steps 200``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_config5 import run_kind  # noqa: E402

CHECKS = (25, 220)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pivots", type=int, default=220)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(HERE, "bench16k.json"))
    a = ap.parse_args()
    import make_config5
    make_config5.CHECKPOINTS = tuple(k for k in CHECKS if k < a.pivots)
    rec = run_kind("uniform", a.pivots, a.threads, 16383, 16383)
    rec.pop("cycle", None)
    with open(a.out, "w") as f:
        json.dump({"generator": "tests/golden/make_bench16k.py", "oracle": "oracle/simplex_oracle.c",
                   "hash": "sha256(rows[:n, :m+1] C-order fp64) || f-row[:m]", **rec}, f)
        f.write("\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
