"""Drive a dense (pick, pivot) pair with the reference's host semantics and record a trajectory
in the same shape as ``make_golden.trajectory`` (simplex.py:184-198 with a cap).

Used to check the numpy / C oracles against the fixtures.  Host-side rules mirrored here:
labels (simplex.py:30-33, 152), ``find_optimum`` (:51-68), ``f`` (:48-49) and the two
IndexError cases of ``recalculate_matrix`` when ``len(function)`` is not m or m+1.
"""
from __future__ import annotations

import numpy as np

from golden_util import dense_hash

PIVOT, OPTIMUM, INCORRECT, NOT_CONVERGE, FSHORT = 0, 1, 2, 3, 4
MESSAGES = {INCORRECT: "incorrect system", NOT_CONVERGE: "simplex method does not converge"}


def run_trajectory(T, n, m, flen, function, pick, pivot, cap):
    row = ["x%d" % k for k in range(1, m + 1)] + ["-b"]
    col = ["y%d" % k for k in range(1, n + 1)] + ["f"]

    def opt():
        vals = []
        for name in ("x1", "x2"):
            vals.append(float(T[col.index(name), m]) if name in col else 0)
        return vals

    steps = [{"hash": dense_hash(T, n, flen), "x1": 0, "x2": 0, "optimum": 0}]
    outcome = None
    for _ in range(cap):
        st, r, c = pick(T, n, m, flen)
        if st in MESSAGES:
            outcome = {"kind": "error", "message": MESSAGES[st]}
            break
        if st == FSHORT:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        if st == OPTIMUM:
            try:
                x1, x2 = opt()
                function[0] * x1 + function[1] * x2
            except IndexError:
                outcome = {"kind": "exception", "type": "IndexError"}
                break
            outcome = {"kind": "optimum"}
            break
        steps[-1]["i"], steps[-1]["j"] = r, c
        row[c], col[r] = col[r], row[c]
        if flen > m + 1 or (flen < m and c >= flen):
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        T = pivot(T, r, c)
        x1, x2 = opt()
        try:
            f = function[0] * x1 + function[1] * x2
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"hash": dense_hash(T, n, flen), "x1": x1, "x2": x2, "optimum": f})
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"steps": steps, "outcome": outcome, "row": row, "column": col, "T": T}
