"""Generate ``tests/golden/intzero.json`` by IMPORTING the reference solver: LPs given as Python
ints (and ints mixed with floats, including -0.0), whose first pivot the reference computes in
int arithmetic (simplex.py:155-175) -- the case where a zero result can carry the other sign
than in fp64.  Runs only in the build container, where ``/root/reference`` exists::

    python tests/golden/make_intzero.py

Each record: the input (ints as JSON ints, floats as ``float.hex``), and per step of
get_solution's loop (simplex.py:184-198, capped) the pivot ``(i, j)``, the full table (signs of
zeros included: ``float.hex(-0.0)`` is ``-0x0.0p+0``), ``x1, x2, optimum``, and the outcome.
``sign_differs``: whether the reference's tables differ from an all-float run of the same LP in
any zero's sign (the cases this fixture exists for).
"""
from __future__ import annotations

import copy
import json
import math
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF_SRC, enc, enc_input, enc_table, load_reference  # noqa: E402


def run(simplex, cons, func, cap):
    sm = simplex.SimplexMethod(copy.deepcopy(cons), list(func))
    steps = [{"table": enc_table(sm.table), "x1": enc(0), "x2": enc(0), "optimum": enc(0)}]
    raw = [copy.deepcopy(sm.table)]
    outcome = None
    for _ in range(cap):
        try:
            ok, i, j, _e = sm.pick_element()
        except ValueError as exc:
            outcome = {"kind": "error", "message": str(exc)}
            break
        if not ok:
            outcome = {"kind": "optimum"}
            break
        steps[-1]["i"], steps[-1]["j"] = i, j
        sm.recalculate_matrix()
        x1, x2 = sm.find_optimum()
        steps.append({"table": enc_table(sm.table), "x1": enc(x1), "x2": enc(x2),
                      "optimum": enc(sm.f(x1, x2))})
        raw.append(copy.deepcopy(sm.table))
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"steps": steps, "outcome": outcome, "row": sm.row, "column": sm.column}, raw


def zero_signs(tables):
    return [[[math.copysign(1.0, v) if v == 0 else 0.0 for v in r] for r in t] for t in tables]


def main():
    simplex = load_reference()
    rnd = random.Random(20261017)
    cases = []
    pools = {
        "int": [0, 0, 0, 1, -1, 2, -2, 3, -3, 5, 7],
        "mixed": [0, 0, 1, -1, 2, -3, 5, 0.0, -0.0, 1.5, -2.5, 0.25],
    }
    want = {"int": 70, "mixed": 70}
    for kind, pool in pools.items():
        made = tries = 0
        while made < want[kind] and tries < 5000:
            tries += 1
            n, m = rnd.randint(2, 7), rnd.randint(2, 7)
            cons = [[rnd.choice(pool) for _ in range(m + 1)] for _ in range(n)]
            fpool = [0, -1, -2, 1, 3] if kind == "int" else [0, -1, -2, 1, 0.0, -0.0, -1.5]
            func = [rnd.choice(fpool) for _ in range(m)]
            rec, raw = run(simplex, cons, func, cap=30)
            if len(rec["steps"]) < 2:
                continue                          # no pivot: nothing int-specific to pin
            fl = [[float(x) for x in r] for r in cons]
            _, raw_f = run(simplex, fl, [float(x) for x in func], cap=30)
            differs = zero_signs(raw) != zero_signs(raw_f)
            if made >= want[kind] // 2 and not differs:
                continue                          # keep the second half to the sign cases
            rec.update({"kind": kind, "n": n, "m": m, "input": enc_input(cons, func),
                        "sign_differs": differs})
            cases.append(rec)
            made += 1
    # larger int tables (the block / resident / sharded paths at forced policies on the GPU):
    # integer-valued, ~30 % zeros, b >= 0 feasible at the origin plus a few negative rows
    for (n, m, seed) in [(24, 24, 1), (40, 33, 2), (64, 64, 3)]:
        r2 = random.Random(seed)
        cons = [[r2.choice([0, 0, 0, 1, -1, 2, -2, 3, 4, -5]) for _ in range(m)]
                + [r2.choice([0, 1, 2, 3, -1])] for _ in range(n)]
        func = [r2.choice([0, -1, -2, -3, 1]) for _ in range(m)]
        rec, raw = run(simplex, cons, func, cap=12)
        fl = [[float(x) for x in r] for r in cons]
        _, raw_f = run(simplex, fl, [float(x) for x in func], cap=12)
        rec.update({"kind": "int_large", "n": n, "m": m, "input": enc_input(cons, func),
                    "sign_differs": zero_signs(raw) != zero_signs(raw_f)})
        cases.append(rec)
    path = os.path.join(HERE, "intzero.json")
    with open(path, "w") as fh:
        json.dump(cases, fh, separators=(",", ":"))
    print(path, os.path.getsize(path), len(cases), "cases,",
          sum(c["sign_differs"] for c in cases), "with zero signs differing from fp64")


if __name__ == "__main__":
    if not os.path.isdir(REF_SRC):
        print("reference not present; fixtures are committed, nothing to do")
        sys.exit(0)
    main()
