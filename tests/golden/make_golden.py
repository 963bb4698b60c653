"""Generate the committed golden fixtures by IMPORTING the reference solver.

Runs only in the build container, where ``/root/reference`` exists (the GPU box has no copy of
the reference; it only sees the JSON this script wrote).  Usage::

    python tests/golden/make_golden.py            # rewrites tests/golden/*.json

What is recorded (all floats as ``float.hex`` strings, Python ints as JSON ints):

* ``examples.json``   - the reference's own demo LP and the five commented LPs
  (simplex.py:205-238), as full ``get_solution()`` lists (every ``Info`` field, trailing ``Error``);
* ``random.json``     - seeded dense LPs (feasible-at-origin and mixed-sign ``b``, square and
  rectangular, 8..64), trajectory ``(i, j)`` per step, per-step SHA-256 of the table bytes,
  ``x1, x2, optimum`` per step, terminal outcome, final table for the small ones;
* ``ties.json``       - small LPs over {+-2, +-1, +-0.5, +-0.0, 3} that hammer the ratio-test ties;
* ``degenerate.json`` - integer degenerate LPs (the §8d config-5 generator) capped at K pivots;
* ``edge.json``       - NaN / inf entries, ``len(function)`` in {m-1, m+1}, m = 1, n = 1;
* ``large256.json``   - one 256x256 random LP, 300 pivots, per-step ``(i, j)`` and SHA-256.

The per-step loop for the capped cases is the body of ``get_solution`` (simplex.py:184-198)
driven through the reference's own ``pick_element`` / ``recalculate_matrix``.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import struct
import sys

import numpy as np

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))


def enc(v):
    if isinstance(v, bool):
        return v
    if isinstance(v, int):
        return v
    if isinstance(v, float):
        return float.hex(v)
    if v is None:
        return None
    raise TypeError(type(v))


CANON_NAN = float("nan")


def table_hash(table) -> str:
    """SHA-256 of the table's fp64 bytes, every NaN canonicalised (NaN payload and sign are not
    part of the contract: x86 and gfx950 propagate them differently)."""
    h = hashlib.sha256()
    for row in table:
        vals = [float(x) for x in row]
        vals = [v if v == v else CANON_NAN for v in vals]
        h.update(struct.pack("<%dd" % len(vals), *vals))
    return h.hexdigest()


def enc_table(table):
    return [[enc(x) for x in row] for row in table]


def load_reference():
    sys.path.insert(0, REF_SRC)
    import simplex  # noqa: E402  (the reference module)
    return simplex


def full_solution(simplex, constraints, function):
    sm = simplex.SimplexMethod([list(r) for r in constraints], list(function))
    out = []
    try:
        res = sm.get_solution()
    except Exception as exc:  # IndexError from f() when m < 2, etc. (simplex.py:49)
        return [{"kind": "exception", "type": type(exc).__name__}]
    for item in res:
        if isinstance(item, simplex.Error):
            out.append({"kind": "error", "message": str(item)})
        else:
            out.append({"kind": "info", "row": item.row, "column": item.column,
                        "table": enc_table(item.table), "i": item.i, "j": item.j,
                        "x1": enc(item.x1), "x2": enc(item.x2), "optimum": enc(item.optimum)})
    return out


def trajectory(simplex, constraints, function, cap, keep_final=False):
    """get_solution's loop (simplex.py:184-198) with a pivot cap; records hashes per step."""
    sm = simplex.SimplexMethod([list(r) for r in constraints], list(function))
    steps = [{"hash": table_hash(sm.table), "x1": enc(0), "x2": enc(0), "optimum": enc(0)}]
    outcome = None
    for _ in range(cap):
        try:
            ok, i, j, _e = sm.pick_element()
        except ValueError as exc:
            outcome = {"kind": "error", "message": str(exc)}
            break
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        if not ok:
            outcome = {"kind": "optimum"}
            break
        steps[-1]["i"], steps[-1]["j"] = i, j
        sm.recalculate_matrix()
        x1, x2 = sm.find_optimum()
        try:
            f = sm.f(x1, x2)
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"hash": table_hash(sm.table), "x1": enc(x1), "x2": enc(x2),
                      "optimum": enc(f)})
    if outcome is None:
        outcome = {"kind": "cap"}
    rec = {"steps": steps, "outcome": outcome, "row": sm.row, "column": sm.column}
    if keep_final:
        rec["final_table"] = enc_table(sm.table)
    return rec


def lp_uniform(rng, n, m, mixed=False):
    A = rng.uniform(-1.0, 1.0, size=(n, m))
    b = rng.uniform(-1.0, 1.0, size=n) if mixed else rng.uniform(0.1, 1.0, size=n)
    c = rng.uniform(-1.0, 1.0, size=m)
    cons = [list(map(float, A[i])) + [float(b[i])] for i in range(n)]
    return cons, list(map(float, c))


def lp_ties(rng, n, m):
    vals = np.array([2.0, -2.0, 1.0, -1.0, 0.5, -0.5, 0.0, -0.0, 3.0])
    A = rng.choice(vals, size=(n, m))
    b = rng.choice(vals, size=n)
    c = rng.choice(vals, size=m)
    cons = [list(map(float, A[i])) + [float(b[i])] for i in range(n)]
    return cons, list(map(float, c))


def lp_degenerate(rng, n, m, mixed=False):
    A = rng.integers(-2, 3, size=(n, m)).astype(float)
    if mixed:
        b = rng.integers(-2, 3, size=n).astype(float)
    else:
        b = np.where(rng.random(n) < 0.9, 0.0, rng.integers(1, 3, size=n).astype(float))
    c = rng.integers(-2, 3, size=m).astype(float)
    cons = [list(map(float, A[i])) + [float(b[i])] for i in range(n)]
    return cons, list(map(float, c))


EXAMPLES = {
    # simplex.py:231-234 (the __main__ demo; ints on purpose, as in the reference)
    "main": ([[1, 1, -2], [-1, 1, 1.5], [1, -2, 4]], [-1, -1]),
    # simplex.py:205-209
    "ex1": ([[-39.70, -96.00, 4060.80], [-45.50, 45.30, 600.60], [45.50, -7.40, -54.60],
             [24.20, 45.10, -1091.42]], [-1, -1]),
    # simplex.py:210-215
    "ex2": ([[12.50, -26.60, 726.78], [-26.40, -18.40, 1814.48], [-6, 41.80, -81.00],
             [22.30, 16.20, -780.76], [17.50, -3.60, -105.43]], [2.4, -1.15]),
    # simplex.py:216-223
    "ex3": ([[-39.00, 93.10, 113.10], [-45.50, 89.90, 250.25], [-45.50, 67.00, 441.35],
             [-45.50, 47.20, 746.20], [-45.50, 24.90, 1392.30], [-45.50, 12.90, 1810.90],
             [-45.50, 45.50, -45.50]], [-1, -2.45]),
    # simplex.py:224-225
    "ex4": ([[-1.00, -1.00, -1]], [-1, 0]),
    # simplex.py:226-229
    "ex5": ([[-45.50, 12.20, 1810.90], [-44.20, 56.30, -73.19], [2.50, -92.60, 3764.32]],
            [-1, -2.45]),
    # simplex.py:235-238 (commented alternative demo)
    "alt": ([[1, 1, -2], [-1, 1, 2], [0, -1, 2]], [-1, 0]),
}


def enc_input(cons, func):
    return {"constraints": [[enc(x) for x in r] for r in cons], "function": [enc(x) for x in func]}


def main():
    simplex = load_reference()
    out = {}

    ex = {}
    for name, (cons, func) in EXAMPLES.items():
        ex[name] = {"input": enc_input(cons, func), "solution": full_solution(simplex, cons, func)}
    out["examples.json"] = ex

    rnd = []
    rng = np.random.default_rng(20250620)
    shapes = [(8, 8), (12, 12), (16, 16), (24, 24), (32, 32), (48, 48), (64, 64), (40, 17),
              (17, 40), (5, 30), (30, 5)]
    for (n, m) in shapes:
        for mixed in (False, True):
            for rep in range(2 if n * m <= 1024 else 1):
                cons, func = lp_uniform(rng, n, m, mixed)
                rec = trajectory(simplex, cons, func, cap=1500, keep_final=(n * m <= 576))
                rec.update({"n": n, "m": m, "mixed": mixed, "input": enc_input(cons, func)})
                rnd.append(rec)
    out["random.json"] = rnd

    ties = []
    rng = np.random.default_rng(7)
    for k in range(240):
        n = int(rng.integers(1, 9))
        m = int(rng.integers(1, 7))
        cons, func = lp_ties(rng, n, m)
        rec = trajectory(simplex, cons, func, cap=60, keep_final=True)
        rec.update({"n": n, "m": m, "input": enc_input(cons, func)})
        ties.append(rec)
    out["ties.json"] = ties

    deg = []
    rng = np.random.default_rng(5)
    for (n, m, mixed) in [(16, 16, False), (16, 16, True), (32, 32, False), (32, 32, True),
                          (24, 40, False), (64, 64, False), (12, 6, True), (6, 12, True)]:
        for rep in range(3):
            cons, func = lp_degenerate(rng, n, m, mixed)
            rec = trajectory(simplex, cons, func, cap=120, keep_final=True)
            rec.update({"n": n, "m": m, "mixed": mixed, "input": enc_input(cons, func)})
            deg.append(rec)
    out["degenerate.json"] = deg

    edge = {}
    nan, inf = float("nan"), float("inf")
    cases = {
        # NaN in the entering column of the FIRST candidate row: the NaN ratio sticks
        "nan_first_candidate": ([[nan, -1.0, 1.0], [-1.0, 1.0, 2.0], [-2.0, 1.0, 1.0]], [-1.0, -1.0]),
        # NaN ratio on a later candidate row: ignored
        "nan_later_candidate": ([[-1.0, 1.0, 2.0], [nan, 1.0, 1.0], [-2.0, 1.0, 1.0]], [-1.0, -1.0]),
        "nan_b_first": ([[-1.0, 1.0, nan], [-1.0, 1.0, 2.0], [-2.0, 1.0, 1.0]], [-1.0, -1.0]),
        "inf_b": ([[-1.0, 1.0, inf], [-1.0, 1.0, 2.0], [-2.0, 1.0, 1.0]], [-1.0, -1.0]),
        "neg_inf_coeff": ([[-inf, 1.0, 3.0], [-1.0, 1.0, 2.0], [-2.0, 1.0, 1.0]], [-1.0, -1.0]),
        "nan_objective": ([[-1.0, 1.0, 2.0], [-2.0, 1.0, 1.0]], [nan, -1.0]),
        # len(function) == m + 1: the f-row has a real "-b" entry that is updated too
        "flen_m_plus_1": ([[-1.0, 1.0, 2.0], [1.0, -2.0, 1.0], [-2.0, -1.0, 6.0]], [-1.0, -1.0, 5.0]),
        # len(function) == m - 1 with no negative in it: the reference indexes past its end
        "flen_short_indexerror": ([[-1.0, 1.0, 1.0, 2.0], [1.0, -2.0, 1.0, 1.0]], [1.0, 2.0]),
        # len(function) == m - 1 with a negative inside it: runs normally
        "flen_short_ok": ([[-1.0, 1.0, 1.0, 2.0], [1.0, -2.0, -1.0, 1.0], [-1.0, -1.0, -1.0, 4.0]],
                          [-1.0, 2.0]),
        # m == 1: f() indexes function[1] -> IndexError (simplex.py:49)
        "m_equals_1": ([[-1.0, 2.0], [-2.0, 3.0]], [-1.0]),
        "n_equals_1": ([[-1.0, -2.0, 4.0]], [-1.0, -3.0]),
        "unbounded": ([[1.0, -1.0, 2.0], [2.0, 1.0, 1.0]], [-1.0, 1.0]),
        "already_optimal": ([[1.0, -1.0, 2.0], [2.0, 1.0, 1.0]], [1.0, 1.0]),
        "zero_column": ([[0.0, -1.0, 2.0], [0.0, 1.0, 1.0]], [-1.0, 1.0]),
        "neg_zero_b": ([[-1.0, 1.0, -0.0], [-1.0, -1.0, 2.0]], [-1.0, -1.0]),
        "incorrect_system": ([[-1.0, -1.0, -1.0], [1.0, 1.0, 2.0]], [-1.0, -1.0]),
    }
    for name, (cons, func) in cases.items():
        edge[name] = {"input": enc_input(cons, func),
                      "solution": full_solution_capped(simplex, cons, func, cap=40)}
    out["edge.json"] = edge

    rng = np.random.default_rng(256)
    cons, func = lp_uniform(rng, 255, 255)
    rec = trajectory(simplex, cons, func, cap=300)
    rec.update({"n": 255, "m": 255, "generator": "uniform A~U(-1,1) b~U(0.1,1) c~U(-1,1)",
                "input": enc_input(cons, func)})
    out["large256.json"] = rec

    for fname, obj in out.items():
        with open(os.path.join(HERE, fname), "w") as fh:
            json.dump(obj, fh, separators=(",", ":"))
        print(fname, os.path.getsize(os.path.join(HERE, fname)))


def full_solution_capped(simplex, cons, func, cap):
    """Like full_solution, but refuses to hang on cycling inputs (runs trajectory first)."""
    probe = trajectory(simplex, cons, func, cap=cap)
    if probe["outcome"]["kind"] == "cap":
        probe["capped"] = True
        return {"trajectory": probe}
    return {"full": full_solution(simplex, cons, func), "trajectory": probe}


if __name__ == "__main__":
    if not os.path.isdir(REF_SRC):
        print("reference not present; fixtures are committed, nothing to do")
        sys.exit(0)
    main()
