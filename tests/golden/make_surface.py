"""Generate ``surface.json`` by IMPORTING the reference solver: per-step golden vectors for the
parts of the drop-in surface that the trajectory fixtures do not pin (tests/test_surface.py,
tests/test_gpu_parity.py):

* ``print_table()`` (simplex.py:41-46) -- the exact text the reference prints before the first
  pivot and after every pivot (labels, tabs, ``round(val, 6)``);
* ``step()`` -- the build's addition (one ``pick_element`` + pivot) has no reference twin; its
  return value is pick_element's tuple (simplex.py:91, :101-103, :141) and its effect
  recalculate_matrix's (simplex.py:143-177), so the vectors record the reference's
  ``pick_element()`` tuple at every step, then call ``recalculate_matrix()``.

Runs only in the build container, where ``/root/reference`` exists (the GPU box sees only the
JSON).  Usage: ``python tests/golden/make_surface.py``.
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import (EXAMPLES, REF_SRC, enc, enc_input, load_reference,  # noqa: E402
                         lp_degenerate, lp_ties, lp_uniform)


def _printed(sm) -> str:
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        sm.print_table()
    return buf.getvalue()


def surface_case(simplex, cons, func, cap):
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
    steps = [{"printed": _printed(sm)}]
    outcome = None
    for _ in range(cap):
        try:
            res = sm.pick_element()
        except ValueError as exc:
            outcome = {"kind": "error", "message": str(exc)}
            break
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps[-1]["pick"] = [bool(res[0])] + [enc(x) for x in res[1:]]
        if not res[0]:
            outcome = {"kind": "optimum"}
            break
        try:
            sm.recalculate_matrix()
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"printed": _printed(sm)})
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"input": enc_input(cons, func), "steps": steps, "outcome": outcome,
            "row": sm.row, "column": sm.column}


def main():
    simplex = load_reference()
    out = {}
    # the reference's example LPs, as floats (the UI converts its inputs, main.py:311)
    for name, (cons, func) in EXAMPLES.items():
        cons = [[float(x) for x in r] for r in cons]
        func = [float(x) for x in func]
        out[name] = surface_case(simplex, cons, func, cap=40)
    nan, inf = float("nan"), float("inf")
    out["nan_inf"] = surface_case(simplex, [[nan, -1.0, 1.0], [-1.0, inf, 2.0],
                                            [-2.0, 1.0, 1.0]], [-1.0, -1.0], cap=10)
    out["tiny_values"] = surface_case(simplex, [[1e-9, -3.0, 1e-7], [-2.5e-7, 1.0, 7.1234567],
                                                [-2.0, 1e12, 1.0]], [-1.0, -1.0], cap=10)
    rng = np.random.default_rng(4141)
    for k in range(12):
        cons, func = lp_ties(rng, int(rng.integers(2, 7)), int(rng.integers(2, 6)))
        out[f"ties{k}"] = surface_case(simplex, cons, func, cap=30)
    for k in range(4):
        cons, func = lp_uniform(rng, 6 + 3 * k, 5 + 2 * k, mixed=bool(k & 1))
        out[f"uniform{k}"] = surface_case(simplex, cons, func, cap=60)
    for k in range(4):
        cons, func = lp_degenerate(rng, 8, 6, mixed=bool(k & 1))
        out[f"degenerate{k}"] = surface_case(simplex, cons, func, cap=30)
    path = os.path.join(HERE, "surface.json")
    with open(path, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("surface.json", os.path.getsize(path), len(out), "cases")


if __name__ == "__main__":
    if not os.path.isdir(REF_SRC):
        print("reference not present; fixtures are committed, nothing to do")
        sys.exit(0)
    main()
