"""Pin the CPU oracle (pure-Python, numpy and C restatements) to the reference's own outputs.

The fixtures were produced by importing /root/reference/src/simplex.py (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import (dec, dec_input, dec_table, load, same_table, same_value,
                         table_hash, trajectory_cap, trajectory_cases)
from dense_driver import run_trajectory
from oracle import c_oracle, numpy_oracle, restated

CASES = list(trajectory_cases())


def _check_steps(label, got, rec):
    exp = rec["steps"]
    assert len(got["steps"]) == len(exp), (label, len(got["steps"]), len(exp))
    for k, (g, e) in enumerate(zip(got["steps"], exp)):
        assert g["hash"] == e["hash"], (label, "table differs at step", k)
        assert g.get("i") == e.get("i") and g.get("j") == e.get("j"), (label, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(g[key], dec(e[key])), (label, k, key, g[key], e[key])
    assert got["outcome"] == rec["outcome"], (label, got["outcome"], rec["outcome"])
    assert got["row"] == rec["row"] and got["column"] == rec["column"], label


@pytest.mark.parametrize("name", list(load("examples.json")))
def test_restated_examples_full_solution(name):
    case = load("examples.json")[name]
    cons, func = dec_input(case["input"])
    s = restated.Solver([list(r) for r in cons], list(func))
    got = s.get_solution()
    exp = case["solution"]
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert g["kind"] == e["kind"]
        if e["kind"] == "error":
            assert g["message"] == e["message"]
            continue
        assert g["row"] == e["row"] and g["column"] == e["column"]
        assert g["i"] == e["i"] and g["j"] == e["j"]
        assert same_table(g["table"], dec_table(e["table"]))
        for key in ("x1", "x2", "optimum"):
            assert same_value(g[key], dec(e[key]))


def _restated_trajectory(cons, func, cap):
    s = restated.Solver([list(r) for r in cons], list(func))
    steps = [{"hash": table_hash(s.table), "x1": 0, "x2": 0, "optimum": 0}]
    outcome = None
    for _ in range(cap):
        try:
            ok, i, j, _e = s.pick_element()
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
        try:
            s.recalculate_matrix()
            x1, x2 = s.find_optimum()
            f = s.f(x1, x2)
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"hash": table_hash(s.table), "x1": x1, "x2": x2, "optimum": f})
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"steps": steps, "outcome": outcome, "row": s.row, "column": s.column}


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_restated_trajectories(case):
    label, cons, func, rec = case
    _check_steps(label, _restated_trajectory(cons, func, trajectory_cap(rec)), rec)


def _dense(cons, func):
    T, n, m, flen = numpy_oracle.to_dense(cons, func)
    return T, n, m, flen


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_numpy_oracle_trajectories(case):
    label, cons, func, rec = case
    T, n, m, flen = _dense(cons, func)
    got = run_trajectory(T, n, m, flen, func, numpy_oracle.pick, numpy_oracle.pivot,
                         trajectory_cap(rec))
    _check_steps(label, got, rec)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_c_oracle_trajectories(case):
    label, cons, func, rec = case
    T, n, m, flen = _dense(cons, func)
    got = run_trajectory(T, n, m, flen, func, c_oracle.pick,
                         lambda T, r, c: c_oracle.pivot(T, r, c), trajectory_cap(rec))
    _check_steps(label, got, rec)


@pytest.mark.parametrize("which", ["numpy", "c"])
def test_large256_trajectory(which):
    rec = load("large256.json")
    cons, func = dec_input(rec["input"])
    T, n, m, flen = _dense(cons, func)
    if which == "numpy":
        pk, pv = numpy_oracle.pick, numpy_oracle.pivot
    else:
        pk, pv = c_oracle.pick, (lambda T, r, c: c_oracle.pivot(T, r, c, threads=4))
    got = run_trajectory(T, n, m, flen, func, pk, pv, trajectory_cap(rec))
    _check_steps("large256", got, rec)


def test_c_run_matches_numpy_run():
    """The C ping-pong driver reproduces the numpy trajectory and final table bitwise."""
    rec = load("large256.json")
    cons, func = dec_input(rec["input"])
    T, n, m, flen = _dense(cons, func)
    Tc, stc, donec, logc = c_oracle.run(T, n, m, flen, 200, threads=2)
    Tn = T.copy()
    logn = []
    Tn, stn, donen = numpy_oracle.run(Tn, n, m, flen, 200, log=logn)
    assert (stc, donec) == (stn, donen)
    assert np.array_equal(logc, np.array(logn, dtype=np.int32))
    assert np.array_equal(Tc.view(np.int64), Tn.view(np.int64))
