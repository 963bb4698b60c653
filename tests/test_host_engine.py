"""The host engine (``smx_host_*`` in libsmx.so, ``simplex_mi355x/host.py``): the drop-in
``SimplexMethod`` on a machine without an MI355X (``backend == "host"``; BASELINE.json
configs[0], the reference UI's flow main.py:308-313).  Runs in the CPU suite: every committed
golden fixture (made by importing /root/reference/src/simplex.py) through the product surface,
bit for bit, and the native chained loop against the C oracle.  Nothing here touches a GPU.
"""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import (dec, dec_input, dec_table, load, same_table, same_value, table_hash,
                         trajectory_cap, trajectory_cases)


def _sm(cons, func):
    import simplex
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cpu")
    assert sm.backend == "host"
    return sm


@pytest.mark.parametrize("name", list(load("examples.json")))
def test_host_examples_get_solution(name):
    """Every Info field of get_solution() for the reference's own example LPs."""
    import simplex
    case = load("examples.json")[name]
    cons, func = dec_input(case["input"])
    got = _sm(cons, func).get_solution()
    exp = case["solution"]
    ints = any(isinstance(x, int) for r in cons for x in r)
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        if e["kind"] == "error":
            assert isinstance(g, simplex.Error) and str(g) == e["message"]
            continue
        assert isinstance(g, simplex.Info)
        assert (g.row, g.column, g.i, g.j) == (e["row"], e["column"], e["i"], e["j"])
        assert same_table(g.table, dec_table(e["table"]), signed_zero=not ints)
        for key in ("x1", "x2", "optimum"):
            assert same_value(getattr(g, key), dec(e[key]), signed_zero=not ints)


def test_host_ui_flow_demo_lp():
    """main.py:308-313: floats in, SimplexMethod(y, c).get_solution(), the last Info read."""
    import simplex
    y = [[1.0, 1.0, -2.0], [-1.0, 1.0, 1.5], [1.0, -2.0, 4.0]]
    c = [-1.0, -1.0]
    res = simplex.SimplexMethod(y, c).get_solution()   # no device on this machine: host
    assert not isinstance(res[-1], simplex.Error)
    assert (res[-1].x1, res[-1].x2, res[-1].optimum) == (7.0, 5.5, -12.5)


def _trajectory(cons, func, cap):
    sm = _sm(cons, func)
    steps = [{"hash": table_hash(sm.table), "x1": 0, "x2": 0, "optimum": 0}]
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
        try:
            sm.recalculate_matrix()
            x1, x2 = sm.find_optimum()
            f = sm.f(x1, x2)
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"hash": table_hash(sm.table), "x1": x1, "x2": x2, "optimum": f})
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"steps": steps, "outcome": outcome, "row": sm.row, "column": sm.column}


CASES = list(trajectory_cases())


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_host_fixture_trajectories(case):
    label, cons, func, rec = case
    got = _trajectory(cons, func, trajectory_cap(rec))
    exp = rec["steps"]
    assert len(got["steps"]) == len(exp), (label, len(got["steps"]), len(exp))
    for k, (g, e) in enumerate(zip(got["steps"], exp)):
        assert g["hash"] == e["hash"], (label, "table differs at step", k)
        assert (g.get("i"), g.get("j")) == (e.get("i"), e.get("j")), (label, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(g[key], dec(e[key])), (label, k, key)
    assert got["outcome"] == rec["outcome"], label
    assert got["row"] == rec["row"] and got["column"] == rec["column"], label


def test_host_large256_trajectory():
    rec = load("large256.json")
    cons, func = dec_input(rec["input"])
    got = _trajectory(cons, func, trajectory_cap(rec))
    assert [s["hash"] for s in got["steps"]] == [s["hash"] for s in rec["steps"]]


@pytest.mark.parametrize("kind,n,m,k", [("uniform", 120, 90, 300), ("mixed", 100, 140, 300),
                                        ("degenerate", 64, 64, 200),
                                        ("degenerate_mixed", 50, 30, 200)])
def test_host_chained_loop_vs_oracle(kind, n, m, k):
    """solve(record_history=False): the native loop (smx_host_run) against the C oracle."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 3, n, m)
    sm = _sm(T[:n].tolist(), T[n, :m].tolist())
    out = sm.solve(record_history=False, max_pivots=k, chunk=64)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    D = sm._dev.download()
    assert np.array_equal(D[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(D[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
    if done < k:
        assert sm.status in ("optimum", "error")
    else:
        assert sm.status == "cap"
    assert len(out) >= 2


def test_host_is_never_chosen_with_a_device(monkeypatch):
    """With a HIP device present the default backend is the device (the host engine is opt-in
    there): simulate a device and check the selection rule."""
    import torch
    from simplex_mi355x import engine
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    assert engine._use_host(None) is False
    assert engine._use_host("cuda:0") is False
    assert engine._use_host("cpu") is True
