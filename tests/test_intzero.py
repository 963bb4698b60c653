"""Integer inputs: the reference keeps the caller's Python ints until its first pivot and computes
that pivot in int arithmetic (simplex.py:155-175), where some zero results take the other sign
than in fp64.  ``tests/golden/intzero.json`` (made by importing the reference,
``tests/golden/make_intzero.py``): 143 int and mixed int / float LPs, every step's full table
with the signs of zeros, 120 of them differing from an all-float run.  Checked bit for bit,
signed zeros included, through the oracle restatement, the host engine (CPU suite) and every
device path (``-m gpu``: eager and lazy get_solution, chained solve with the launch chain, the
LDS-resident loop and block pivots, row-sharded devices).
"""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import dec, dec_input, dec_table, load, same_table, same_value

CASES = load("intzero.json")
SMALL = [k for k, c in enumerate(CASES) if c["kind"] != "int_large"]
LARGE = [k for k, c in enumerate(CASES) if c["kind"] == "int_large"]


def _check_solution(got, case, simplex):
    steps = case["steps"]
    infos = [g for g in got if not isinstance(g, simplex.Error)]
    assert len(infos) == len(steps), (len(infos), len(steps))
    for k, (g, e) in enumerate(zip(infos, steps)):
        assert (g.i, g.j) == (e.get("i"), e.get("j")), k
        assert same_table(g.table, dec_table(e["table"]), signed_zero=True), k
        for key in ("x1", "x2", "optimum"):
            assert same_value(getattr(g, key), dec(e[key]), signed_zero=True), (k, key)
    if case["outcome"]["kind"] == "error":
        assert isinstance(got[-1], simplex.Error)
        assert str(got[-1]) == case["outcome"]["message"]


def _cap(case):
    # get_solution(max_pivots) stops at the cap exactly where the fixture's capped loop did
    return len(case["steps"]) - 1 if case["outcome"]["kind"] == "cap" else None


def test_fixture_has_sign_cases():
    assert sum(c["sign_differs"] for c in CASES) >= 100
    assert {c["kind"] for c in CASES} == {"int", "mixed", "int_large"}


@pytest.mark.parametrize("k", range(len(CASES)))
def test_oracle_restatement_int_semantics(k):
    """The oracle restatement on the caller's ints (Python arithmetic, as simplex.py) reproduces
    the reference's tables, signed zeros included."""
    from oracle import restated
    case = CASES[k]
    cons, func = dec_input(case["input"])
    s = restated.Solver([list(r) for r in cons], list(func))
    for k2, e in enumerate(case["steps"]):
        assert same_table(s.table, dec_table(e["table"]), signed_zero=True), k2
        if "i" not in e:
            break
        st = restated.pick(s.table, s.n, s.m, s.invalid_index)
        assert st[0] == "pivot" and (st[1], st[2]) == (e["i"], e["j"])
        s.table = restated.pivot(s.table, st[1], st[2])


def test_int_entries_mask():
    from simplex_mi355x.engine import _int_entries
    d = np.zeros((3, 3))
    assert _int_entries([[1.0, 2.0, 3.0], [0.5, 1.5, 2.0]], [1.0, 2.0], 2, d) is None
    assert _int_entries([[1, 2, 3], [0, True, 2]], [1, 2], 2, d) is True
    assert _int_entries([np.array([1, 2, 3]), [np.int64(0), 1, 2]], [1, 2], 2, d) is True
    mk = _int_entries([[1, 2.0, 3], [0.5, 1.5, 2.0]], [1.0, -0.0], 2, d)
    assert mk.tolist() == [[1, 0, 1], [0, 0, 0], [0, 0, 0]]
    big = np.full((3, 3), float(1 << 26))
    with pytest.warns(RuntimeWarning, match="2\\^26"):
        _int_entries([[1 << 26, 1, 1], [1, 1, 1]], [1, 1], 2, big)


@pytest.mark.parametrize("k", SMALL + LARGE)
def test_host_engine_get_solution(k):
    import simplex
    case = CASES[k]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cpu")
    _check_solution(sm.get_solution(max_pivots=_cap(case)), case, simplex)


@pytest.mark.parametrize("k", SMALL[::7] + LARGE)
def test_host_engine_chained_solve(k):
    """solve(record_history=False): the int table's first pivot runs alone, then the chain."""
    import simplex
    case = CASES[k]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cpu")
    out = sm.solve(record_history=False, max_pivots=_cap(case), chunk=5)
    last = case["steps"][-1]
    assert same_table(out[1].table, dec_table(last["table"]), signed_zero=True)


def test_host_engine_float_input_unchanged():
    """An all-float copy of an int LP keeps fp64's zero signs (no fix applied)."""
    import simplex
    case = next(c for c in CASES if c["sign_differs"] and c["kind"] == "int")
    cons, func = dec_input(case["input"])
    fl = simplex.SimplexMethod([[float(x) for x in r] for r in cons], [float(x) for x in func],
                               device="cpu")
    got = fl.get_solution(max_pivots=_cap(case))
    ref = [dec_table(e["table"]) for e in case["steps"]]
    assert all(same_table(g.table, t, signed_zero=False) for g, t in zip(got, ref))
    assert not all(same_table(g.table, t, signed_zero=True) for g, t in zip(got, ref))


# ---- device paths ----------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("k", SMALL + LARGE)
def test_gpu_get_solution_eager(k):
    import simplex
    case = CASES[k]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cuda:0")
    assert sm.backend == "hip"
    _check_solution(sm.get_solution(max_pivots=_cap(case), lazy=False), case, simplex)


@pytest.mark.gpu
@pytest.mark.parametrize("k", SMALL[::5] + LARGE)
def test_gpu_get_solution_lazy(k):
    """The chained loop with device history: first pivot alone + fix, x-ring of pivot 0 re-read,
    tables replayed from the checkpoint with the fix."""
    import simplex
    case = CASES[k]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cuda:0")
    got = sm.get_solution(max_pivots=_cap(case), lazy=True, chunk=4)
    # the chunks realign after the lone first pivot: a checkpoint every 4 pivots, not only at 0
    hist = got[0]._history
    assert sorted(hist.ckpt) == [s for s in range(0, sm.pivots + 1, 4)], sorted(hist.ckpt)
    _check_solution(got, case, simplex)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["launch", "resident", "block"])
@pytest.mark.parametrize("k", SMALL[::9] + LARGE)
def test_gpu_chained_solve_paths(k, path):
    import simplex
    from simplex_mi355x import _lib
    case = CASES[k]
    cons, func = dec_input(case["input"])
    prev_r = _lib.tune_resident(0 if path == "resident" else -1)
    prev_b = _lib.tune_block(4 if path == "block" else 1)
    try:
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cuda:0")
        assert (sm._dev.block_plan() is not None) == (path == "block")
        assert (sm._dev.resident_plan() is not None) == (path == "resident")
        out = sm.solve(record_history=False, max_pivots=_cap(case), chunk=6)
        last = case["steps"][-1]
        assert same_table(out[1].table, dec_table(last["table"]), signed_zero=True)
        assert sm.pivot_log == [(e["i"], e["j"]) for e in case["steps"][:-1]]
    finally:
        _lib.tune_resident(prev_r)
        _lib.tune_block(prev_b)


@pytest.mark.gpu
@pytest.mark.parametrize("k", SMALL[::11] + LARGE)
def test_gpu_row_sharded(k):
    """devices=[0, 0] (two row blocks, copy exchange): eager get_solution and chained solve."""
    import simplex
    case = CASES[k]
    cons, func = dec_input(case["input"])
    if case["n"] < 2:
        pytest.skip("one constraint row")
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=["cuda:0", "cuda:0"])
    _check_solution(sm.get_solution(max_pivots=_cap(case), lazy=False), case, simplex)
    sm2 = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=["cuda:0", "cuda:0"])
    out = sm2.solve(record_history=False, max_pivots=_cap(case), chunk=5)
    assert same_table(out[1].table, dec_table(case["steps"][-1]["table"]), signed_zero=True)
