"""GPU: batched small LPs (one wavefront per LP) against the reference's fixtures and the oracle."""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import pytest

from golden_util import (dec, dec_input, dec_table, load, same_table, same_value, table_hash,
                         trajectory_cap, trajectory_cases)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


def test_batch_examples_full_solution():
    from simplex_mi355x.batch import solve_batch
    import simplex
    ex = load("examples.json")
    names = list(ex)
    probs = [dec_input(ex[k]["input"]) for k in names]
    results, statuses = solve_batch(probs, max_pivots=50)
    for name, got in zip(names, results):
        exp = ex[name]["solution"]
        # int inputs (the demo LP) go through SimplexMethod, which reproduces the reference's
        # int first pivot: zero signs included
        assert len(got) == len(exp), name
        for g, e in zip(got, exp):
            if e["kind"] == "error":
                assert isinstance(g, simplex.Error) and str(g) == e["message"]
                continue
            assert (g.row, g.column, g.i, g.j) == (e["row"], e["column"], e["i"], e["j"])
            assert same_table(g.table, dec_table(e["table"]), signed_zero=True), name
            for key in ("x1", "x2", "optimum"):
                assert same_value(getattr(g, key), dec(e[key]), signed_zero=True)


def test_batch_every_trajectory_fixture():
    """All ~320 capped trajectory fixtures in as few launches as there are distinct caps."""
    from simplex_mi355x.batch import solve_batch
    import simplex
    groups = defaultdict(list)
    for label, cons, func, rec in trajectory_cases():
        groups[trajectory_cap(rec)].append((label, cons, func, rec))
    checked = 0
    for cap, cases in groups.items():
        results, statuses = solve_batch([(c, f) for _, c, f, _ in cases], max_pivots=cap)
        for (label, cons, func, rec), got, st in zip(cases, results, statuses):
            outcome = rec["outcome"]
            if outcome["kind"] == "exception":
                assert isinstance(got, IndexError) or st == "exception" or \
                    len(got) - 1 < len(rec["steps"]), label
                continue
            infos = [g for g in got if isinstance(g, simplex.Info)]
            assert [table_hash(i.table) for i in infos] == [s["hash"] for s in rec["steps"]], label
            for i, s in zip(infos, rec["steps"]):
                assert (i.i, i.j) == (s.get("i"), s.get("j")), label
                for key in ("x1", "x2", "optimum"):
                    assert same_value(getattr(i, key), dec(s[key])), (label, key)
            if outcome["kind"] == "error":
                assert str(got[-1]) == outcome["message"] and st == "error"
            elif outcome["kind"] == "optimum":
                assert st == "optimum"
            else:
                assert st == "cap"
            assert infos[-1].row == rec["row"] and infos[-1].column == rec["column"]
            checked += 1
    assert checked > 250


def test_batch_large_random_vs_oracle():
    """20 000 UI-shaped LPs (m = 2, n = 3..20, mixed signs) in one launch; a sample of them
    checked bit for bit (final table, pivot log, status) against the C oracle."""
    from simplex_mi355x.batch import solve_batch
    from oracle import c_oracle
    rng = np.random.default_rng(123)
    probs = []
    for k in range(20000):
        n = int(rng.integers(3, 21))
        A = rng.uniform(-50, 50, size=(n, 2))
        b = rng.uniform(-100, 400, size=n)
        c = rng.uniform(-3, 3, size=2)
        probs.append(([list(map(float, A[i])) + [float(b[i])] for i in range(n)],
                      list(map(float, c))))
    results, statuses = solve_batch(probs, max_pivots=64, history=False)
    st_code = {"optimum": 1, "error": None, "cap": 0}
    for k in range(0, 20000, 97):
        cons, func = probs[k]
        n = len(cons)
        T = np.zeros((n + 1, 3))
        T[:n] = cons
        T[n, :2] = func
        Tref, st, done, log = c_oracle.run(T, n, 2, 2, 64)
        got = results[k]
        final = got[1]
        assert np.array_equal(np.array(final.table[:n]).view(np.int64), Tref[:n].view(np.int64))
        if statuses[k] == "optimum":
            assert st == 1
        elif statuses[k] == "error":
            assert st in (2, 3) and str(got[-1]) == ("incorrect system" if st == 2 else
                                                     "simplex method does not converge")
        else:
            assert st == 0 and done == 64


def test_batch_no_history_matches_solve():
    from simplex_mi355x.batch import solve_batch
    import simplex
    recs = [r for r in load("random.json") if r["outcome"]["kind"] != "cap" and r["n"] < 64]
    probs = [dec_input(r["input"]) for r in recs]
    results, statuses = solve_batch(probs, max_pivots=2000, history=False)
    for (cons, func), got in zip(probs, results):
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
        exp = sm.solve(record_history=False, chunk=64)
        assert len(got) == len(exp)
        assert (got[0].i, got[0].j) == (exp[0].i, exp[0].j)
        assert same_table(got[1].table, exp[1].table)
        assert same_value(got[1].optimum, exp[1].optimum)
        assert got[1].row == exp[1].row and got[1].column == exp[1].column


def test_batch_int_inputs_signed_zeros():
    """Int and mixed int / float LPs (tests/golden/intzero.json, made by importing the reference):
    solve_batch returns exactly SimplexMethod's get_solution, signed zeros of the int first pivot
    included (such problems leave the batch kernel for SimplexMethod)."""
    from simplex_mi355x.batch import solve_batch
    import simplex
    cases = [c for c in load("intzero.json")
             if c["kind"] != "int_large" and c["outcome"]["kind"] != "cap"][::2]
    probs = [dec_input(c["input"]) for c in cases]
    results, statuses = solve_batch(probs, max_pivots=64)
    checked = 0
    for case, got in zip(cases, results):
        steps = case["steps"]
        infos = [g for g in got if not isinstance(g, simplex.Error)]
        assert len(infos) == len(steps)
        if case["outcome"]["kind"] == "error":
            assert str(got[-1]) == case["outcome"]["message"]
        for g, e in zip(infos, steps):
            assert (g.i, g.j) == (e.get("i"), e.get("j"))
            assert same_table(g.table, dec_table(e["table"]), signed_zero=True)
        checked += 1
    assert checked > 20
