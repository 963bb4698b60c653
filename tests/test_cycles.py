"""The opt-in cycle detector (simplex_mi355x.basis) on the reference's cycling fixtures."""
from __future__ import annotations

import pytest

from golden_util import load
from simplex_mi355x.basis import BasisTracker


def _layout(n, m, pivots):
    row = ["x%d" % k for k in range(1, m + 1)]
    col = ["y%d" % k for k in range(1, n + 1)]
    out = [(tuple(row), tuple(col))]
    for r, c in pivots:
        row[c], col[r] = col[r], row[c]          # simplex.py:152
        out.append((tuple(row), tuple(col)))
    return out


def _cycling():
    for name in ("degenerate.json", "random.json"):
        for k, rec in enumerate(load(name)):
            if rec["outcome"]["kind"] == "cap":
                yield f"{name}:{k}", rec


@pytest.mark.parametrize("label,rec", list(_cycling()), ids=[x[0] for x in _cycling()])
def test_tracker_agrees_with_explicit_label_layouts(label, rec):
    n, m = rec["n"], rec["m"]
    piv = [(s["i"], s["j"]) for s in rec["steps"][:-1]]
    lay = _layout(n, m, piv)
    first = {}
    expect = None
    for t, L in enumerate(lay):
        if L in first:
            expect = (first[L], t - first[L])
            break
        first[L] = t
    tr = BasisTracker(n, m)
    got = None
    for r, c in piv:
        got = tr.pivot(r, c)
        if got:
            break
    assert got == expect, (label, got, expect)


def test_known_period_two_cycle():
    rec = load("degenerate.json")[0]
    tr = BasisTracker(rec["n"], rec["m"])
    for s in rec["steps"][:-1]:
        if tr.pivot(s["i"], s["j"]):
            break
    assert tr.cycle == (3, 2)
