"""The rest of the drop-in surface, pinned per step to vectors made by importing the reference
(tests/golden/make_surface.py -> surface.json):

* ``print_table()`` (simplex.py:41-46): the exact printed text before the first pivot and after
  every pivot (labels, tabs, round(val, 6), NaN/inf, tiny and huge values);
* ``step()`` -- the build's addition (north_star's step()/solve() surface): its return value is the
  reference's ``pick_element()`` tuple at that step (simplex.py:91, :101-103, :141) and its effect
  ``recalculate_matrix()``'s (the next print_table and the labels); it raises the reference's
  ValueError strings (simplex.py:89, :139).

Every engine: ``host`` (CPU suite), ``hip`` and ``sharded`` (three row blocks,
``devices=[0, 0, 0]``) on the MI355X (-m gpu).
"""
from __future__ import annotations

import contextlib
import io

import pytest

from golden_util import dec, dec_input, load

SURFACE = load("surface.json")
BACKENDS = [pytest.param("host", id="host"),
            pytest.param("hip", id="hip", marks=pytest.mark.gpu),
            pytest.param("sharded", id="sharded", marks=pytest.mark.gpu)]


def _sm(cons, func, backend):
    import simplex
    if backend in ("hip", "sharded"):
        import torch
        if not torch.cuda.is_available():
            pytest.skip("needs an MI355X")
        if backend == "hip":
            sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cuda:0")
        else:   # three row blocks on the one GPU of the test box (copy exchange)
            sm = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=[0, 0, 0])
    else:
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func), device="cpu")
    assert sm.backend == backend
    return sm


def _printed(sm) -> str:
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        sm.print_table()
    return buf.getvalue()


def _same(a, b):
    if isinstance(a, float) and isinstance(b, float) and a != a and b != b:
        return True
    return type(a) is type(b) and a == b and str(a) == str(b)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("name", list(SURFACE))
def test_step_and_print_table(name, backend):
    rec = SURFACE[name]
    cons, func = dec_input(rec["input"])
    sm = _sm(cons, func, backend)
    steps = rec["steps"]
    outcome = None
    for k, st in enumerate(steps):
        assert _printed(sm) == st["printed"], (name, k)
        if "pick" not in st:
            break
        exp = [st["pick"][0]] + [dec(x) for x in st["pick"][1:]]
        got = sm.step()
        assert len(got) == 4 and got[0] is exp[0], (name, k, got, exp)
        for g, e in zip(got[1:], exp[1:]):
            assert _same(g, e), (name, k, got, exp)
        if not got[0]:
            outcome = {"kind": "optimum"}
            break
    if outcome is None and rec["outcome"]["kind"] == "error":
        with pytest.raises(ValueError) as ei:
            sm.step()
        assert str(ei.value) == rec["outcome"]["message"]
        outcome = rec["outcome"]
    if rec["outcome"]["kind"] == "optimum":
        assert outcome == {"kind": "optimum"}
    assert sm.row == rec["row"] and sm.column == rec["column"]
