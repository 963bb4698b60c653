"""GPU: row sharding behind the drop-in surface -- ``SimplexMethod(..., devices=[...])``
(simplex_mi355x/multi.py, the native multi-device driver smx_mshard_run, include/smx.h).

The reference's only caller is ``SimplexMethod(y, c).get_solution()`` (main.py:313 ->
simplex.py:179-199).  On the one-GPU test box the ranks share device 0 (``devices=[0, 0, 0, 0]``),
so the exchange is the event-ordered copy form of smx_mshard_run; the kernels, the per-rank
buffers and streams and the protocol are those of a multi-GPU run (distinct devices exchange by a
grouped RCCL all-gather instead).  Bit for bit against the committed fixtures (made by importing
/root/reference/src/simplex.py), the C oracle and the single-device engine.
"""
from __future__ import annotations

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


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name", list(load("examples.json")))
def test_multi_examples_get_solution(name, world):
    """The UI call, main.py:313, on row blocks: every Info field of get_solution()."""
    import simplex
    case = load("examples.json")[name]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=[0] * world)
    assert sm.backend == "sharded" and sm._dev.exchange == "copy"
    got = sm.get_solution()
    exp = case["solution"]
    ints = any(isinstance(x, int) for r in cons for x in r)
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        if e["kind"] == "error":
            assert isinstance(g, simplex.Error) and str(g) == e["message"]
            continue
        assert (g.row, g.column, g.i, g.j) == (e["row"], e["column"], e["i"], e["j"])
        assert same_table(g.table, dec_table(e["table"]), signed_zero=not ints)
        for key in ("x1", "x2", "optimum"):
            assert same_value(getattr(g, key), dec(e[key]), signed_zero=not ints)


CASES = [c for k, c in enumerate(trajectory_cases()) if k % 5 == 0]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_multi_fixture_trajectories(case):
    """pick_element / recalculate_matrix / find_optimum on 3 row blocks, every step's table hash
    and (i, j, x1, x2, optimum) against the fixtures."""
    import simplex
    label, cons, func, rec = case
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=[0, 0, 0])
    steps = [{"hash": table_hash(sm.table), "x1": 0, "x2": 0, "optimum": 0}]
    outcome = None
    for _ in range(trajectory_cap(rec)):
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
    outcome = outcome or {"kind": "cap"}
    exp = rec["steps"]
    assert len(steps) == len(exp), (label, len(steps), len(exp))
    for k, (g, e) in enumerate(zip(steps, exp)):
        assert g["hash"] == e["hash"], (label, k)
        assert (g.get("i"), g.get("j")) == (e.get("i"), e.get("j")), (label, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(g[key], dec(e[key])), (label, k, key)
    assert outcome == rec["outcome"], label
    assert sm.row == rec["row"] and sm.column == rec["column"]


@pytest.mark.parametrize("kind,n,m,world,k", [
    ("uniform", 2047, 2047, 4, 40),        # 5 blocks of 8
    ("mixed", 1500, 900, 3, 37),            # phase 1, a ragged block
    ("degenerate", 1023, 1023, 2, 60),
    ("degenerate_mixed", 600, 300, 5, 45),
])
def test_multi_chained_vs_oracle(kind, n, m, world, k):
    """solve(record_history=False) on row blocks (smx_mshard_run, 8 pivots per sweep): pivots,
    status and the whole table bit for bit against the C oracle."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 11, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), devices=[0] * world)
    sm.solve(record_history=False, max_pivots=k, chunk=k)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    D = sm._dev.download()
    assert np.array_equal(D[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(D[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
    assert sm.status == ("cap" if done == k else sm.status)


def test_multi_lazy_get_solution_matches_single_device():
    """get_solution(max_pivots=...) above the lazy threshold: the sharded chain's per-step (i, j),
    labels, x1/x2/optimum (x-history merged from the owners of the label rows) equal the
    single-device engine's; tables materialised from the gathered checkpoints equal the C
    oracle's at the same step."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import lp
    n, m, k = 1500, 1200, 30
    T = lp.dense_tableau("uniform", 5, n, m)
    cons, func = T[:n].tolist(), T[n, :m].tolist()
    one = simplex.SimplexMethod(cons, func, device="cuda:0").get_solution(max_pivots=k, chunk=8)
    sm = simplex.SimplexMethod(cons, func, devices=[0, 0, 0, 0])
    got = sm.get_solution(max_pivots=k, chunk=8)
    assert len(got) == len(one) == k + 1
    for a, b in zip(got, one):
        assert (a.i, a.j, a.row, a.column) == (b.i, b.j, b.row, b.column)
        assert np.array_equal(np.float64([a.x1, a.x2, a.optimum]).view(np.int64),
                              np.float64([b.x1, b.x2, b.optimum]).view(np.int64))
    for step in (0, 13, k):
        Tref, _, done, _ = c_oracle.run(T, n, m, m, step, threads=8)
        assert done == step
        tab = got[step].table
        assert table_hash(tab) == table_hash(Tref[:n].tolist() + [Tref[n, :m].tolist()])


def test_multi_pick_is_read_only():
    """pick_element() twice without a pivot leaves the table and the state alone (the control
    blocks are restored), then recalculate_matrix() pivots once."""
    import simplex
    from simplex_mi355x import lp
    n = m = 300
    T = lp.dense_tableau("uniform", 2, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), devices=[0, 0])
    sm.solve(record_history=False, max_pivots=3)
    h0 = table_hash(sm.table)
    a = sm.pick_element()
    b = sm.pick_element()
    assert a[:3] == b[:3] and table_hash(sm.table) == h0 and sm.pivots == 3
    sm.recalculate_matrix()
    assert sm.pivots == 4 and sm.pivot_log[-1] == (a[1], a[2])
    ref = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), device="cuda:0")
    ref.solve(record_history=False, max_pivots=4)
    assert ref.pivot_log == sm.pivot_log and table_hash(ref.table) == table_hash(sm.table)


@pytest.mark.parametrize("light", [0, 1])
def test_multi_rccl_exchange_world1_vs_oracle(light):
    """The branch a real multi-GPU node takes (distinct devices -> exchange="rccl"), run at world
    size 1: ncclCommInitAll on one device, then one host thread per device enqueuing its rank's
    chain on its own communicator: per pivot the all-gather of the send slots (full,
    smx_tune_shard_xchg(0)) or the header all-gather + k_bsh_pick + the int64 MAX all-reduce of
    the pivot row (light, smx_tune_shard_xchg(1)); smx_mshard_run, reached from
    SimplexMethod(..., devices=[0], exchange="rccl") as main.py:313 would call it.
    Pivot log and the whole table bit for bit against the C oracle, then the reference's own
    example LP through get_solution()."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    prev = _lib.tune_shard_xchg(light)
    try:
        for kind, n, m, k in (("uniform", 2047, 2047, 41), ("mixed", 1500, 900, 37)):
            T = lp.dense_tableau(kind, 11, n, m)
            sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), devices=[0],
                                       exchange="rccl")
            assert sm.backend == "sharded" and sm._dev.exchange == "rccl"
            sm.solve(record_history=False, max_pivots=k, chunk=k)
            Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
            assert sm.pivot_log == [tuple(map(int, x)) for x in log], kind
            D = sm._dev.download()
            assert np.array_equal(D[:n].view(np.int64), Tref[:n].view(np.int64)), kind
            assert np.array_equal(D[n, :m].view(np.int64), Tref[n, :m].view(np.int64)), kind
            sm._dev.close()
        case = load("examples.json")["ex2"]
        cons, func = dec_input(case["input"])
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func), devices=[0],
                                   exchange="rccl")
        got = sm.solve(record_history=False)
        last = [s for s in case["solution"] if s["kind"] == "info"][-1]
        assert same_table(got[-1].table, dec_table(last["table"]))
        sm._dev.close()
    finally:
        _lib.tune_shard_xchg(prev)


@pytest.mark.parametrize("kind,n,m,world,k,chunk", [
    ("uniform", 2047, 2047, 4, 48, 16),      # one captured graph, replayed three times
    ("mixed", 1500, 900, 3, 36, 12),         # phase 1
    ("degenerate", 1023, 1023, 8, 40, 20),
])
def test_multi_graph_chain_vs_oracle(kind, n, m, world, k, chunk):
    """Ranks sharing one device with graph_chain (smx_mshard_graph_create: the chain captured
    once, every event of the capture recorded exactly once): pivots and the whole table bit for
    bit against the C oracle, the graph replayed for every chunk."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 13, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), devices=[0] * world)
    sm._dev.graph_chain = True
    sm.solve(record_history=False, max_pivots=k, chunk=chunk)
    assert len(sm._dev._graphs) >= 1
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    D = sm._dev.download()
    assert np.array_equal(D[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(D[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
