"""GPU parity of pipelined block chains (smx_tune_block_pipe, csrc/smx_kernels.hip
launch_block_chain_pipe): block b+1 is planned on a second stream from block b's input table
(every chain prefixed by block b's pivots) while block b is swept out of place.  Bit-exact
against the unpipelined block chain, the one-pivot chain and the C oracle -- pivot logs, tables,
control blocks and the x-history ring -- for ragged-first blocks, terminal outcomes in any block
(the settle kernel), graph replays and the timed path; both planner forms (the register prefix
form k_blk_step_pfx after blocks of 12 / 20, the LDS-rolled k_blk_step_lag) and the CU partition
(smx_tune_block_pipe_cus: planner and sweeps on CU-masked streams, eager chains).
"""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import dec_input, load, table_hash

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


@pytest.fixture
def modes():
    """set(P, pipe) for one test (resident loop off); restores the library policies."""
    from simplex_mi355x import _lib
    prev = (_lib.tune_block(-1), _lib.tune_block_pipe(-1), _lib.tune_resident(-2),
            _lib.tune_block_pipe_cus(-1, -1))
    _lib.tune_resident(-1)

    def set_(P, pipe, cus=(0, 0)):
        _lib.tune_block(P)
        _lib.tune_block_pipe(pipe)
        _lib.tune_block_pipe_cus(*cus)
    yield set_
    _lib.tune_block(prev[0])
    _lib.tune_block_pipe(prev[1])
    _lib.tune_resident(prev[2])
    _lib.tune_block_pipe_cus(prev[3], 0)


def _state(sm, k):
    c = sm._dev.read_ctl()
    sp = int(c["npivots"]) & 1
    return (sm.pivot_log, sm.status, int(c["npivots"]), int(c["term"]), int(c["sel_status"]),
            int(c["sel_r"]), int(c["sel_c"]), int(c["negb"][sp]), int(c["negf"][sp]),
            sm._dev.download().view(np.int64).tobytes(),
            sm._dev.read_xhist(0, min(k, int(c["npivots"]))).view(np.int64).tobytes())


@pytest.mark.parametrize("P", [2, 3, 5, 8, 12, 20])
def test_pipe_equals_unpipelined_on_fixtures(modes, P):
    """Every non-capped random fixture, chunks of 3P+1 pivots (ragged first block, several
    blocks, terminal outcomes inside any of them): the pipelined chain leaves exactly the
    unpipelined chain's pivots, control block, table and x-history."""
    import simplex
    seen = 0
    for rec in load("random.json"):
        if rec["outcome"]["kind"] == "cap":
            continue
        cons, func = dec_input(rec["input"])
        if len(func) < 2:
            continue
        out = []
        for pipe in (1, 0):
            modes(P, pipe)
            sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
            sm.solve(record_history=False, chunk=3 * P + 1)
            out.append(_state(sm, 1 << 16))
        assert out[0] == out[1], rec.get("label")
        seen += 1
    assert seen > 10


@pytest.mark.parametrize("kind,n,m,k,chunk,P", [
    ("uniform", 1023, 1023, 203, 203, 8),      # 26 blocks, ragged first (3)
    ("uniform", 2047, 2047, 64, 64, 8),        # whole blocks only
    ("mixed", 1023, 1023, 301, 150, 5),        # phase 1 first
    ("degenerate", 511, 511, 300, 100, 4),
    ("degenerate_mixed", 600, 300, 300, 77, 6),
    ("uniform", 999, 3000, 150, 50, 3),
    ("uniform", 3001, 998, 150, 50, 7),
    ("uniform", 65535, 255, 40, 40, 8),
])
def test_pipe_vs_oracle(modes, kind, n, m, k, chunk, P):
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    modes(P, 1)
    T = lp.dense_tableau(kind, 5, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    assert sm._dev.block_plan()[1] == P
    sm.solve(record_history=False, max_pivots=k, chunk=chunk)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("graph", [True, False])
def test_pipe_graph_eager_and_history(modes, graph):
    """Graph replays and eager launches of the pipelined chain, continued by host steps and
    more chains: pivots, table and x-history equal the one-pivot chain's."""
    from simplex_mi355x import lp
    import simplex
    n, m = 900, 700
    T = lp.dense_tableau("mixed", 4, n, m)
    modes(4, 1)
    a = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    a.solve(record_history=False, max_pivots=45, chunk=45, graph=graph)
    for _ in range(2):
        ok, i, j, _e = a.pick_element()
        assert ok
        a.recalculate_matrix()
    a.solve(record_history=False, max_pivots=31, chunk=31, graph=graph)
    modes(1, 0)
    b = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    b.solve(record_history=False, max_pivots=78, chunk=78)
    assert a.pivot_log == b.pivot_log
    assert np.array_equal(a._dev.download().view(np.int64), b._dev.download().view(np.int64))
    assert np.array_equal(a._dev.read_xhist(0, 78).view(np.int64),
                          b._dev.read_xhist(0, 78).view(np.int64))


def test_pipe_lazy_history_equals_eager(modes):
    import simplex
    recs = [r for r in load("random.json") if r["outcome"]["kind"] != "cap"]
    for rec in recs[:8]:
        cons, func = dec_input(rec["input"])
        modes(3, 1)
        lazy = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=True, chunk=11)
        modes(1, 0)
        eager = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=False)
        assert len(lazy) == len(eager)
        for a, b in zip(lazy, eager):
            assert isinstance(a, simplex.Error) == isinstance(b, simplex.Error)
            if isinstance(b, simplex.Error):
                assert str(a) == str(b)
                continue
            assert (a.i, a.j, a.row, a.column) == (b.i, b.j, b.row, b.column)
            assert table_hash(a.table) == table_hash(b.table)


@pytest.mark.parametrize("k", [20, 33])
def test_pipe_timed_run_16k_prefix_vs_oracle(modes, k):
    """The bench path at the headline size: smx_block_run_timed through the pipelined chain
    (blocks 4+8+8 and 1+8+8+8+8), the whole 16383^2 table bit-exact against the C oracle."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    from simplex_mi355x.device import DeviceTableau
    modes(0, 1)
    n = m = 16383
    T = lp.dense_tableau("uniform", 0, n, m)
    dev = DeviceTableau(T, n, m, m)
    assert dev.block_plan()[1] == 20   # 1-4 GiB: up to 20 per sweep
    sw, tot = dev.run_block_timed(k, 8)
    assert len(sw) == -(-k // 8) and tot > 0
    ctl = dev.sync_state()
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert int(ctl["npivots"]) == done == k
    assert np.array_equal(dev.read_log(0, k), log)
    got = dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


# The register prefix form (pipe 1 after blocks of 12 / 20) against the LDS-rolled form (pipe 2)
# and the C oracle, unpartitioned and on a CU partition (4 CUs per XCD, 32 planner workgroups);
# eager chains (a partition does not survive stream capture), then a graph replay of the same.
@pytest.mark.parametrize("kind,n,m,k,P", [
    ("uniform", 2047, 2047, 64, 20),           # 4 + 20 + 20 + 20: the rolled form plans block 1
    ("uniform", 1535, 1791, 72, 12),           # whole blocks: every later block in prefix form
    ("mixed", 1023, 1023, 130, 20),            # phase 1 first
    ("degenerate", 1023, 1023, 120, 12),       # zero pivot-row entries, exact fallbacks
    ("degenerate_mixed", 1200, 600, 100, 20),
    ("uniform", 65535, 255, 60, 20),           # tall: several rows per planner thread
])
@pytest.mark.parametrize("pipe,cus", [(1, (0, 0)), (1, (4, 32)), (2, (4, 32))])
def test_pipe_prefix_form_vs_oracle(modes, kind, n, m, k, P, pipe, cus):
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    T = lp.dense_tableau(kind, 7, n, m)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    for graph in (False, True):
        modes(P, pipe, cus)
        sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
        assert sm._dev.block_plan()[1] == P
        sm.solve(record_history=False, max_pivots=k, chunk=k, graph=graph)
        assert sm.pivots == done, (graph, sm.pivots, done, st)
        assert sm.pivot_log == [tuple(map(int, x)) for x in log], graph
        got = sm._dev.download()
        assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64)), graph
        assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64)), graph


def test_pipe_partition_knob():
    from simplex_mi355x import _lib
    prev = _lib.tune_block_pipe_cus(-1, -1)
    try:
        assert _lib.tune_block_pipe_cus(17, 0) == -1        # out of range: unchanged
        assert _lib.tune_block_pipe_cus(4, 32) == prev
        assert _lib.tune_block_pipe_cus(-1, -1) == 4
    finally:
        _lib.tune_block_pipe_cus(prev, 0)
