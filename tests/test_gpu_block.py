"""GPU parity of block pivots (smx_block_run, csrc/smx_block.hpp): P pivots planned from the
block's input table and applied in one HBM sweep; every test runs with both planners: the window
planner (the default: the first columns of every row kept current step by step, k_blk_wstep) and
the register-form chains (k_blk_step<L>).  Bit-exact against the golden fixtures, the C
oracle and the one-pivot-per-sweep chain, for block sizes 1..24, both sweep layouts (pivot-row
slices in registers / in LDS, smx_tune_block_form), ragged last blocks, terminal outcomes inside
a block, the x-history ring and interleaving with host steps.
"""
from __future__ import annotations

import numpy as np
import pytest

from golden_util import dec_input, load, table_hash, trajectory_cap, trajectory_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


@pytest.fixture(autouse=True, params=[0, 2, 1], ids=["wplan", "wstep", "register"])
def planner_form(request):
    """Every test three times: the window planner as one persistent launch per block (k_blk_wplan,
    the default where eligible), the window planner's launch form (k_blk_wstep, planner 2) and the
    register-form chains (k_blk_step<L>, planner 1) -- the same bits every way."""
    from simplex_mi355x import _lib
    prev = _lib.tune_block_planner(request.param, 0)
    yield request.param
    _lib.tune_block_planner(prev, 0)


@pytest.fixture
def block_mode():
    """Set smx_tune_block for one test (resident loop off, so small tables take the block path)
    and restore both policies afterwards."""
    from simplex_mi355x import _lib
    prev_b = _lib.tune_block(-1)
    prev_r = _lib.tune_resident(-2)
    _lib.tune_resident(-1)
    yield _lib.tune_block
    _lib.tune_block(prev_b)
    _lib.tune_resident(prev_r)


@pytest.fixture
def sweep_form():
    """Set smx_tune_block_form (sweep layout 0 auto / 4 registers / 5 LDS / 6 LDS work items)
    for one test."""
    from simplex_mi355x import _lib
    prev = _lib.tune_block_form(-1)
    yield _lib.tune_block_form
    _lib.tune_block_form(prev)


CASES = list(trajectory_cases())


def _solve(cons, func, cap, chunk):
    import simplex
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
    out = sm.solve(record_history=False, max_pivots=cap, chunk=chunk)
    last = out[-2] if sm.status == "error" else out[-1]
    return sm, (sm.pivot_log, sm.status, str(out[-1]) if sm.status == "error" else None,
                table_hash(last.table))


@pytest.mark.parametrize("P,form", [(2, 0), (3, 5), (3, 6), (4, 0), (8, 0), (8, 5), (11, 0),
                                    (16, 0), (16, 4), (20, 0), (20, 6), (24, 5)])
def test_every_fixture_block_vs_chain_vs_reference(block_mode, sweep_form, P, form):
    """Every trajectory fixture: block chain == one-pivot chain == the reference's pivots, with
    chunks that end inside and at block boundaries and terminal outcomes inside blocks."""
    sweep_form(form)
    n_blk = 0
    for label, cons, func, rec in CASES:
        if len(func) not in (len(cons[0]) - 1, len(cons[0])) or len(func) < 2:
            continue   # the reference raises IndexError there (f() needs x1, x2)
        cap = trajectory_cap(rec)
        block_mode(P)
        sm, a = _solve(cons, func, cap, 7)
        n_blk += sm._dev.block_plan() is not None
        block_mode(1)
        _, b = _solve(cons, func, cap, 7)
        assert a == b, label
        exp = [(s["i"], s["j"]) for s in rec["steps"] if "i" in s and s["i"] is not None]
        assert a[0] == exp[:len(a[0])], label
        if rec["outcome"]["kind"] in ("optimum", "error"):
            assert a[3] == rec["steps"][-1]["hash"], label
    assert n_blk > 250


@pytest.mark.parametrize("P,nwin", [(3, 2), (8, 2), (5, 4), (12, 9)])
def test_every_fixture_small_window(block_mode, planner_form, P, nwin):
    """The window planner with a window of a few columns (the first nwin - 1 and the "-b" column):
    entering, phase-1 and pivot columns past it take the fallbacks (win_colvals / win_chain from
    the block's input table) -- every trajectory fixture still equals the one-pivot chain and the
    reference's pivots."""
    from simplex_mi355x import _lib
    if planner_form == 1:
        pytest.skip("window planner only")
    _lib.tune_block_planner(planner_form, nwin)
    n_blk = 0
    for label, cons, func, rec in CASES:
        if len(func) not in (len(cons[0]) - 1, len(cons[0])) or len(func) < 2:
            continue
        cap = trajectory_cap(rec)
        block_mode(P)
        sm, a = _solve(cons, func, cap, 7)
        n_blk += sm._dev.block_plan() is not None
        block_mode(1)
        _, b = _solve(cons, func, cap, 7)
        assert a == b, label
        exp = [(s["i"], s["j"]) for s in rec["steps"] if "i" in s and s["i"] is not None]
        assert a[0] == exp[:len(a[0])], label
    assert n_blk > 250


@pytest.mark.parametrize("nwin", [2, 3, 17])
@pytest.mark.parametrize("kind,n,m,k,chunk,P", [
    ("uniform", 1023, 1023, 120, 60, 12),
    ("mixed", 700, 900, 200, 61, 7),           # phase 1: first positive past the window
    ("degenerate", 511, 511, 150, 75, 8),
    ("degenerate_mixed", 600, 300, 150, 75, 6),
    ("mixed", 255, 4095, 60, 60, 20),
])
def test_window_fallbacks_vs_oracle(block_mode, planner_form, kind, n, m, k, chunk, P, nwin):
    """Window planner, small windows on BASELINE-shaped generators: pivots and the whole table bit
    for bit against the C oracle whichever columns fall outside the window."""
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    import simplex
    if planner_form == 1:
        pytest.skip("window planner only")
    _lib.tune_block_planner(planner_form, nwin)
    block_mode(P)
    T = lp.dense_tableau(kind, 13, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    assert sm._dev.block_plan()[1] == P
    sm.solve(record_history=False, max_pivots=k, chunk=chunk)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("kind,n,m,k,chunk,P", [
    ("uniform", 1023, 1023, 203, 64, 4),
    ("uniform", 1023, 1023, 120, 120, 8),
    ("uniform", 999, 3000, 150, 50, 3),        # wide, odd C
    ("uniform", 3001, 998, 150, 50, 5),        # tall, odd C
    ("mixed", 1023, 1023, 400, 100, 4),        # phase 1 first
    ("mixed", 700, 900, 200, 61, 7),
    ("degenerate", 511, 511, 300, 100, 4),     # zero ratios, -0.0 classes
    ("degenerate_mixed", 600, 300, 300, 100, 6),
    ("uniform", 65535, 255, 40, 20, 4),        # very tall
    ("mixed", 255, 65535, 40, 20, 4),          # very wide, phase 1
    ("uniform", 2047, 2047, 100, 100, 16),     # 16 pivots per sweep, ragged last block
    ("mixed", 1500, 1100, 160, 80, 13),
    ("degenerate", 700, 700, 200, 200, 12),
    ("uniform", 2047, 2047, 110, 110, 20),     # LDS layout from 13 pivots on
    ("mixed", 1500, 1100, 160, 80, 24),
    ("degenerate_mixed", 900, 1300, 150, 75, 22),
    ("uniform", 255, 65535, 48, 48, 24),       # 512 chunks per row: one workgroup each
])
@pytest.mark.parametrize("form", [0, 4, 5, 6])
def test_block_vs_oracle(block_mode, sweep_form, kind, n, m, k, chunk, P, form):
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    if form == 4 and P > 16:
        pytest.skip("register layout: up to 16 pivots tested")
    sweep_form(form)
    block_mode(P)
    T = lp.dense_tableau(kind, 11, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    assert sm._dev.block_plan()[1] == P
    sm.solve(record_history=False, max_pivots=k, chunk=chunk)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("P", [10, 12, 16, 20, 24])
@pytest.mark.parametrize("form", [4, 5, 6])
def test_block_bounded_fast_path_edges_vs_oracle(block_mode, sweep_form, P, form):
    """The one-row sweep's unchecked fast path (smx_block.hpp, kBndSpan) next to its fallbacks in
    one table: rows scaled past 2^101 (input bound), rows scaled to ~2^-60 (small numerators),
    columns scaled to ~2^-99 (pivot-row values below 2^-100: the chunk falls back), exact zeros
    (zero multipliers and pivot-row values), signed zeros -- bit-exact against the C oracle."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    sweep_form(form)
    block_mode(P)
    n = m = 1023
    T = lp.dense_tableau("uniform", 5, n, m)
    T[0:40] *= 2.0 ** 102
    T[40:90] *= 2.0 ** -60
    T[:, 200:260] *= 2.0 ** -99
    T[300:340, 500:540] = 0.0
    T[340:350, 600:640] = -0.0
    T[500:900, 700] = 0.0
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    assert sm._dev.block_plan()[1] == P
    k = 4 * P + 3
    sm.solve(record_history=False, max_pivots=k, chunk=k)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("P", [1, 2, 5, 8, 16])
def test_graph_and_eager_block_chains_agree(block_mode, P):
    from simplex_mi355x import lp
    import simplex
    block_mode(P if P > 1 else 2)
    T = lp.dense_tableau("mixed", 3, 700, 900)
    a = simplex.SimplexMethod(T[:700].tolist(), T[700, :900].tolist())
    b = simplex.SimplexMethod(T[:700].tolist(), T[700, :900].tolist())
    a._dev.block = P
    b._dev.block = P
    a.solve(record_history=False, max_pivots=96, chunk=32, graph=True)
    b.solve(record_history=False, max_pivots=96, chunk=32, graph=False)
    block_mode(1)
    c = simplex.SimplexMethod(T[:700].tolist(), T[700, :900].tolist())
    c.solve(record_history=False, max_pivots=96, chunk=32)
    assert a.pivot_log == b.pivot_log == c.pivot_log
    ga, gb, gc = (x._dev.download().view(np.int64) for x in (a, b, c))
    assert np.array_equal(ga, gb) and np.array_equal(ga, gc)


def test_block_history_and_host_steps(block_mode):
    """block chunk -> host pick_element/recalculate_matrix -> block chunk: control block state
    carries over; the device x-history ring written by the planner equals the one-pivot chain's
    and the lazy get_solution equals the eager one."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    block_mode(4)
    n, m = 300, 260
    T = lp.dense_tableau("mixed", 9, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    sm.solve(record_history=False, max_pivots=17, chunk=17)
    for _ in range(3):
        ok, i, j, _e = sm.pick_element()
        assert ok
        sm.recalculate_matrix()
    sm.solve(record_history=False, max_pivots=22, chunk=11)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 42, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    xa = sm._dev.read_xhist(0, 42)
    block_mode(1)
    ref = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    ref.solve(record_history=False, max_pivots=42, chunk=42)
    assert np.array_equal(xa.view(np.int64), ref._dev.read_xhist(0, 42).view(np.int64))
    recs = [r for r in load("random.json") if r["outcome"]["kind"] != "cap"]
    for rec in recs[:6]:
        cons, func = dec_input(rec["input"])
        block_mode(3)
        lazy = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=True, chunk=5)
        block_mode(1)
        eager = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=False)
        assert len(lazy) == len(eager)
        for a, b in zip(lazy, eager):
            assert isinstance(a, simplex.Error) == isinstance(b, simplex.Error)
            if isinstance(b, simplex.Error):
                assert str(a) == str(b)
                continue
            assert (a.i, a.j, a.row, a.column) == (b.i, b.j, b.row, b.column)
            assert np.array_equal(np.float64([a.x1, a.x2, a.optimum]).view(np.int64),
                                  np.float64([b.x1, b.x2, b.optimum]).view(np.int64))
            assert table_hash(a.table) == table_hash(b.table)


def test_block_terminal_state_matches_chain(block_mode):
    """A chain that stops inside a block leaves the same control block (status, selection,
    first-negative slots, pivot count) and table as the one-pivot chain."""
    import simplex
    seen = 0
    for rec in load("random.json"):
        if rec["outcome"]["kind"] == "cap":
            continue
        cons, func = dec_input(rec["input"])
        ctls = []
        for P in (5, 1):
            block_mode(P)
            sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
            sm.solve(record_history=False, chunk=12)
            c = sm._dev.read_ctl()
            sp = int(c["npivots"]) & 1          # the slot of the table the chain stopped at
            ctls.append((int(c["npivots"]), int(c["term"]), int(c["sel_status"]),
                         int(c["sel_r"]), int(c["sel_c"]), int(c["negb"][sp]),
                         int(c["negf"][sp]), table_hash(sm.table)))
        assert ctls[0] == ctls[1], ctls
        seen += 1
    assert seen > 10


@pytest.mark.parametrize("n,m,k,P", [(8191, 8191, 23, 12), (16383, 16383, 9, 20),
                                     (16383, 16383, 20, 20), (16383, 16383, 47, 20),
                                     (3071, 3071, 13, 10)])
def test_block_full_size_prefix_vs_oracle(block_mode, planner_form, n, m, k, P):
    """BASELINE sizes through the default policy: with the launch-form planners 10, 12 or --
    1-4 GiB tables -- 20 pivots per sweep at most, blocks of near-equal size (23 = 12 + 11, 9 = one
    block, 20 = one block of 20 in the LDS layout (k_blk_sweep<20, 5>), 47 = 16 + 16 + 15, 13 =
    7 + 6); with the persistent planner 24 (23, 9, 20 = one block, 47 = 24 + 23, 13 = one)."""
    from simplex_mi355x import lp, _lib
    from simplex_mi355x.device import DeviceTableau
    from oracle import c_oracle
    block_mode(0)
    T = lp.dense_tableau("uniform", 0, n, m)
    dev = DeviceTableau(T, n, m, m)
    assert dev.block_plan()[1] == (24 if planner_form == 0 else P)
    dev.run(k, graph=False)
    ctl = dev.sync_state()
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert int(ctl["npivots"]) == done == k
    assert np.array_equal(dev.read_log(0, k), log)
    got = dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("kind,k", [("degenerate", 20), ("degenerate", 41), ("uniform", 20),
                                    ("degenerate_mixed", 41)])
def test_block_wide_table_vs_oracle(block_mode, planner_form, kind, k):
    """A 1 GiB table 4096 x 32768 (config 5's width: 256 chunks of 128 columns per row) through
    the default policy, 24 pivots per sweep in the LDS layout (the persistent planner; its column
    slices of 128 leave the pivot rows to k_blk_prows), integer degenerate data included (zeros:
    the zero-extended division; exact paths): 20 = one block, 41 = 21 + 20 (the launch-form
    planners: 20 per sweep, 41 = 14 + 14 + 13)."""
    from simplex_mi355x import lp
    from simplex_mi355x.device import DeviceTableau
    from oracle import c_oracle
    block_mode(0)
    n, m = 4095, 32767
    T = lp.dense_tableau(kind, 5, n, m)
    dev = DeviceTableau(T, n, m, m)
    assert dev.block_plan()[1] == (24 if planner_form == 0 else 20)
    dev.run(k, graph=False)
    ctl = dev.sync_state()
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert int(ctl["npivots"]) == done
    assert np.array_equal(dev.read_log(0, done), log)
    got = dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


def test_block_plan_policy(block_mode, planner_form):
    from simplex_mi355x import _lib
    if planner_form != 0:
        pytest.skip("the policy of each planner form is checked below")
    block_mode(0)
    # the persistent planner's tables (up to 32,768 rows): 24; beyond, the launch-form policy
    assert _lib.block_plan([16384, 16383, 16383, 16383, 16383, 0, 64])[1] == 24   # 2 GiB
    assert _lib.block_plan([32768, 32767, 32767, 32767, 32767, 0, 64])[1] == 24   # 8 GiB
    assert _lib.block_plan([32768, 65535, 65535, 32767, 32767, 0, 64])[1] == 20   # config 5
    assert _lib.block_plan([8192, 8191, 8191, 8191, 8191, 0, 32])[1] == 24
    assert _lib.block_plan([3072, 3071, 3071, 3071, 3071, 0, 12])[1] == 24
    prev = _lib.tune_block_planner(2, 0)   # the launch form: round 5's policy
    try:
        assert _lib.block_plan([16384, 16383, 16383, 16383, 16383, 0, 64])[1] == 20
        assert _lib.block_plan([8192, 8191, 8191, 8191, 8191, 0, 32])[1] == 12
        assert _lib.block_plan([3072, 3071, 3071, 3071, 3071, 0, 12])[1] == 10
    finally:
        _lib.tune_block_planner(prev, 0)
    assert _lib.block_plan([2048, 2047, 2047, 2047, 2047, 0, 8]) is None    # below 48 MiB
    assert _lib.block_plan([1024, 1023, 1023, 1023, 1023, 0, 4]) is None
    assert _lib.block_plan([1024, 1023, 1023, 1023, 1023, 0, 4], 6)[1] == 6
    assert _lib.block_plan([1024, 100, 1023, 1023, 1023, 0, 4], 4) is None  # sharded
    assert _lib.block_plan([1024, 1023, 1023, 1023, 1023, 0, 4], 24)[1] == 24
    assert _lib.block_plan([1024, 1023, 1023, 1023, 1023, 0, 4], 25) is None
    block_mode(1)
    assert _lib.block_plan([16384, 16383, 16383, 16383, 16383, 0, 64]) is None


def test_deferred_timed_launch_vs_oracle(block_mode):
    """The bench's timed form: block_timed_launcher's launch() only enqueues (smx_block_run_timed
    with NULL outputs), read() waits and returns the sweep times; the table bit-exact against
    the C oracle, and a read without a deferred launch is refused."""
    import ctypes

    import torch
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    from simplex_mi355x.device import DeviceTableau
    block_mode(0)
    n = m = 3071
    k = 13
    T = lp.dense_tableau("uniform", 0, n, m)
    dev = DeviceTableau(T, n, m, m)
    P = dev.block_plan()[1]
    launch, read = dev.block_timed_launcher(k, P)
    launch()
    torch.cuda.synchronize()
    sw, tot = read()
    assert len(sw) == -(-k // P) and (sw > 0).all() and tot >= float(sw.sum())
    f = ctypes.c_float()
    assert _lib.load().smx_block_timed_read(len(sw), (ctypes.c_float * len(sw))(),
                                            ctypes.byref(f)) != 0      # already read
    ctl = dev.sync_state()
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert int(ctl["npivots"]) == done == k
    assert np.array_equal(dev.read_log(0, k), log)
    got = dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


_NOFREE_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [{repo!r}, {repo!r} + '/simplex-method-solver_amd', {repo!r} + '/tests']
import simplex
from oracle import c_oracle
from simplex_mi355x import lp
n = m = 3071
T = lp.dense_tableau('uniform', 7, n, m)
sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist(), device='cuda:0')
assert sm._dev.block_plan() is not None
sm.solve(record_history=False, max_pivots=24, chunk=12, graph=True)   # captured block graphs
Tref, st, done, log = c_oracle.run(T, n, m, m, 24, threads=8)
assert sm.pivot_log == [tuple(map(int, x)) for x in log]
D = sm._dev.download()
assert np.array_equal(D[:n].view(np.int64), Tref[:n].view(np.int64))
print('nofree ok', len(sm._dev._graphs))
"""


def test_nofree_knob_with_captured_block_graph():
    """SMX_BLK_NOFREE=1 (the A/B knob that turns the sweep's bounded fast path off) set in a fresh
    process, then block graphs captured: round 2 saw hipError 901 (capture invalidated) here
    because the knob's device-symbol write ran inside the capture; it now runs in
    smx_block_bytes, before any capture.  The captured chain stays bit-exact vs the C oracle."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SMX_BLK_NOFREE="1")
    out = subprocess.run([sys.executable, "-c", _NOFREE_SCRIPT.format(repo=repo)], env=env,
                         capture_output=True, text=True, timeout=300, cwd=repo)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "nofree ok" in out.stdout


def test_block_graph_replays_and_tall_table(block_mode, planner_form):
    """ONE captured graph of a block chain replayed many times continues the trajectory bit for
    bit; a table with more rows than planner threads (65,537 > 256 x 256 rows)."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    block_mode(6)
    n, m = 1500, 1100
    T = lp.dense_tableau("uniform", 21, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    sm.solve(record_history=False, max_pivots=120, chunk=12, graph=True)   # 10 replays
    assert len(sm._dev._graphs) <= 2
    Tref, st, done, log = c_oracle.run(T, n, m, m, 120, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    n, m = 65537, 63
    T = lp.dense_tableau("uniform", 22, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    sm.solve(record_history=False, max_pivots=30, chunk=30)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 30, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))


@pytest.mark.parametrize("kind", ["uniform", "mixed"])
def test_zero_pivot_chain_publishes_state(block_mode, kind):
    """smx_block_run with k = 0: the chain start (k_blk_start) and the publish alone (no block,
    so no pivot-column pass to carry it) -- ctl's negb / negf of the parity slot are the table's
    first negative "-b" row and f-row column (simplex.py:72-76, :94-98), the table untouched."""
    import torch
    from simplex_mi355x import _lib, lp, ops
    from simplex_mi355x.device import DeviceTableau
    block_mode(8)
    n, m = 3000, 2000
    T = lp.dense_tableau(kind, 9, n, m)
    dev = DeviceTableau(T, n, m, m)
    plan = dev.block_plan()
    assert plan is not None and plan[1] == 8
    blk = dev._blk_for(plan)
    with torch.cuda.stream(dev.stream):
        ops.block_run(dev.buf, dev.ctl, blk, dev.log, dev.xhist, dev.shape, 0, 0, plan[1])
    torch.cuda.synchronize()
    c = dev.read_ctl()
    neg_b = np.nonzero(T[:n, m] < 0.0)[0]
    neg_f = np.nonzero(T[n, :m] < 0.0)[0]
    assert int(c["negb"][0]) == (int(neg_b[0]) if len(neg_b) else _lib.NONE)
    assert int(c["negf"][0]) == (int(neg_f[0]) if len(neg_f) else _lib.NONE)
    assert int(c["npivots"]) == 0 and int(c["term"]) == 0
    assert np.array_equal(dev.download()[:n + 1, :m + 1].view(np.int64),
                          T[:n + 1, :m + 1].view(np.int64))
