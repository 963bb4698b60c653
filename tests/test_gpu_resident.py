"""GPU parity of the on-chip resident pivot loop (smx_resident_run, csrc/smx_resident.hpp): the
whole get_solution loop (simplex.py:184-198) in one persistent launch with the rows in LDS.
Bit-exact against the golden fixtures, the C oracle and the launch chain (smx_run), for every
workgroup count, and interleaved with the host-driven step path.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from golden_util import dec_input, load, table_hash, trajectory_cap, trajectory_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


@pytest.fixture
def resident_mode():
    """Set smx_tune_resident for one test and restore the automatic policy afterwards."""
    from simplex_mi355x import _lib
    prev = _lib.tune_resident(-2)
    yield _lib.tune_resident
    _lib.tune_resident(prev)


CASES = list(trajectory_cases())


def _solve(cons, func, cap, chunk):
    import simplex
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
    out = sm.solve(record_history=False, max_pivots=cap, chunk=chunk)
    last = out[-2] if sm.status == "error" else out[-1]
    return sm, (sm.pivot_log, sm.status, str(out[-1]) if sm.status == "error" else None,
                table_hash(last.table))


def test_every_fixture_resident_vs_chain_vs_reference(resident_mode):
    """Every trajectory fixture: resident loop == launch chain == the reference's pivots."""
    n_res = 0
    for label, cons, func, rec in CASES:
        if len(func) not in (len(cons[0]) - 1, len(cons[0])) or len(func) < 2:
            continue   # the reference raises IndexError there (f() needs x1, x2)
        cap = trajectory_cap(rec)
        resident_mode(0)
        sm, a = _solve(cons, func, cap, 5)
        n_res += sm._dev.resident_plan() is not None
        resident_mode(-1)
        _, b = _solve(cons, func, cap, 5)
        assert a == b, label
        exp = [(s["i"], s["j"]) for s in rec["steps"] if "i" in s and s["i"] is not None]
        assert a[0] == exp[:len(a[0])], label
        if rec["outcome"]["kind"] in ("optimum", "error"):
            assert a[3] == rec["steps"][-1]["hash"], label
    assert n_res > 250


def test_hand_off_timeout_recovers_on_launch_chain(resident_mode):
    """A resident chain whose hand-off spin times out (forced here: smx_tune_resident_timeout(0))
    leaves its table undefined; the host restores the chain's input from the snapshot it took,
    reruns the same pivots on the launch chain and keeps that tableau off the resident loop --
    results bit-exact against the C oracle, across several chunks."""
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    import simplex
    n, m, k = 511, 511, 90
    T = lp.dense_tableau("mixed", 9, n, m)
    resident_mode(0)
    L = _lib.load()
    prev = int(L.smx_tune_resident_timeout(0))
    assert prev > 0
    try:
        sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
        assert sm._dev.resident_plan() is not None
        sm.solve(record_history=False, max_pivots=k, chunk=30)
    finally:
        assert int(L.smx_tune_resident_timeout(prev)) == 0
    assert sm._dev.resident_fallbacks == 1
    assert sm._dev.resident is False
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("wg", [1, 3, 7, 64, 255, 256])
def test_workgroup_counts_agree(resident_mode, wg):
    """Any grid (1 .. 256 workgroups, ragged last row block) gives the same bits."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    n, m, k = 100, 120, 150     # one workgroup holds all 101 x 121 doubles in LDS
    T = lp.dense_tableau("mixed", 5, n, m)
    resident_mode(wg)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    G, rpw = sm._dev.resident_plan()[1][:2]
    assert G <= wg and G * rpw >= n > (G - 1) * rpw
    sm.solve(record_history=False, max_pivots=k, chunk=k)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("kind,n,m,k", [
    ("uniform", 1023, 1023, 500),
    ("uniform", 1919, 1919, 200),      # largest square that fits (8 rows per workgroup)
    ("uniform", 999, 3000, 150),       # 16 columns per thread, odd C
    ("uniform", 3001, 998, 150),       # 12 rows per workgroup
    ("mixed", 1023, 1023, 400),        # phase 1 first
    ("degenerate", 511, 511, 300),     # zero ratios, -0.0 classes
    ("degenerate_mixed", 600, 300, 300),
    ("uniform", 5, 4095, 40),          # widest eligible row
])
def test_resident_vs_oracle(resident_mode, kind, n, m, k):
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    resident_mode(0)
    T = lp.dense_tableau(kind, 11, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    assert sm._dev.resident_plan() is not None
    sm.solve(record_history=False, max_pivots=k, chunk=k)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


def test_too_large_falls_back_to_chain(resident_mode):
    from simplex_mi355x import _lib
    resident_mode(0)
    # 2048^2 does not fit in LDS (9 rows + the staged pivot row per workgroup), 1920^2 does;
    # more than 4096 columns never (13-bit phase-1 column in the record)
    assert _lib.resident_plan([2048, 2047, 2047, 2047, 2047, 0, 8]) is None
    assert _lib.resident_plan([1920, 1919, 1919, 1919, 1919, 0, 8]) is not None
    assert _lib.resident_plan([4112, 10, 10, 4096, 4096, 0, 16]) is None
    assert _lib.resident_plan([4096, 10, 10, 4095, 4095, 0, 16]) is not None
    # sharded shapes never run resident
    assert _lib.resident_plan([1024, 100, 1023, 1023, 1023, 0, 4]) is None
    resident_mode(-1)
    assert _lib.resident_plan([1024, 1023, 1023, 1023, 1023, 0, 4]) is None


def test_interleaved_with_host_steps_and_lazy_history(resident_mode):
    """resident chunk -> host pick_element/recalculate_matrix -> resident chunk: the control
    block (first-negative slots, label positions, pivot index) carries over; lazy history
    (x1, x2 from the device ring) equals the eager get_solution."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    import simplex
    resident_mode(0)
    n, m = 300, 260
    T = lp.dense_tableau("mixed", 9, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    sm.solve(record_history=False, max_pivots=17, chunk=17)
    for _ in range(3):
        ok, i, j, _e = sm.pick_element()
        assert ok
        sm.recalculate_matrix()
    sm.solve(record_history=False, max_pivots=20, chunk=9)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 40, threads=8)
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    recs = [r for r in load("random.json") if r["outcome"]["kind"] != "cap"]
    for rec in recs[:6]:
        cons, func = dec_input(rec["input"])
        lazy = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=True, chunk=4)
        resident_mode(-1)
        eager = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(
            lazy=False)
        resident_mode(0)
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


def test_fastdiv_matches_hardware_division():
    """The resident update divides by the pivot element with the hardware division sequence's
    denominator half hoisted (smx_resident.hpp, fd_div): bit-identical to x / e on 24 M operand
    pairs -- random mantissas and signs with exponents spanning the window and beyond, all-ones /
    power-of-two / next-to-power-of-two mantissas, tableau-like values, zeros, infs, NaNs."""
    import torch
    from simplex_mi355x import _lib
    rng = np.random.default_rng(123)
    N = 1 << 22

    def mk(exp_lo, exp_hi, mant=None):
        m = rng.random(N) + 1.0 if mant is None else mant
        x = np.ldexp(m, rng.integers(exp_lo, exp_hi, N))
        return np.where(rng.random(N) < 0.5, -x, x)

    ones = np.full(N, 2.0 - 2.0 ** -52)
    nums = [mk(-140, 140), mk(-130, 131, ones), mk(-3, 4), mk(-128, -120), mk(125, 131),
            rng.uniform(-1, 1, N) * rng.uniform(-1, 1, N) - rng.uniform(-1, 1, N)]
    dens = [mk(-140, 140), mk(-3, 4), mk(-130, 131, ones), mk(-2, 2, np.full(N, 1.0)),
            mk(-2, 2, np.full(N, 1.0 + 2.0 ** -52)), rng.uniform(-1, 1, N)]
    num = np.concatenate(nums)
    den = np.concatenate(dens)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 1e308, -1e-308])
    num[:64] = np.resize(special, 64)
    den[64:128] = np.resize(special[2:], 64)
    tn = torch.from_numpy(num).cuda()
    td = torch.from_numpy(den).cuda()
    out = torch.zeros(2, dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().smx_fastdiv_check(tn.data_ptr(), td.data_ptr(), num.size,
                                             out.data_ptr(), torch.cuda.current_stream().cuda_stream),
               "smx_fastdiv_check")
    inside, bad = (int(x) for x in out.cpu())
    assert bad == 0
    assert inside > num.size // 2


def test_fastdiv_bounded_domain_matches_hardware_division():
    """The block sweep's unchecked fast path (smx_block.hpp, kBndSpan) divides with no window
    check when the pivot elements, pivot-row values and multipliers are bounded, which keeps
    every numerator at +0 or inside [2^-254, 2^410) and the pivot element inside [2^-100, 2^101):
    the hoisted-reciprocal sequence must equal x / e bit for bit on that whole domain -- random
    mantissas and signs across it, its edges, all-ones and power-of-two mantissas, +0."""
    import torch
    from simplex_mi355x import _lib
    rng = np.random.default_rng(321)
    N = 1 << 22

    def mk(exp_lo, exp_hi, mant=None):
        m = rng.random(N) + 1.0 if mant is None else mant
        x = np.ldexp(m, rng.integers(exp_lo, exp_hi, N))
        return np.where(rng.random(N) < 0.5, -x, x)

    ones = np.full(N, 2.0 - 2.0 ** -52)
    nums = [mk(-254, 410), mk(-254, -240), mk(395, 410), mk(-254, 410, ones),
            mk(-254, 410, np.full(N, 1.0)), mk(-3, 4)]
    dens = [mk(-100, 101), mk(90, 101), mk(-100, -90), mk(-100, 101, ones),
            mk(-100, 101, np.full(N, 1.0 + 2.0 ** -52)), rng.uniform(-1, 1, N)]
    num = np.concatenate(nums)
    den = np.concatenate(dens)
    num[::97] = 0.0                    # +0 numerators (a zero numerator is never -0 there)
    # the zero-extended domain of the flag-form sweep: -0 numerators over both signs of e, the
    # -0.0 values of the edge fixtures, and numerators down to 2^-456 -- the kernel checks both
    # zero-safe sequences there (fd_zero, and fd_zneg with its sign folded back), bad0 counting a
    # pair either one gets wrong
    edge_zero = [v for rec in load("edge.json").values()
                 for row in dec_input(rec["input"])[0] for v in row if v == 0.0]
    assert any(math.copysign(1.0, v) < 0 for v in edge_zero)
    zn = np.concatenate([np.full(N // 4, -0.0), np.full(N // 4, 0.0), mk(-456, -400),
                         np.resize(np.array(edge_zero), N // 4)])
    zd = np.concatenate([mk(-100, 101) for _ in range(4)])[:zn.size]
    num = np.concatenate([num, zn])
    den = np.concatenate([den, zd])
    tn = torch.from_numpy(num).cuda()
    td = torch.from_numpy(den).cuda()
    out = torch.zeros(4, dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().smx_fastdiv_check_bounded(
        tn.data_ptr(), td.data_ptr(), num.size, out.data_ptr(),
        torch.cuda.current_stream().cuda_stream), "smx_fastdiv_check_bounded")
    inside, bad, inside0, bad0 = (int(x) for x in out.cpu())
    assert bad == 0 and bad0 == 0
    assert inside > 0.7 * num.size and inside0 > 0.95 * num.size


def test_two_resident_chains_on_separate_streams(resident_mode):
    """Two solvers, each on its own stream, enqueue resident chains that overlap in time: every
    workgroup of a chain must be resident at once (256 of them each at 1023^2), so the library
    orders resident launches on a device one after the other -- without that the two chains
    would split the CUs and wait on each other's workgroups until the hand-off timeout.  Both
    must finish without a timeout and equal the oracle."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    from simplex_mi355x.device import DeviceTableau
    import torch
    resident_mode(256)   # every CU: two such chains can never be resident together
    n = m = 1023
    k = 150
    Ts = [lp.dense_tableau(kind, 21, n, m) for kind in ("uniform", "mixed")]
    devs = [DeviceTableau(T, n, m, m) for T in Ts]
    for d in devs:
        assert d.resident_plan() is not None and d.resident_plan()[1][0] == 256
    torch.cuda.synchronize()
    for rnd in range(3):                  # interleaved enqueues, no host sync in between
        for d in devs:
            d.run(k // 3, graph=False)
    for d, T in zip(devs, Ts):
        ctl = d.sync_state()              # raises on a resident hand-off timeout
        Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
        assert int(ctl["npivots"]) == done
        assert np.array_equal(d.read_log(0, done), log)
        got = d.download()
        assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))


@pytest.mark.parametrize("kind,n,m,k", [
    ("uniform", 1023, 1023, 300),
    ("mixed", 700, 650, 250),          # phase 1 rows, published before their bulk update
    ("degenerate", 511, 511, 200),
    ("uniform", 5, 4095, 40),
])
def test_resident_round3_loop_vs_overlapped(resident_mode, kind, n, m, k):
    """smx_tune_resident_overlap(0) (every step fully updated before the next record) and the
    default overlapped loop (bulk update under the next hand-off): same pivots, same table bits,
    both equal to the C oracle."""
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    import simplex
    resident_mode(0)
    T = lp.dense_tableau(kind, 5, n, m)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    prev = _lib.tune_resident_overlap(-1)   # (2: automatic)
    try:
        for ovl in (0, 1):
            _lib.tune_resident_overlap(ovl)
            sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
            assert sm._dev.resident_plan() is not None
            sm.solve(record_history=False, max_pivots=k, chunk=k)
            assert sm.pivot_log == [tuple(map(int, x)) for x in log], ovl
            got = sm._dev.download()
            assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64)), ovl
            assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64)), ovl
    finally:
        _lib.tune_resident_overlap(prev)
