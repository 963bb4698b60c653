"""GPU: the HIP shard kernels for P simulated ranks in one process on one device (the all-gather
done by a device copy), against the unsharded C oracle, bit for bit -- all three pivot forms:
unfused (k_select/k_pack/k_update<kShard>), fused (k_la_prime/k_pack<fused>/
k_update<kShardFused>) and the overlapped chain's halves (k_shard_la + k_pack_ahead, then the
sweep without look-ahead workgroups).  The native RCCL driver is covered at world size 1
(tools/check_native_shard.py) and the multi-process protocol by the gloo tests."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


MODES = {"overlap": (True, True), "fused": (True, False), "unfused": (False, False)}


def _simulate(T, n, m, k, P, mode="overlap", bes=None):
    import torch
    from simplex_mi355x.sharded import HipShardBackend, row_range
    if bes is None:
        bes = []
        for p in range(P):
            lo, hi = row_range(n, p, P)
            local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
            fused, overlap = MODES[mode]
            bes.append(HipShardBackend(local, n, m, m, lo, P, fused=fused, overlap=overlap))
    for _ in range(k):
        for be in bes:
            with be.stream_ctx():
                be.begin()
        torch.cuda.synchronize()
        allsend = torch.cat([be.send for be in bes])
        for be in bes:
            be.recv.copy_(allsend)
        torch.cuda.synchronize()
        for be in bes:
            with be.stream_ctx():
                be.finish()
    torch.cuda.synchronize()
    states = [be.state() for be in bes]
    logs = [be.log(0, s["npivots"]) for be, s in zip(bes, states)]
    tables = [be.local_table() for be in bes]
    full = np.concatenate([t[:-1] for t in tables] + [tables[0][-1:]], axis=0)
    return states, logs, tables, full, bes


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("kind,n,m,k,P", [
    ("uniform", 1023, 1023, 80, 2),
    ("uniform", 1001, 777, 80, 3),
    ("uniform", 2047, 2047, 40, 8),
    ("mixed", 700, 600, 120, 4),
    ("degenerate", 511, 511, 120, 4),
    ("degenerate_mixed", 300, 500, 120, 5),
    ("uniform", 40, 30, 78, 3),   # step 26 pivots on row 26 = rank 2's first row: on rank 1
                                  # r - row0 == its f-row replica's local index (regression)
    ("mixed", 5, 7, 30, 8),       # fewer constraint rows than ranks: some ranks own none
    ("uniform", 4095, 4095, 24, 2),   # 64 MiB per shard
    ("degenerate_mixed", 9, 3, 40, 4),
])
def test_hip_shards_match_oracle(kind, n, m, k, P, mode):
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 7, n, m)
    states, logs, tables, full, _ = _simulate(T, n, m, k, P, mode)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    for s, lg in zip(states, logs):
        assert s["npivots"] == done
        assert np.array_equal(lg, log)
    for t in tables[1:]:   # every f-row replica identical
        assert np.array_equal(t[-1, :m].view(np.int64), tables[0][-1, :m].view(np.int64))
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(full[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


@pytest.mark.parametrize("mode", list(MODES))
def test_hip_shards_terminal_outcome(mode):
    """A run that ends (optimum or error) stops identically on every rank."""
    from oracle import c_oracle
    from simplex_mi355x import lp
    n, m = 40, 30
    T = lp.dense_tableau("uniform", 2, n, m)
    states, logs, tables, full, _ = _simulate(T, n, m, 400, 3, mode)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 400)
    assert done < 400
    for s in states:
        assert s["term"] and s["status"] == st and s["npivots"] == done
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))


def test_native_rccl_driver_world1():
    """libsmx.so's own RCCL communicator + stream-ordered all-gather (1-rank job)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(repo, "tools", "check_native_shard.py")],
                         capture_output=True, text=True, timeout=600, cwd=repo)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


def test_hip_shards_fused_then_unfused():
    """Fused steps, smx_fused_publish, then unfused steps continue the same trajectory."""
    import ctypes
    import torch
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    n, m, P = 600, 500, 3
    T = lp.dense_tableau("mixed", 11, n, m)
    _, _, _, _, bes = _simulate(T, n, m, 37, P, mode="fused")
    L = _lib.load()
    for be in bes:
        d = be.dev
        _lib.check(L.smx_fused_publish(ctypes.byref(be._shape), d.step & 1, d.ctl.data_ptr(),
                                       d.parts.data_ptr(), d.stream.cuda_stream), "publish")
        be.fused = be.overlap = False
    torch.cuda.synchronize()
    states, logs, tables, full, _ = _simulate(T, n, m, 45, P, bes=bes)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 82, threads=8)
    for s_, lg in zip(states, logs):
        assert s_["npivots"] == done
        assert np.array_equal(lg, log)
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))


def _nan_tables():
    """The gloo tests' NaN cases (simplex.py:117-121: a NaN first candidate sticks; a NaN that
    is not the global first candidate is ignored)."""
    n, m = 6, 3
    A = np.zeros((n + 1, m + 1))
    A[:, :m] = [[0, 1, 1], [0, -1, 2], [0, 1, -1], [np.nan, 1, 1], [-1, 1, 1], [-2, 1, 1],
                [-1, -1, -1]]
    A[:n, m] = [1, 2, 3, 1, 1, 1]
    n2, m2 = 6, 2
    B = np.zeros((n2 + 1, m2 + 1))
    B[:n2, 0] = [0, 0, -4, np.nan, -1, -3]
    B[:n2, 1] = [1, 1, 1, 1, 1, 1]
    B[:n2, m2] = [1, 1, 8, 1, 1, 1]
    B[n2, :m2] = [-1, -1]
    return [(A, n, m), (B, n2, m2)]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("P", [2, 3])
def test_hip_shards_nan_first_candidate(mode, case, P):
    from oracle import c_oracle
    T, n, m = _nan_tables()[case]
    states, logs, tables, full, _ = _simulate(T, n, m, 3, P, mode)
    Tref, st, done, log = c_oracle.run(T, n, m, m, 3)
    for s_, lg in zip(states, logs):
        assert s_["npivots"] == done
        assert np.array_equal(lg, log)
    assert np.array_equal(np.nan_to_num(full[:n]).view(np.int64),
                          np.nan_to_num(Tref[:n]).view(np.int64))
    assert np.array_equal(np.isnan(full[:n]), np.isnan(Tref[:n]))


@pytest.mark.parametrize("kind,n", [("uniform", 4095), ("mixed", 4096)])
def test_hip_shards_folded_pack(kind, n):
    """smx_tune_fold(0): the fused update's last look-ahead workgroup packs the next step."""
    from oracle import c_oracle
    from simplex_mi355x import _lib, lp
    L = _lib.load()
    m, k, P = 4095, 24, 2
    prev = L.smx_tune_fold(0)
    try:
        T = lp.dense_tableau(kind, 7, n, m)
        states, logs, tables, full, bes = _simulate(T, n, m, k, P, "fused")
        assert all(L.smx_shard_folds_pack(__import__("ctypes").byref(b._shape)) for b in bes)
    finally:
        L.smx_tune_fold(prev)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    for s_, lg in zip(states, logs):
        assert s_["npivots"] == done
        assert np.array_equal(lg, log)
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
