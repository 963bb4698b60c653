"""GPU parity at BASELINE.json's multi-GPU configs, at their real shapes:

* config 4 -- a 16384 x 16384 tableau row-sharded over 2 and then 4 ranks (block pivots, 8 per
  sweep, and the one-pivot fused protocol), bit for bit against the unsharded C oracle over a
  prefix with a ragged last block;
* config 5 -- a 65536 x 32768 degenerate tableau (both degenerate generators), the unsharded HIP
  path against the C oracle AT FULL SIZE over 209 pivots through the committed fixture
  tests/golden/config5.json (made in the build container by tests/golden/make_config5.py: the
  oracle's pivot log, its basis-cycle report and the table's SHA-256 after pivots 20, 60, 140 and
  209), and the same chain row-sharded over 8 ranks identical to it, row by row.

The ranks are simulated in one process on the one GPU of the test box: every rank is its own
``BlockShardBackend`` / ``HipShardBackend`` (own buffers, own stream), the all-gather is a device
copy of the concatenated send slots (tests/test_gpu_block_sharded.py), so the very kernels of the
multi-GPU run see the very bytes an RCCL all-gather would hand them.  Reference semantics:
/root/reference/src/simplex.py:70-177 (selection + update), :179-199 (the loop).
Host memory at config 5: the 17.2 GB table, the oracle's two 17.2 GB buffers and one download.
"""
from __future__ import annotations

import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


def _free():
    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _rows_equal_on_device(bes, dev, n, m):
    """Every rank's rows (and its f-row replica) equal the unsharded table's, compared on the
    device as int64 bit patterns (no 17 GB downloads)."""
    import torch
    from simplex_mi355x.sharded import row_range
    full = dev.cur()
    C = m + 1
    for p, be in enumerate(bes):
        lo, hi = row_range(n, p, len(bes))
        loc = be.dev.cur()
        a = loc[:hi - lo, :C].contiguous().view(torch.int64)
        b = full[lo:hi, :C].contiguous().view(torch.int64)
        assert torch.equal(a, b), f"rank {p}: rows {lo}..{hi} differ"
        fa = loc[hi - lo, :m].contiguous().view(torch.int64)
        fb = full[n, :m].contiguous().view(torch.int64)
        assert torch.equal(fa, fb), f"rank {p}: f-row replica differs"


def _cycle(n, m, log):
    from simplex_mi355x.basis import BasisTracker
    tr = BasisTracker(n, m)
    for r, c in log:
        if tr.pivot(int(r), int(c)):
            break
    return tr.cycle


# ----------------------------------------------------------------------------------------------
# config 4: 16384 x 16384 row-sharded across 2 then 4 ranks
@pytest.fixture(scope="module")
def table16k():
    from simplex_mi355x import lp
    from oracle import c_oracle
    n = m = 16383
    T = lp.dense_tableau("uniform", 0, n, m)
    k = 11   # one block of 8 + a ragged block of 3
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert done == k
    yield T, Tref, log
    del T, Tref
    gc.collect()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_config4_block_sharded_16k(table16k, world):
    """16384^2, 8 pivots per sweep on every rank, 11 pivots (8 + a ragged 3): pivots and the
    whole table bit for bit against the unsharded C oracle."""
    from test_gpu_block_sharded import _backends, _lockstep, _result
    T, Tref, log = table16k
    n = m = 16383
    bes = _backends(T, n, m, world, 8)
    _lockstep(bes, 8, 8)
    _lockstep(bes, 3, 8)
    states, logs, tables, full = _result(bes)
    for s, lg in zip(states, logs):
        assert s["npivots"] == 11 and not s["term"]
        assert np.array_equal(lg, log)
    for t in tables[1:]:
        assert np.array_equal(t[-1, :m].view(np.int64), tables[0][-1, :m].view(np.int64))
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(full[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
    del bes, full, tables
    _free()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_config4_one_pivot_sharded_16k(table16k, world):
    """16384^2 with the one-pivot protocol (fused pack -> all-gather -> fused update per pivot),
    11 pivots: bit for bit against the C oracle."""
    from test_gpu_sharded import _simulate
    T, Tref, log = table16k
    n = m = 16383
    states, logs, tables, full, bes = _simulate(T, n, m, 11, world, "fused")
    for s, lg in zip(states, logs):
        assert s["npivots"] == 11
        assert np.array_equal(lg, log)
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(full[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
    del bes, full, tables
    _free()


# ----------------------------------------------------------------------------------------------
# config 5: 65536 x 32768 row-sharded across 8 ranks, degenerate / anti-cycling stress
@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["degenerate", "degenerate_mixed"])
def test_config5_sharded_65536x32768(kind):
    """The unsharded block chain (20 pivots per sweep, the window planner) against the C oracle's
    full-size run (fixture): every pivot, the cycle report, the whole table after 20, 60, 140 and
    209 pivots; 8 simulated ranks (8 pivots per sweep, the register planner and the exchange of
    the multi-GPU run) identical to it after 9 and 209 pivots."""
    from golden_util import load, table_sha256
    from simplex_mi355x import lp
    from simplex_mi355x.device import DeviceTableau
    from test_gpu_block_sharded import _backends, _lockstep
    fx = [c for c in load("config5.json")["cases"] if c["kind"] == kind][0]
    n, m, world, P = 65535, 32767, 8, 8
    assert (fx["n"], fx["m"], fx["seed"]) == (n, m, 0)
    T = lp.dense_tableau(kind, 0, n, m)
    dev = DeviceTableau(T, n, m, m, log_cap=1 << 12)
    assert dev.block_plan()[1] == 20           # the unsharded path: up to 20 pivots per sweep (8 GiB)
    bes = _backends(T, n, m, world, P)
    del T
    gc.collect()
    done = 0
    for stop in (9, 20, 60, 140, fx["pivots"]):
        dev.run(stop - done, graph=False)
        ctl = dev.sync_state()
        assert int(ctl["npivots"]) == stop and not ctl["term"], (stop, int(ctl["npivots"]))
        if stop == 9:
            _lockstep(bes, 9, P)
        elif stop == fx["pivots"]:
            _lockstep(bes, stop - 9, P)
        done = stop
        assert dev.read_log(0, stop).tolist() == fx["log"][:stop], stop
        if str(stop) in fx["sha256"]:
            got = dev.download()
            assert table_sha256(got, n, m) == fx["sha256"][str(stop)], stop
            del got
            gc.collect()
        if stop == 9:
            for be in bes:
                assert be.state()["npivots"] == 9
                assert be.log(0, 9).tolist() == fx["log"][:9]
            _rows_equal_on_device(bes, dev, n, m)
    total = fx["pivots"]
    cyc = _cycle(n, m, dev.read_log(0, total))
    assert (list(cyc) if cyc else None) == fx["cycle"]
    for be in bes:
        s = be.state()
        assert s["npivots"] == total and not s["term"]
        assert be.log(0, total).tolist() == fx["log"]
    _rows_equal_on_device(bes, dev, n, m)
    print(f"config 5 ({kind}): {total} pivots, basis cycle {cyc} = the oracle's")
    del bes, dev
    _free()
