"""GPU: block pivots on row-sharded tableaux (smx_bshard_*, csrc/smx_block.hpp) for P simulated
ranks in one process on one device, the all-gather done by a device copy, driven in lockstep by
the protocol of sharded.run_block_protocol -- against the unsharded C oracle, bit for bit.  The
multi-process driver runs over gloo in tests/test_sharded_gloo.py; the native RCCL chain
(smx_bshard_run) at world size 1 through bench.py --sharded below."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


def _backends(T, n, m, world, pivots):
    from simplex_mi355x.sharded import BlockShardBackend, row_range
    bes = []
    for p in range(world):
        lo, hi = row_range(n, p, world)
        local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
        bes.append(BlockShardBackend(local, n, m, m, lo, world, pivots=pivots))
    return bes


def _lockstep(bes, k, P, light=False):
    """run_block_protocol for every simulated rank at once (the exchange is a device copy).
    light: the headers are copied, every rank picks, and the pivot-row buffers are reduced with
    MAX over their int64 bit patterns (what the RCCL all-reduce of the light exchange does)."""
    import torch
    hdr = 8
    for be in bes:
        with be.stream_ctx():
            be.prime()
    parity = bes[0].parity()
    done = bn = 0
    while done < k:
        pb = min(P, k - done)
        for step in range(1, pb + 1):
            for be in bes:
                with be.stream_ctx():
                    be.pack(step - 1, pb, bn, parity)
            torch.cuda.synchronize()
            if not light:
                allsend = torch.cat([be.send for be in bes])
                for be in bes:
                    be.recv.copy_(allsend)
                torch.cuda.synchronize()
                for be in bes:
                    with be.stream_ctx():
                        be.decide(step, pb, parity, bn)
                continue
            allhdr = torch.cat([be.send[:hdr] for be in bes])
            for be in bes:
                be.recv[:len(bes) * hdr].copy_(allhdr)
            torch.cuda.synchronize()
            for q, be in enumerate(bes):
                with be.stream_ctx():
                    be.pick(q)
            torch.cuda.synchronize()
            rowmax = torch.stack([be.row.view(torch.int64) for be in bes]).amax(dim=0)
            for be in bes:
                be.row.view(torch.int64).copy_(rowmax)
            torch.cuda.synchronize()
            for be in bes:
                with be.stream_ctx():
                    be.decide_light(step, pb, parity, bn)
        for be in bes:
            with be.stream_ctx():
                be.sweep(pb, parity)
        parity = (parity + pb) & 1
        done += pb
        bn += 1
    for be in bes:
        with be.stream_ctx():
            be.publish(parity, bn)
    torch.cuda.synchronize()


def _result(bes):
    states = [be.state() for be in bes]
    logs = [be.log(0, s["npivots"]) for be, s in zip(bes, states)]
    tables = [be.local_table() for be in bes]
    full = np.concatenate([t[:-1] for t in tables] + [tables[0][-1:]], axis=0)
    return states, logs, tables, full


@pytest.mark.parametrize("kind,n,m,world,P,chunks", [
    ("uniform", 1023, 1023, 2, 8, [40, 21]),
    ("uniform", 1001, 777, 3, 5, [60]),
    ("uniform", 2047, 2047, 8, 8, [32]),
    ("mixed", 700, 600, 4, 3, [50, 50]),       # phase 1 first
    ("degenerate", 511, 511, 4, 8, [120]),
    ("degenerate_mixed", 300, 500, 5, 6, [60, 60]),
    ("uniform", 40, 30, 3, 4, [78]),           # pivot row = first row of the next rank
    ("mixed", 5, 7, 8, 8, [30]),               # fewer constraint rows than ranks
    ("uniform", 4095, 4095, 2, 8, [24]),
    ("degenerate_mixed", 9, 3, 4, 2, [40]),
])
@pytest.mark.parametrize("light", [False, True])
def test_block_shards_match_oracle(kind, n, m, world, P, chunks, light):
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 7, n, m)
    bes = _backends(T, n, m, world, P)
    for chunk in chunks:
        _lockstep(bes, chunk, P, light)
        if bes[0].state()["term"]:
            break
    states, logs, tables, full = _result(bes)
    k = sum(chunks)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    for s, lg in zip(states, logs):
        assert s["npivots"] == done
        assert np.array_equal(lg, log)
        if s["term"]:
            assert s["status"] == st
    for t in tables[1:]:   # every f-row replica identical
        assert np.array_equal(t[-1, :m].view(np.int64), tables[0][-1, :m].view(np.int64))
    assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(full[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


def test_block_shards_terminal_outcomes():
    """Every non-capped random fixture on 2 and 3 simulated ranks: same pivots, outcome status
    and final table as the oracle (terminal outcomes land inside blocks)."""
    from golden_util import dec_input, load
    from oracle import c_oracle
    seen = 0
    for rec in load("random.json"):
        if rec["outcome"]["kind"] == "cap":
            continue
        cons, func = dec_input(rec["input"])
        n, m = len(cons), len(cons[0]) - 1
        if len(func) != m:
            continue
        T = np.zeros((n + 1, m + 1))
        T[:n] = np.array(cons, dtype=np.float64)
        T[n, :m] = np.array(func, dtype=np.float64)
        Tref, st, done, log = c_oracle.run(T, n, m, m, 10_000, threads=4)
        world = 2 + seen % 2
        bes = _backends(T, n, m, world, 3 + seen % 4)
        # three more blocks after the one holding the terminal outcome: a stopped chain's later
        # blocks decode stale headers and must touch nothing (smx_block.hpp, the stopped return)
        P = bes[0].pivots
        _lockstep(bes, done + 2 + 3 * P, P, light=bool(seen % 3 == 1))
        states, logs, tables, full = _result(bes)
        assert states[0]["npivots"] == done
        assert np.array_equal(logs[0], log)
        assert states[0]["term"] and states[0]["status"] == st
        assert np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
        seen += 1
    assert seen > 10


@pytest.mark.parametrize("xchg", ["full", "light"])
def test_native_block_shard_chain_world1(xchg):
    """bench.py --sharded at world size 1: smx_bshard_run_timed with libsmx's own RCCL
    communicator, 8 pivots per sweep, both exchanges (light: header all-gather, pick, max
    all-reduce on int64); the trajectory must stay valid."""
    env = dict(os.environ)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--sharded",
                          "--size", "2048", "--steps", "40", "--warmup", "8", "--xchg", xchg,
                          "--no-cpu-baseline"], capture_output=True, text=True, env=env,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["trajectory_valid"] and d["n_gpus"] == 1
    assert d["config"]["pivots_per_sweep"] == 8
    assert d["config"]["exchange"] == xchg


@pytest.mark.parametrize("light", [False, True])
def test_block_shards_edge_fixtures(light):
    """The edge fixtures (NaN first / later ratio candidates, inf, -0.0 "-b", m = 1, n = 1) on 2
    and 3 simulated ranks, both exchanges: the NaN-first row travels as row A of its owner."""
    from golden_util import dec_input, load
    from oracle import c_oracle
    seen = 0
    for label, rec in load("edge.json").items():
        cons, func = dec_input(rec["input"])
        n, m = len(cons), len(cons[0]) - 1
        if len(func) != m or m < 1:
            continue
        T = np.zeros((n + 1, m + 1))
        T[:n] = np.array(cons, dtype=np.float64)
        T[n, :m] = np.array(func, dtype=np.float64)
        Tref, st, done, log = c_oracle.run(T, n, m, m, 200, threads=2)
        for world in (2, 3):
            bes = _backends(T, n, m, world, 3)
            _lockstep(bes, min(done + 2, 200), 3, light)
            states, logs, tables, full = _result(bes)
            assert states[0]["npivots"] == done, label
            assert np.array_equal(logs[0], log)
            # NaN payloads / signs are not part of the contract: NaN
            # positions must agree, every other element bit for bit
            a, b = full[:n], Tref[:n]
            assert np.array_equal(np.isnan(a), np.isnan(b)), label
            ok = ~np.isnan(a)
            assert np.array_equal(a[ok].view(np.int64), b[ok].view(np.int64)), label
        seen += 1
    assert seen >= 5


def test_native_block_shard_chain_both_exchanges_vs_oracle():
    """smx_bshard_run with libsmx's own RCCL communicator at world size 1, full and light
    exchange, eagerly and replayed from captured hipGraphs (smx_bshard_graph_create, RCCL
    collectives inside the graph), against the C oracle (tools/check_native_bshard.py, its own
    process)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_native_bshard.py")],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-3000:])
    assert out.stdout.count(" ok") == 20, out.stdout
    assert out.stdout.count("graph ") == 10, out.stdout
