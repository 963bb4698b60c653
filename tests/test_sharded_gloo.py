"""World-size 2 and 3 runs of the sharded protocol over gloo on CPU (no GPU needed).

Each rank owns a contiguous row block plus the f-row replica (simplex_mi355x.sharded), runs the
product driver ShardedSolver with the numpy mirror of the HIP kernels, and the gathered result
must equal the unsharded C oracle bit for bit (trajectory and final table).
"""
from __future__ import annotations

import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "simplex-method-solver_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from shard_numpy_backend import NumpyShardBackend
    from simplex_mi355x.sharded import ShardedSolver, row_range

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    T = np.load(os.path.join(outdir, "T.npy"))
    n, m, k = case["n"], case["m"], case["k"]
    lo, hi = row_range(n, rank, world)
    local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
    be = NumpyShardBackend(local, n, m, m, lo, world)
    solver = ShardedSolver(be)
    st = solver.run(k)
    gathered = [None] * world
    dist.all_gather_object(gathered, be.local_table()[:-1].copy())
    if rank == 0:
        full = np.concatenate(gathered + [be.local_table()[-1:]], axis=0)
        np.save(os.path.join(outdir, "out.npy"), full)
        with open(os.path.join(outdir, "out.json"), "w") as fh:
            json.dump({"state": st, "log": be.log(0, st["npivots"]).tolist()}, fh)
    dist.barrier()
    dist.destroy_process_group()


def _case_T(kind, n, m, seed):
    from simplex_mi355x import lp
    return lp.dense_tableau(kind, seed, n, m)


CASES = [
    ("uniform", 64, 48, 60, 2),
    ("uniform", 61, 70, 60, 3),
    ("mixed", 50, 50, 80, 2),
    ("mixed", 47, 33, 80, 3),
    ("degenerate", 40, 30, 60, 2),
    ("degenerate_mixed", 45, 25, 60, 3),
    ("mixed", 2, 6, 20, 3),           # fewer constraint rows than ranks: rank 0 owns none
]


@pytest.mark.parametrize("kind,n,m,k,world", CASES)
def test_sharded_protocol_matches_oracle(tmp_path, kind, n, m, k, world):
    from oracle import c_oracle
    T = _case_T(kind, n, m, 3)
    _run(tmp_path, T, n, m, k, world)
    _compare(tmp_path, T, n, m, k)


def _run(tmp_path, T, n, m, k, world):
    np.save(tmp_path / "T.npy", T)
    case = {"n": n, "m": m, "k": k}
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)


def _compare(tmp_path, T, n, m, k):
    from oracle import c_oracle
    Tref, st, done, log = c_oracle.run(T, n, m, m, k)
    got = np.load(tmp_path / "out.npy")
    meta = json.load(open(tmp_path / "out.json"))
    assert meta["state"]["npivots"] == done
    assert meta["log"] == log.tolist()
    if meta["state"]["term"]:
        assert meta["state"]["status"] == st
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


def test_sharded_nan_first_candidate_on_second_rank(tmp_path):
    """Rank 0 has no candidate in the entering column; rank 1's first candidate has a NaN ratio
    (simplex.py:117-121: a NaN first candidate sticks) -> that row must be the pivot."""
    n, m = 6, 3
    T = np.zeros((n + 1, m + 1))
    T[:, :m] = [[0, 1, 1], [0, -1, 2], [0, 1, -1], [np.nan, 1, 1], [-1, 1, 1], [-2, 1, 1],
                [-1, -1, -1]]
    T[:n, m] = [1, 2, 3, 1, 1, 1]
    T[3, m] = 1.0
    _run(tmp_path, T, n, m, 1, 2)
    meta = json.load(open(tmp_path / "out.json"))
    assert meta["log"] == [[3, 0]]


def test_sharded_nan_first_local_but_not_global(tmp_path):
    """Rank 1's local first candidate is NaN but rank 0 has an earlier candidate: the global
    best (which lives on rank 1) must still arrive as rank 1's row B."""
    n, m = 6, 2
    T = np.zeros((n + 1, m + 1))
    T[:n, 0] = [0, 0, -4, np.nan, -1, -3]
    T[:n, 1] = [1, 1, 1, 1, 1, 1]
    T[:n, m] = [1, 1, 8, 1, 1, 1]
    T[n, :m] = [-1, -1]
    _run(tmp_path, T, n, m, 1, 2)
    _compare(tmp_path, T, n, m, 1)


# ---------------------------------------------------------------------------------------------
# block protocol (sharded.run_block_protocol, the driver of smx_bshard_*): pack -> all-gather
# -> decide per pivot, one sweep per block of P, publish -- over gloo with the numpy mirror
def _block_worker(rank, world, port, case, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "simplex-method-solver_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from shard_numpy_backend import NumpyBlockShardBackend
    from simplex_mi355x.sharded import row_range, run_block_protocol

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    T = np.load(os.path.join(outdir, "T.npy"))
    n, m, k, P = case["n"], case["m"], case["k"], case["P"]
    lo, hi = row_range(n, rank, world)
    local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
    be = NumpyBlockShardBackend(local, n, m, m, lo, world, pivots=P)
    done = 0
    for chunk in case["chunks"]:
        if case.get("light"):
            # header all-gather, pick, MAX all-reduce of the pivot row's int64 bit patterns
            hdr = 8
            run_block_protocol(
                be, chunk,
                lambda: dist.all_gather_into_tensor(be.recv[:world * hdr], be.send[:hdr]),
                pivots=P, rank=rank,
                reduce_row=lambda: dist.all_reduce(be.row.view(torch.int64),
                                                   op=dist.ReduceOp.MAX))
        else:
            run_block_protocol(be, chunk, lambda: dist.all_gather_into_tensor(be.recv, be.send),
                               pivots=P)
        done += chunk
    st = be.state()
    gathered = [None] * world
    dist.all_gather_object(gathered, be.local_table()[:-1].copy())
    if rank == 0:
        full = np.concatenate(gathered + [be.local_table()[-1:]], axis=0)
        np.save(os.path.join(outdir, "out.npy"), full)
        with open(os.path.join(outdir, "out.json"), "w") as fh:
            json.dump({"state": st, "log": be.log(0, st["npivots"]).tolist(),
                       "calls": be.calls}, fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("light", [False, True])
@pytest.mark.parametrize("kind,n,m,world,P,chunks", [
    ("uniform", 64, 48, 2, 8, [20, 13]),
    ("mixed", 47, 33, 3, 3, [7, 30]),
    ("degenerate_mixed", 45, 25, 2, 5, [60]),
    ("mixed", 2, 6, 3, 4, [9, 9]),        # rank 0 owns no rows
])
def test_block_protocol_matches_oracle(tmp_path, kind, n, m, world, P, chunks, light):
    """Both exchanges: the full send slots, and the light one (headers + the pivot row by a
    MAX all-reduce over int64 bit patterns, -0.0 included)."""
    T = _case_T(kind, n, m, 3)
    np.save(tmp_path / "T.npy", T)
    k = sum(chunks)
    case = {"n": n, "m": m, "k": k, "P": P, "chunks": chunks, "light": light}
    mp.spawn(_block_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world,
             join=True)
    _compare(tmp_path, T, n, m, k)
    calls = json.load(open(tmp_path / "out.json"))["calls"]
    # per chunk: prime, then blocks of P (last one ragged) of pack/decide pairs, sweep, publish
    exp = []
    for chunk in chunks:
        exp.append(["prime"])
        done = bn = 0
        while done < chunk:
            pb = min(P, chunk - done)
            for step in range(1, pb + 1):
                exp += [["pack", step - 1, pb, bn]]
                if light:
                    exp += [["pick", 0]]
                exp += [["decide", step, pb, bn]]
            exp.append(["sweep", pb, None])
            done += pb
            bn += 1
        exp.append(["publish", None, bn])
    got = [[c[0]] + [None if (c[0], i) in (("sweep", 2), ("publish", 1)) else x
                     for i, x in enumerate(c[1:], 1)] for c in calls]
    assert got == exp
