"""Two PROCESSES on the one GPU run the row-sharded block protocol of a multi-GPU job in lockstep
(VERDICT r5 item 3): each is a rank with its own ``BlockShardBackend`` -- the very kernels the
driver's 8-GPU run launches (smx_bshard_prime / pack / step / sweep / publish, csrc/smx_block.hpp)
-- and its own HIP stream, and the per-pivot exchange goes through torch.distributed across the
process boundary.  RCCL refuses two ranks on one device (ncclInvalidUsage), so the
exchange is host-staged over gloo: the send slot (full exchange) or the header (light exchange) is
copied to the host, all-gathered, and copied into ``recv``; the light exchange's pivot row is then
MAX-all-reduced over its int64 bit patterns (include/smx.h, smx_bshard_pick).  Everything else is
the multi-process path of ``sharded.run_block_protocol``.  Both ranks' rows, the f-row replica and
the pivot log must equal the unsharded C oracle bit for bit (reference semantics:
/root/reference/src/simplex.py:70-199; caller /root/reference/src/main.py:313).
"""
from __future__ import annotations

import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


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
    from simplex_mi355x import _lib
    from simplex_mi355x.sharded import BlockShardBackend, row_range, run_block_protocol

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.cuda.set_device(0)
    T = np.load(os.path.join(outdir, "T.npy"))
    n, m, k, P, xchg = case["n"], case["m"], case["k"], case["P"], case["xchg"]
    lo, hi = row_range(n, rank, world)
    local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
    be = BlockShardBackend(local, n, m, m, lo, world, device="cuda:0", pivots=P)
    dev = be.dev.device
    cnt = be.slot if xchg == "full" else _lib.SHARD_HDR

    def exchange():
        # (inside be.stream_ctx(): the current stream is the rank's solver stream)
        torch.cuda.current_stream().synchronize()
        mine = be.send[:cnt].cpu()
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        be.recv[:world * cnt].copy_(torch.cat(parts).to(dev))

    def reduce_row():
        torch.cuda.current_stream().synchronize()
        row = be.row.cpu().view(torch.int64).clone()
        dist.all_reduce(row, op=dist.ReduceOp.MAX)
        be.row.copy_(row.view(torch.float64).to(dev))

    run_block_protocol(be, k, exchange, pivots=P,
                       reduce_row=reduce_row if xchg == "light" else None, rank=rank)
    torch.cuda.synchronize()
    st = be.state()
    table = be.local_table()
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, table[:hi - lo].copy(), table[hi - lo].copy(),
                                      be.log(0, st["npivots"]).tolist(), st))
    if rank == 0:
        full = np.empty_like(T)
        meta = {"states": [], "logs": [], "frow_equal": True}
        for lo_p, hi_p, rows_p, frow_p, log_p, st_p in gathered:
            full[lo_p:hi_p] = rows_p
            meta["states"].append(st_p)
            meta["logs"].append(log_p)
        full[n] = gathered[0][3]
        for g in gathered[1:]:
            meta["frow_equal"] &= bool(np.array_equal(g[3][:m].view(np.int64),
                                                      gathered[0][3][:m].view(np.int64)))
        np.save(os.path.join(outdir, "out.npy"), full)
        with open(os.path.join(outdir, "out.json"), "w") as fh:
            json.dump(meta, fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,n,m,k,P", [
    ("uniform", 4095, 4095, 30, 8),        # BASELINE-shaped, blocks of 8 + a ragged 6
    ("mixed", 2047, 3071, 40, 12),         # phase 1 first
])
@pytest.mark.parametrize("xchg", ["full", "light"])
def test_two_process_block_protocol_vs_oracle(tmp_path, kind, n, m, k, P, xchg):
    from oracle import c_oracle
    from simplex_mi355x import lp
    T = lp.dense_tableau(kind, 5, n, m)
    np.save(tmp_path / "T.npy", T)
    case = {"n": n, "m": m, "k": k, "P": P, "xchg": xchg}
    mp.spawn(_worker, args=(2, _free_port(), case, str(tmp_path)), nprocs=2, join=True)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    got = np.load(tmp_path / "out.npy")
    meta = json.load(open(tmp_path / "out.json"))
    for s, lg in zip(meta["states"], meta["logs"]):
        assert s["npivots"] == done
        assert lg == log.tolist()
    assert meta["frow_equal"]
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))
