"""The multi-GPU bench line's extra records on CPU (no GPU, gloo world 2): what RCCL formed
(sharded.comm_record, through a stub communicator) and the cpu_baseline block of rank 0
(sharded.sharded_cpu_baseline, through a stub baseline function) -- the keys the driver's
N > 1 lines carry (bench.py --gpus N)."""
from __future__ import annotations

import json
import os
import socket
from types import SimpleNamespace

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _StubComm:
    def __init__(self, count, rank, device):
        self._v = (count, rank, device)

    def info(self):
        return self._v


def _worker(rank, world, port, outdir, bad):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "simplex-method-solver_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from simplex_mi355x.sharded import comm_record
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    # bad: rank 1 reports a communicator of one rank on rank 0's device
    comm = _StubComm(1, 0, 0) if (bad and rank == 1) else _StubComm(world, rank, rank)
    rec = comm_record(comm, device_index=rank)
    with open(os.path.join(outdir, f"rec{rank}.json"), "w") as fh:
        json.dump(rec, fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bad", [False, True])
def test_comm_record_world2(tmp_path, bad):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), bad), nprocs=2, join=True)
    recs = [json.load(open(tmp_path / f"rec{r}.json")) for r in range(2)]
    assert recs[0] == recs[1]          # every rank gathers the same record
    rec = recs[0]
    assert rec["consistent"] is (not bad)
    assert rec["rccl_ranks"] == 2
    assert [r["rank"] for r in rec["ranks"]] == [0, 1]
    for r in rec["ranks"]:
        for k in ("comm_count", "comm_user_rank", "comm_device", "hip_device", "host"):
            assert k in r
    if not bad:
        assert [r["comm_device"] for r in rec["ranks"]] == [0, 1]


def test_sharded_cpu_baseline_scopes():
    import numpy as np
    from simplex_mi355x import lp
    from simplex_mi355x.sharded import row_range, sharded_cpu_baseline
    seen = []

    def stub(T, n, m, seconds):
        seen.append((T.shape, n, m, seconds, T.copy()))
        return {"value": 1.0, "unit": "pivots/s", "cores": 1, "kind": "port", "sample": "stub"}

    args = SimpleNamespace(kind="uniform", seed=3, cpu_seconds=2.0)
    n, m = 63, 47
    lo, hi = row_range(n, 0, 4)
    full = sharded_cpu_baseline(stub, args, n, m, lo, hi)
    assert full["scope"].startswith("full 64x48") and full["kind"] == "port"
    shape, nn, mm, sec, T = seen[-1]
    assert shape == (64, 48) and (nn, mm, sec) == (63, 47, 2.0)
    assert np.array_equal(T, lp.dense_tableau("uniform", 3, n, m))
    part = sharded_cpu_baseline(stub, args, n, m, lo, hi, full_limit_bytes=1024)
    assert part["scope"].startswith("rank 0's row block")
    shape, nn, mm, sec, T = seen[-1]
    assert shape == (hi - lo + 1, 48) and nn == hi - lo
    ref = lp.dense_tableau("uniform", 3, n, m)
    assert np.array_equal(T[:-1], ref[lo:hi]) and np.array_equal(T[-1], ref[-1])
