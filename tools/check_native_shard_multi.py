"""Native RCCL shard driver with WORLD_SIZE > 1 on whatever GPUs exist (ranks share a device when
there are fewer GPUs than ranks): every rank runs its row block through libsmx's own RCCL
communicator, and rank 0 compares the gathered trajectory and table with the C oracle.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
           --master-port 29555 tools/check_native_shard_multi.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from simplex_mi355x import lp  # noqa: E402
from simplex_mi355x.sharded import HipShardBackend, RcclComm, ShardedSolver, row_range  # noqa


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")        # bootstrap only; the data path is libsmx's RCCL
    ok = True
    cases = (("uniform", 1023, 777, 120), ("mixed", 600, 500, 150), ("degenerate", 300, 300, 100),
             ("uniform", 40, 30, 400), ("mixed", 5, 7, 30))
    modes = (("fused", True), ("unfused", False))
    for (mode, fused), (kind, n, m, k) in [(md, c) for md in modes for c in cases]:
        T = lp.dense_tableau(kind, 5, n, m)
        lo, hi = row_range(n, rank, world)
        local = np.concatenate([T[lo:hi], T[n:n + 1]], axis=0)
        be = HipShardBackend(local, n, m, m, lo, world, device=f"cuda:{dev}", fused=fused)
        comm = RcclComm()
        st = ShardedSolver(be, comm=comm).run(k)
        tab = be.local_table()
        parts = [None] * world
        dist.all_gather_object(parts, (tab[:-1], be.log(0, st["npivots"]), st))
        if rank == 0:
            from oracle import c_oracle
            full = np.concatenate([p[0] for p in parts] + [tab[-1:]], axis=0)
            Tref, s_ref, done, log = c_oracle.run(T, n, m, m, k, threads=8)
            same = all(p[2]["npivots"] == done and np.array_equal(p[1], log) for p in parts)
            same &= np.array_equal(full[:n].view(np.int64), Tref[:n].view(np.int64))
            same &= (not st["term"]) or st["status"] == s_ref
            print(mode, kind, n, m, "world", world, "pivots", st["npivots"], done,
                  "ok" if same else "MISMATCH", flush=True)
            ok &= bool(same)
        comm.close()
        dist.barrier()
    flag = [ok]
    dist.broadcast_object_list(flag, src=0)
    dist.destroy_process_group()
    sys.exit(0 if flag[0] else 1)


if __name__ == "__main__":
    main()
