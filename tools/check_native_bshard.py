"""Native RCCL block-shard chain (smx_bshard_run), 1-rank job, both exchanges: trajectory and
table vs the C oracle (bit for bit).  Run as a subprocess by tests/test_gpu_block_sharded.py
(it initialises torch.distributed).  The light exchange runs its real collectives here: the
header all-gather, k_bsh_pick and the MAX all-reduce over int64 of the pivot row."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]
for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29543"), ("RANK", "0"),
             ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
    os.environ.setdefault(k, v)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import c_oracle  # noqa: E402
from simplex_mi355x import _lib, lp  # noqa: E402
from simplex_mi355x.sharded import BlockShardBackend, RcclComm  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
ok = True
cases = (("uniform", 1023, 777, 120, 8), ("mixed", 600, 500, 150, 5),
         ("degenerate", 300, 300, 100, 3), ("uniform", 40, 30, 400, 8),
         ("mixed", 2047, 2047, 40, 8))
for xmode, name in ((0, "full"), (1, "light")):
    _lib.tune_shard_xchg(xmode)
    for kind, n, m, k, P in cases:
        T = lp.dense_tableau(kind, 5, n, m)
        Tref, s_ref, done, log = c_oracle.run(T, n, m, m, k, threads=8)
        # eager: smx_bshard_run; graph: two replays of captured chains of k // 3 pivots (the
        # second from the other parity when k // 3 is odd), then the rest eagerly
        for how in ("eager", "graph"):
            be = BlockShardBackend(T, n, m, m, 0, 1, device="cuda:0", pivots=P)
            comm = RcclComm()
            if how == "eager":
                be.run_native(k, comm)
            else:
                kk = max(1, k // 3)
                be.run_graph(kk, comm)
                be.run_graph(kk, comm)
                if k > 2 * kk:
                    be.run_native(k - 2 * kk, comm)
            st = be.state()
            got = be.local_table()
            same = (st["npivots"] == done and np.array_equal(be.log(0, done), log)
                    and np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
                    and (not st["term"] or st["status"] == s_ref))
            print(name, how, kind, n, m, P, "pivots", st["npivots"], done,
                  "ok" if same else "MISMATCH", flush=True)
            ok &= same
            be.drop_graphs()
            comm.close()
_lib.tune_shard_xchg(-1)
dist.destroy_process_group()
sys.exit(0 if ok else 1)
