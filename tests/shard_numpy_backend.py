"""CPU stand-in for HipShardBackend, used only by the gloo tests of the sharded protocol.

It mirrors the HIP kernels' semantics and buffer layouts exactly (k_select + k_pack ->
smx_shard_begin, k_update<kShard> with its in-kernel header merge -> smx_shard_finish;
include/smx.h), so the
Python driver (simplex_mi355x.sharded.ShardedSolver) and its collective run unchanged over
gloo on CPU tensors.  The arithmetic follows oracle/numpy_oracle.py (simplex.py:149-177).
"""
from __future__ import annotations

import numpy as np
import torch

NONE = 0x7F7F7F7F
HDR = 8
PIVOT, OPTIMUM, INCORRECT, NOT_CONVERGE, FSHORT = 0, 1, 2, 3, 4


def _better(a, b):
    """Candidate order of the ratio test (cls, idx, v); True if a is strictly better."""
    if a[0] != b[0]:
        return a[0] < b[0]
    if a[0] == 0:
        return a[2] > b[2] or (a[2] == b[2] and a[1] > b[1])
    return a[1] < b[1]


class NumpyShardBackend:
    def __init__(self, local_T, n, m, flen, row0, world, ld=None):
        self.rows = local_T.shape[0] - 1
        self.n, self.m, self.flen, self.row0, self.world = n, m, flen, row0, world
        self.C = m + 1
        self.ld = ld if ld is not None else ((self.C + 15) // 16) * 16
        self.T = np.zeros((self.rows + 1, self.ld))
        self.T[:, :self.C] = local_T[:, :self.C]
        self.fscan = min(flen, m)
        self.slot = HDR + 2 * self.ld
        self.send = torch.zeros(self.slot, dtype=torch.float64)
        self.recv = torch.zeros(world * self.slot, dtype=torch.float64)
        self.step = 0
        self.negb = [NONE, NONE]
        self.negf = [NONE, NONE]
        self.term = False
        self.status, self.r, self.c = 5, NONE, NONE
        self.npivots = 0
        self.pivots = []
        self.negb[0], self.negf[0] = self._scan(self.T)

    def stream_ctx(self):
        import contextlib
        return contextlib.nullcontext()

    def _scan(self, T):
        b = np.flatnonzero(T[:self.rows, self.m] < 0)
        f = np.flatnonzero(T[self.rows, :self.fscan] < 0)
        return (self.row0 + int(b[0]) if b.size else NONE), (int(f[0]) if f.size else NONE)

    # -- k_select + k_pack ------------------------------------------------------------------
    def begin(self):
        if self.term:
            return
        p = self.step & 1
        self.negb[p ^ 1] = NONE
        self.negf[p ^ 1] = NONE
        negb, c = self.negb[p], self.negf[p]
        first, first_v, best = NONE, 0.0, (3, NONE, 0.0)
        if negb == NONE and c != NONE:
            a = self.T[:self.rows, c]
            cand = np.flatnonzero(a != 0)
            if cand.size:
                with np.errstate(all="ignore"):
                    v = self.T[cand, self.m] / a[cand]
                first, first_v = self.row0 + int(cand[0]), float(v[0])
                for i, vi in zip(cand, v):
                    if np.isnan(vi):
                        continue
                    cls = 0 if vi < 0 else (1 if vi == 0 else 2)
                    x = (cls, self.row0 + int(i), float(vi))
                    if _better(x, best):
                        best = x
        p1 = NONE   # phase 1: the owner scans its own first-negative-b row (simplex.py:81-85)
        if negb != NONE:
            pos = np.flatnonzero(self.T[negb - self.row0, :self.m] > 0)
            p1 = int(pos[0]) if pos.size else NONE
        send = self.send.numpy()
        send[:HDR] = [negb, first, first_v, best[0], best[1], best[2], c, p1]
        if first != NONE and np.isnan(first_v):
            send[HDR:HDR + self.ld] = self.T[first - self.row0]
        rb = negb if negb != NONE else (best[1] if best[0] < 3 else NONE)
        if rb != NONE:
            send[HDR + self.ld:HDR + 2 * self.ld] = self.T[rb - self.row0]

    # -- k_merge + k_update<kShard> ---------------------------------------------------------
    def _merge(self, recv):
        """merge_headers over recv = [world][stride] (headers first): (status, r, c, owner,
        offset of the winning row in the owner's send slot)."""
        gnegb, owner_b, gfirst, owner_f, fv = NONE, -1, NONE, -1, 0.0
        best, owner_best, c = (3, NONE, 0.0), -1, NONE
        for q in range(self.world):
            h = recv[q]
            if int(h[0]) < gnegb:
                gnegb, owner_b = int(h[0]), q
            if int(h[1]) < gfirst:
                gfirst, fv, owner_f = int(h[1]), h[2], q
            o = (int(h[3]), int(h[4]), h[5])
            if _better(o, best):
                best, owner_best = o, q
            c = int(h[6])
        r, owner, off = NONE, -1, 0
        if gnegb != NONE:
            r, owner, off = gnegb, owner_b, HDR + self.ld
            c = int(recv[owner_b, 7])
            status = PIVOT if c != NONE else INCORRECT
        elif c == NONE:
            status = FSHORT if self.flen < self.m else OPTIMUM
        elif gfirst == NONE:
            status = NOT_CONVERGE
        elif np.isnan(fv):
            status, r, owner, off = PIVOT, gfirst, owner_f, HDR
        elif best[0] >= 2:
            status = NOT_CONVERGE
        else:
            status, r, owner, off = PIVOT, best[1], owner_best, HDR + self.ld
        return status, r, c, owner, off

    def finish(self, ev_before=None, ev_after=None):
        recv = self.recv.numpy().reshape(self.world, self.slot)
        self._apply(recv, None)

    def _apply(self, recv, row):
        """the pivot from the merged headers; row = the pivot row (light exchange) or None (it
        is read from the gathered slots)"""
        p = self.step & 1
        self.step += 1
        if self.term:
            return
        status, r, c, owner, off = self._merge(recv)
        if status == PIVOT and row is None:
            row = recv[owner, off:off + self.ld]
        self.status, self.r, self.c = status, r, c
        if status != PIVOT:
            self.term = True
            return
        self.pivots.append((r, c))
        self.npivots += 1
        pr = row[:self.C].copy()
        e = pr[c]
        T = self.T[:, :self.C]
        pc = T[:, c].copy()
        with np.errstate(all="ignore"):
            N = T * e
            N -= np.multiply.outer(pc, pr)
            N /= e
            N[:, c] = pc / e
            rl = r - self.row0
            if 0 <= rl < self.rows:
                N[rl, :] = -T[rl, :] / e
                N[rl, c] = 1.0 / e
        self.T[:, :self.C] = N
        self.negb[p ^ 1], self.negf[p ^ 1] = self._scan(self.T)

    def state(self):
        return {"npivots": self.npivots, "term": self.term, "status": self.status,
                "r": self.r, "c": self.c}

    def log(self, start, stop):
        return np.array(self.pivots[start:stop], dtype=np.int32).reshape(-1, 2)

    def local_table(self):
        return self.T[:, :self.C].copy()


class NumpyBlockShardBackend(NumpyShardBackend):
    """CPU stand-in for sharded.BlockShardBackend.  The block protocol exchanges the same slots
    as the one-pivot protocol (header + rows A / B as values of T_{k+D}); the HIP kernels derive
    those rows from the block's input table by chains of the update expression, this mirror by
    keeping its rows materialised after every pivot -- the same values -- so pack is begin(),
    decide is finish(), and the sweep has nothing left to do."""

    def __init__(self, *args, pivots=8, **kw):
        super().__init__(*args, **kw)
        self.P = pivots          # (self.pivots is the mirror's pivot log)
        self.calls = []

    def parity(self):
        return self.step & 1

    def prime(self):
        self.calls.append(("prime",))

    def pack(self, step, pivots, block, parity):
        assert parity == (self.step - step) & 1, "pack on the block's input parity"
        self.calls.append(("pack", step, pivots, block))
        self.begin()

    def decide(self, step, pivots, parity, block):
        self.calls.append(("decide", step, pivots, block))
        self.finish()

    # -- the light exchange (smx_bshard_pick / smx_bshard_step_light) --------------------------
    @property
    def row(self):
        return self.recv[self.world * HDR:self.world * HDR + self.ld]

    def pick(self, rank):
        self.calls.append(("pick", rank))
        if self.term:
            return
        hdrs = self.recv.numpy()[:self.world * HDR].reshape(self.world, HDR)
        status, r, c, owner, off = self._merge(hdrs)
        out = self.row.numpy().view(np.int64)
        if status == PIVOT and owner == rank:
            out[:] = self.send.numpy()[off:off + self.ld].view(np.int64)
        else:
            out[:] = np.iinfo(np.int64).min

    def decide_light(self, step, pivots, parity, block):
        self.calls.append(("decide", step, pivots, block))
        hdrs = self.recv.numpy()[:self.world * HDR].reshape(self.world, HDR)
        self._apply(hdrs, self.row.numpy().copy())

    def sweep(self, pivots, parity):
        self.calls.append(("sweep", pivots, parity))

    def publish(self, parity, block):
        self.calls.append(("publish", parity, block))
