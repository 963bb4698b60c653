"""A tableau row-partitioned over several devices of ONE process: ``SimplexMethod(...,
devices=[...])``.

The reference has one caller, ``SimplexMethod(y, c).get_solution()`` (main.py:313 ->
simplex.py:179-199); this puts the row-sharded engine behind exactly that surface.  Rank p of
``len(devices)`` owns the constraint rows ``[p*n/P, (p+1)*n/P)`` (sharded.row_range) on
``devices[p]`` with its own stream and a replica of the f-row, and the ranks run the block protocol
of the multi-process engine (smx_bshard_*, csrc/smx_block.hpp): per pivot every rank packs its
header and candidate rows, the send slots are exchanged, every rank merges them identically and
logs the pivot; every ``pivots`` pivots one sweep per rank applies them.  The exchange is native
(``smx_mshard_run``, include/smx.h):

* distinct devices -- one grouped RCCL all-gather per pivot over ``ncclCommInitAll``
  communicators (xGMI);
* repeated devices (e.g. ``devices=[0, 0, 0, 0]`` on a one-GPU box) -- RCCL refuses two ranks on
  one GPU, so every rank copies every send slot into its receive buffer, ordered by events.

Step-wise calls (``pick_element`` / ``recalculate_matrix`` / ``step``) are the same protocol with
one pivot per block: ``pick`` plans the pivot (records, exchange, merge) without touching the
table, restoring the control blocks if it is not followed by an apply; ``apply_selected`` sweeps
and publishes.  The x-history ring of each rank holds the label rows it owns
(include/smx.h, smx_bshard_*); :meth:`read_xhist` takes every value from the owner of the label's
row, tracked from the pivot log like simplex.py:152 moves the labels.  Lazy ``get_solution``
tables (engine.History) are checkpointed as whole gathered tables on ``devices[0]``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .device import Graph, int_first_fix
from .sharded import BlockShardBackend, row_range


def _norm(d) -> torch.device:
    if isinstance(d, int):
        return torch.device("cuda", d)
    d = torch.device(d)
    if d.type != "cuda":
        raise ValueError(f"devices must be HIP devices, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def _move(code: int, r: int, c: int) -> int:
    """Label position code after pivot (r, c): row p >= 0, column j as -(j+1) (simplex.py:152)."""
    if code == -(c + 1):
        return r
    if code == r:
        return -(c + 1)
    return code


class MultiTableau:
    """The DeviceTableau surface SimplexMethod uses, over P row blocks on P (device, stream)s."""

    is_host = False

    def __init__(self, dense: np.ndarray, n: int, m: int, flen: int, devices, *,
                 pivots: int | None = None, log_cap: int = 1 << 16, exchange: str | None = None,
                 graph_chain: bool = False):
        if not torch.cuda.is_available():
            raise RuntimeError("simplex_mi355x needs an MI355X (HIP device); there is no CPU path")
        L = _lib.load()
        self.devices = [_norm(d) for d in devices]
        self.world = P = len(self.devices)
        if P < 1:
            raise ValueError("devices must name at least one device")
        self.n, self.m, self.flen = n, m, flen
        self.rows = n
        self.C = m + 1
        self.P = int(pivots) if pivots else 8   # the sharded protocol pays one exchange per pivot
        if not 1 <= self.P <= _lib.BLOCK_MAX:
            raise ValueError(f"pivots per sweep must be 1..{_lib.BLOCK_MAX}")
        self.ranges = [row_range(n, p, P) for p in range(P)]
        self.ranks = []
        for p, dev in enumerate(self.devices):
            lo, hi = self.ranges[p]
            local = np.concatenate([dense[lo:hi], dense[n:n + 1]], axis=0)
            with torch.cuda.device(dev):
                self.ranks.append(BlockShardBackend(local, n, m, flen, lo, P, device=dev,
                                                    log_cap=log_cap, pivots=self.P))
        r0 = self.ranks[0].dev
        self.ld = r0.ld
        self.device = self.devices[0]
        self.stream = r0.stream
        self.log_cap = log_cap
        self.shape = [self.ld, n, n, m, flen, 0, L.smx_nparts_for(n, m)]
        distinct = len({(d.index) for d in self.devices}) == P
        self.exchange = exchange or ("rccl" if distinct and P > 1 else "copy")
        self._comms = None
        if self.exchange == "rccl":
            comms = (ctypes.c_void_p * P)()
            devs = (ctypes.c_int32 * P)(*[d.index for d in self.devices])
            _lib.check(L.smx_mshard_comms(comms, P, devs), "smx_mshard_comms")
            self._comms = [comms[p] for p in range(P)]
        self._structs = self._rank_structs()
        self._aborted = False     # smx_mshard_run aborted the communicators (see _native)
        # opt-in: chained runs of ranks sharing ONE device (copy exchange) replay a captured graph
        # per (parity, k) -- one host call per chain instead of ~3N per pivot
        # (smx_mshard_graph_create); other layouts enqueue eagerly
        self.graph_chain = bool(graph_chain) and self.exchange == "copy" and \
            len({d.index for d in self.devices}) == 1 and P <= 16
        self._graphs = {}
        self.step = 0
        self._term = False
        self._saved = None        # control blocks before a pick() not yet applied
        self._xcodes = self._initial_codes()
        self._xstep = 0           # pivot count _xcodes describes
        self._xck = {0: self._xcodes}   # label codes at earlier read_xhist stops (see there)

    # -- native rank table --------------------------------------------------------------------
    def _rank_structs(self):
        arr = (_lib.Rank * self.world)()
        for p, be in enumerate(self.ranks):
            d = be.dev
            a = arr[p]
            a.device = self.devices[p].index
            a.stream = d.stream.cuda_stream
            a.buf0, a.buf1 = d.buf[0].data_ptr(), d.buf[1].data_ptr()
            a.ctl = d.ctl.data_ptr()
            a.blk, a.blk_bytes = be.blk.data_ptr(), be._nbytes
            a.send, a.recv = be.send.data_ptr(), be.recv.data_ptr()
            a.log, a.xhist, a.log_cap = d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap
            a.comm = self._comms[p] if self._comms else None
            a.shape = _lib.Shape(*d.shape)
        return arr

    def _native(self, k: int, pivots: int, graph: bool = False) -> None:
        if graph and self.graph_chain:
            key = (self.step & 1, int(k), int(pivots))
            g = self._graphs.get(key)
            if g is None:
                h = ctypes.c_void_p()
                _lib.check(_lib.load().smx_mshard_graph_create(
                    self._structs, self.world, self.step & 1, int(k), int(pivots),
                    ctypes.byref(h)), "smx_mshard_graph_create")
                g = self._graphs[key] = Graph(h.value)
            g.launch(self.ranks[0].dev.stream.cuda_stream)
            return
        if self._aborted:
            raise RuntimeError("MultiTableau: its RCCL communicators were aborted by an earlier "
                               "failed run; build a new MultiTableau")
        err = _lib.load().smx_mshard_run(
            self._structs, self.world, self.step & 1, int(k), int(pivots),
            _lib.XCHG_RCCL if self.exchange == "rccl" else _lib.XCHG_COPY)
        if err == _lib.ERR_COMMS_ABORTED:
            # aborted (and freed) by the library: no handle may reach RCCL again -- not through
            # the rank table either (a later run() passed the freed handles)
            self._comms = None
            for p in range(self.world):
                self._structs[p].comm = None
            self._aborted = True
        _lib.check(err, "smx_mshard_run")

    def _sync(self) -> None:
        for dev in self.devices:
            torch.cuda.synchronize(dev)

    # -- data movement ------------------------------------------------------------------------
    def upload(self, dense: np.ndarray) -> None:
        self.settle()
        n = self.n
        for p, be in enumerate(self.ranks):
            lo, hi = self.ranges[p]
            be.dev.upload(np.concatenate([dense[lo:hi], dense[n:n + 1]], axis=0))
        self.step = 0
        self._term = False
        self._saved = None
        self._xcodes = self._initial_codes()
        self._xstep = 0
        self._xck = {0: self._xcodes}

    def settle(self) -> None:
        for be in self.ranks:
            be.dev.settle()

    def cur(self) -> torch.Tensor:
        """The whole current table gathered on devices[0] (rows, then rank 0's f-row)."""
        self._sync()
        parts = []
        for p, be in enumerate(self.ranks):
            lo, hi = self.ranges[p]
            parts.append(be.dev.cur()[:hi - lo].to(self.device))
        lo, hi = self.ranges[0]
        parts.append(self.ranks[0].dev.cur()[hi - lo:hi - lo + 1].to(self.device))
        return torch.cat(parts)

    def download(self) -> np.ndarray:
        self._sync()
        tabs = [be.dev.download() for be in self.ranks]
        out = [t[:hi - lo] for t, (lo, hi) in zip(tabs, self.ranges)]
        out.append(tabs[0][-1:])
        return np.concatenate(out)

    def _owner(self, i: int) -> tuple[int, int]:
        """(rank, local row) of global row i; the f-row (i == n) from rank 0's replica."""
        if i == self.n:
            lo, hi = self.ranges[0]
            return 0, hi - lo
        for p, (lo, hi) in enumerate(self.ranges):
            if lo <= i < hi:
                return p, i - lo
        raise IndexError(i)

    def values(self, idx) -> list[float]:
        out = []
        for i, j in idx:
            p, li = self._owner(i)
            out.extend(self.ranks[p].dev.values([(li, j)]))
        return out

    def read_log(self, start: int, stop: int) -> np.ndarray:
        return self.ranks[0].dev.read_log(start, stop)

    def _initial_codes(self):
        return [(-1 if self.m >= 1 else None), (-2 if self.m >= 2 else None)]

    def read_xhist(self, start: int, stop: int) -> np.ndarray:
        """(x1, x2) after pivots start..stop-1, each from the rank owning the label's row."""
        if stop <= start:
            return np.zeros((0, 2), dtype=np.float64)
        if start != self._xstep:
            # re-derive the label positions at `start`: from the nearest earlier stop whose
            # codes were kept, replaying the pivots after it -- which must still be in the
            # device's log ring (log_cap entries; older ones are overwritten)
            s0 = max(k for k in self._xck if k <= start)
            if max(self.step, stop) - s0 > self.log_cap:
                raise RuntimeError(
                    f"x-history from pivot {start}: the pivots after {s0} are no longer in the "
                    f"device log ring (log_cap = {self.log_cap}); read the history in order")
            codes = list(self._xck[s0])
            for r, c in self.read_log(s0, start):
                codes = [None if x is None else _move(x, int(r), int(c)) for x in codes]
            self._xcodes, self._xstep = codes, start
        log = self.read_log(start, stop)
        rings = [be.dev.read_xhist(start, stop) for be in self.ranks]
        out = np.zeros((stop - start, 2), dtype=np.float64)
        codes = self._xcodes
        for t, (r, c) in enumerate(log):
            codes = [None if x is None else _move(x, int(r), int(c)) for x in codes]
            for q, x in enumerate(codes):
                if x is not None and x >= 0:
                    p, _ = self._owner(x)
                    out[t, q] = rings[p][t, q]
        self._xcodes, self._xstep = codes, stop
        self._xck[stop] = codes
        if len(self._xck) > 64:   # keep the start and the newest stops
            for k in sorted(self._xck)[1:-32]:
                del self._xck[k]
        return out

    def block_plan(self):
        return None

    def resident_plan(self):
        return None

    # -- pivot loop ---------------------------------------------------------------------------
    def _restore(self) -> None:
        if self._saved is not None:
            for be, saved in zip(self.ranks, self._saved):
                with be.stream_ctx():
                    be.dev.ctl.copy_(saved)
            self._saved = None

    def pick(self):
        """pick_element: plan one pivot on every rank (records, exchange, merge); the table is
        untouched and the control blocks are restored unless apply_selected() follows."""
        self.settle()
        self._restore()
        if self._term:
            self.clear_term()
        self._saved = []
        for be in self.ranks:
            with be.stream_ctx():
                self._saved.append(be.dev.ctl.clone())
        # run_block_protocol's first step of a one-pivot block: prime, pack, exchange, step
        parity = self.step & 1
        for be in self.ranks:
            with be.stream_ctx():
                be.prime()
                be.pack(0, 1, 0, parity)
        self._exchange()
        for be in self.ranks:
            with be.stream_ctx():
                be.decide(1, 1, parity, 0)
        c = self.ranks[0].dev.read_ctl()
        st, r, cc, e = int(c["sel_status"]), int(c["sel_r"]), int(c["sel_c"]), float(c["sel_e"])
        if st != _lib.PIVOT:
            self._restore()
        return st, r, cc, e

    def _exchange(self) -> None:
        """All-gather of the send slots for the step-wise calls: the same bytes smx_mshard_run
        exchanges, as (peer) device copies with the host waiting -- step-wise picks are the
        UI-sized path; chained pivots (run) exchange natively without host synchronisation."""
        self._sync()
        allsend = torch.cat([be.send.to(self.device) for be in self.ranks])
        for be in self.ranks:
            be.recv.copy_(allsend.to(be.recv.device))
        self._sync()

    def apply_selected(self) -> None:
        if self._saved is None:
            raise RuntimeError("apply_selected() without a pivot selected by pick()")
        parity = self.step & 1
        for be in self.ranks:
            with be.stream_ctx():
                be.sweep(1, parity)
                be.publish(parity ^ 1, 1)
        self._saved = None
        self.step += 1

    def int_first_fix(self, mask, r: int, c: int) -> None:
        """After the table's first pivot: the int semantics of its zero results on every rank
        (smx_int_first_fix with T0's pivot row copied from its owner; simplex.py:155-175)."""
        self._sync()
        p0 = (self.step - 1) & 1
        owner, rl = self._owner(r)
        src = self.ranks[owner].dev.buf[p0][rl]
        n = self.n
        for q, be in enumerate(self.ranks):
            lo, hi = self.ranges[q]
            d = be.dev
            local = None if mask is None else np.concatenate([mask[lo:hi], mask[n:n + 1]])
            with torch.cuda.device(d.device), be.stream_ctx():
                prow = src.to(d.device)
                int_first_fix(d.buf[p0], d.buf[p0 ^ 1], self.C, local,
                              rl if q == owner else -1, c, prow,
                              None if mask is None else mask[r])
        self._sync()

    def forced(self, r: int, c: int) -> None:
        raise NotImplementedError("forced pivots are a single-device microbenchmark")

    def run(self, k: int, graph: bool = True) -> None:
        """k chained pivots of the block protocol on every rank (no host synchronisation)."""
        if k <= 0:
            return
        self.settle()
        self._restore()
        if self._term:
            self.clear_term()
        self._native(k, self.P, graph=graph)
        for be in self.ranks:
            be.dev.step += k
            be.dev._pending = True
        self.step += k

    def sync_state(self):
        states = [be.dev.sync_state() for be in self.ranks]
        c = states[0]
        for s in states[1:]:   # every rank must have reached the same decision
            if int(s["npivots"]) != int(c["npivots"]) or bool(s["term"]) != bool(c["term"]):
                raise RuntimeError("row-sharded ranks diverged (pivot count / terminal state)")
        self.step = int(c["npivots"])
        self._term = bool(c["term"])
        return c

    def clear_term(self) -> None:
        for be in self.ranks:
            be.dev.clear_term()
        self._term = False

    def close(self) -> None:
        for g in getattr(self, "_graphs", {}).values():
            g.destroy()
        self._graphs = {}
        if self._comms:
            L = _lib.load()
            for h in self._comms:
                L.smx_comm_destroy(h)
            self._comms = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
