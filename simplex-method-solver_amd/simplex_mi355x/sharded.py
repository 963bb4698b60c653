"""Row-sharded pivot engine: one process per GPU, one exchange per pivot over RCCL (xGMI).

Partitioning: rank p owns the contiguous constraint rows
``[p*n/P, (p+1)*n/P)`` (all C columns) plus a replica of the f-row, so the entering column of
phase 2 (simplex.py:94-98) is decided locally and identically everywhere.  Per pivot:

1. ``smx_shard_begin``  : local ratio-test partials (simplex.py:105-136 over the local rows), then
   the send slot = [header | row A | row B] (include/smx.h): the local first-negative "-b" row
   (phase 1, simplex.py:72-76) or the local best ratio row, and the local first candidate row
   when its ratio is NaN (that one wins only if it is the globally first candidate, :117-121);
2. ``all_gather_into_tensor(recv, send)`` : the only collective (RCCL; gloo in the CPU tests).
   It carries the ratio-test minimum AND the pivot row in one message: the winner's row is
   already in ``recv`` on every rank, so no second broadcast and no host round trip;
3. ``smx_shard_finish`` : every rank merges the P headers identically (phase decision, global
   arg-min, phase-1 column scan of the winning row, simplex.py:81-85), then pivots its rows and
   its f-row replica with the winning row (simplex.py:149-177).

Stream-ordered end to end: the host never waits inside the loop; the outcome is read from the
control block every ``chunk`` pivots, like the single-GPU path.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import socket
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, lp, ops
from .device import DeviceTableau, Graph


def row_range(n: int, rank: int, world: int) -> tuple[int, int]:
    return rank * n // world, (rank + 1) * n // world


class RcclComm:
    """This rank's own RCCL communicator for the native shard driver (smx_comm_*).

    The 128-byte unique id is made on rank 0 and broadcast over the already-initialised
    torch.distributed group; after that every collective of the pivot loop is issued by
    libsmx.so on the solver stream (no torch stream hand-offs)."""

    def __init__(self, group=None):
        L = _lib.load()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            _lib.check(L.smx_comm_unique_id(uid), "smx_comm_unique_id")
        box = [bytes(uid.raw)]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = ctypes.create_string_buffer(box[0], 128)
        h = ctypes.c_void_p()
        _lib.check(L.smx_comm_init(ctypes.byref(h), self.world, uid, self.rank), "smx_comm_init")
        self.handle = h.value

    def info(self) -> tuple[int, int, int]:
        """(ncclCommCount, ncclCommUserRank, ncclCommCuDevice) of this communicator."""
        cnt, rk, dv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(_lib.load().smx_comm_info(self.handle, ctypes.byref(cnt), ctypes.byref(rk),
                                             ctypes.byref(dv)), "smx_comm_info")
        return cnt.value, rk.value, dv.value

    def close(self):
        if self.handle:
            _lib.load().smx_comm_destroy(self.handle)
            self.handle = None


class HipShardBackend:
    """This rank's slice of the tableau in HBM plus the exchange buffers.

    ``fused`` (default: the library's chain mode, smx_tune_fused): a pivot is fused pack ->
    all-gather -> fused update, with the next step's look-ahead records written by the update
    (no select kernel); otherwise select + pack -> all-gather -> update.  ``overlap`` (fused
    only, off by default): the native chain (run_native*) runs the next step's look-ahead and
    all-gather on a second stream under the sweep -- slower on this stack, see DESIGN.md §12."""

    def __init__(self, local_T: np.ndarray, n: int, m: int, flen: int, row0: int, world: int,
                 device=None, log_cap: int = 1 << 16, fused: bool | None = None,
                 overlap: bool = False):
        self.dev = DeviceTableau(local_T, n, m, flen, device=device, row0=row0, n_global=n,
                                 log_cap=log_cap)
        self.world = world
        self.slot = ops.shard_slot(self.dev.ld)
        with torch.cuda.stream(self.dev.stream):
            self.send = torch.zeros(self.slot, dtype=torch.float64, device=self.dev.device)
            # two gather slots: the overlapped native chain alternates them by step parity;
            # the per-step path (begin / all-gather / finish) uses the first
            self._recv2 = torch.zeros(2 * world * self.slot, dtype=torch.float64,
                                      device=self.dev.device)
            self.recv = self._recv2[:world * self.slot]
        self._shape = ops.make_shape(self.dev.shape)
        self.fused = _lib.fused_enabled() if fused is None else bool(fused)
        # True / "events": the exchange stream synchronised by events; "values": by stream
        # memory operations on device counters
        self.overlap = overlap if (overlap and self.fused) else False
        self._records = False   # look-ahead records of step dev.step are in dev.parts
        self._packed = False    # overlap form: send already holds step dev.step's pack

    def stream_ctx(self):
        return torch.cuda.stream(self.dev.stream)

    def begin(self) -> None:
        d = self.dev
        L = _lib.load()
        if self.fused:
            p = d.step & 1
            if self._packed:
                return          # packed by the previous finish (fused update / shard_ahead)
            if not self._records:
                _lib.check(L.smx_shard_fused_prime(
                    d.buf[p].data_ptr(), ctypes.byref(self._shape), p, d.ctl.data_ptr(),
                    d.parts.data_ptr(), d.stream.cuda_stream), "smx_shard_fused_prime")
                self._records = True
            _lib.check(L.smx_shard_fused_begin(
                d.buf[p].data_ptr(), ctypes.byref(self._shape), p, d.ctl.data_ptr(),
                d.parts.data_ptr(), self.send.data_ptr(), d.stream.cuda_stream),
                "smx_shard_fused_begin")
            return
        _lib.check(L.smx_shard_begin(
            d.buf[d.step & 1].data_ptr(), ctypes.byref(self._shape), d.step & 1,
            d.ctl.data_ptr(), d.parts.data_ptr(), self.send.data_ptr(), d.stream.cuda_stream),
            "smx_shard_begin")

    def finish(self, ev_before=None, ev_after=None) -> None:
        d = self.dev
        p = d.step & 1
        if self.overlap:
            L = _lib.load()
            # step k+1's records + pack from T_k (the native chain runs this on its exchange
            # stream, concurrently with the sweep), then step k's sweep
            _lib.check(L.smx_shard_ahead(
                d.buf[p].data_ptr(), ctypes.byref(self._shape), p, self.recv.data_ptr(),
                self.world, d.ctl.data_ptr(), d.parts.data_ptr(), self.send.data_ptr(),
                d.stream.cuda_stream), "smx_shard_ahead")
            if ev_before is not None:
                ev_before.record(d.stream)
            _lib.check(L.smx_shard_sweep(
                d.buf[p].data_ptr(), d.buf[p ^ 1].data_ptr(), self.recv.data_ptr(), self.world,
                ctypes.byref(self._shape), p, d.ctl.data_ptr(), d.log.data_ptr(), d.log_cap,
                d.stream.cuda_stream), "smx_shard_sweep")
            if ev_after is not None:
                ev_after.record(d.stream)
            self._packed = True
            d.step += 1
            d._pending = True
            return
        if self.fused:
            # the update's last look-ahead workgroup also packs the next step into send
            _lib.check(_lib.load().smx_shard_fused_finish(
                d.buf[p].data_ptr(), d.buf[p ^ 1].data_ptr(), self.recv.data_ptr(), self.world,
                ctypes.byref(self._shape), p, d.ctl.data_ptr(), d.parts.data_ptr(),
                self.send.data_ptr(), d.log.data_ptr(), d.log_cap,
                ev_before.cuda_event if ev_before is not None else None,
                ev_after.cuda_event if ev_after is not None else None, d.stream.cuda_stream),
                "smx_shard_fused_finish")
            self._packed = bool(_lib.load().smx_shard_folds_pack(ctypes.byref(self._shape)))
            d.step += 1
            d._pending = True
            return
        _lib.check(_lib.load().smx_shard_finish(
            d.buf[p].data_ptr(), d.buf[p ^ 1].data_ptr(), self.recv.data_ptr(), self.world,
            ctypes.byref(self._shape), p, d.ctl.data_ptr(), d.log.data_ptr(), d.log_cap,
            ev_before.cuda_event if ev_before is not None else None,
            ev_after.cuda_event if ev_after is not None else None, d.stream.cuda_stream),
            "smx_shard_finish")
        d.step += 1
        d._pending = True

    def _chain_mode(self):
        """Run the native chain in this backend's mode (smx_tune_fused is process-wide)."""
        L = _lib.load()
        mode = (3 if self.overlap == "values" else 2) if self.overlap else 1
        prev = L.smx_tune_fused(mode if self.fused else 0)
        return L, prev

    def run_native(self, k: int, comm: "RcclComm") -> None:
        """k pivots, all-gathers issued by libsmx.so on the solver stream (no host sync)."""
        d = self.dev
        L, prev = self._chain_mode()
        try:
            _lib.check(L.smx_shard_run(
                d.buf[0].data_ptr(), d.buf[1].data_ptr(), ctypes.byref(self._shape), d.step & 1,
                k, d.ctl.data_ptr(), d.parts.data_ptr(), self.send.data_ptr(),
                self._recv2.data_ptr(), self.world, comm.handle, d.log.data_ptr(), d.log_cap,
                d.stream.cuda_stream), "smx_shard_run")
        finally:
            L.smx_tune_fused(prev)
        d.step += k
        d._pending = True
        self._records = self._packed = False   # the native chain may keep fewer records

    def run_native_timed(self, k: int, comm: "RcclComm"):
        """Like run_native, with HIP events around every update kernel (synchronous)."""
        d = self.dev
        upd = (ctypes.c_float * k)()
        tot = ctypes.c_float()
        L, prev = self._chain_mode()
        try:
            _lib.check(L.smx_shard_run_timed(
                d.buf[0].data_ptr(), d.buf[1].data_ptr(), ctypes.byref(self._shape), d.step & 1,
                k, d.ctl.data_ptr(), d.parts.data_ptr(), self.send.data_ptr(),
                self._recv2.data_ptr(), self.world, comm.handle, d.log.data_ptr(), d.log_cap,
                d.stream.cuda_stream, upd, ctypes.byref(tot)), "smx_shard_run_timed")
        finally:
            L.smx_tune_fused(prev)
        d.step += k
        d._pending = True
        self._records = self._packed = False
        return np.frombuffer(upd, dtype=np.float32).copy(), float(tot.value)

    def state(self) -> dict:
        c = self.dev.sync_state()
        return {"npivots": int(c["npivots"]), "term": bool(c["term"]),
                "status": int(c["sel_status"]), "r": int(c["sel_r"]), "c": int(c["sel_c"])}

    def log(self, start: int, stop: int) -> np.ndarray:
        return self.dev.read_log(start, stop)

    def local_table(self) -> np.ndarray:
        return self.dev.download()


class BlockShardBackend:
    """This rank's row block for BLOCK pivots (smx_bshard_*, csrc/smx_block.hpp): per pivot the
    rank packs its header + candidate rows as values of T_{k+D} derived from the block's input,
    one all-gather exchanges the slots (the layout of the one-pivot protocol above), and the step
    kernel merges them, records the pivot and prepares the next step; every ``pivots`` pivots
    ONE sweep applies them all to the rank's rows.  Same methods for the numpy mirror of the
    gloo tests (tests/shard_numpy_backend.py, NumpyBlockShardBackend)."""

    def __init__(self, local_T: np.ndarray, n: int, m: int, flen: int, row0: int, world: int,
                 device=None, log_cap: int = 1 << 16, pivots: int = 8):
        self.dev = DeviceTableau(local_T, n, m, flen, device=device, row0=row0, n_global=n,
                                 log_cap=log_cap, block=0)
        self.world = world
        self.pivots = int(pivots)
        self.slot = ops.shard_slot(self.dev.ld)
        self._shape = ops.make_shape(self.dev.shape)
        nbytes = int(_lib.load().smx_bshard_bytes(ctypes.byref(self._shape)))
        if nbytes <= 0:
            raise ValueError(f"shape {self.dev.shape} is not eligible for sharded block pivots")
        with torch.cuda.stream(self.dev.stream):
            self.send = torch.zeros(self.slot, dtype=torch.float64, device=self.dev.device)
            self.recv = torch.zeros(world * self.slot, dtype=torch.float64,
                                    device=self.dev.device)
            self.blk = torch.zeros((nbytes + 7) // 8, dtype=torch.int64, device=self.dev.device)
        self._nbytes = nbytes

    def stream_ctx(self):
        return torch.cuda.stream(self.dev.stream)

    # -- the step-wise protocol (include/smx.h, smx_bshard_*) ---------------------------------
    def parity(self) -> int:
        return self.dev.step & 1

    def prime(self) -> None:
        d = self.dev
        _lib.check(_lib.load().smx_bshard_prime(
            d.buf[d.step & 1].data_ptr(), ctypes.byref(self._shape), d.step & 1,
            d.ctl.data_ptr(), self.blk.data_ptr(), self._nbytes, d.stream.cuda_stream),
            "smx_bshard_prime")

    def pack(self, step: int, pivots: int, block: int, parity: int) -> None:
        d = self.dev
        _lib.check(_lib.load().smx_bshard_pack(
            d.buf[parity].data_ptr(), ctypes.byref(self._shape), step, pivots, block,
            d.ctl.data_ptr(), self.blk.data_ptr(), self._nbytes, self.send.data_ptr(),
            d.stream.cuda_stream), "smx_bshard_pack")

    def decide(self, step: int, pivots: int, parity: int, block: int) -> None:
        """smx_bshard_step: merge the gathered slots, record pivot ``step - 1`` of the block,
        prepare step ``step``."""
        d = self.dev
        _lib.check(_lib.load().smx_bshard_step(
            d.buf[parity].data_ptr(), ctypes.byref(self._shape), step, pivots, parity, block,
            self.recv.data_ptr(), self.world, d.ctl.data_ptr(), self.blk.data_ptr(),
            self._nbytes, d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap,
            d.stream.cuda_stream), "smx_bshard_step")

    # -- the light exchange: header all-gather, pick, max all-reduce of one row ----------------
    @property
    def row(self) -> torch.Tensor:
        """The pivot-row buffer of the light exchange (after the gathered headers in recv)."""
        h = self.world * _lib.SHARD_HDR
        return self.recv[h:h + self.dev.ld]

    def pick(self, rank: int) -> None:
        """smx_bshard_pick: the owner of the winning row copies it into ``row``, the others
        fill it with the bit pattern 0x8000000000000000 (a MAX all-reduce on int64 follows)."""
        d = self.dev
        _lib.check(_lib.load().smx_bshard_pick(
            self.recv.data_ptr(), ctypes.byref(self._shape), self.world, rank,
            self.send.data_ptr(), self.row.data_ptr(), d.stream.cuda_stream), "smx_bshard_pick")

    def decide_light(self, step: int, pivots: int, parity: int, block: int) -> None:
        """smx_bshard_step_light: decide from the gathered headers, pivot row from ``row``."""
        d = self.dev
        _lib.check(_lib.load().smx_bshard_step_light(
            d.buf[parity].data_ptr(), ctypes.byref(self._shape), step, pivots, parity, block,
            self.recv.data_ptr(), self.row.data_ptr(), self.world, d.ctl.data_ptr(),
            self.blk.data_ptr(), self._nbytes, d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap,
            d.stream.cuda_stream), "smx_bshard_step_light")

    def sweep(self, pivots: int, parity: int) -> None:
        d = self.dev
        _lib.check(_lib.load().smx_bshard_sweep(
            d.buf[parity].data_ptr(), d.buf[parity ^ 1].data_ptr(), ctypes.byref(self._shape),
            pivots, self.blk.data_ptr(), self._nbytes, d.stream.cuda_stream), "smx_bshard_sweep")
        d.step += pivots
        d._pending = True

    def publish(self, parity: int, block: int) -> None:
        d = self.dev
        _lib.check(_lib.load().smx_bshard_publish(
            ctypes.byref(self._shape), parity, block, d.ctl.data_ptr(), self.blk.data_ptr(),
            self._nbytes, d.stream.cuda_stream), "smx_bshard_publish")

    # -- the native chain (libsmx issues the all-gathers) -------------------------------------
    def run_native(self, k: int, comm: "RcclComm") -> None:
        d = self.dev
        _lib.check(_lib.load().smx_bshard_run(
            d.buf[0].data_ptr(), d.buf[1].data_ptr(), ctypes.byref(self._shape), d.step & 1, k,
            self.pivots, d.ctl.data_ptr(), self.blk.data_ptr(), self._nbytes,
            self.send.data_ptr(), self.recv.data_ptr(), self.world, comm.handle,
            d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap, d.stream.cuda_stream),
            "smx_bshard_run")
        d.step += k
        d._pending = True

    def graph(self, k: int, comm: "RcclComm") -> Graph:
        """run_native's chain of k pivots captured as a hipGraph (smx_bshard_graph_create), for
        the current parity; cached per (parity, k, comm)."""
        d = self.dev
        # the exchange form is baked in at capture time, and a communicator handle can be reused
        # after close: key on both (close() / drop_graphs() free the cache)
        key = (d.step & 1, int(k), id(comm), comm.handle, _lib.tune_shard_xchg(-2))
        graphs = self.__dict__.setdefault("_graphs", {})
        if key not in graphs:
            h = ctypes.c_void_p()
            _lib.check(_lib.load().smx_bshard_graph_create(
                d.buf[0].data_ptr(), d.buf[1].data_ptr(), ctypes.byref(self._shape), d.step & 1,
                k, self.pivots, d.ctl.data_ptr(), self.blk.data_ptr(), self._nbytes,
                self.send.data_ptr(), self.recv.data_ptr(), self.world, comm.handle,
                d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap, d.stream.cuda_stream,
                ctypes.byref(h)), "smx_bshard_graph_create")
            graphs[key] = Graph(h.value)
        return graphs[key]

    def run_graph(self, k: int, comm: "RcclComm") -> None:
        """run_native(k, comm) as one replay of the captured chain (one host call)."""
        g = self.graph(k, comm)
        g.launch(self.dev.stream.cuda_stream)
        self.dev.step += k
        self.dev._pending = True

    def drop_graphs(self) -> None:
        for g in self.__dict__.pop("_graphs", {}).values():
            g.destroy()

    def close(self) -> None:
        """Free the captured chains (they hold the communicator they were captured with)."""
        self.drop_graphs()

    def run_native_timed(self, k: int, comm: "RcclComm"):
        """Like run_native, with HIP events around every sweep (synchronous)."""
        d = self.dev
        nb = -(-k // self.pivots)
        sw = (ctypes.c_float * nb)()
        tot = ctypes.c_float()
        _lib.check(_lib.load().smx_bshard_run_timed(
            d.buf[0].data_ptr(), d.buf[1].data_ptr(), ctypes.byref(self._shape), d.step & 1, k,
            self.pivots, d.ctl.data_ptr(), self.blk.data_ptr(), self._nbytes,
            self.send.data_ptr(), self.recv.data_ptr(), self.world, comm.handle,
            d.log.data_ptr(), d.xhist.data_ptr(), d.log_cap, d.stream.cuda_stream, sw,
            ctypes.byref(tot)),
            "smx_bshard_run_timed")
        d.step += k
        d._pending = True
        return np.frombuffer(sw, dtype=np.float32).copy(), float(tot.value)

    def state(self) -> dict:
        c = self.dev.sync_state()
        return {"npivots": int(c["npivots"]), "term": bool(c["term"]),
                "status": int(c["sel_status"]), "r": int(c["sel_r"]), "c": int(c["sel_c"])}

    def log(self, start: int, stop: int) -> np.ndarray:
        return self.dev.read_log(start, stop)

    def local_table(self) -> np.ndarray:
        return self.dev.download()


def rank_block_pivots(rows: int, m: int) -> int:
    """Pivots per sweep on one rank's row block: the single-GPU policy (smx_block_bytes, i.e.
    block_pivots in libsmx) applied to an unsharded table of the rank's size; 8 where that policy
    would not use blocks (a small rank table still saves sweeps at 8)."""
    ld = -(-(m + 1) // 16) * 16
    shape = [ld, rows, rows, m, m, 0, _lib.load().smx_nparts_for(rows, m)]
    plan = _lib.block_plan(shape, 0) if rows >= 1 else None
    # at most 12 per sweep on a rank: the sharded planner's per-pivot exchange makes its share
    # larger than the single-GPU policy's 1-4 GiB band (20) was measured for
    return min(plan[1], 12) if plan is not None else 8


def run_block_protocol(be, k: int, exchange, pivots: int | None = None, reduce_row=None,
                       rank: int | None = None) -> None:
    """k pivots of the block protocol on one rank's backend with any exchange: prime; per block
    of P pivots, P times pack -> exchange -> step, then one sweep; publish.  Full exchange
    (``reduce_row`` None): ``exchange()`` all-gathers ``be.send`` into ``be.recv``.  Light
    exchange: ``exchange()`` all-gathers the SHARD_HDR-double headers of ``be.send`` into the
    start of ``be.recv``, ``be.pick(rank)`` fills ``be.row``, ``reduce_row()`` all-reduces it with
    MAX over its int64 bit patterns, ``be.decide_light`` steps.  Stream-ordered, no host
    synchronisation."""
    P = int(pivots if pivots is not None else be.pivots)
    with be.stream_ctx():
        be.prime()
        parity = be.parity()
        done = bn = 0
        while done < k:
            pb = min(P, k - done)
            for step in range(1, pb + 1):
                be.pack(step - 1, pb, bn, parity)
                exchange()
                if reduce_row is None:
                    be.decide(step, pb, parity, bn)
                else:
                    be.pick(rank)
                    reduce_row()
                    be.decide_light(step, pb, parity, bn)
            be.sweep(pb, parity)
            parity = (parity + pb) & 1
            done += pb
            bn += 1
        be.publish(parity, bn)


class ShardedSolver:
    """The per-pivot protocol over any backend with begin/finish/state and a send/recv pair.

    With ``comm`` (an ``RcclComm``) and the HIP backend, ``run`` uses the native driver
    (libsmx.so issues select / pack / ncclAllGather / update on the solver stream); otherwise each
    pivot is begin -> torch.distributed all-gather -> finish (the path the gloo tests run)."""

    def __init__(self, backend, group=None, allgather=None, comm=None):
        self.be = backend
        self.group = group
        self._allgather = allgather
        self.comm = comm

    def _exchange(self) -> None:
        if self._allgather is not None:
            self._allgather(self.be.recv, self.be.send)
        else:
            dist.all_gather_into_tensor(self.be.recv, self.be.send, group=self.group)

    def pivot(self, ev_before=None, ev_after=None) -> None:
        """Enqueue one pivot (no host synchronisation)."""
        with self.be.stream_ctx():
            self.be.begin()
            self._exchange()
            self.be.finish(ev_before, ev_after)

    def run(self, k: int) -> dict:
        if self.comm is not None:
            self.be.run_native(k, self.comm)
        else:
            for _ in range(k):
                self.pivot()
        return self.be.state()


def _enqueue_probe(be: BlockShardBackend, comm: "RcclComm", k: int, reps: int = 3) -> dict:
    """Host enqueue time per pivot of the per-rank chain, eager (smx_bshard_run: prime, per pivot
    pack + RCCL + step launches, per block a sweep) against one replay of the same chain captured
    as a hipGraph, next to the device time per pivot (HIP events on the solver stream).  Runs
    after the timed region (the trajectory continues; every rank issues the same sequence); the
    median of ``reps`` runs per mode."""
    st = be.dev.stream
    out = {"pivots_per_run": k, "runs": reps}
    with torch.cuda.stream(st):
        be.graph(k, comm)            # capture for both parities before timing anything
        if k % 2:
            be.run_native(k, comm)
            be.graph(k, comm)
        torch.cuda.synchronize()
        for mode in ("eager", "graph"):
            host, dev = [], []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                t0 = time.perf_counter()
                if mode == "eager":
                    be.run_native(k, comm)
                else:
                    be.run_graph(k, comm)
                host.append(time.perf_counter() - t0)
                e1.record(st)
                e1.synchronize()
                dev.append(e0.elapsed_time(e1) * 1e-3)
            out[f"{mode}_host_us_per_pivot"] = float(np.median(host)) * 1e6 / k
            out[f"{mode}_device_us_per_pivot"] = float(np.median(dev)) * 1e6 / k
    out["npivots_after"] = int(be.state()["npivots"])
    be.drop_graphs()
    return out


# ---------------------------------------------------------------------------------------------
# bench.py --gpus N (launched by torch.distributed.run, one rank per GPU)
def comm_record(comm, device_index: int, group=None) -> dict:
    """What RCCL actually formed, from every rank (gathered; collective over `group`):
    ``rccl_ranks`` = rank 0's ncclCommCount, and per rank its torch rank, ncclCommUserRank,
    ncclCommCount, ncclCommCuDevice and the HIP device it runs on.  ``consistent``: every rank
    sees the same count, equal to the torch world size, the user ranks are a permutation of
    0..N-1 and no two ranks share a device."""
    count, user_rank, comm_dev = comm.info()
    mine = {"rank": dist.get_rank(group), "comm_count": int(count),
            "comm_user_rank": int(user_rank), "comm_device": int(comm_dev),
            "hip_device": int(device_index), "host": socket.gethostname()}
    world = dist.get_world_size(group)
    allr = [None] * world
    dist.all_gather_object(allr, mine, group=group)
    ok = (all(r["comm_count"] == world for r in allr)
          and sorted(r["comm_user_rank"] for r in allr) == list(range(world))
          and len({(r["host"], r["comm_device"]) for r in allr}) == world)
    return {"rccl_ranks": allr[0]["comm_count"], "consistent": bool(ok), "ranks": allr}


def sharded_cpu_baseline(cpu_baseline_fn, args, n: int, m: int, lo: int, hi: int,
                         full_limit_bytes: int = 4 << 30):
    """cpu_baseline of the multi-GPU line (rank 0, after the timed region): the CPU restatement
    on the FULL tableau when it fits ``full_limit_bytes`` (16384^2: 2 GiB), else on rank 0's own
    row block plus the f-row as an LP of its own (65536 x 32768: 17 GB); ``scope`` says which."""
    R, C = n + 1, m + 1
    seconds = float(getattr(args, "cpu_seconds", 15.0))
    if 8 * R * C <= full_limit_bytes:
        T = lp.dense_tableau(args.kind, args.seed, n, m)
        out = cpu_baseline_fn(T, n, m, seconds)
        out["scope"] = f"full {R}x{C} tableau (the same LP every rank holds a row block of)"
    else:
        nloc = hi - lo
        T = np.zeros((nloc + 1, C), dtype=np.float64)
        T[:-1] = lp.dense_rows(args.kind, args.seed, n, m, lo, hi)
        T[-1, :m] = lp.objective(args.kind, args.seed, m)
        out = cpu_baseline_fn(T, nloc, m, seconds)
        out["scope"] = (f"rank 0's row block (rows {lo}..{hi - 1} + the f-row, {nloc + 1}x{C}) as "
                        f"an LP of its own: the full {R}x{C} tableau is "
                        f"{8 * R * C / 2**30:.1f} GiB")
    return out


def bench_main(args, metric, peak_gbs, cpu_baseline_fn=None, load_traffic=None):
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511"), ("RANK", "0"),
                 ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
        os.environ.setdefault(k, v)   # plain `python bench.py --sharded` = a 1-rank job
    local_rank = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if not dist.is_initialized():
        dist.init_process_group("nccl", device_id=device)
    rank, world = dist.get_rank(), dist.get_world_size()
    R = args.rows if getattr(args, "rows", None) else args.size
    C = args.cols if getattr(args, "cols", None) else args.size
    n, m = R - 1, C - 1
    lo, hi = row_range(n, rank, world)
    local = np.zeros((hi - lo + 1, m + 1), dtype=np.float64)
    local[:-1] = lp.dense_rows(args.kind, args.seed, n, m, lo, hi)
    local[-1, :m] = lp.objective(args.kind, args.seed, m)
    pivots = getattr(args, "pivots", None)
    if pivots is None:
        pivots = rank_block_pivots(hi - lo, m)
    pivots = int(pivots or 1)
    block = pivots > 1
    xmode = {"auto": -1, "full": 0, "light": 1}[getattr(args, "xchg", "auto") or "auto"]
    _lib.tune_shard_xchg(xmode)
    light = block and (world >= 4 if xmode < 0 else xmode == 1)
    if block:
        be = BlockShardBackend(local, n, m, m, lo, world, device=device,
                               log_cap=max(1 << 16, args.warmup + args.steps), pivots=pivots)
        nsw = -(-args.steps // pivots)    # blocks of near-equal size (block_size in libsmx)
    else:
        be = HipShardBackend(local, n, m, m, lo, world, device=device,
                             log_cap=max(1 << 16, args.warmup + args.steps))
    del local
    comm = RcclComm()
    _lib.check(_lib.load().smx_timer_reserve(2 * args.steps + 2), "smx_timer_reserve")
    if args.warmup:
        if block:
            be.run_native(args.warmup, comm)
        else:
            ShardedSolver(be, comm=comm).run(args.warmup)
        be.state()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    upd_ms, tot_ms = be.run_native_timed(args.steps, comm)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = be.state()
    cycle = None
    if rank == 0:
        from .basis import BasisTracker
        tr = BasisTracker(n, m)
        for r, c in be.log(0, st["npivots"]):
            if tr.pivot(int(r), int(c)):
                cycle = {"first_step": tr.cycle[0], "period": tr.cycle[1]}
                break
    upd_ms = np.asarray(upd_ms, dtype=np.float64)
    stats = torch.tensor([elapsed, float(upd_ms.mean()),
                          float(st["npivots"] == args.warmup + args.steps and not st["term"])],
                         dtype=torch.float64, device=device)
    mx = stats.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mn = stats.clone()
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    wall = float(mx[0])
    enqueue = None
    if block and getattr(args, "enqueue_probe", False):
        # opt-in (it captures RCCL graphs and runs ~7x --steps more pivots after the timed
        # region): a failure is recorded in the line instead of losing the metric
        try:
            enqueue = _enqueue_probe(be, comm, args.steps)
        except Exception as exc:   # noqa: BLE001 -- reported, not raised
            enqueue = {"error": f"{type(exc).__name__}: {exc}"}
    rccl = comm_record(comm, device.index)
    local_bytes = 16.0 * (hi - lo + 1) * C
    ld = be.dev.ld
    # bytes each rank receives per pivot: full = every rank's slot (8 + 2 ld doubles); light =
    # the headers plus a ring all-reduce of one row (~2 (N - 1) / N rows)
    xbytes = (8 * world * 8 + 2.0 * (world - 1) / world * ld * 8) if light else \
        (world * (8 + 2 * ld) * 8)
    if rank == 0:
        avg_upd = float(upd_ms.mean()) * 1e-3
        achieved = local_bytes / avg_upd / 1e9
        workload = f"{R}x{C} dense fp64 tableau, {args.kind} random LP seed {args.seed}"
        traffic = load_traffic(None, f"{R}x{C}/{world}") if load_traffic else None
        out = {
            "metric": metric,
            "value": args.steps / wall,
            "unit": "pivots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: seeded dense random LP, each rank generates its own row block "
                    "on the host and uploads it to its HBM before timing (no dataset)",
            "config": {"workload": workload, "rows": R, "cols": C, "n": n, "m": m,
                       "parallelism": f"row-shard x{world} (RCCL exchange per pivot, issued "
                                      "natively on the solver stream)",
                       "rows_per_rank": hi - lo,
                       "pivots_per_sweep": pivots if block else 1,
                       "kernels_per_pivot": (2 * args.steps + nsw) / args.steps if block
                       else (2 if be.fused else 3),
                       "gather_overlapped_with_sweep": False if block else be.overlap,
                       "exchange": "light" if light else "full",
                       "collectives_per_pivot": 2 if light else 1,
                       "exchange_bytes_per_pivot_per_rank": xbytes},
            "equiv_one_pass_gbs": 16.0 * R * C / (wall / args.steps) / 1e9,
            "equiv_one_pass_note": "16 B/element/pivot of the whole tableau over wall time per "
                                   "pivot; not HBM traffic (block sweeps move 16 B/element once "
                                   "per P pivots, spread over the ranks)",
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak_gbs, "unit": "GB/s",
                         "frac": achieved / peak_gbs, "traffic": traffic,
                         "kernel": (f"k_blk_sweep<{-(-args.steps // nsw)}>" if block else
                                    ("k_update<kShardFused>" if be.fused else "k_update<kShard>"))
                                   + " (rank 0)",
                         "pivots_per_launch": args.steps / nsw if block else 1,
                         "algorithmic_bytes_per_launch": local_bytes,
                         "avg_kernel_ms": avg_upd * 1e3,
                         "max_rank_avg_kernel_ms": float(mx[1]),
                         "planner_exchange_ms_per_pivot":
                             (tot_ms - float(upd_ms.sum())) / args.steps},
            "trajectory_valid": bool(mn[2] > 0.5),
            "basis_cycle": cycle,
            "host_enqueue": enqueue,
            "rccl_ranks": rccl["rccl_ranks"],
            "rccl": rccl,
            "cpu_baseline": None,
        }
        if cpu_baseline_fn is not None and not getattr(args, "no_cpu_baseline", False):
            out["cpu_baseline"] = sharded_cpu_baseline(cpu_baseline_fn, args, n, m, lo, hi)
        print(json.dumps(out), flush=True)
    dist.barrier()
    if block:
        be.close()   # captured chains reference comm: free them before it
    comm.close()
    dist.destroy_process_group()


@contextlib.contextmanager
def _null():
    yield
