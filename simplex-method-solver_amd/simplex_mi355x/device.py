"""Device-resident tableau: HBM layout, control block and the pivot launches.

Layout in HBM (one object per tableau, owned by torch tensors):

* ``buf``   : ``float64[2][R][ld]`` ping-pong tableaux; step ``s`` reads ``buf[s & 1]`` and writes
  ``buf[(s+1) & 1]`` (the reference is out of place as well: deepcopy at simplex.py:149/177).
  ``R = rows + 1`` (constraint rows, then the f-row), ``C = m + 1`` used columns, ``ld`` = C
  rounded up to an even count and to 16 doubles (128-B rows, 16-B ``double2`` lanes).
* ``ctl``   : 128-B ``struct smx_ctl`` (first-negative slots, selection, pivot counter).
* ``parts`` : 2 x ``nparts`` 32-B ``struct smx_part`` records (select partials; the fused
  chain's look-ahead records, double-buffered by parity).
* ``log``   : ``int32[log_cap][2]`` ring of applied pivots ``(r, c)``, drained by the host.
* ``xhist`` : ``float64[log_cap][2]`` ring of ``(x1, x2)`` of the tableau after each pivot
  (find_optimum, simplex.py:51-68), written by the update kernel itself.
* ``xch``   : exchange buffer of the on-chip resident loop (records + candidate rows), allocated
  on first use for tableaux whose rows fit in LDS (``_lib.resident_plan``).
* ``blk``   : scratch of the block-pivot chain (pivot rows, per-row multipliers, records, the
  running f-row), allocated on first use for tableaux it applies to (``_lib.block_plan``).

Chained pivots run one of three ways: tableaux that fit on chip (about R x C <= 2048^2) run the
whole chunk in ONE persistent launch that keeps the rows in LDS (``smx_resident_run``); tables
that stream from HBM (>= 64 MiB) replay a hipGraph of block pivots -- several pivots planned from
the table, then applied in one sweep (``smx_block_graph_create``); the rest replay a hipGraph of
one fused update kernel per pivot (``smx_graph_*``).

All launches go to one dedicated HIP stream per tableau; the host synchronises only when it
reads the control block.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, ops


def leading_dim(C: int, pad_to: int = 16) -> int:
    """Row stride in doubles: C rounded up to a multiple of ``pad_to`` (>= 4, so every 32-B
    lane group of the VEC=4 update variants stays inside the row)."""
    pad_to = max(4, pad_to - pad_to % 4)
    return ((C + pad_to - 1) // pad_to) * pad_to


class Graph:
    """A captured chain of k pivots (hipGraph); replayed by :meth:`launch`."""

    def __init__(self, handle: int):
        self.handle = handle

    def launch(self, stream: int) -> None:
        _lib.check(_lib.load().smx_graph_launch(self.handle, stream), "smx_graph_launch")

    def destroy(self) -> None:
        if self.handle:
            _lib.load().smx_graph_destroy(self.handle)
            self.handle = None


def int_first_fix(T0: torch.Tensor, T1: torch.Tensor, C: int, mask, r: int, c: int,
                  prow: torch.Tensor | None = None, maskr=None) -> None:
    """The int semantics of the zero results of a table's first pivot T0 -> T1
    (``smx_int_first_fix``, csrc/smx_intfirst.hpp; simplex.py:155-175 on the caller's ints), on
    the current stream.  ``T0`` / ``T1``: ``float64[rows][ld]`` on one device; ``mask``: uint8
    ``[rows][C]`` host array (nonzero = the caller passed an int there) or None when every entry
    is an int; ``r``: the local pivot row (-1: held by another rank, whose T0 row is ``prow``);
    ``maskr``: the pivot row's mask when it is not a row of ``mask``."""
    rows, ld = int(T0.shape[0]), int(T0.shape[1])
    dev = T0.device
    if prow is None:
        prow = T0[r]
    md = mr = None
    if mask is not None:
        md = torch.from_numpy(np.ascontiguousarray(mask, dtype=np.uint8)).to(dev)
        if maskr is None:
            mr = md[r]
    if maskr is not None:
        mr = torch.from_numpy(np.ascontiguousarray(maskr, dtype=np.uint8)).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.load().smx_int_first_fix(
        T0.data_ptr(), T1.data_ptr(), ld, rows, int(C), int(r), int(c), prow.data_ptr(),
        None if md is None else md.data_ptr(), int(C), None if mr is None else mr.data_ptr(),
        stream), "smx_int_first_fix")


class DeviceTableau:
    """A dense fp64 tableau in HBM plus the state of the pivot loop."""

    def __init__(self, dense: np.ndarray, n: int, m: int, flen: int, *, device=None,
                 row0: int = 0, n_global: int | None = None, log_cap: int = 1 << 16,
                 pad_to: int = 16, ld_extra: int = 0, defer_upload: bool = False,
                 resident: bool | None = None, block: int | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("simplex_mi355x needs an MI355X (HIP device); there is no CPU path")
        _lib.load()
        rows = dense.shape[0] - 1
        C = m + 1
        if dense.shape[1] < C and not defer_upload:
            raise ValueError("dense tableau narrower than m + 1")
        self.device = torch.device(device if device is not None else "cuda")
        self.rows, self.n, self.m, self.flen, self.row0 = rows, (n if n_global is None else n_global), m, flen, row0
        self.C = C
        self.ld = leading_dim(C, pad_to) + ld_extra
        self.nparts = _lib.load().smx_nparts_for(rows, m)
        self.shape = [self.ld, rows, self.n, m, flen, row0, self.nparts]
        self.stream = torch.cuda.Stream(self.device)
        with torch.cuda.stream(self.stream):
            self.buf = torch.zeros((2, rows + 1, self.ld), dtype=torch.float64, device=self.device)
            self.ctl = torch.zeros(_lib.CTL_BYTES // 8, dtype=torch.int64, device=self.device)
            # 2 x nparts: the fused chain double-buffers the partials by parity
            self.parts = torch.zeros(2 * self.nparts * _lib.PART_BYTES // 8, dtype=torch.int64,
                                     device=self.device)
            self.log = torch.zeros(2 * log_cap, dtype=torch.int32, device=self.device)
            self.xhist = torch.zeros(2 * log_cap, dtype=torch.float64, device=self.device)
        self.log_cap = log_cap
        self.step = 0
        self._pending = False   # chained pivots enqueued whose outcome the host has not read
        self._term = False      # a terminal outcome may be latched in ctl.term
        self._graphs: dict[tuple[int, int], Graph] = {}
        # None: the library's policy (smx_tune_resident); False: always the launch chain
        self.resident = resident
        self._xch = None
        self._epoch = 0
        # the input of a resident chain not yet confirmed (buffer, control block, step, pivots):
        # on a hand-off timeout sync_state restores it and reruns the pivots on the launch chain
        self._res_snap = None
        self.resident_fallbacks = 0
        # None: the library's policy (smx_tune_block); 0: never; 1..16: pivots per sweep
        self.block = block
        self._blk = None
        if not defer_upload:
            self.upload(dense)

    # -- data movement --------------------------------------------------------------------
    def upload(self, dense: np.ndarray) -> None:
        """Copy a host tableau into buf[0] and prime the control block (pivot count = 0)."""
        host = torch.from_numpy(np.ascontiguousarray(dense[:, :self.C], dtype=np.float64))
        with torch.cuda.stream(self.stream):
            self.buf.zero_()
            self.buf[0, :, :self.C].copy_(host)
            self.step = 0
            ops.reset(self.buf[0], self.ctl, self.shape, 0, 1)
        self._pending = False
        self._term = False

    def reset_state(self) -> None:
        """Prime the control block for whatever buf[0] now holds (pivot count = 0)."""
        with torch.cuda.stream(self.stream):
            self.step = 0
            ops.reset(self.buf[0], self.ctl, self.shape, 0, 1)
        self._pending = False
        self._term = False

    def settle(self) -> None:
        """Make the host step counter exact after chained pivots (one control-block read)."""
        if self._pending:
            self.sync_state()

    def cur(self) -> torch.Tensor:
        self.settle()
        return self.buf[self.step & 1]

    def download(self) -> np.ndarray:
        with torch.cuda.stream(self.stream):
            out = self.cur()[:, :self.C].cpu().numpy()
        return out

    def values(self, idx) -> list[float]:
        """Host copies of selected elements [(i, j), ...] of the current tableau."""
        if not idx:
            return []
        ii = torch.tensor([i for i, _ in idx], device=self.device)
        jj = torch.tensor([j for _, j in idx], device=self.device)
        with torch.cuda.stream(self.stream):
            return self.cur()[ii, jj].cpu().tolist()

    def read_ctl(self) -> np.void:
        with torch.cuda.stream(self.stream):
            raw = self.ctl.cpu().numpy()
        return raw.view(_lib.CTL_DTYPE)[0]

    def read_log(self, start: int, stop: int) -> np.ndarray:
        """Pivots start..stop-1 (absolute counts) from the device ring."""
        return self._ring(self.log, start, stop, np.int32)

    def read_xhist(self, start: int, stop: int) -> np.ndarray:
        """(x1, x2) after pivots start..stop-1 (absolute counts) from the device ring."""
        return self._ring(self.xhist, start, stop, np.float64)

    def _ring(self, buf, start, stop, dtype):
        if stop <= start:
            return np.zeros((0, 2), dtype=dtype)
        if stop - start > self.log_cap:
            raise RuntimeError("pivot log overrun: drain the log more often")
        pos = np.arange(start, stop) % self.log_cap
        lo, hi = int(pos.min()), int(pos.max()) + 1
        with torch.cuda.stream(self.stream):
            ring = buf.view(-1, 2)[lo:hi].cpu().numpy()
        return ring[pos - lo]

    def set_label_positions(self, x1code: int, x2code: int) -> None:
        """Tell the device where labels x1/x2 sit (after a host-side re-labelling)."""
        with torch.cuda.stream(self.stream):
            _lib.check(_lib.load().smx_set_xpos(self.ctl.data_ptr(), self.step & 1, x1code,
                                                x2code, self.stream.cuda_stream), "smx_set_xpos")

    # -- pivot loop -----------------------------------------------------------------------
    def select(self) -> None:
        with torch.cuda.stream(self.stream):
            ops.select(self.cur(), self.ctl, self.parts, self.shape, self.step & 1)

    def pick(self):
        """pick_element on the device: returns (status, r, c, e); synchronises."""
        self.settle()
        if self._term:
            self.clear_term()
        with torch.cuda.stream(self.stream):
            p = self.step & 1
            ops.select(self.cur(), self.ctl, self.parts, self.shape, p)
            ops.finalize(self.cur(), self.ctl, self.parts, self.shape, p)
        c = self.read_ctl()
        return int(c["sel_status"]), int(c["sel_r"]), int(c["sel_c"]), float(c["sel_e"])

    def apply_selected(self) -> None:
        """recalculate_matrix with the selection of the last select() (no host sync)."""
        self.settle()
        p = self.step & 1
        with torch.cuda.stream(self.stream):
            ops.update(self.buf[p], self.buf[p ^ 1], self.ctl, self.parts, self.log, self.xhist,
                       self.shape, p)
        self.step += 1

    def run(self, k: int, graph: bool = True) -> None:
        """Enqueue k chained pivots (no host sync).  Call :meth:`sync_state` afterwards."""
        if k <= 0:
            return
        self.settle()
        if self._term:
            self.clear_term()
        p = self.step & 1
        plan = self.resident_plan()
        bplan = self.block_plan() if plan is None else None
        with torch.cuda.stream(self.stream):
            if plan is not None:
                xch, epoch = self._xch_for(plan), self._next_epoch()
                # a copy of the chain's input (tables up to ~1920^2: <= 30 MB, ~0.1 % of the
                # chain's time) so a hand-off timeout is recoverable (sync_state)
                self._res_snap = (self.buf[p].clone(), self.ctl.clone(), self.step, k)
                ops.resident_run(self.buf, self.ctl, xch, self.log, self.xhist, self.shape, p,
                                 k, epoch)
            elif bplan is not None:
                blk = self._blk_for(bplan)
                if graph:
                    g = self._graphs.get((p, k, "blk", bplan[1]))
                    if g is None:
                        g = self._make_block_graph(p, k, bplan[1])
                    g.launch(self.stream.cuda_stream)
                else:
                    ops.block_run(self.buf, self.ctl, blk, self.log, self.xhist, self.shape, p,
                                  k, bplan[1])
            elif graph:
                g = self._graphs.get((p, k))
                if g is None:
                    g = self._make_graph(p, k)
                g.launch(self.stream.cuda_stream)
            else:
                ops.run(self.buf, self.ctl, self.parts, self.log, self.xhist, self.shape, p, k)
        # optimistic: if the chain stops early every later kernel is a no-op, and sync_state()
        # replaces this with the device's exact count
        self.step += k
        self._pending = True

    def resident_plan(self):
        """The resident loop's (exchange bytes, (workgroups, rows per workgroup, columns per
        thread, LDS bytes)) when :meth:`run` will use it, else None."""
        if self.resident is False:
            return None
        return _lib.resident_plan(self.shape)

    def block_plan(self):
        """(scratch bytes, pivots per sweep) of the block-pivot chain when :meth:`run` will use
        it (the resident loop takes precedence), else None."""
        if self.block == 0:
            return None
        return _lib.block_plan(self.shape, self.block or 0)

    def _blk_for(self, plan) -> torch.Tensor:
        nbytes = plan[0]
        if self._blk is None or self._blk.numel() * 8 < nbytes:
            with torch.cuda.stream(self.stream):
                self._blk = torch.zeros((nbytes + 7) // 8, dtype=torch.int64, device=self.device)
        return self._blk

    def _make_block_graph(self, parity: int, k: int, pivots: int) -> Graph:
        import ctypes
        h = ctypes.c_void_p()
        sh = ops.make_shape(self.shape)
        blk = self._blk
        _lib.check(_lib.load().smx_block_graph_create(
            self.buf[0].data_ptr(), self.buf[1].data_ptr(), ctypes.byref(sh), parity, k, pivots,
            self.ctl.data_ptr(), blk.data_ptr(), blk.numel() * 8, self.log.data_ptr(),
            self.xhist.data_ptr(), self.log_cap, self.stream.cuda_stream, ctypes.byref(h)),
            "smx_block_graph_create")
        g = Graph(h.value)
        self._graphs[(parity, k, "blk", pivots)] = g
        return g

    def block_timed_launcher(self, k: int, pivots: int):
        """``run_block_timed`` in two calls: the host preparation (shape, plan, scratch) is done
        here; returns (launch, read).  ``launch()`` only enqueues the chain with its HIP events
        (smx_block_run_timed with NULL outputs); ``read()`` waits for the chain's last event and
        returns (per-sweep ms array, device ms of the whole chain).  A timed region can bracket
        launch() and its own synchronize, with the event readout after it."""
        import ctypes
        self.settle()
        if self._term:
            self.clear_term()
        p = self.step & 1
        nb = -(-k // pivots)
        plan = _lib.block_plan(self.shape, pivots)
        if plan is None:
            raise ValueError(f"shape {self.shape} is not eligible for block pivots")
        blk = self._blk_for(plan)
        sh = ops.make_shape(self.shape)
        L = _lib.load()
        args = (self.buf[0].data_ptr(), self.buf[1].data_ptr(), ctypes.byref(sh), p, k, pivots,
                self.ctl.data_ptr(), blk.data_ptr(), blk.numel() * 8, self.log.data_ptr(),
                self.xhist.data_ptr(), self.log_cap, self.stream.cuda_stream)

        def launch() -> None:
            _lib.check(L.smx_block_run_timed(*args, None, None), "smx_block_run_timed")
            self.step += k
            self._pending = True

        def read():
            sw = (ctypes.c_float * nb)()
            tot = ctypes.c_float()
            _lib.check(L.smx_block_timed_read(nb, sw, ctypes.byref(tot)), "smx_block_timed_read")
            return np.frombuffer(sw, dtype=np.float32).copy(), float(tot.value)

        launch.shape = sh   # keeps the ctypes shape alive as long as the closures
        return launch, read

    def run_block_timed(self, k: int, pivots: int):
        """k chained pivots in blocks of ``pivots`` with HIP events around every sweep
        (synchronous).  Returns (per-sweep ms array, device ms of the whole chain)."""
        launch, read = self.block_timed_launcher(k, pivots)
        launch()
        return read()

    def _xch_for(self, plan) -> torch.Tensor:
        nbytes = plan[0]
        if self._xch is None or self._xch.numel() * 8 < nbytes:
            with torch.cuda.stream(self.stream):
                self._xch = torch.zeros((nbytes + 7) // 8, dtype=torch.int64, device=self.device)
            self._epoch = 0
        return self._xch

    def _next_epoch(self) -> int:
        """Tag of the next resident launch; the exchange buffer is re-zeroed when tags wrap."""
        self._epoch += 1
        if self._epoch > _lib.RESIDENT_EPOCHS:
            with torch.cuda.stream(self.stream):
                self._xch.zero_()
            self._epoch = 1
        return self._epoch

    def prepare(self, k: int) -> None:
        """Capture (without running) the k-pivot graph the next ``run(k)`` will replay (or
        allocate the resident loop's exchange buffer)."""
        self.settle()
        p = self.step & 1
        plan = self.resident_plan()
        if plan is not None:
            self._xch_for(plan)
            return
        bplan = self.block_plan()
        if bplan is not None:
            self._blk_for(bplan)
            if (p, k, "blk", bplan[1]) not in self._graphs:
                with torch.cuda.stream(self.stream):
                    self._make_block_graph(p, k, bplan[1])
            return
        if (p, k) not in self._graphs:
            with torch.cuda.stream(self.stream):
                self._make_graph(p, k)

    def run_timed(self, k: int):
        """k chained pivots with HIP events around every update kernel (synchronous).
        Returns (per-update-kernel ms array, device ms of the whole chain)."""
        import ctypes
        self.settle()
        if self._term:
            self.clear_term()
        p = self.step & 1
        upd = (ctypes.c_float * k)()
        tot = ctypes.c_float()
        sh = ops.make_shape(self.shape)
        _lib.check(_lib.load().smx_run_timed(
            self.buf[0].data_ptr(), self.buf[1].data_ptr(), ctypes.byref(sh), p, k,
            self.ctl.data_ptr(), self.parts.data_ptr(), self.log.data_ptr(),
            self.xhist.data_ptr(), self.log_cap, self.stream.cuda_stream, upd,
            ctypes.byref(tot)), "smx_run_timed")
        self.step += k
        self._pending = True
        return np.frombuffer(upd, dtype=np.float32).copy(), float(tot.value)

    def sync_state(self) -> np.void:
        """Read the control block and set the host step counter to the device pivot count."""
        c = self.read_ctl()
        snap, self._res_snap = self._res_snap, None
        if int(c["dec"][0][0]) & _lib.RESIDENT_TIMEOUT:
            self._pending = False
            if snap is None:
                raise RuntimeError("a workgroup hand-off timed out (resident pivot loop or "
                                   "persistent planner; the tableau on the device is undefined)")
            # the chain's workgroups could not all be resident at once (or one stalled): put
            # its input back and run the same pivots on the launch chain, for good on this
            # tableau -- the same decisions and arithmetic, so the same results
            buf_in, ctl_in, step0, k = snap
            with torch.cuda.stream(self.stream):
                self.buf[step0 & 1].copy_(buf_in)
                self.ctl.copy_(ctl_in)
            del buf_in, ctl_in
            self.step = step0
            self._term = False
            self.resident = False
            self.resident_fallbacks += 1
            self.run(k)
            return self.sync_state()
        self.step = int(c["npivots"])
        self._pending = False
        self._term = bool(c["term"])
        return c

    def clear_term(self) -> None:
        """Re-arm the chain after a terminal outcome (the table is unchanged by it)."""
        with torch.cuda.stream(self.stream):
            self.ctl.view(torch.int32)[4] = 0   # smx_ctl.term (byte offset 16)
        self._term = False

    def _make_graph(self, parity: int, k: int) -> Graph:
        import ctypes
        h = ctypes.c_void_p()
        sh = ops.make_shape(self.shape)
        b0, b1 = self.buf[0].data_ptr(), self.buf[1].data_ptr()
        _lib.check(_lib.load().smx_graph_create(
            b0, b1, ctypes.byref(sh), parity, k, self.ctl.data_ptr(), self.parts.data_ptr(),
            self.log.data_ptr(), self.xhist.data_ptr(), self.log_cap, self.stream.cuda_stream,
            ctypes.byref(h)),
            "smx_graph_create")
        g = Graph(h.value)
        self._graphs[(parity, k)] = g
        return g

    def forced(self, r: int, c: int) -> None:
        """Forced pivot (no selection, no bookkeeping): buf[s&1] -> buf[(s+1)&1]."""
        self.settle()
        p = self.step & 1
        with torch.cuda.stream(self.stream):
            ops.update_forced(self.buf[p], self.buf[p ^ 1], self.shape, r, c)
        self.step += 1

    def int_first_fix(self, mask, r: int, c: int, prow: torch.Tensor | None = None,
                      maskr=None) -> None:
        """After the table's first pivot (buf[(step - 1) & 1] -> buf[step & 1]): the int
        semantics of its zero results (see :func:`int_first_fix`).  ``r``: local pivot row."""
        self.settle()
        p0 = (self.step - 1) & 1
        with torch.cuda.stream(self.stream):
            int_first_fix(self.buf[p0], self.buf[p0 ^ 1], self.C, mask, r, c, prow, maskr)

    def close(self) -> None:
        for g in self._graphs.values():
            g.destroy()
        self._graphs.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
