"""Thin PyTorch-ROCm custom ops over the C ABI (``include/smx.h``).

Each op passes ``tensor.data_ptr()`` and the current HIP stream to ``libsmx.so`` and is
registered with ``torch.library.custom_op`` so the pivot kernels are first-class torch ops
(``torch.ops.smx.update`` ...).  Every op checks on the host that the operands have the shapes
the kernel and its grid assume before anything is launched.

``shape`` is ``[ld, rows, n, m, flen, row0, nparts]`` (``struct smx_shape``).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

Tensor = torch.Tensor


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Tensor) -> int:
    return t.data_ptr()


def make_shape(shape) -> _lib.Shape:
    ld, rows, n, m, flen, row0, nparts = (int(x) for x in shape)
    return _lib.Shape(ld, rows, n, m, flen, row0, nparts)


def _table_ok(t: Tensor, shape, name: str) -> None:
    ld, rows, n, m = int(shape[0]), int(shape[1]), int(shape[2]), int(shape[3])
    if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous float64 CUDA tensor")
    if t.dim() != 2 or t.shape[0] != rows + 1 or t.shape[1] != ld:
        raise ValueError(f"{name}: shape {tuple(t.shape)} != ({rows + 1}, {ld})")
    if ld % 2 or ld < m + 1 or ((m + 1) % 2 and ld < m + 2):
        raise ValueError(f"{name}: leading dimension {ld} invalid for m={m}")
    if not (0 <= rows <= n):
        raise ValueError(f"{name}: rows={rows} n={n}")


def _bytes_ok(t: Tensor, nbytes: int, name: str) -> None:
    if not t.is_cuda or not t.is_contiguous() or t.numel() * t.element_size() < nbytes:
        raise ValueError(f"{name}: needs a contiguous CUDA buffer of >= {nbytes} bytes")


def _parts_ok(parts: Tensor, shape, slots: int = 1) -> None:
    nparts = int(shape[6])
    if not 1 <= nparts <= 64:
        raise ValueError(f"nparts={nparts} out of range [1, 64]")
    _bytes_ok(parts, slots * nparts * _lib.PART_BYTES, "parts")


def _log_cap(log: Tensor) -> int:
    if log.dtype != torch.int32 or not log.is_cuda or not log.is_contiguous():
        raise ValueError("log: expected a contiguous int32 CUDA tensor")
    return log.numel() // 2


@torch.library.custom_op("smx::reset", mutates_args=("ctl",))
def reset(T: Tensor, ctl: Tensor, shape: list[int], parity: int, clear_count: int) -> None:
    """Prime the control block for a freshly uploaded tableau (simplex.py:25-39 set-up)."""
    _table_ok(T, shape, "T")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_reset(_ptr(T), ctypes.byref(sh), parity, clear_count, _ptr(ctl),
                                     _stream()), "smx_reset")


@torch.library.custom_op("smx::select", mutates_args=("ctl", "parts"))
def select(T: Tensor, ctl: Tensor, parts: Tensor, shape: list[int], parity: int) -> None:
    """pick_element partials (simplex.py:70-141)."""
    _table_ok(T, shape, "T")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _parts_ok(parts, shape)
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_select(_ptr(T), ctypes.byref(sh), parity, _ptr(ctl), _ptr(parts),
                                      _stream()), "smx_select")


@torch.library.custom_op("smx::finalize", mutates_args=("ctl",))
def finalize(T: Tensor, ctl: Tensor, parts: Tensor, shape: list[int], parity: int) -> None:
    """pick_element outcome into ctl.sel_* (simplex.py:89, 91, 101-103, 138-141)."""
    _table_ok(T, shape, "T")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _parts_ok(parts, shape)
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_finalize(_ptr(T), ctypes.byref(sh), parity, _ptr(ctl),
                                        _ptr(parts), _stream()), "smx_finalize")


def _xhist_ok(xhist: Tensor, log: Tensor) -> None:
    if xhist.dtype != torch.float64 or not xhist.is_cuda or not xhist.is_contiguous() or \
            xhist.numel() < log.numel():
        raise ValueError("xhist: expected a contiguous float64 CUDA tensor as long as log")


@torch.library.custom_op("smx::update", mutates_args=("tout", "ctl", "log", "xhist"))
def update(tin: Tensor, tout: Tensor, ctl: Tensor, parts: Tensor, log: Tensor, xhist: Tensor,
           shape: list[int], parity: int) -> None:
    """recalculate_matrix (simplex.py:143-177) from tin into tout; logs (r, c) and the new
    tableau's (x1, x2) (find_optimum, simplex.py:51-68) into the history rings."""
    _table_ok(tin, shape, "tin")
    _table_ok(tout, shape, "tout")
    if tin.data_ptr() == tout.data_ptr():
        raise ValueError("update is out of place: tin and tout must differ")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _parts_ok(parts, shape)
    _xhist_ok(xhist, log)
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_update(_ptr(tin), _ptr(tout), ctypes.byref(sh), parity, _ptr(ctl),
                                      _ptr(parts), _ptr(log), _ptr(xhist), _log_cap(log),
                                      _stream()), "smx_update")


@torch.library.custom_op("smx::run", mutates_args=("buf", "ctl", "parts", "log", "xhist"))
def run(buf: Tensor, ctl: Tensor, parts: Tensor, log: Tensor, xhist: Tensor, shape: list[int],
        parity: int, k: int) -> None:
    """k chained pivots (the loop of get_solution, simplex.py:184-198) on buf[0]/buf[1]."""
    if buf.dim() != 3 or buf.shape[0] != 2:
        raise ValueError("buf must be (2, R, ld)")
    _table_ok(buf[0], shape, "buf[0]")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _parts_ok(parts, shape, 2)      # the fused chain double-buffers the partials
    _xhist_ok(xhist, log)
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_run(_ptr(buf[0]), _ptr(buf[1]), ctypes.byref(sh), parity, k,
                                   _ptr(ctl), _ptr(parts), _ptr(log), _ptr(xhist),
                                   _log_cap(log), _stream()), "smx_run")


@torch.library.custom_op("smx::resident_run",
                         mutates_args=("buf", "ctl", "xch", "log", "xhist"))
def resident_run(buf: Tensor, ctl: Tensor, xch: Tensor, log: Tensor, xhist: Tensor,
                 shape: list[int], parity: int, k: int, epoch: int) -> None:
    """k pivots of the get_solution loop (simplex.py:184-198) in one persistent launch with the
    tableau held in LDS (smx_resident_run); ``xch`` is the zero-initialised exchange buffer of
    ``_lib.resident_plan(shape)[0]`` bytes and ``epoch`` (1..4095) tags this launch's
    hand-offs (the caller rotates it and re-zeroes ``xch`` when it wraps)."""
    if not 1 <= epoch <= _lib.RESIDENT_EPOCHS or not 0 <= k < (1 << 20) - 1:
        raise ValueError(f"resident_run: epoch {epoch} / k {k} out of range")
    if buf.dim() != 3 or buf.shape[0] != 2:
        raise ValueError("buf must be (2, R, ld)")
    _table_ok(buf[0], shape, "buf[0]")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _xhist_ok(xhist, log)
    plan = _lib.resident_plan(shape)
    if plan is None:
        raise ValueError(f"shape {list(shape)} is not eligible for the resident pivot loop")
    _bytes_ok(xch, plan[0], "xch")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_resident_run(
        _ptr(buf[0]), _ptr(buf[1]), ctypes.byref(sh), parity, k, _ptr(ctl), _ptr(xch),
        xch.numel() * xch.element_size(), epoch, _ptr(log), _ptr(xhist), _log_cap(log),
        _stream()),
        "smx_resident_run")


@torch.library.custom_op("smx::block_run", mutates_args=("buf", "ctl", "blk", "log", "xhist"))
def block_run(buf: Tensor, ctl: Tensor, blk: Tensor, log: Tensor, xhist: Tensor,
              shape: list[int], parity: int, k: int, pivots: int) -> None:
    """k pivots of the get_solution loop (simplex.py:184-198) in blocks of ``pivots`` per HBM
    sweep (smx_block_run): each block's decisions are planned from its input table, then one
    sweep applies them all.  ``blk`` is scratch of ``_lib.block_plan(shape)[0]`` bytes."""
    if not 1 <= pivots <= _lib.BLOCK_MAX or k < 0:
        raise ValueError(f"block_run: pivots {pivots} / k {k} out of range")
    if buf.dim() != 3 or buf.shape[0] != 2:
        raise ValueError("buf must be (2, R, ld)")
    _table_ok(buf[0], shape, "buf[0]")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    _xhist_ok(xhist, log)
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_block_run(
        _ptr(buf[0]), _ptr(buf[1]), ctypes.byref(sh), parity, k, pivots, _ptr(ctl), _ptr(blk),
        blk.numel() * blk.element_size(), _ptr(log), _ptr(xhist), _log_cap(log), _stream()),
        "smx_block_run")


@torch.library.custom_op("smx::update_forced", mutates_args=("tout",))
def update_forced(tin: Tensor, tout: Tensor, shape: list[int], r: int, c: int) -> None:
    """Forced pivot (r, c): the update kernel alone, for roofline measurement."""
    _table_ok(tin, shape, "tin")
    _table_ok(tout, shape, "tout")
    if not (0 <= r < int(shape[1]) and 0 <= c <= int(shape[3])):
        raise ValueError("forced pivot out of range")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_update_forced(_ptr(tin), _ptr(tout), ctypes.byref(sh), r, c,
                                             _stream()), "smx_update_forced")


def shard_slot(ld: int) -> int:
    """Doubles per rank in the all-gather buffers: header + candidate rows A and B."""
    return _lib.SHARD_HDR + 2 * ld


@torch.library.custom_op("smx::shard_pack", mutates_args=("send",))
def shard_pack(T: Tensor, ctl: Tensor, parts: Tensor, send: Tensor, shape: list[int],
               parity: int) -> None:
    """Local header + candidate rows into the all-gather send slot."""
    _table_ok(T, shape, "T")
    _parts_ok(parts, shape)
    _bytes_ok(send, shard_slot(int(shape[0])) * 8, "send")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_shard_pack(_ptr(T), ctypes.byref(sh), parity, _ptr(ctl),
                                          _ptr(parts), _ptr(send), _stream()), "smx_shard_pack")


@torch.library.custom_op("smx::shard_merge", mutates_args=("ctl", "log"))
def shard_merge(recv: Tensor, ctl: Tensor, log: Tensor, shape: list[int], parity: int,
                nranks: int) -> None:
    """Identical global decision on every rank from the gathered headers."""
    _bytes_ok(recv, nranks * shard_slot(int(shape[0])) * 8, "recv")
    _bytes_ok(ctl, _lib.CTL_BYTES, "ctl")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_shard_merge(_ptr(recv), nranks, ctypes.byref(sh), parity,
                                           _ptr(ctl), _ptr(log), _log_cap(log), _stream()),
               "smx_shard_merge")


@torch.library.custom_op("smx::shard_update", mutates_args=("tout", "ctl", "log"))
def shard_update(tin: Tensor, tout: Tensor, recv: Tensor, ctl: Tensor, log: Tensor,
                 shape: list[int], parity: int, nranks: int) -> None:
    """Merge the gathered headers (identically on every rank) and pivot the local rows and the
    f-row replica with the winning row from recv."""
    _table_ok(tin, shape, "tin")
    _table_ok(tout, shape, "tout")
    _bytes_ok(recv, nranks * shard_slot(int(shape[0])) * 8, "recv")
    sh = make_shape(shape)
    _lib.check(_lib.load().smx_shard_update(_ptr(tin), _ptr(tout), _ptr(recv), nranks,
                                            ctypes.byref(sh), parity, _ptr(ctl), _ptr(log),
                                            _log_cap(log), _stream()), "smx_shard_update")
