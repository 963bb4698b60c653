"""Host tableau: the pivot loop on the CPU, for machines without an MI355X.

The reference's real workload is the PyQt5 UI's 2-variable LP with a handful of constraints
(main.py:308-313, BASELINE.json configs[0]); a desktop without an MI355X must still run it.
``HostTableau`` keeps the device tableau's layout (``float64[2][R][ld]`` ping-pong, f-row padding
past ``flen``) in host memory and drives the host engine of ``libsmx.so`` (``smx_host_*``,
``csrc/smx_host.hpp``): the same decisions and the same per-element expression as the HIP kernels,
so its trajectories are bit-identical to the device's and to the reference's
(tests/test_surface.py, tests/test_host_engine.py).

It offers the subset of :class:`~simplex_mi355x.device.DeviceTableau` that ``SimplexMethod``
uses.  ``SimplexMethod`` picks it only when no HIP device exists (or for ``device="cpu"``); on a
machine with an MI355X every tableau is a ``DeviceTableau``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .device import leading_dim


class HostTableau:
    """A dense fp64 tableau in host memory plus the state of the pivot loop."""

    is_host = True

    def __init__(self, dense: np.ndarray, n: int, m: int, flen: int, *, log_cap: int = 1 << 16):
        self._L = _lib.load()
        self.rows = self.n = n
        self.m, self.flen, self.row0 = m, flen, 0
        self.C = m + 1
        self.ld = leading_dim(self.C, 4)
        self.device = "cpu"
        self.shape = [self.ld, n, n, m, flen, 0, 1]
        self._shape = _lib.Shape(*self.shape)
        self.buf = np.zeros((2, n + 1, self.ld), dtype=np.float64)
        self.log_cap = log_cap
        self._log = np.zeros((0, 2), dtype=np.int32)
        self.step = 0
        self._sel = None
        self._term = False
        self._status = _lib.IDLE
        self.upload(dense)

    # -- data movement --------------------------------------------------------------------
    def upload(self, dense: np.ndarray) -> None:
        self.buf[:] = 0.0
        self.buf[0, :, :self.C] = np.asarray(dense, dtype=np.float64)[:, :self.C]
        self.step = 0
        self._log = np.zeros((0, 2), dtype=np.int32)
        self._sel = None
        self._term = False
        self._status = _lib.IDLE

    def settle(self) -> None:
        pass

    def cur(self) -> np.ndarray:
        return self.buf[self.step & 1]

    def download(self) -> np.ndarray:
        return self.cur()[:, :self.C].copy()

    def values(self, idx) -> list[float]:
        T = self.cur()
        return [float(T[i, j]) for i, j in idx]

    def read_log(self, start: int, stop: int) -> np.ndarray:
        return self._log[start:stop]

    def block_plan(self):
        return None

    def resident_plan(self):
        return None

    # -- pivot loop -----------------------------------------------------------------------
    def _ptr(self, a: np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)

    def pick(self):
        """pick_element: (status, r, c, e)."""
        self._term = False
        rc = np.zeros(2, dtype=np.int32)
        st = int(self._L.smx_host_select(self._ptr(self.cur()), ctypes.byref(self._shape),
                                         self._ptr(rc)))
        r, c = int(rc[0]), int(rc[1])
        self._sel = (r, c) if st == _lib.PIVOT else None
        self._status = st
        e = float(self.cur()[r, c]) if st == _lib.PIVOT else 0.0
        return st, r, c, e

    def apply_selected(self) -> None:
        """recalculate_matrix with the selection of the last pick()."""
        if self._sel is None:
            raise RuntimeError("apply_selected() without a pivot selected by pick()")
        r, c = self._sel
        p = self.step & 1
        _lib.check(self._L.smx_host_pivot(self._ptr(self.buf[p]), self._ptr(self.buf[p ^ 1]),
                                          ctypes.byref(self._shape), r, c), "smx_host_pivot")
        self._log = np.concatenate([self._log, np.array([[r, c]], dtype=np.int32)])
        self.step += 1
        self._sel = None

    def forced(self, r: int, c: int) -> None:
        self._sel = (r, c)
        self.apply_selected()

    def run(self, k: int, graph: bool = True) -> None:
        """k chained pivots (get_solution's loop, simplex.py:184-198) in one native call."""
        if k <= 0:
            return
        log = np.zeros((k, 2), dtype=np.int32)
        st = ctypes.c_int32()
        done = int(self._L.smx_host_run(self._ptr(self.buf[0]), self._ptr(self.buf[1]),
                                        ctypes.byref(self._shape), self.step & 1, int(k),
                                        self._ptr(log), ctypes.byref(st)))
        self._log = np.concatenate([self._log, log[:done]])
        self.step += done
        self._status = int(st.value)
        self._term = self._status != _lib.IDLE
        self._sel = None

    def int_first_fix(self, mask, r: int, c: int) -> None:
        """After the table's first pivot: the int semantics of its zero results
        (``smx_host_int_first_fix``, csrc/smx_intfirst.hpp; simplex.py:155-175 on ints)."""
        p0 = (self.step - 1) & 1
        md = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        T0 = self.buf[p0]
        _lib.check(self._L.smx_host_int_first_fix(
            self._ptr(T0), self._ptr(self.buf[p0 ^ 1]), self.ld, self.n + 1, self.C, r, c,
            self._ptr(T0[r]), None if md is None else self._ptr(md), self.C,
            None if md is None else self._ptr(md[r])), "smx_host_int_first_fix")

    def sync_state(self) -> dict:
        return {"npivots": self.step, "term": self._term, "sel_status": self._status}

    def clear_term(self) -> None:
        self._term = False

    def close(self) -> None:
        pass
