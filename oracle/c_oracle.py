"""CPU ORACLE (test infrastructure only) — ctypes binding of ``oracle/_build/libsmx_oracle.so``.

The C restatement of simplex.py:70-199 (see ``simplex_oracle.c``).  Used by ``tests/`` as a fast
checker at sizes the pure-Python restatement cannot reach, by ``smoke()`` and by ``bench.py``'s
``cpu_baseline`` leg.  Never imported by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsmx_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i32, i64, dp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
        L.smx_oracle_pick.argtypes = [dp, i64, i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.smx_oracle_pick.restype = ctypes.c_int
        L.smx_oracle_pivot.argtypes = [dp, dp, i64, i32, i32, i32, i32, i32]
        L.smx_oracle_pivot.restype = None
        L.smx_oracle_run.argtypes = [dp, dp, i64, i32, i32, i32, i64, dp,
                                     ctypes.POINTER(i32), ctypes.POINTER(i32), i32]
        L.smx_oracle_run.restype = i64
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.c_void_p)


def pick(T: np.ndarray, n: int, m: int, flen: int):
    r, c = ctypes.c_int32(), ctypes.c_int32()
    st = lib().smx_oracle_pick(_ptr(T), T.shape[1], n, m, flen, ctypes.byref(r), ctypes.byref(c))
    return st, r.value, c.value


def pivot(T: np.ndarray, r: int, c: int, out: np.ndarray | None = None, threads: int = 1):
    if out is None:
        out = np.empty_like(T)
    lib().smx_oracle_pivot(_ptr(T), _ptr(out), T.shape[1], T.shape[0], T.shape[1], r, c, threads)
    return out


def run(T: np.ndarray, n: int, m: int, flen: int, max_pivots: int, threads: int = 1,
        want_log: bool = True):
    """Pivot until terminal or ``max_pivots``; returns ``(T_final, status, pivots, log)``."""
    A = np.ascontiguousarray(T, dtype=np.float64).copy()
    B = np.empty_like(A)
    log = np.zeros((max(max_pivots, 1), 2), dtype=np.int32) if want_log else None
    which, status = ctypes.c_int32(), ctypes.c_int32()
    done = lib().smx_oracle_run(_ptr(A), _ptr(B), A.shape[1], n, m, flen, max_pivots,
                                log.ctypes.data_as(ctypes.c_void_p) if want_log else None,
                                ctypes.byref(which), ctypes.byref(status), threads)
    final = A if which.value == 0 else B
    return final, status.value, int(done), (log[:done] if want_log else None)
