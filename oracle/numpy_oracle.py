"""CPU ORACLE (test infrastructure only) — numpy restatement of the reference pivot loop.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this
module.  It is the checker for the HIP engine, never part of the product path.

Dense form of ``/root/reference/src/simplex.py`` (jqnfxa/Simplex-Method-Solver @ 2025-06-20):

* the tableau is a row-major ``float64`` array ``T[R][C]``, ``R = n+1`` (constraint rows + the
  f-row), ``C = m+1`` (variables + the "-b" column).  The reference's f-row has ``len(function)``
  entries (``flen``; the UI passes ``flen = m``, main.py:312); positions ``j >= flen`` of the
  f-row are padding that is computed but never read (simplex.py:94-98 scans ``j < m`` only and no
  selection reads the f-row's last entry);
* :func:`pick` restates ``pick_element`` (simplex.py:70-141) with the leaving-row state machine
  (simplex.py:105-141) written as an arg-min over the total order
  ``key = (0, -v, -i)`` if ``v < 0``, ``(1, i)`` if ``v == 0``, ``(2, i)`` if ``v > 0``
  plus the NaN rule "a NaN ratio of the FIRST candidate sticks, later NaNs are ignored"
  (simplex.py:117-121 vs the comparisons at :123-136);
* :func:`pivot` restates ``recalculate_matrix`` steps 1-4 (simplex.py:155-175): separate numpy
  ufunc passes, so each multiply, subtract and divide is rounded on its own (no FMA) and the
  result is bit-identical to the Python float loops.

Pinned against the reference's own outputs by ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import numpy as np

# status codes shared with include/smx.h
PIVOT, OPTIMUM, INCORRECT, NOT_CONVERGE, FSHORT = 0, 1, 2, 3, 4


def pick(T: np.ndarray, n: int, m: int, flen: int):
    """Return ``(status, r, c)`` for the dense tableau ``T`` (see module doc)."""
    b = T[:n, m]
    neg = np.flatnonzero(b < 0)                            # simplex.py:72-76
    if neg.size:
        r = int(neg[0])
        pos = np.flatnonzero(T[r, :m] > 0)                 # simplex.py:81-85
        if not pos.size:
            return INCORRECT, r, -1                        # simplex.py:88-89
        return PIVOT, r, int(pos[0])
    scan = min(m, flen)
    negf = np.flatnonzero(T[n, :scan] < 0)                 # simplex.py:94-98
    if not negf.size:
        # the reference indexes function[idx] for idx < m: IndexError if flen < m
        return (FSHORT if flen < m else OPTIMUM), -1, -1
    c = int(negf[0])
    a = T[:n, c]
    cand = np.flatnonzero(a != 0)                          # simplex.py:112-113 (NaN != 0)
    if not cand.size:
        return NOT_CONVERGE, -1, c                         # simplex.py:138-139 (first_try)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        v = b[cand] / a[cand]                              # simplex.py:115
    if np.isnan(v[0]):
        return PIVOT, int(cand[0]), c                      # first NaN sticks
    ok = ~np.isnan(v)
    cls0 = ok & (v < 0)
    if cls0.any():
        vmax = v[cls0].max()
        last = np.flatnonzero(cls0 & (v == vmax))[-1]      # ties go to the LAST row (:133)
        return PIVOT, int(cand[last]), c
    zero = ok & (v == 0)
    if zero.any():
        return PIVOT, int(cand[np.flatnonzero(zero)[0]]), c
    return NOT_CONVERGE, -1, c                             # best key in class 2


def pivot(T: np.ndarray, r: int, c: int, out: np.ndarray | None = None) -> np.ndarray:
    """Out-of-place update of simplex.py:149-177; returns the new table."""
    e = T[r, c]
    pr = T[r, :].copy()
    pc = T[:, c].copy()
    with np.errstate(all="ignore"):
        N = np.multiply(T, e, out=out)                     # t*e        (rounded)
        N -= np.multiply.outer(pc, pr)                     # - pr*pc    (rounded each)
        N /= e                                             # / e        (rounded)
        N[r, :] = -pr / e                                  # step 1
        N[:, c] = pc / e                                   # step 2
        N[r, c] = 1.0 / e                                  # step 3
    return N


def to_dense(constraints, function) -> tuple[np.ndarray, int, int, int]:
    """Pack the reference's list-of-lists input (simplex.py:36-39) into ``(T, n, m, flen)``."""
    n = len(constraints)
    m = len(constraints[0]) - 1
    flen = len(function)
    T = np.zeros((n + 1, m + 1), dtype=np.float64)
    for i, row in enumerate(constraints):
        T[i, :] = row
    k = min(flen, m + 1)
    T[n, :k] = function[:k]
    return T, n, m, flen


def from_dense(T: np.ndarray, n: int, flen: int) -> list:
    """Unpack to the reference's ragged layout (f-row trimmed back to ``flen`` entries)."""
    rows = T[:n].tolist()
    rows.append(T[n, :flen].tolist())
    return rows


def run(T: np.ndarray, n: int, m: int, flen: int, max_pivots: int, log=None):
    """Pivot until a terminal status or ``max_pivots``; returns ``(T, status, pivots)``."""
    done = 0
    while done < max_pivots:
        st, r, c = pick(T, n, m, flen)
        if st != PIVOT:
            return T, st, done
        if log is not None:
            log.append((r, c))
        T = pivot(T, r, c)
        done += 1
    return T, PIVOT, done
