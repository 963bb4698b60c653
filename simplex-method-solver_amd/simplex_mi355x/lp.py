"""Seeded dense LP generators (the §8d benchmark/parity inputs), shardable by row block.

Rows are produced in blocks of ``BLOCK`` rows, block ``k`` from ``default_rng([seed, k])``, so a
rank can build exactly its own row range of the global LP without materialising the rest.
Tableau convention of the reference (simplex.py:36-39): constraint row i = [a_i1 .. a_im, b_i]
meaning y_i = a_i . x + b_i >= 0, then the f-row = c (len m, the UI's layout, main.py:312).
"""
from __future__ import annotations

import numpy as np

BLOCK = 1024


def _block(kind: str, seed: int, k: int, nrows: int, m: int) -> np.ndarray:
    rng = np.random.default_rng([seed, k])
    out = np.empty((nrows, m + 1), dtype=np.float64)
    if kind == "uniform":          # A~U(-1,1), b~U(0.1,1): feasible at the origin (phase 2)
        out[:, :m] = rng.uniform(-1.0, 1.0, size=(nrows, m))
        out[:, m] = rng.uniform(0.1, 1.0, size=nrows)
    elif kind == "mixed":          # b~U(-1,1): phase 1 first
        out[:, :m] = rng.uniform(-1.0, 1.0, size=(nrows, m))
        out[:, m] = rng.uniform(-1.0, 1.0, size=nrows)
    elif kind == "degenerate":     # §8d config 5: A in [-2,2], b = 0 w.p. 0.9 else {1,2}
        out[:, :m] = rng.integers(-2, 3, size=(nrows, m))
        out[:, m] = np.where(rng.random(nrows) < 0.9, 0.0, rng.integers(1, 3, size=nrows))
    elif kind == "degenerate_mixed":
        out[:, :m] = rng.integers(-2, 3, size=(nrows, m))
        out[:, m] = rng.integers(-2, 3, size=nrows)
    else:
        raise ValueError(kind)
    return out


def objective(kind: str, seed: int, m: int) -> np.ndarray:
    rng = np.random.default_rng([seed, 1 << 30])
    if kind.startswith("degenerate"):
        return rng.integers(-2, 3, size=m).astype(np.float64)
    return rng.uniform(-1.0, 1.0, size=m)


def dense_rows(kind: str, seed: int, n: int, m: int, row_lo: int = 0, row_hi: int | None = None,
               ld: int | None = None, out: np.ndarray | None = None) -> np.ndarray:
    """Constraint rows [row_lo, row_hi) of the global n x (m+1) LP, width ld (zero padded);
    written into ``out`` (shape (row_hi - row_lo, >= m+1), zero padded by the caller) if given."""
    row_hi = n if row_hi is None else row_hi
    width = m + 1 if ld is None else ld
    if out is None:
        out = np.zeros((row_hi - row_lo, width), dtype=np.float64)
    k0, k1 = row_lo // BLOCK, (row_hi + BLOCK - 1) // BLOCK

    def fill(k):
        lo, hi = k * BLOCK, min(n, (k + 1) * BLOCK)
        blk = _block(kind, seed, k, hi - lo, m)
        a, b = max(lo, row_lo), min(hi, row_hi)
        if a < b:
            out[a - row_lo:b - row_lo, :m + 1] = blk[a - lo:b - lo]

    if (row_hi - row_lo) * m < (1 << 24):
        for k in range(k0, k1):
            fill(k)
        return out
    # every block has its own generator, so the blocks are independent: fill them on threads
    # (numpy's generators release the GIL; a 65536 x 32768 table: ~38 s -> a few seconds)
    import os
    from concurrent.futures import ThreadPoolExecutor
    workers = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(fill, range(k0, k1)))
    return out


def dense_tableau(kind: str, seed: int, n: int, m: int, row_lo: int = 0,
                  row_hi: int | None = None) -> np.ndarray:
    """Rows [row_lo, row_hi) plus the f-row (objective, len m) as the last row (one allocation:
    a 65536 x 32768 tableau is 17 GB)."""
    row_hi = n if row_hi is None else row_hi
    T = np.zeros((row_hi - row_lo + 1, m + 1), dtype=np.float64)
    dense_rows(kind, seed, n, m, row_lo, row_hi, out=T[:-1])
    T[-1, :m] = objective(kind, seed, m)
    return T
