"""Batched small LPs: many ``get_solution`` runs in one kernel launch.

The reference UI solves 2-variable LPs with a handful of constraints (main.py:309-313); on the
GPU one such solve is pure launch latency.  ``solve_batch`` packs up to millions of small problems
(n <= 63 constraints, m + 1 <= 64 columns) and runs each one's whole pivot loop inside one
wavefront of ``k_batch`` (csrc/smx_batch.hpp).  Per problem the result is exactly what
``SimplexMethod(constraints, function).get_solution()`` returns (simplex.py:179-199): the list of
``Info`` snapshots (labels, table, i/j, x1/x2/optimum) with the trailing ``Error`` on the two
``ValueError`` outcomes.  Problems outside the batch kernel's envelope (bigger, ragged, or with a
``len(function)`` the reference would index out of range) go through ``SimplexMethod`` one by one
-- still on the device.
"""
from __future__ import annotations

import gc

import numpy as np
import torch

from . import _lib
from .engine import MESSAGES, Error, Info, SimplexMethod

MAX_ROWS = 64      # one wavefront: rows 0..n (f-row = lane n)
MAX_COLS = 64      # register-resident row of at most 64 doubles


def _eligible(cons, func) -> bool:
    if not cons:
        return False
    m = len(cons[0]) - 1
    n = len(cons)
    if n + 1 > MAX_ROWS or m + 1 > MAX_COLS or m < 1:
        return False
    if any(len(r) != m + 1 for r in cons):
        return False
    flen = len(func)
    # int entries: the reference's first pivot runs in int arithmetic, whose zero signs differ
    # from fp64's (engine._int_entries); SimplexMethod applies that fix, k_batch does not
    return flen in (m, m + 1) and flen >= 2 and not _has_ints(cons, func)


def _has_ints(cons, func) -> bool:
    """Any entry an int (Python int / bool, numpy integer scalar or integer row), as
    engine._int_entries counts them."""
    for row in (*cons, func):
        if isinstance(row, np.ndarray):
            if row.dtype.kind in "iub":
                return True
            continue
        for x in row:
            if type(x) is not float and isinstance(x, (int, np.integer)):
                return True
    return False


def _labels(n, m):
    row = ['x' + str(k) for k in range(1, m + 1)] + ['-b']
    col = ['y' + str(k) for k in range(1, n + 1)] + ['f']
    return row, col


def _fallback(cons, func, max_pivots, history):
    try:
        sm = SimplexMethod(cons, func)
        if history:
            return sm.get_solution(max_pivots=max_pivots), sm.status
        return sm.solve(record_history=False, max_pivots=max_pivots), sm.status
    except IndexError as exc:        # where the reference itself raises (simplex.py:49, 95, 159)
        return exc, "exception"


def solve_batch_arrays(tabs: np.ndarray, dims: np.ndarray, max_pivots: int = 256,
                       history: bool = False, device=None) -> dict:
    """Array-level batch solve (no Python objects per problem).

    ``tabs``: float64 [B][Rmax][ldb], problem k in rows 0..n_k (f-row = row n_k), columns
    0..m_k; ``dims``: int32 [B][3] = (n, m, len(function)) with every problem inside the kernel's
    envelope (see ``eligible``).  Returns numpy arrays: ``final`` (same layout as tabs),
    ``status`` (SMX_* codes; SMX_PIVOT = max_pivots reached), ``npivots``, ``rc`` [B][P][2],
    ``xv`` [B][P][2] (x1, x2 after each pivot) and, with ``history``, ``snaps``
    [sum(npivots)][Rmax][ldb] -- problem k's tables after each of its pivots are
    ``snaps[snap_off[k]:snap_off[k + 1]]`` (compacted on the device before the copy back).
    """
    if not torch.cuda.is_available():
        raise RuntimeError("simplex_mi355x needs an MI355X (HIP device); there is no CPU path")
    tabs = np.ascontiguousarray(tabs, dtype=np.float64)
    dims = np.ascontiguousarray(dims, dtype=np.int32)
    B, Rmax, ldb = tabs.shape
    if dims.shape != (B, 3):
        raise ValueError("dims must be int32 [B][3]")
    if B and (Rmax > MAX_ROWS or ldb > MAX_COLS or (dims[:, 0] + 1 > Rmax).any() or
              (dims[:, 1] + 1 > ldb).any() or (dims[:, 1] < 1).any() or (dims[:, 0] < 1).any()):
        raise ValueError("a problem is outside the batch kernel's envelope")
    P = int(max_pivots)
    L = _lib.load()
    dev = torch.device(device if device is not None else "cuda")
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        d_tabs = torch.from_numpy(tabs).to(dev)
        d_dims = torch.from_numpy(dims).to(dev)
        d_out = torch.empty_like(d_tabs)
        d_rc = torch.zeros((B, max(P, 1), 2), dtype=torch.int32, device=dev)
        d_xv = torch.zeros((B, max(P, 1), 2), dtype=torch.float64, device=dev)
        d_snaps = (torch.empty((B, max(P, 1), Rmax, ldb), dtype=torch.float64, device=dev)
                   if history else None)
        d_st = torch.zeros(B, dtype=torch.int32, device=dev)
        d_np = torch.zeros(B, dtype=torch.int32, device=dev)
        _lib.check(L.smx_batch_solve(
            d_tabs.data_ptr(), d_dims.data_ptr(), B, Rmax, ldb, P, d_out.data_ptr(),
            d_rc.data_ptr(), d_xv.data_ptr(), d_snaps.data_ptr() if history else None,
            d_st.data_ptr(), d_np.data_ptr(), stream.cuda_stream), "smx_batch_solve")
        res = {"final": d_out.cpu().numpy(), "rc": d_rc.cpu().numpy(),
               "xv": d_xv.cpu().numpy(), "status": d_st.cpu().numpy(),
               "npivots": d_np.cpu().numpy()}
        if history:
            steps = torch.arange(max(P, 1), device=dev)[None, :] < d_np[:, None]
            res["snaps"] = d_snaps[steps].cpu().numpy()
            res["snap_off"] = np.concatenate([[0], np.cumsum(res["npivots"], dtype=np.int64)])
    return res


def pack(problems):
    """(constraints, function) lists -> (tabs, dims) for solve_batch_arrays."""
    B = len(problems)
    dims = np.zeros((B, 3), dtype=np.int32)
    for q, (c, f) in enumerate(problems):
        dims[q] = (len(c), len(c[0]) - 1, len(f))
    Rmax = int(dims[:, 0].max()) + 1
    ldb = int(dims[:, 1].max()) + 1
    tabs = np.zeros((B, Rmax, ldb), dtype=np.float64)
    for q, (c, f) in enumerate(problems):
        n, m = len(c), len(c[0]) - 1
        tabs[q, :n, :m + 1] = c
        tabs[q, n, :min(len(f), m + 1)] = f[:m + 1]
    return tabs, dims


def solve_batch(problems, max_pivots: int = 256, history: bool = True, device=None):
    """Solve every ``(constraints, function)``; returns ``(results, statuses)``.

    ``results[k]`` is the ``get_solution()`` list of problem k (``history=False``: only the
    initial and the final ``Info``, like ``SimplexMethod.solve(record_history=False)``), or the
    ``IndexError`` the reference would raise.  ``statuses[k]`` is ``"optimum"``, ``"error"``,
    ``"cap"`` (``max_pivots`` reached) or ``"exception"``."""
    problems = list(problems)
    if not torch.cuda.is_available():
        raise RuntimeError("simplex_mi355x needs an MI355X (HIP device); there is no CPU path")
    results = [None] * len(problems)
    statuses = [None] * len(problems)
    idx = [k for k, (c, f) in enumerate(problems) if _eligible(c, f)]
    batched = set(idx)
    for k, (c, f) in enumerate(problems):
        if k not in batched:
            results[k], statuses[k] = _fallback(c, f, max_pivots, history)
    if not idx:
        return results, statuses
    tabs, dims = pack([problems[k] for k in idx])
    out = solve_batch_arrays(tabs, dims, max_pivots, history, device)
    P = int(max_pivots)
    # Hundreds of thousands of fresh, acyclic lists: pause the cyclic collector while they are
    # built, or its generational passes rescan the growing result set (5x slower at 20k LPs).
    gc_was_on = gc.isenabled()
    gc.disable()
    try:
        for q, k in enumerate(idx):
            results[k], statuses[k] = _assemble(
                problems[k], dims[q], out["final"][q], out["rc"][q], out["xv"][q],
                out["snaps"][out["snap_off"][q]:out["snap_off"][q + 1]] if history else None,
                int(out["status"][q]), int(out["npivots"][q]), P)
    finally:
        if gc_was_on:
            gc.enable()
    return results, statuses


def _table(T, n, flen, m):
    rows = T[:n, :m + 1].tolist()
    rows.append(T[n, :min(flen, m + 1)].tolist())
    return rows


def _tables(S, n, flen, m):
    """All snapshots of one LP as Python lists in one conversion (f-row cut to len(function))."""
    tabs = S[:, :n + 1, :m + 1].tolist()
    if flen < m + 1:
        for t in tabs:
            t[n] = t[n][:flen]
    return tabs


def _assemble(problem, dims, final, rc, xv, snaps, status, np_, P):
    """Build the get_solution list (simplex.py:179-199) from the device outputs."""
    cons, func = problem
    n, m, flen = (int(v) for v in dims)
    row, col = _labels(n, m)
    f0, f1 = func[0], func[1]                                # simplex.py:48-49
    # snapshot #0 keeps the caller's values and types (simplex.py:181); rows of numbers, so a
    # row-wise copy is the deep copy
    res = [Info.owning(row, col, [list(r) for r in cons] + [list(func)], None, None, 0, 0, 0)]
    rcl = rc[:np_].tolist()
    xvl = xv[:np_].tolist()
    tables = _tables(snaps[:np_], n, flen, m) if snaps is not None else None
    x1 = x2 = 0
    for s in range(np_):
        r, c = rcl[s]
        if tables is not None or s == 0:
            res[-1].i, res[-1].j = r, c                      # simplex.py:194-195
        row[c], col[r] = col[r], row[c]                      # simplex.py:152
        x1 = xvl[s][0] if 'x1' in col else 0                 # simplex.py:51-68
        x2 = xvl[s][1] if 'x2' in col else 0
        if tables is not None:
            res.append(Info.owning(row, col, tables[s], None, None, x1, x2, f0 * x1 + f1 * x2))
    if tables is None:  # like SimplexMethod.solve(record_history=False): initial + final
        res.append(Info.owning(row, col, _table(final, n, flen, m), None, None, x1, x2,
                               f0 * x1 + f1 * x2))
    if status == _lib.OPTIMUM:
        return res, "optimum"
    if status in MESSAGES:
        res.append(Error(MESSAGES[status]))
        return res, "error"
    if status == _lib.PIVOT and np_ >= P:
        return res, "cap"
    raise RuntimeError(f"unexpected batch status {status}")
