"""``SimplexMethod`` / ``Info`` / ``Error`` -- the reference's solver surface, backed by HBM.

Mirrors ``/root/reference/src/simplex.py`` (jqnfxa/Simplex-Method-Solver @ 2025-06-20):
same constructor, attributes, method names, return tuples, snapshot objects and error
strings, so ``main.py:13`` (``from simplex import SimplexMethod, Error``) and
``table_widget.py:7`` (``from simplex import Info``) work unchanged through the ``simplex.py``
drop-in next to this package.  The tableau lives on the MI355X; every selection and every
pivot is a HIP kernel (``ops.py`` -> ``libsmx.so``).  On a machine with no HIP device at all (a
desktop running the reference UI's 2-variable LPs) the same library's host engine runs the
loop instead (``host.py``, ``backend == "host"``, bit-identical decisions and arithmetic); a
machine with an MI355X never takes it unless asked (``device="cpu"``).

Additions (not in the reference, all opt-in): ``step()`` (one pick + pivot), ``solve()``
(``get_solution`` with an optional pivot cap, or the chained no-history fast path),
``pivots`` / ``pivot_log`` and ``status``.

Deliberate differences, all on inputs the reference UI never produces (main.py:309-312 always
passes rectangular float rows and ``len(function) == m``):
* ragged constraint rows raise ``ValueError`` (the device tableau is dense);
* integer inputs are held as fp64 on the device.  The reference keeps them as Python ints until
  its first pivot, whose int arithmetic gives some zero results the opposite sign from fp64
  (-0 is the int 0; an int product 0 * -3 is +0): the first pivot of a table with int entries
  is followed by ``smx_int_first_fix`` (csrc/smx_intfirst.hpp), which rewrites exactly those
  zeros, so the tables match the reference's bits (tests/golden/intzero.json).  That holds
  while every int is below 2^26 in magnitude (products and differences exact in fp64); larger
  ints get a ``RuntimeWarning``: the reference computes their products exactly, fp64 rounds.
"""
from __future__ import annotations

import copy
import gc

import numpy as np

from . import _lib
from .basis import BasisTracker
from .device import DeviceTableau

MESSAGES = {_lib.INCORRECT: "incorrect system",                  # simplex.py:89
            _lib.NOT_CONVERGE: "simplex method does not converge"}  # simplex.py:139


class Error:
    """simplex.py:4-9."""

    def __init__(self, error_string):
        self.error_string = error_string

    def __str__(self):
        return self.error_string


class Info:
    """simplex.py:12-21: one step snapshot (labels and table copied)."""

    def __init__(self, row, column, table, i, j, x1, x2, optimum):
        self.row = row.copy()
        self.column = column.copy()
        self.table = copy.deepcopy(table)
        self.i = i
        self.j = j
        self.x1 = x1
        self.x2 = x2
        self.optimum = optimum

    @classmethod
    def owning(cls, row, column, table, i, j, x1, x2, optimum):
        """The same snapshot for a table the caller just built and hands over (fresh lists of
        Python floats from the device download): labels are copied, the table is not
        deep-copied again -- the observable object is identical."""
        self = cls.__new__(cls)
        self.row = row.copy()
        self.column = column.copy()
        self.table = table
        self.i = i
        self.j = j
        self.x1 = x1
        self.x2 = x2
        self.optimum = optimum
        return self


class LazyInfo(Info):
    """An ``Info`` whose ``table`` is materialised on first access from the device history
    (checkpoint + replay of the logged pivots with the bit-identical update kernel), so a
    get_solution history of a large tableau costs O(pivots) host memory, not O(pivots x R x C)."""

    def __init__(self, row, column, history, step, i, j, x1, x2, optimum, table=None):
        self.row = row.copy()
        self.column = column.copy()
        self._history = history
        self._step = step
        self._table = table
        self.i = i
        self.j = j
        self.x1 = x1
        self.x2 = x2
        self.optimum = optimum

    @property
    def table(self):
        if self._table is None:
            self._table = self._history.table(self._step)
        return self._table

    @table.setter
    def table(self, value):
        self._table = value


class History:
    """Device checkpoints of the tableau every ``every`` pivots (within ``budget_bytes``) plus
    the host copy of the pivot log; ``table(step)`` replays from the nearest checkpoint."""

    def __init__(self, solver, every=256, budget_bytes=8 << 30):
        import torch
        self.sm = solver
        self.dev = solver._dev
        self.every = max(1, int(every))
        self.budget = budget_bytes
        self.ckpt = {}
        self.base = solver.pivots          # pivot count at the start of this history
        self._torch = torch
        self._scratch = None
        self.checkpoint(self.base)

    def _bytes(self):
        return sum(t.numel() * 8 for t in self.ckpt.values())

    def checkpoint(self, step):
        dev = self.dev
        if step in self.ckpt or (step - self.base) % self.every and step != self.base:
            return
        one = (dev.rows + 1) * dev.ld * 8
        if self.ckpt and self._bytes() + one > self.budget:
            return
        with self._torch.cuda.stream(dev.stream):
            self.ckpt[step] = dev.cur().clone()

    def checkpoint_now(self):
        """Checkpoint the current device table regardless of spacing (budget permitting)."""
        dev = self.dev
        step = self.sm.pivots
        one = (dev.rows + 1) * dev.ld * 8
        if step in self.ckpt or (self.ckpt and self._bytes() + one > self.budget):
            return
        with self._torch.cuda.stream(dev.stream):
            self.ckpt[step] = dev.cur().clone()

    def table(self, step):
        dev, torch = self.dev, self._torch
        s0 = max(k for k in self.ckpt if k <= step)
        log = self.sm.pivot_log
        with torch.cuda.stream(dev.stream):
            if self._scratch is None:
                self._scratch = torch.empty((2, dev.rows + 1, dev.ld), dtype=torch.float64,
                                            device=dev.device)
            sc = self._scratch
            sc[0].copy_(self.ckpt[s0])
            from . import ops
            ih = self.sm._int_hist
            for t in range(s0, step):
                a = (t - s0) & 1
                r, c = log[t]
                ops.update_forced(sc[a], sc[a ^ 1], dev.shape, r, c)
                if t == 0 and ih is not None:   # the caller's ints: their first pivot's zeros
                    from .device import int_first_fix
                    int_first_fix(sc[a], sc[a ^ 1], dev.C, ih[0], ih[1], ih[2])
            T = sc[(step - s0) & 1][:, :dev.C].cpu().numpy()
        rows = T[:self.sm.n].tolist()
        rows.append(T[self.sm.n, :min(self.sm.flen, self.sm.m + 1)].tolist())
        return rows


def _dense_from_lists(constraints, function, m):
    n = len(constraints)
    T = np.zeros((n + 1, m + 1), dtype=np.float64)
    if n:
        T[:n, :] = np.asarray(constraints, dtype=np.float64)
    k = min(len(function), m + 1)
    if k:
        T[n, :k] = np.asarray(function[:k], dtype=np.float64)
    return T


INT_EXACT = 1 << 26   # |int| below this: the first pivot's int products are exact in fp64


def _int_entries(constraints, function, m, dense):
    """Which tableau entries the caller passed as ints (Python ``int`` / ``bool``, numpy integer
    scalars or integer rows): None when none, True when all of them, else a uint8 mask
    ``[n + 1][m + 1]``."""
    rows = list(constraints) + [function]
    n = len(constraints)
    kinds = []
    for row in rows:
        if isinstance(row, np.ndarray):
            kinds.append(1 if row.dtype.kind in "iub" else 0)
            continue
        ts = set(map(type, row))
        ints = {t for t in ts if issubclass(t, (int, np.integer))}
        kinds.append(0 if not ints else (1 if ints == ts else 2))
    if not any(kinds):
        return None
    if all(k == 1 for k in kinds):   # (f-row padding is never an operand: int or not alike)
        mask = True
        big = float(np.abs(dense[:n + 1, :m + 1]).max(initial=0.0)) >= INT_EXACT
    else:
        mask = np.zeros((n + 1, m + 1), dtype=np.uint8)
        for i, (row, k) in enumerate(zip(rows, kinds)):
            if k == 1:
                mask[i, :min(len(row), m + 1)] = 1
            elif k == 2:
                mask[i, :min(len(row), m + 1)] = [isinstance(x, (int, np.integer))
                                                  for x in row[:m + 1]]
        big = float(np.abs(np.where(mask != 0, dense[:n + 1, :m + 1], 0.0)).max(initial=0.0)) \
            >= INT_EXACT
    if big:
        import warnings
        warnings.warn("simplex_mi355x: integer inputs of magnitude >= 2^26: the reference forms "
                      "their first-pivot products in exact integer arithmetic, this engine in "
                      "fp64 (the results may differ in the last bits)", RuntimeWarning,
                      stacklevel=3)
    return mask


def _use_host(device) -> bool:
    """The host engine runs a tableau only on request (``device="cpu"``) or when this machine has
    no HIP device at all -- then with a one-time ``RuntimeWarning``, and ``SimplexMethod.backend``
    reads "host"; with an MI355X present every tableau lives in HBM."""
    if device is not None:
        return str(device) == "cpu"
    import torch
    if torch.cuda.is_available():
        return False
    global _warned_host
    if not _warned_host:
        _warned_host = True
        import warnings
        warnings.warn("simplex_mi355x: no HIP device is visible, so SimplexMethod runs on the host "
                      "engine (backend == 'host'); pass device='cpu' to choose it explicitly",
                      RuntimeWarning, stacklevel=3)
    return True


_warned_host = False


class SimplexMethod:
    """simplex.py:24-199 on an MI355X-resident tableau (or, on a machine without one, on the
    host engine of the same library: ``backend == "host"``)."""

    def __init__(self, constraints, function, device=None, devices=None, pivots=None,
                 exchange=None):
        # simplex.py:26-33 (IndexError on an empty constraint list, like the reference)
        self.n = len(constraints)
        self.m = len(constraints[0]) - 1
        self.invalid_index = 1 + max(self.n, self.m)
        self.function = function
        self.row = ['x' + str(_) for _ in range(1, self.m + 1)]
        self.column = ['y' + str(_) for _ in range(1, self.n + 1)]
        self.row.append('-b')
        self.column.append('f')
        if any(len(c) != self.m + 1 for c in constraints):
            raise ValueError("ragged constraint rows: the device tableau is dense "
                             f"(every row must have m + 1 = {self.m + 1} entries)")
        # simplex.py:36-39: the caller's rows (and function) by reference, until the first pivot
        self._initial = [constraint for constraint in constraints]
        self._initial.append(function)
        self.flen = len(function)
        dense = _dense_from_lists(constraints, function, self.m)
        if devices is not None:
            # row sharding behind the same surface: rank p's rows on devices[p] (multi.py)
            from .multi import MultiTableau
            self._dev = MultiTableau(dense, self.n, self.m, self.flen, devices, pivots=pivots,
                                     exchange=exchange)
        elif _use_host(device):
            from .host import HostTableau
            self._dev = HostTableau(dense, self.n, self.m, self.flen)
        else:
            self._dev = DeviceTableau(dense, self.n, self.m, self.flen, device=device)
        self._pristine = True
        # int entries of the caller's table (None / True / mask): pending until the first pivot,
        # then kept with its (r, c) for history replays (_int_first_fix)
        self._int0 = _int_entries(constraints, function, self.m, dense)
        self._int_hist = None
        self.pivot_log: list[tuple[int, int]] = []
        self.status = "ready"
        self.cycle = None          # (first step of a repeated basis, period) when detected
        self._tracker = None

    @classmethod
    def from_file(cls, path, device=None):
        """Load a problem file: the reference UI's ``.txt`` (main.py:402-495; objective =
        gradient[:-1], main.py:312) or a binary ``.smx`` tableau streamed straight into HBM."""
        from . import problem_io
        if path.endswith(".smx"):
            dev = problem_io.load_device(path, device=device)
            return cls._from_device(dev)
        return cls(*problem_io.solver_inputs_txt(path), device=device)

    @classmethod
    def _from_device(cls, dev):
        """A SimplexMethod around an already-resident tableau (no host lists of the table)."""
        self = cls.__new__(cls)
        self.n, self.m, self.flen = dev.rows, dev.m, dev.flen
        self.invalid_index = 1 + max(self.n, self.m)
        with __import__("torch").cuda.stream(dev.stream):
            self.function = dev.buf[0, self.n, :min(dev.flen, dev.C)].cpu().tolist()
        self.row = ['x' + str(_) for _ in range(1, self.m + 1)] + ['-b']
        self.column = ['y' + str(_) for _ in range(1, self.n + 1)] + ['f']
        self._initial = None
        self._dev = dev
        self._pristine = False
        self._int0 = self._int_hist = None
        self.pivot_log = []
        self.status = "ready"
        self.cycle = None
        self._tracker = None
        return self

    # ---------------------------------------------------------------- state views --------
    @property
    def table(self):
        """The current tableau as the reference's list of lists (f-row has len(function))."""
        if self._pristine:
            return self._initial
        T = self._dev.download()
        rows = T[:self.n].tolist()
        rows.append(T[self.n, :min(self.flen, self.m + 1)].tolist())
        return rows

    def _snapshot(self, x1, x2, optimum) -> Info:
        """Info of the current state (simplex.py:181, :197-198).  A downloaded table is a fresh
        list of fresh floats, so it is handed over instead of deep-copied a second time; the
        pristine table (the caller's own lists) is deep-copied like the reference does."""
        if self._pristine:
            return Info(self.row, self.column, self.table, None, None, x1, x2, optimum)
        return Info.owning(self.row, self.column, self.table, None, None, x1, x2, optimum)

    @table.setter
    def table(self, value):
        cons, func = value[:-1], value[-1]
        if any(len(c) != self.m + 1 for c in cons) or len(cons) != self.n:
            raise ValueError("table shape does not match this problem")
        self._initial = list(value)
        self.flen = len(func)
        dense = _dense_from_lists(cons, func, self.m)
        self._dev.upload(dense)
        self._pristine = True
        self._int0 = _int_entries(cons, func, self.m, dense)
        self._int_hist = None

    @property
    def backend(self) -> str:
        """"hip" (the tableau is in HBM, every pivot a HIP kernel), "sharded" (row blocks on
        several devices, ``devices=[...]``) or "host" (no HIP device)."""
        if getattr(self._dev, "is_host", False):
            return "host"
        return "sharded" if hasattr(self._dev, "ranks") else "hip"

    @property
    def pivots(self) -> int:
        return len(self.pivot_log)

    def print_table(self):
        """simplex.py:41-46."""
        table = self.table
        print("\t", end='')
        print("\t".join(self.row))
        for row in range(self.n + 1):
            print(self.column[row], end='\t')
            print("\t".join([str(round(val, 6)) for val in table[row]]))

    def f(self, x1, x2):
        """simplex.py:48-49 (on the ORIGINAL objective list)."""
        return self.function[0] * x1 + self.function[1] * x2

    def _last_of_rows(self, rows):
        if self._pristine:
            return [self._initial[i][-1] for i in rows]
        last = [(i, self.m if i < self.n else min(self.flen, self.m + 1) - 1) for i in rows]
        return self._dev.values(last)

    def find_optimum(self) -> (float, float):
        """simplex.py:51-68."""
        def index_of(s):
            for row in range(len(self.column)):
                if self.column[row] == s:
                    return row
            return self.invalid_index

        x1_i = index_of('x1')
        x2_i = index_of('x2')
        want = [i for i in (x1_i, x2_i) if i != self.invalid_index]
        vals = dict(zip(want, self._last_of_rows(want)))
        x1 = vals[x1_i] if x1_i != self.invalid_index else 0
        x2 = vals[x2_i] if x2_i != self.invalid_index else 0
        return x1, x2

    # ---------------------------------------------------------------- the hot path -------
    def pick_element(self) -> (bool, int, int, float):
        """simplex.py:70-141: selection kernels on the device, outcome mapped to the
        reference's return tuple / ValueError."""
        status, r, c, e = self._dev.pick()
        if status == _lib.PIVOT:
            if self._pristine:
                e = self._initial[r][c]
            return True, r, c, e
        if status == _lib.OPTIMUM:
            x1, x2 = self.find_optimum()
            return False, x1, x2, self.f(x1, x2)
        if status in MESSAGES:
            raise ValueError(MESSAGES[status])
        if status == _lib.FSHORT:
            # the reference indexes function[idx] past its end (simplex.py:95-96)
            raise IndexError("list index out of range")
        raise RuntimeError(f"unexpected selection status {status}")

    def _apply(self, r, c):
        """The part of recalculate_matrix after its pick_element (simplex.py:149-177)."""
        self.row[c], self.column[r] = self.column[r], self.row[c]   # simplex.py:152
        if self.flen > self.m + 1 or (self.flen < self.m and c >= self.flen):
            # the reference's step 2 / step 4 index the f-row out of range (simplex.py:159-175)
            raise IndexError("list index out of range")
        first_int = self._pristine and self._int0 is not None
        self._dev.apply_selected()
        if first_int:
            self._int_first_fix(r, c)
        self._pristine = False
        self.pivot_log.append((r, c))

    def _int_first_fix(self, r, c):
        """The first pivot of a table with int entries just ran (r, c): give its zero results
        the signs the reference's int arithmetic gives them (smx_int_first_fix)."""
        mask = None if self._int0 is True else self._int0
        self._dev.int_first_fix(mask, r, c)
        self._int_hist = (mask, r, c)
        self._int0 = None

    def _int_first_after_run(self, before, done):
        """After a chained run that began at the caller's table: the int fix of its first pivot
        (the chained loops run that pivot alone while one is pending).  True when applied."""
        if self._int0 is None or before != 0 or done < 1 or not self._pristine:
            return False
        r, c = (int(x) for x in self._dev.read_log(0, 1)[0])
        self._int_first_fix(r, c)
        return True

    def recalculate_matrix(self):
        """simplex.py:143-177."""
        _is_successful, r, c, _ = self.pick_element()
        if not _is_successful:
            return
        self._apply(r, c)

    def _track(self, r, c, detect_cycles):
        """Feed a pivot to the opt-in cycle detector; True when the basis has repeated."""
        if not detect_cycles:
            return False
        if self._tracker is None:
            self._tracker = BasisTracker(self.n, self.m)
            for rr, cc in self.pivot_log[:-1]:
                self._tracker.pivot(rr, cc)
        if self._tracker.pivot(r, c) is not None:
            self.cycle = self._tracker.cycle
            return True
        return False

    LAZY_ELEMENTS = 1 << 20   # above this many tableau entries get_solution snapshots lazily

    def get_solution(self, max_pivots=None, detect_cycles=False, lazy=None, chunk=256):
        """simplex.py:179-199.  Opt-in additions (defaults = the reference's behaviour):
        ``max_pivots`` bounds the loop (the list ends, ``status == 'cap'``); ``detect_cycles``
        ends it when the basis repeats (``status == 'cycle'``, ``self.cycle``).  ``lazy``
        (default: automatic above ``LAZY_ELEMENTS`` entries) runs the chained device loop and
        returns ``LazyInfo`` snapshots whose tables are materialised on access."""
        if lazy is None:
            lazy = (self.n + 1) * (self.m + 1) > self.LAZY_ELEMENTS
        lazy = lazy and self.backend != "host"   # device checkpoints + replay need a device
        if lazy and self.flen in (self.m, self.m + 1) and self.flen >= 2:
            return self._get_solution_lazy(max_pivots, detect_cycles, chunk)
        # every snapshot is a fresh acyclic list of lists: pause the cyclic collector so its
        # passes do not rescan the growing history (the reference pays that; the result is equal)
        gc_was_on = gc.isenabled()
        gc.disable()
        try:
            return self._get_solution_eager(max_pivots, detect_cycles)
        finally:
            if gc_was_on:
                gc.enable()

    def _get_solution_eager(self, max_pivots, detect_cycles):
        result = []
        result.append(self._snapshot(0, 0, 0))
        done = 0
        while True:
            try:
                is_successful, i, j, e = self.pick_element()
            except ValueError as exc:
                result.append(Error(str(exc)))
                self.status = "error"
                return result
            if not is_successful:
                self.status = "optimum"
                break
            if max_pivots is not None and done >= max_pivots:
                self.status = "cap"
                break
            result[-1].i = i
            result[-1].j = j
            self._apply(i, j)   # recalculate_matrix() without re-running the selection
            done += 1
            x1, x2 = self.find_optimum()
            result.append(self._snapshot(x1, x2, self.f(x1, x2)))
            if self._track(i, j, detect_cycles):
                self.status = "cycle"
                break
        return result

    def _get_solution_lazy(self, max_pivots, detect_cycles, chunk):
        """get_solution's loop (simplex.py:184-198) chained on the device; the (i, j) of every
        step and its (x1, x2) come from the device rings, tables from History on demand."""
        hist = History(self, every=chunk)
        first = LazyInfo(self.row, self.column, hist, self.pivots, None, None, 0, 0, 0,
                         table=copy.deepcopy(self.table) if self._pristine else None)
        result = [first]
        dev = self._dev
        budget = float("inf") if max_pivots is None else int(max_pivots)
        start = self.pivots
        status = None
        while self.pivots - start < budget:
            # chunks end on multiples of `chunk` from the history's base, where hist.checkpoint
            # keeps a table: after an int table's lone first pivot the next chunk is one shorter,
            # so the later checkpoints are taken (else every replay starts at step 0)
            k = chunk - (self.pivots - start) % chunk
            k = int(min(k, budget - (self.pivots - start), dev.log_cap))
            if self._int0 is not None and self._pristine:
                k = 1                      # the first pivot of an int table runs alone
            before = dev.step
            dev.run(k, graph=(k == chunk))
            ctl = dev.sync_state()
            done = int(ctl["npivots"])
            fixed = self._int_first_after_run(before, done)
            logs = dev.read_log(before, done)
            xs = dev.read_xhist(before, done)
            cycled = False
            for (r, c), (v1, v2) in zip(logs, xs):
                r, c = int(r), int(c)
                result[-1].i, result[-1].j = r, c
                self.row[c], self.column[r] = self.column[r], self.row[c]   # simplex.py:152
                self.pivot_log.append((r, c))
                self._pristine = False
                if fixed:                  # the ring holds the pre-fix values of pivot 0
                    x1, x2 = self.find_optimum()
                    fixed = False
                else:
                    x1 = float(v1) if 'x1' in self.column else 0            # simplex.py:51-68
                    x2 = float(v2) if 'x2' in self.column else 0
                result.append(LazyInfo(self.row, self.column, hist, self.pivots, None, None,
                                       x1, x2, self.f(x1, x2)))
                cycled = self._track(r, c, detect_cycles) or cycled   # stop after this chunk
            hist.checkpoint(self.pivots)
            if cycled:
                status = "cycle"
                break
            if ctl["term"]:
                status = int(ctl["sel_status"])
                break
        if status is None:
            self.status = "cap"
        elif status == "cycle":
            self.status = "cycle"
        elif status == _lib.OPTIMUM:
            self.status = "optimum"
        elif status in MESSAGES:
            self.status = "error"
            result.append(Error(MESSAGES[status]))
        return result

    # ---------------------------------------------------------------- additions ----------
    def step(self):
        """One pick + pivot; returns pick_element's tuple (raises like it)."""
        res = self.pick_element()
        if res[0]:
            self._apply(res[1], res[2])
        return res

    def solve(self, record_history=True, max_pivots=None, chunk=256, graph=True,
              detect_cycles=False):
        """``get_solution`` (record_history=True) or the chained fast path: pivots run on the
        device in chunks of ``chunk`` with no host synchronisation inside a chunk; returns
        ``[Info(initial, i/j of the first pivot), Info(final)]`` plus a trailing ``Error``.
        ``detect_cycles`` stops at the end of the chunk in which the basis first repeats."""
        if record_history:
            return self.get_solution(max_pivots=max_pivots, detect_cycles=detect_cycles)
        if self.flen not in (self.m, self.m + 1) or self.flen < 2:
            return self._solve_stepwise(max_pivots, detect_cycles)
        big = (self.n + 1) * (self.m + 1) > self.LAZY_ELEMENTS and self.backend != "host"
        hist = History(self, every=1 << 62) if big else None    # one checkpoint: the start
        if big:
            first = LazyInfo(self.row, self.column, hist, self.pivots, None, None, 0, 0, 0)
        else:
            first = self._snapshot(0, 0, 0)
        start = self.pivots
        budget = float("inf") if max_pivots is None else int(max_pivots)
        dev = self._dev
        status = None
        while self.pivots - start < budget:
            k = int(min(chunk, budget - (self.pivots - start), dev.log_cap))
            if self._int0 is not None and self._pristine:
                k = 1                      # the first pivot of an int table runs alone
            before = dev.step
            dev.run(k, graph=graph and k == chunk)
            ctl = dev.sync_state()
            done = int(ctl["npivots"])
            self._int_first_after_run(before, done)
            cycled = False
            for r, c in dev.read_log(before, done):
                r, c = int(r), int(c)
                self.row[c], self.column[r] = self.column[r], self.row[c]
                self.pivot_log.append((r, c))
                cycled = self._track(r, c, detect_cycles) or cycled
            if done > 0:
                self._pristine = False
            if ctl["term"]:
                status = int(ctl["sel_status"])
                break
            if cycled:
                status = "cycle"
                break
        out = [first]
        if self.pivots > start:
            first.i, first.j = self.pivot_log[start]
        x1, x2 = self.find_optimum()
        if big:   # the final table is the current device table: materialise it on access
            hist.checkpoint_now()
            out.append(LazyInfo(self.row, self.column, hist, self.pivots, None, None, x1, x2,
                                self.f(x1, x2)))
        else:
            out.append(self._snapshot(x1, x2, self.f(x1, x2)))
        if status is None:
            self.status = "cap"
        elif status == "cycle":
            self.status = "cycle"
        elif status == _lib.OPTIMUM:
            self.status = "optimum"
        elif status in MESSAGES:
            self.status = "error"
            out.append(Error(MESSAGES[status]))
        else:
            raise RuntimeError(f"unexpected terminal status {status}")
        return out

    def _solve_stepwise(self, max_pivots, detect_cycles=False):
        first = self._snapshot(0, 0, 0)
        out = [first]
        done = 0
        while max_pivots is None or done < max_pivots:
            try:
                ok, i, j, _ = self.pick_element()
            except ValueError as exc:
                x1, x2 = self.find_optimum()
                out.append(self._snapshot(x1, x2, self.f(x1, x2)))
                out.append(Error(str(exc)))
                self.status = "error"
                return out
            if not ok:
                break
            if done == 0:
                first.i, first.j = i, j
            self._apply(i, j)
            done += 1
            if self._track(i, j, detect_cycles):
                break
        if self.cycle is not None and detect_cycles:
            self.status = "cycle"
        else:
            self.status = "optimum" if (max_pivots is None or done < max_pivots) else "cap"
        x1, x2 = self.find_optimum()
        out.append(self._snapshot(x1, x2, self.f(x1, x2)))
        return out
