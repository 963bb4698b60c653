"""CPU ORACLE (test infrastructure only) — pure-Python restatement of the reference solver.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(``simplex-method-solver_amd/simplex_mi355x``) never imports it.

This restates ``/root/reference/src/simplex.py`` (jqnfxa/Simplex-Method-Solver @ 2025-06-20)
operation for operation on Python ``list``-of-``list`` tableaux:

* :func:`pick`  follows ``SimplexMethod.pick_element``     (simplex.py:70-141), state machine kept
  in its sequential form (the numpy oracle uses the equivalent key-argmin form, so the two
  restatements check each other);
* :func:`pivot` follows ``SimplexMethod.recalculate_matrix`` (simplex.py:143-177): out-of-place,
  every right-hand side read from the OLD table, per element ``(t*e - pr*pc)/e`` with each
  operation rounded separately (Python floats never fuse a multiply-add);
* :class:`Solver` follows ``__init__`` / ``find_optimum`` / ``f`` / ``get_solution``
  (simplex.py:25-39, 48-68, 179-199) but returns plain dict snapshots.

Parity is pinned: ``tests/test_oracle_golden.py`` checks this module bit-for-bit against the
fixtures in ``tests/golden/`` that ``tests/golden/make_golden.py`` produced by importing the
reference itself.
"""
from __future__ import annotations

import copy

INCORRECT_SYSTEM = "incorrect system"                      # simplex.py:89
NOT_CONVERGE = "simplex method does not converge"          # simplex.py:139


def pick(table, n, m, invalid_index):
    """Return ``('pivot', r, c)`` or ``('optimum',)``; raise ValueError like simplex.py:70-141."""
    # phase 1: first row whose last entry (the "-b" column) is negative (simplex.py:72-76)
    r = invalid_index
    for i in range(n):
        if table[i][-1] < 0:
            r = i
            break
    if r != invalid_index:
        # first strictly positive coefficient in that row (simplex.py:81-85)
        for j in range(m):
            if table[r][j] > 0:
                return ("pivot", r, j)
        raise ValueError(INCORRECT_SYSTEM)                 # simplex.py:88-89
    # phase 2 entering column: first negative objective coefficient (simplex.py:94-98)
    c = invalid_index
    for j in range(m):
        if table[-1][j] < 0:
            c = j
            break
    if c == invalid_index:
        return ("optimum",)                                # simplex.py:101-103
    # leaving row: the reference's sequential state machine (simplex.py:107-136)
    best_row, best_val, seen = invalid_index, 1, False
    for i in range(n):
        a = table[i][c]
        if a == 0:
            continue
        v = table[i][-1] / a
        if not seen:
            best_row, best_val, seen = i, v, True
        elif v == 0 and best_val > 0:
            best_row, best_val = i, v
        elif v < 0 <= best_val:
            best_row, best_val = i, v
        elif best_val <= v < 0:
            best_row, best_val = i, v
    if not seen or best_val > 0:                           # simplex.py:138-139
        raise ValueError(NOT_CONVERGE)
    return ("pivot", best_row, c)


def pivot(table, r, c):
    """Out-of-place modified Jordan step of simplex.py:149-177; returns the new table."""
    old = table
    e = old[r][c]
    new = copy.deepcopy(old)                               # simplex.py:149
    new[r] = [-x / e for x in old[r]]                      # step 1, simplex.py:155-156
    for i in range(len(new)):                              # step 2, simplex.py:159-160
        new[i][c] = old[i][c] / e
    new[r][c] = 1.0 / e                                    # step 3, simplex.py:163
    prow = old[r]
    for i in range(len(new)):                              # step 4, simplex.py:166-175
        if i == r:
            continue
        pc = old[i][c]
        row_old, row_new = old[i], new[i]
        for j in range(len(row_new)):
            if j == c:
                continue
            row_new[j] = (row_old[j] * e - prow[j] * pc) / e
    return new


class Solver:
    """List-based mirror of the reference ``SimplexMethod`` state (simplex.py:25-39)."""

    def __init__(self, constraints, function):
        self.n = len(constraints)
        self.m = len(constraints[0]) - 1
        self.invalid_index = 1 + max(self.n, self.m)
        self.function = function
        self.row = ["x%d" % k for k in range(1, self.m + 1)] + ["-b"]
        self.column = ["y%d" % k for k in range(1, self.n + 1)] + ["f"]
        self.table = list(constraints) + [function]

    def f(self, x1, x2):                                   # simplex.py:48-49
        return self.function[0] * x1 + self.function[1] * x2

    def find_optimum(self):                                # simplex.py:51-68
        vals = []
        for name in ("x1", "x2"):
            try:
                k = self.column.index(name)
            except ValueError:
                vals.append(0)
                continue
            vals.append(self.table[k][-1])
        return vals[0], vals[1]

    def pick_element(self):
        res = pick(self.table, self.n, self.m, self.invalid_index)
        if res[0] == "optimum":
            x1, x2 = self.find_optimum()
            return False, x1, x2, self.f(x1, x2)
        _, r, c = res
        return True, r, c, self.table[r][c]

    def recalculate_matrix(self):
        ok, r, c, _ = self.pick_element()
        if not ok:
            return
        self.row[c], self.column[r] = self.column[r], self.row[c]   # simplex.py:152
        self.table = pivot(self.table, r, c)

    def snapshot(self, i=None, j=None, x1=0, x2=0, optimum=0):
        return {"kind": "info", "row": list(self.row), "column": list(self.column),
                "table": copy.deepcopy(self.table), "i": i, "j": j,
                "x1": x1, "x2": x2, "optimum": optimum}

    def get_solution(self, max_pivots=None):
        """simplex.py:179-199; ``max_pivots`` (not in the reference) bounds cycling inputs."""
        out = [self.snapshot()]
        done = 0
        while True:
            try:
                ok, i, j, _ = self.pick_element()
            except ValueError as exc:
                out.append({"kind": "error", "message": str(exc)})
                return out
            if not ok:
                return out
            if max_pivots is not None and done >= max_pivots:
                out.append({"kind": "cap"})
                return out
            out[-1]["i"], out[-1]["j"] = i, j
            self.recalculate_matrix()
            done += 1
            x1, x2 = self.find_optimum()
            out.append(self.snapshot(None, None, x1, x2, self.f(x1, x2)))
