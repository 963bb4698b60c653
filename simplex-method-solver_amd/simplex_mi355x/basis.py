"""Cycle detection for the pivot loop (opt-in; the reference has none and loops forever,
simplex.py:184-198, on degenerate inputs - SURVEY §8a-7).

The state that decides the rest of a trajectory is the basis laid out on the tableau: which label
sits at each row position (``column`` list, simplex.py:31) and each column position (``row``
list, simplex.py:30).  A pivot ``(r, c)`` swaps the labels at row position r and column position c
(simplex.py:152).  The tracker keeps ``H = XOR_p mix(p, label(p))`` over all positions and updates
it in O(1) per pivot, so it works from the device's pivot log at any tableau size.  A repeated
``H`` means the same basis in the same positions, i.e. the simplex method has cycled; detection
only observes the trajectory, it never changes a pivot.
"""
from __future__ import annotations

_MASK = (1 << 64) - 1


def _mix(x: int) -> int:
    """splitmix64 finaliser."""
    x = (x + 0x9E3779B97F4A7C15) & _MASK
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK
    return x ^ (x >> 31)


class BasisTracker:
    """Incremental hash of the label layout; ``pivot()`` returns a cycle when the basis repeats."""

    def __init__(self, n: int, m: int):
        self.n, self.m = n, m
        # label ids: x_j -> j (0..m-1), y_i -> m + i; positions: column j -> j, row i -> m + i
        self.col_label = list(range(m))             # label at column position j
        self.row_label = [m + i for i in range(n)]  # label at row position i
        h = 0
        for j in range(m):
            h ^= self._z(j, j)
        for i in range(n):
            h ^= self._z(m + i, m + i)
        self.h = h
        self.step = 0
        self.seen = {h: 0}
        self.cycle = None   # (first step of the repeated basis, period)

    @staticmethod
    def _z(pos: int, label: int) -> int:
        return _mix((pos << 32) ^ label)

    def pivot(self, r: int, c: int):
        a, b = self.row_label[r], self.col_label[c]
        pr, pc = self.m + r, c
        self.h ^= self._z(pr, a) ^ self._z(pc, b) ^ self._z(pr, b) ^ self._z(pc, a)
        self.row_label[r], self.col_label[c] = b, a
        self.step += 1
        prev = self.seen.get(self.h)
        if prev is not None and self.cycle is None:
            self.cycle = (prev, self.step - prev)
        else:
            self.seen[self.h] = self.step
        return self.cycle
