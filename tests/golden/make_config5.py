"""Generate ``tests/golden/config5.json``: BASELINE config 5 (65536 x 32768 degenerate tableaux,
SURVEY.md §8d) pinned at FULL size against the C oracle, so the GPU test compares the HIP path
with the oracle instead of with itself.  Runs in the build container only
(the oracle needs two 17.2 GB buffers and ~10 minutes per generator on 8 cores)::

    python tests/golden/make_config5.py [--pivots 209] [--threads 8]

For each generator (``degenerate``, ``degenerate_mixed``; seed 0, ``simplex_mi355x.lp``) the
oracle (``oracle/simplex_oracle.c``, the restatement of simplex.py:70-199 pinned by the other
fixtures) runs get_solution's loop (simplex.py:184-198) for up to ``--pivots`` pivots and the
fixture records

* ``log``: every pivot ``(r, c)`` (simplex.py:194-195);
* ``cycle``: the first repeat of the basis laid out on the tableau (label at every row and column
  position, moved by simplex.py:152), as ``[first step, period]``, found by comparing the exact
  label arrays (a SHA-256 of each state's int32 labels as the dictionary key) -- independent of
  the product's ``basis.BasisTracker``;
* ``sha256``: at pivots 20, 60, 140 and at the end, the SHA-256 of the table's bytes as the
  reference holds them: the n constraint rows of m + 1 fp64 values (C order), then the f-row's
  first m values (its last entry is padding, simplex.py:36-39 / main.py:312).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))

from oracle import c_oracle  # noqa: E402
from simplex_mi355x import lp  # noqa: E402

N, M, SEED = 65535, 32767, 0
CHECKPOINTS = (20, 60, 140)


def table_sha256(T: np.ndarray, n: int, m: int) -> str:
    """SHA-256 of rows 0..n-1 (m + 1 values each) then the f-row's first m values."""
    h = hashlib.sha256()
    step = 1024
    for lo in range(0, n, step):
        h.update(np.ascontiguousarray(T[lo:min(n, lo + step), :m + 1]).tobytes())
    h.update(np.ascontiguousarray(T[n, :m]).tobytes())
    return h.hexdigest()


def cycle_of(n: int, m: int, log) -> list | None:
    """First repeat of the label layout (exact arrays; simplex.py:152 moves the labels)."""
    col = np.arange(m, dtype=np.int32)               # x_j at column position j
    row = np.arange(m, m + n, dtype=np.int32)        # y_i at row position i

    def key():
        return hashlib.sha256(col.tobytes() + row.tobytes()).digest()

    seen = {key(): 0}
    for s, (r, c) in enumerate(log, start=1):
        row[r], col[c] = col[c], row[r]
        k = key()
        if k in seen:
            return [seen[k], s - seen[k]]
        seen[k] = s
    return None


def run_kind(kind: str, pivots: int, threads: int, n: int = N, m: int = M) -> dict:
    t0 = time.time()
    A = lp.dense_tableau(kind, SEED, n, m)
    B = np.empty_like(A)
    L = c_oracle.lib()
    ld = A.shape[1]
    log = np.zeros((pivots, 2), dtype=np.int32)
    which, status = ctypes.c_int32(), ctypes.c_int32()
    cur, nxt = A, B
    done = 0
    sha = {}
    st = 0
    marks = [k for k in CHECKPOINTS if k < pivots] + [pivots]
    for k in marks:
        want = k - done
        got = L.smx_oracle_run(cur.ctypes.data_as(ctypes.c_void_p), nxt.ctypes.data_as(ctypes.c_void_p),
                               ld, n, m, m, want, log[done:].ctypes.data_as(ctypes.c_void_p),
                               ctypes.byref(which), ctypes.byref(status), threads)
        done += int(got)
        if which.value == 1:
            cur, nxt = nxt, cur
        st = status.value
        sha[str(done)] = table_sha256(cur, n, m)
        print(f"{kind}: {done} pivots, status {st}, {time.time() - t0:.0f} s", flush=True)
        if got < want:
            break
    log = log[:done]
    return {
        "kind": kind, "seed": SEED, "n": n, "m": m, "pivots": done, "status": st,
        "log": log.tolist(), "cycle": cycle_of(n, m, log.tolist()), "sha256": sha,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pivots", type=int, default=209)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--kinds", default="degenerate,degenerate_mixed")
    ap.add_argument("--out", default=os.path.join(HERE, "config5.json"))
    ap.add_argument("--shape", default=f"{N}x{M}", help="n x m (a smaller shape: a dry run)")
    a = ap.parse_args()
    c_oracle.build()
    recs = []
    for kind in a.kinds.split(","):
        n, m = (int(v) for v in a.shape.split("x"))
        recs.append(run_kind(kind, a.pivots, a.threads, n, m))
    with open(a.out, "w") as f:
        json.dump({"generator": "tests/golden/make_config5.py", "oracle": "oracle/simplex_oracle.c",
                   "hash": "sha256(rows[:n, :m+1] C-order fp64) || f-row[:m]",
                   "cases": recs}, f)
        f.write("\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
