"""Helpers to read the committed golden fixtures (tests/golden/*.json, made by make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import math
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def dec(v):
    """float.hex strings -> float, ints stay ints, None stays None."""
    if isinstance(v, str):
        return float.fromhex(v)
    return v


def dec_table(t):
    return [[dec(x) for x in row] for row in t]


def dec_input(inp):
    return dec_table(inp["constraints"]), [dec(x) for x in inp["function"]]


CANON_NAN = float("nan")


def table_hash(table) -> str:
    """SHA-256 of the fp64 bytes, NaNs canonicalised (same rule as make_golden.table_hash)."""
    h = hashlib.sha256()
    for row in table:
        vals = [float(x) for x in row]
        vals = [v if v == v else CANON_NAN for v in vals]
        h.update(struct.pack("<%dd" % len(vals), *vals))
    return h.hexdigest()


def canon(T: np.ndarray) -> np.ndarray:
    """Copy with every NaN replaced by the canonical quiet NaN 0x7ff8000000000000."""
    T = np.array(T, dtype="<f8", copy=True)
    T[np.isnan(T)] = np.nan
    return T


def dense_hash(T: np.ndarray, n: int, flen: int) -> str:
    """Hash of a dense tableau in the reference's ragged layout (f-row trimmed to flen)."""
    h = hashlib.sha256()
    T = canon(T)
    h.update(T[:n].tobytes())
    h.update(T[n, :flen].tobytes())
    return h.hexdigest()


def table_sha256(T: np.ndarray, n: int, m: int) -> str:
    """SHA-256 of a dense tableau as the full-size fixtures hash it (tests/golden/make_config5.py,
    make_bench16k.py): rows 0..n-1 with m + 1 values each in C order, then the f-row's first m."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(T[:n, :m + 1]))
    h.update(np.ascontiguousarray(T[n, :m]))
    return h.hexdigest()


def same_value(a, b, signed_zero=True) -> bool:
    """Bitwise float equality (NaN == NaN; -0.0 != 0.0 unless signed_zero=False)."""
    if isinstance(a, int) and isinstance(b, int):
        return a == b
    a, b = float(a), float(b)
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    if a == 0 and b == 0 and signed_zero:
        return math.copysign(1, a) == math.copysign(1, b)
    return a == b


def same_table(t1, t2, signed_zero=True) -> bool:
    if len(t1) != len(t2):
        return False
    for r1, r2 in zip(t1, t2):
        if len(r1) != len(r2):
            return False
        if not all(same_value(a, b, signed_zero) for a, b in zip(r1, r2)):
            return False
    return True


def all_int_input(cons, func) -> bool:
    return all(isinstance(x, int) for r in cons for x in r) or all(isinstance(x, int) for x in func)


def trajectory_cases():
    """Every fixture that has a capped trajectory: yields (label, constraints, function, rec)."""
    for k, rec in enumerate(load("random.json")):
        yield f"random{k}_{rec['n']}x{rec['m']}", *dec_input(rec["input"]), rec
    for k, rec in enumerate(load("ties.json")):
        yield f"ties{k}", *dec_input(rec["input"]), rec
    for k, rec in enumerate(load("degenerate.json")):
        yield f"deg{k}_{rec['n']}x{rec['m']}", *dec_input(rec["input"]), rec
    for name, rec in load("edge.json").items():
        yield f"edge_{name}", *dec_input(rec["input"]), rec["solution"]["trajectory"]


def trajectory_cap(rec) -> int:
    """Pivots to run so a replay ends exactly where the fixture ended (terminal pick included)."""
    pivots = len(rec["steps"]) - 1
    return pivots if rec["outcome"]["kind"] == "cap" else pivots + 1


def check_txt_example(sm_cls, tmp_path, name, device=None):
    """Write examples.json[name] as the reference UI's .txt, load it through
    ``sm_cls.from_file`` and compare every get_solution() step with the reference's answer."""
    from simplex_mi355x import problem_io
    case = load("examples.json")[name]
    cons, func = dec_input(case["input"])
    p = str(tmp_path / f"{name}.txt")
    # the UI's gradient row carries a third entry (main.py:312 drops it: c = grad[:-1])
    problem_io.save_txt(p, cons, list(func) + [0.0], 5)
    got = sm_cls.from_file(p, device=device).get_solution()
    exp = case["solution"]
    # the file holds floats: the reference ran integer inputs as ints, which can differ from the
    # float run only in the sign of a zero (see test_examples_get_solution)
    ints = any(isinstance(x, int) for r in cons for x in r)
    assert len(got) == len(exp), name
    for k, (g, e) in enumerate(zip(got, exp)):
        if e["kind"] == "error":
            assert type(g).__name__ == "Error" and str(g) == e["message"], (name, k)
            continue
        assert g.row == e["row"] and g.column == e["column"], (name, k)
        assert (g.i, g.j) == (e["i"], e["j"]), (name, k)
        assert same_table(g.table, dec_table(e["table"]), signed_zero=not ints), (name, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(getattr(g, key), dec(e[key]), signed_zero=not ints), (name, k, key)
