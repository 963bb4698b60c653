"""GPU parity: the HIP engine (through the C ABI / torch custom ops) against the reference's golden
fixtures and the pinned CPU oracle.  Bit-exact: every table compared as int64 bit patterns
(SHA-256 of the bytes), every pivot (i, j) and outcome identical.
"""
from __future__ import annotations

import os
import numpy as np
import pytest

from golden_util import (check_txt_example, dec, dec_input, dec_table, dense_hash, load, same_table,
                         same_value, table_hash, trajectory_cap, trajectory_cases)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


def _engine():
    import simplex_mi355x
    return simplex_mi355x


# ----------------------------------------------------------------------------------------------
# 1. the reference's own example LPs: every Info field of get_solution()
@pytest.mark.parametrize("name", list(load("examples.json")))
def test_examples_get_solution(name):
    import simplex  # the drop-in module (simplex-method-solver_amd/simplex.py)
    case = load("examples.json")[name]
    cons, func = dec_input(case["input"])
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
    got = sm.get_solution()
    exp = case["solution"]
    ints = any(isinstance(x, int) for r in cons for x in r)
    assert len(got) == len(exp)
    for k, (g, e) in enumerate(zip(got, exp)):
        if e["kind"] == "error":
            assert isinstance(g, simplex.Error) and str(g) == e["message"]
            continue
        assert isinstance(g, simplex.Info)
        assert g.row == e["row"] and g.column == e["column"]
        assert g.i == e["i"] and g.j == e["j"]
        # integer inputs: the reference's int arithmetic may differ in the sign of a zero only
        assert same_table(g.table, dec_table(e["table"]), signed_zero=not ints), (name, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(getattr(g, key), dec(e[key]), signed_zero=not ints)


# ----------------------------------------------------------------------------------------------
# 2. every capped trajectory fixture through pick_element / recalculate_matrix
def _product_trajectory(cons, func, cap):
    import simplex
    sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
    steps = [{"hash": table_hash(sm.table), "x1": 0, "x2": 0, "optimum": 0}]
    outcome = None
    for _ in range(cap):
        try:
            ok, i, j, _e = sm.pick_element()
        except ValueError as exc:
            outcome = {"kind": "error", "message": str(exc)}
            break
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        if not ok:
            outcome = {"kind": "optimum"}
            break
        steps[-1]["i"], steps[-1]["j"] = i, j
        try:
            sm.recalculate_matrix()
            x1, x2 = sm.find_optimum()
            f = sm.f(x1, x2)
        except IndexError:
            outcome = {"kind": "exception", "type": "IndexError"}
            break
        steps.append({"hash": table_hash(sm.table), "x1": x1, "x2": x2, "optimum": f})
    if outcome is None:
        outcome = {"kind": "cap"}
    return {"steps": steps, "outcome": outcome, "row": sm.row, "column": sm.column}


CASES = list(trajectory_cases())


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fixture_trajectories(case):
    label, cons, func, rec = case
    got = _product_trajectory(cons, func, trajectory_cap(rec))
    exp = rec["steps"]
    assert len(got["steps"]) == len(exp), (label, len(got["steps"]), len(exp))
    for k, (g, e) in enumerate(zip(got["steps"], exp)):
        assert g["hash"] == e["hash"], (label, "table differs at step", k)
        assert (g.get("i"), g.get("j")) == (e.get("i"), e.get("j")), (label, k)
        for key in ("x1", "x2", "optimum"):
            assert same_value(g[key], dec(e[key])), (label, k, key)
    assert got["outcome"] == rec["outcome"], label
    assert got["row"] == rec["row"] and got["column"] == rec["column"], label


def test_large256_trajectory():
    rec = load("large256.json")
    cons, func = dec_input(rec["input"])
    got = _product_trajectory(cons, func, trajectory_cap(rec))
    assert [s["hash"] for s in got["steps"]] == [s["hash"] for s in rec["steps"]]
    assert [(s.get("i"), s.get("j")) for s in got["steps"]] == \
        [(s.get("i"), s.get("j")) for s in rec["steps"]]


# ----------------------------------------------------------------------------------------------
# 3. chained fast path (hipGraph) vs the C oracle at sizes the oracle finishes in seconds
def _oracle_run(T, n, m, flen, k):
    from oracle import c_oracle
    return c_oracle.run(T, n, m, flen, k, threads=8)


@pytest.mark.parametrize("kind,n,m,k,chunk", [
    ("uniform", 1023, 1023, 400, 64),
    ("uniform", 2047, 2047, 120, 40),
    ("uniform", 999, 3000, 150, 50),      # wide, odd C = 3001
    ("uniform", 3001, 998, 150, 50),      # tall, odd C = 999
    ("mixed", 1023, 1023, 400, 100),      # phase 1 first
    ("degenerate", 511, 511, 300, 100),   # degenerate, zero ratios
    ("degenerate_mixed", 600, 300, 300, 100),
    ("uniform", 65535, 255, 60, 30),      # very tall: 65536 rows x 256 columns
    ("mixed", 255, 65535, 60, 30),        # very wide: 512 chunks per row, phase 1
])
def test_fast_path_vs_oracle(kind, n, m, k, chunk):
    from simplex_mi355x import lp
    import simplex
    T = lp.dense_tableau(kind, 11, n, m)
    cons, func = T[:n].tolist(), T[n, :m].tolist()
    sm = simplex.SimplexMethod(cons, func)
    sm.solve(record_history=False, max_pivots=k, chunk=chunk)
    Tref, st, done, log = _oracle_run(T, n, m, m, k)
    assert sm.pivots == done
    assert sm.pivot_log == [tuple(map(int, x)) for x in log]
    got = sm._dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


def test_graph_and_eager_chains_agree():
    from simplex_mi355x import lp
    import simplex
    T = lp.dense_tableau("uniform", 3, 700, 900)
    a = simplex.SimplexMethod(T[:700].tolist(), T[700, :900].tolist())
    b = simplex.SimplexMethod(T[:700].tolist(), T[700, :900].tolist())
    a.solve(record_history=False, max_pivots=96, chunk=32, graph=True)
    b.solve(record_history=False, max_pivots=96, chunk=32, graph=False)
    assert a.pivot_log == b.pivot_log
    assert np.array_equal(a._dev.download().view(np.int64), b._dev.download().view(np.int64))


def test_fast_path_terminal_outcomes_match_get_solution():
    """solve(record_history=False) ends with the same Error / optimum as get_solution()."""
    import simplex
    for rec in load("random.json"):
        if rec["outcome"]["kind"] == "cap":
            continue
        cons, func = dec_input(rec["input"])
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
        out = sm.solve(record_history=False, chunk=16)
        exp = rec["outcome"]
        if exp["kind"] == "error":
            assert isinstance(out[-1], simplex.Error) and str(out[-1]) == exp["message"]
        else:
            assert sm.status == "optimum"
        assert table_hash(sm.table) == rec["steps"][-1]["hash"]
        assert sm.row == rec["row"] and sm.column == rec["column"]


# ----------------------------------------------------------------------------------------------
# 4. the update kernel alone (forced pivots, any column incl. the "-b" column) vs the oracle
@pytest.mark.parametrize("n,m", [(1, 1), (2, 1), (5, 2), (63, 64), (64, 63), (200, 129), (1025, 777)])
def test_forced_update_vs_oracle(n, m):
    from oracle import c_oracle
    from simplex_mi355x.device import DeviceTableau
    rng = np.random.default_rng(n * 1000 + m)
    T = rng.standard_normal((n + 1, m + 1))
    T[rng.random(T.shape) < 0.05] = 0.0
    T[rng.random(T.shape) < 0.02] = -0.0
    dev = DeviceTableau(T, n, m, m + 1)
    for (r, c) in [(0, 0), (n - 1, m), (n // 2, m // 2), (0, m)]:
        if T[r, c] == 0:
            T[r, c] = 1.5
            dev.upload(T)
        ref = c_oracle.pivot(T, r, c)
        dev.forced(r, c)
        got = dev.download()
        assert np.array_equal(got.view(np.int64), ref.view(np.int64)), (r, c)
        T = ref
        dev.upload(T)


# ----------------------------------------------------------------------------------------------
# 5. full BASELINE sizes: a short bit-exact prefix against the multithreaded C oracle
@pytest.mark.parametrize("n,m,k", [(8191, 8191, 4), (16383, 16383, 2)])
def test_full_size_prefix_vs_oracle(n, m, k):
    from simplex_mi355x import lp
    from simplex_mi355x.device import DeviceTableau
    from oracle import c_oracle
    T = lp.dense_tableau("uniform", 0, n, m)
    dev = DeviceTableau(T, n, m, m)
    dev.run(k, graph=False)
    ctl = dev.sync_state()
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=16)
    assert int(ctl["npivots"]) == done == k
    got_log = dev.read_log(0, k)
    assert np.array_equal(got_log, log)
    got = dev.download()
    assert np.array_equal(got[:n].view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(got[n, :m].view(np.int64), Tref[n, :m].view(np.int64))


# ----------------------------------------------------------------------------------------------
# 6. opt-in cycle detection on a cycling fixture (the reference itself loops forever here)
def test_solve_detects_basis_cycle():
    import simplex
    rec = load("degenerate.json")[0]
    cons, func = dec_input(rec["input"])
    for history in (True, False):
        sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
        sm.solve(record_history=history, max_pivots=500, chunk=4, detect_cycles=True)
        assert sm.status == "cycle" and sm.cycle == (3, 2)
        exp = [(s["i"], s["j"]) for s in rec["steps"][:len(sm.pivot_log)]]
        assert sm.pivot_log == exp


# ----------------------------------------------------------------------------------------------
# 7. bench.py itself (single path and the RCCL sharded path at world size 1)
def _bench_json(cmd):
    import json
    import subprocess
    import sys
    out = subprocess.run([sys.executable] + cmd, capture_output=True, text=True, timeout=600,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_bench_single_and_sharded_paths():
    for extra in ([], ["--sharded"]):
        rec = _bench_json(["bench.py", "--size", "2048", "--steps", "20", "--warmup", "2",
                           "--no-cpu-baseline"] + extra)
        assert rec["trajectory_valid"] and rec["n_gpus"] == 1 and rec["value"] > 0
        assert rec["roofline"]["bound"] == "hbm" and 0 < rec["roofline"]["frac"] < 1


# ----------------------------------------------------------------------------------------------
# 8. device-resident history: lazy get_solution == eager get_solution, tables bit-identical
def _same_infos(a, b):
    import simplex
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(y, simplex.Error):
            assert isinstance(x, simplex.Error) and str(x) == str(y)
            continue
        assert (x.row, x.column, x.i, x.j) == (y.row, y.column, y.i, y.j)
        assert same_value(x.x1, y.x1) and same_value(x.x2, y.x2)
        assert same_value(x.optimum, y.optimum)
        assert same_table(x.table, y.table)


@pytest.mark.parametrize("k", range(0, 40, 3))
def test_lazy_history_matches_eager_on_fixtures(k):
    import simplex
    rec = load("random.json")[k]
    if rec["outcome"]["kind"] == "cap":
        pytest.skip("cycling fixture")
    cons, func = dec_input(rec["input"])
    eager = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(lazy=False)
    lazy = simplex.SimplexMethod([list(r) for r in cons], list(func)).get_solution(lazy=True,
                                                                                 chunk=7)
    _same_infos(lazy, eager)
    assert [table_hash(i.table) for i in lazy if isinstance(i, simplex.Info)] == \
        [s["hash"] for s in rec["steps"]]


def test_lazy_history_large_tableau_vs_oracle():
    """1200 x 1100 tableau, 90 pivots: automatic lazy mode; tables of chosen steps replayed on the
    device equal the C oracle's tables at those steps bit for bit; x1/x2 per step as well."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import lp
    n, m, k = 1199, 1099, 90
    T = lp.dense_tableau("uniform", 4, n, m)
    sm = simplex.SimplexMethod(T[:n].tolist(), T[n, :m].tolist())
    out = sm.get_solution(max_pivots=k, chunk=32)
    assert sm.status == "cap" and len(out) == k + 1
    for step in (0, 1, 31, 32, 33, 64, 90):
        Tref, st, done, log = c_oracle.run(T, n, m, m, step, threads=8)
        got = np.array(out[step].table[:n])
        assert np.array_equal(got.view(np.int64), Tref[:n].view(np.int64)), step
        assert [tuple(map(int, x)) for x in log] == sm.pivot_log[:step]
    # x1 / x2 per step: the reference's find_optimum on the materialised table
    for step in (5, 47, 90):
        info = out[step]
        tab = info.table
        for name, val in (("x1", info.x1), ("x2", info.x2)):
            exp = tab[info.column.index(name)][-1] if name in info.column else 0
            assert same_value(val, exp)


# ----------------------------------------------------------------------------------------------
# 9. problem files: .txt (the reference UI's format, main.py:386-393 / :402-495) and .smx streamed
#    into HBM, pinned to the reference's own answers (examples.json) and to the C oracle
@pytest.mark.parametrize("name", list(load("examples.json")))
def test_from_file_txt_vs_reference_examples(tmp_path, name):
    """.txt -> SimplexMethod.from_file(...).get_solution() on the GPU equals the reference's own
    get_solution() of that LP (examples.json, generated from /root/reference/src/simplex.py):
    (i, j), labels, tables, x1 / x2 / optimum and the trailing Error of every step.  The .txt
    reader itself restates main.py:415-481 (PyQt5 is absent, so main.py cannot be imported:
    the reader's parity is unpinned; the solver behind it is pinned here)."""
    import simplex
    check_txt_example(simplex.SimplexMethod, tmp_path, name)


def test_from_file_smx_vs_oracle(tmp_path):
    """.smx streamed into HBM, 60 chained pivots: pivot log and the whole final table bit-exact
    against the C oracle (not against a second HIP run)."""
    import simplex
    from oracle import c_oracle
    from simplex_mi355x import lp, problem_io
    n = m = 1500
    k = 60
    T = lp.dense_tableau("uniform", 6, n, m)
    q = str(tmp_path / "big.smx")
    problem_io.save_smx(q, T, n, m, m)
    a = simplex.SimplexMethod.from_file(q)
    assert a.backend == "hip"
    ra = a.solve(record_history=False, max_pivots=k, chunk=30)
    Tref, st, done, log = c_oracle.run(T, n, m, m, k, threads=8)
    assert done == k and a.pivots == k
    assert a.pivot_log == [tuple(map(int, x)) for x in log]
    got = np.array(ra[-1].table[:n])
    assert np.array_equal(got.view(np.int64), Tref[:n].view(np.int64))
    assert np.array_equal(np.array(ra[-1].table[n]).view(np.int64), Tref[n, :m].view(np.int64))
    assert np.array_equal(np.array(ra[0].table[:n]).view(np.int64), T[:n].view(np.int64))


# ----------------------------------------------------------------------------------------------
# 10. the fused chain (look-ahead selection inside the update kernel) == the select+update chain
def test_fused_chain_matches_unfused_on_every_fixture():
    import simplex
    from simplex_mi355x import _lib
    L = _lib.load()
    n_checked = 0
    try:
        for label, cons, func, rec in CASES:
            if len(func) not in (len(cons[0]) - 1, len(cons[0])) or len(func) < 2:
                continue
            runs = []
            for fused in (1, 0):
                L.smx_tune_fused(fused)
                sm = simplex.SimplexMethod([list(r) for r in cons], list(func))
                out = sm.solve(record_history=False, max_pivots=trajectory_cap(rec), chunk=5)
                runs.append((sm.pivot_log, sm.status, table_hash(out[-2 if sm.status == "error"
                                                                    else -1].table)))
            assert runs[0] == runs[1], label
            exp = [(s["i"], s["j"]) for s in rec["steps"][:-1]]
            assert runs[0][0] == exp[:len(runs[0][0])], label
            n_checked += 1
    finally:
        L.smx_tune_fused(1)
    assert n_checked > 250


# ----------------------------------------------------------------------------------------------
# 11. the maintainer-side ctypes stub printed in INTEGRATION.md runs the engine correctly
def test_integration_stub_pivot_loop_vs_oracle():
    import torch
    from oracle import c_oracle
    from simplex_mi355x import lp
    from test_abi import _integration_stub
    ns = _integration_stub()
    n, m, k = 300, 200, 60
    T = lp.dense_tableau("uniform", 3, n, m)
    buf, c, log = ns["pivot_loop"](T[:n].tolist(), T[n, :m].tolist(), k)
    torch.cuda.synchronize()
    Tref, st, done, lref = c_oracle.run(T, n, m, m, k)
    npiv = int(c[5])
    assert npiv == done
    assert np.array_equal(log.cpu().numpy().reshape(-1, 2)[:done], lref)
    got = buf[npiv & 1].cpu().numpy()
    assert np.array_equal(got[:n, :m + 1].view(np.int64), Tref[:n, :m + 1].view(np.int64))
