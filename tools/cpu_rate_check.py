"""Pins the cpu_baseline's pure-Python leg (oracle/restated.py) against the reference's own cost.

bench.py reports a pure-Python CPU rate measured on the GPU box with the restatement, because the
reference cannot travel there.  SURVEY 8d(i) asks that the restatement's ns/element be checked
against the reference's before it stands in.  This script runs in the build container only (where
/root/reference exists): it imports the reference's simplex.py, and times pick_element +
recalculate_matrix (simplex.py:70-177, deepcopy included) and restated.pick + restated.pivot on
the same seeded uniform LPs, alternating the two so clock drift hits both alike.  It writes
profiles/r02/cpu_rate_check.json; tests/test_cpu_rate.py checks the ratio.
usage: python tools/cpu_rate_check.py [--sizes 256,512,1024] [--reps 3]"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))


def load_reference():
    sys.path.insert(0, REF_SRC)
    import simplex  # noqa: E402  (the reference module, build container only)
    return simplex


def lists(T, n, m):
    return [list(map(float, row)) for row in T[:n]] + [list(map(float, T[n, :m]))]


def time_ref(simplex, T, n, m):
    sm = simplex.SimplexMethod(lists(T, n, m)[:n], lists(T, n, m)[n])
    t0 = time.perf_counter()
    sm.recalculate_matrix()   # pick_element + deepcopy + the four steps
    return time.perf_counter() - t0


def time_restated(restated, T, n, m):
    tab = lists(T, n, m)
    t0 = time.perf_counter()
    st = restated.pick(tab, n, m, 1 + max(n, m))
    assert st[0] == "pivot", st
    restated.pivot(tab, st[1], st[2])
    return time.perf_counter() - t0


def measure(sizes, reps):
    from oracle import restated
    from simplex_mi355x import lp
    simplex = load_reference()
    rows = []
    for N in sizes:
        n = m = N - 1
        T = lp.dense_tableau("uniform", 0, n, m)
        ref, res = [], []
        for _ in range(reps):
            ref.append(time_ref(simplex, T, n, m))
            res.append(time_restated(restated, T, n, m))
        el = N * N
        r_ns = min(ref) / el * 1e9
        s_ns = min(res) / el * 1e9
        rows.append({"size": N, "reps": reps, "reference_ns_per_element": r_ns,
                     "restated_ns_per_element": s_ns, "ratio_restated_over_reference": s_ns / r_ns})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,512,1024")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02", "cpu_rate_check.json"))
    a = ap.parse_args()
    if not os.path.isdir(REF_SRC):
        print("reference not present; the committed check stands")
        return
    rows = measure([int(s) for s in a.sizes.split(",")], a.reps)
    rec = {"python": platform.python_version(), "machine": platform.machine(),
           "note": "best of reps, one pivot (pick + pivot with deepcopy) from step 0 of the "
                   "seeded uniform LP, same host, reference and restatement interleaved",
           "rows": rows}
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
