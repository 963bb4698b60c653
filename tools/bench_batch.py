"""Batched small-LP throughput: UI-shaped LPs (m = 2, n = 3..20), one launch.
Reports LPs/s and pivots/s for the device (kernel events) and end to end (host packing + copies),
next to the pure-Python restatement of the reference (oracle/restated.py) on a sample."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "simplex-method-solver_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def make(B, seed=0):
    rng = np.random.default_rng(seed)
    probs = []
    for _ in range(B):
        n = int(rng.integers(3, 21))
        A = rng.uniform(-50, 50, size=(n, 2))
        b = rng.uniform(-100, 400, size=n)
        c = rng.uniform(-3, 3, size=2)
        probs.append(([list(map(float, A[i])) + [float(b[i])] for i in range(n)],
                      list(map(float, c))))
    return probs


def main():
    from simplex_mi355x import _lib
    from simplex_mi355x.batch import pack, solve_batch, solve_batch_arrays
    from oracle import restated
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    probs = make(B)
    tabs, dims = pack(probs)
    solve_batch_arrays(tabs[:1000], dims[:1000], 64)            # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = solve_batch_arrays(tabs, dims, 64)                       # H2D + kernel + D2H
    torch.cuda.synchronize()
    wall_arrays = time.perf_counter() - t0
    t0 = time.perf_counter()
    res, st = solve_batch(probs[:20000], max_pivots=64, history=True)   # Info-object API
    wall_infos = (time.perf_counter() - t0) / 20000 * B
    # device-only: the kernel on resident buffers, timed with HIP events
    L = _lib.load()
    d = lambda a: torch.from_numpy(a).cuda()
    dt, dd = d(tabs), d(dims)
    Rmax, ldb = tabs.shape[1], tabs.shape[2]
    o = torch.empty_like(dt)
    rc = torch.zeros((B, 64, 2), dtype=torch.int32, device="cuda")
    xv = torch.zeros((B, 64, 2), dtype=torch.float64, device="cuda")
    s_ = torch.zeros(B, dtype=torch.int32, device="cuda")
    np_ = torch.zeros(B, dtype=torch.int32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream().cuda_stream
    args = (dt.data_ptr(), dd.data_ptr(), B, Rmax, ldb, 64, o.data_ptr(), rc.data_ptr(),
            xv.data_ptr(), None, s_.data_ptr(), np_.data_ptr(), stream)
    L.smx_batch_solve(*args)
    e0.record()
    for _ in range(10):
        L.smx_batch_solve(*args)
    e1.record()
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / 10
    pivots = int(np_.sum().item())
    sample = probs[:3000]
    t0 = time.perf_counter()
    for c, f in sample:
        restated.Solver([list(r) for r in c], list(f)).get_solution(max_pivots=64)
    cpu = time.perf_counter() - t0
    codes = {0: "cap", 1: "optimum", 2: "incorrect system", 3: "does not converge"}
    print(json.dumps({"what": "batch_small_lps", "lps": B, "pivots": pivots,
                      "kernel_ms": kms, "lps_per_s_device": B / (kms * 1e-3),
                      "pivots_per_s_device": pivots / (kms * 1e-3),
                      "lps_per_s_arrays_end_to_end": B / wall_arrays,
                      "lps_per_s_info_api": B / wall_infos,
                      "cpu_reference_restated_lps_per_s": len(sample) / cpu, "cpu_cores": 1,
                      "statuses": {codes.get(int(k), str(k)): int((out["status"] == k).sum())
                                   for k in np.unique(out["status"])}}), flush=True)


if __name__ == "__main__":
    main()
