"""Small-tableau latency sweep (BASELINE config 2, 1024^2): fused vs select+update chains, blocks
per CU and update variant, each as a captured 200-pivot hipGraph; plus the launch floor of the
box (200 trivial kernels replayed from one torch CUDA graph).
usage: python tools/sweep_small.py [sizes] > out.jsonl"""
import itertools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))
import torch  # noqa: E402
from simplex_mi355x import _lib, lp  # noqa: E402
from simplex_mi355x.device import DeviceTableau  # noqa: E402


def launch_floor(k=200):
    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(k):
                x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (5 * k) * 1e6


def one(T, n, m, k=200, reps=3):
    dev = DeviceTableau(T, n, m, m)
    dev.run(k, graph=True)               # capture + warm
    dev.sync_state()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dev.run(k, graph=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (reps * k)
    st = dev.sync_state()
    ok = int(st["npivots"]) == k * (reps + 1) and not st["term"]
    dev.close()
    return dt * 1e6, ok


def main():
    L = _lib.load()
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1024,2048,4096").split(",")]
    print(json.dumps({"launch_floor_us": launch_floor()}), flush=True)
    for S in sizes:
        n = m = S - 1
        T = lp.dense_tableau("uniform", 0, n, m)
        for fused, bpc, var in itertools.product((1, 0), (3, 4, 5), (0, 1, 9)):
            L.smx_tune_fused(fused)
            L.smx_tune_set(var, bpc)
            us, ok = one(T, n, m)
            print(json.dumps({"size": S, "fused": fused, "bpc": bpc, "variant": var,
                              "us_per_pivot": round(us, 2), "valid": ok}), flush=True)
        L.smx_tune_fused(1)
        L.smx_tune_set(-2, 0)


if __name__ == "__main__":
    main()
