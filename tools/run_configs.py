"""BASELINE configs 2 and 3 with SURVEY 8d's protocol, on one MI355X.
  config 2: 1024x1024, seeds 0..4, K = 1000 pivots after 10 warm-up (the single-kernel-per-pivot
            fused chain, one hipGraph replay), plus a forced-pivot microbench (fixed r, c: the
            update alone, rule cost excluded).
  config 3: 8192x8192, seeds 0..2, K = 200.
Each line: pivots/s, device us per pivot (HIP events around the replay / K), equiv_one_pass_gbs =
16 R C / that (not HBM traffic once a sweep carries several pivots: block pivots, resident loop),
and whether the K pivots ran without reaching a terminal outcome.
usage: python tools/run_configs.py [2,3] > out.jsonl"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from bench import physical_check  # noqa: E402
from simplex_mi355x import lp  # noqa: E402
from simplex_mi355x.device import DeviceTableau  # noqa: E402

CONFIGS = {2: (1024, (0, 1, 2, 3, 4), 1000, 10), 3: (8192, (0, 1, 2), 200, 10)}


def chain(size, seed, k, warm):
    n = m = size - 1
    dev = DeviceTableau(lp.dense_tableau("uniform", seed, n, m), n, m, m,
                        log_cap=max(1 << 16, k + warm))
    dev.run(warm, graph=True)
    dev.sync_state()
    dev.prepare(k)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(dev.stream)
    dev.run(k, graph=True)
    e1.record(dev.stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    st = dev.sync_state()
    done = int(st["npivots"]) - warm
    dev_us = e0.elapsed_time(e1) * 1e3 / max(done, 1)
    rec = {"size": size, "seed": seed, "K": k, "pivots": done, "terminal": bool(st["term"]),
           "pivots_per_s": done / wall, "device_us_per_pivot": dev_us,
           "equiv_one_pass_gbs": 16.0 * size * size / (dev_us * 1e-6) / 1e9}
    dev.close()
    return rec


def forced(size, iters=200):
    """The update alone at a fixed (r, c), replayed from one torch CUDA graph (no launch cost).
    The replay goes to the solver stream the graph was captured on and the events bracket that
    stream (round 3 replayed on torch's current stream while the events sat on the solver stream,
    so they timed nothing: 0.26 us for a 1.07 GB pivot).  physical_check refuses such a line."""
    n = m = size - 1
    dev = DeviceTableau(lp.dense_tableau("uniform", 0, n, m), n, m, m)
    s = dev.stream
    for _ in range(4):
        dev.forced(1, 2)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            dev.forced(1, 2)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        g.replay()
        torch.cuda.synchronize()
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    del g
    dev.close()
    b = 16.0 * size * size
    gbs = physical_check(f"forced update {size}^2", b, us * 1e-6, b)
    return {"size": size, "forced_update_us": us, "gbs": gbs,
            "note": "fixed (r, c) = (1, 2), graph replay on the solver stream, rule cost excluded"}


def main():
    which = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,3").split(",")]
    for cfg in which:
        size, seeds, k, warm = CONFIGS[cfg]
        for seed in seeds:
            print(json.dumps({"config": cfg, **chain(size, seed, k, warm)}), flush=True)
        print(json.dumps({"config": cfg, **forced(size)}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
