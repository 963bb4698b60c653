"""GPU sweep of the update kernel: variants x resident blocks/CU x row padding (forced pivots,
HIP events on the solver stream), plus a torch copy_ reference for the achievable HBM rate.
usage: python tools/tune_update.py [--size 16384] [--iters 20] > gpurun_out/tune.jsonl"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simplex-method-solver_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from simplex_mi355x import _lib  # noqa: E402
from simplex_mi355x.device import DeviceTableau  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pads", default="0,16,64")
    ap.add_argument("--bpcs", default="0,2,3,4,5,6,7,8")
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    L = _lib.load()
    nv = ctypes.c_int32()
    L.smx_tune_get(None, None, ctypes.byref(nv), None, None, None)
    variants = [int(v) for v in args.variants.split(",")] if args.variants else list(range(nv.value))
    n = m = args.size - 1
    R = C = args.size
    bytes_pp = 16.0 * R * C
    rng = np.random.default_rng(0)
    T = rng.uniform(-1, 1, size=(R, C))
    # copy reference: read + write the same byte count as one pivot
    a = torch.empty(R * C, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    a.uniform_()
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"what": "torch_copy", "bytes": bytes_pp, "ms": ms,
                      "gbs": bytes_pp / ms / 1e6}), flush=True)
    del a, b
    torch.cuda.empty_cache()
    for pad in [int(p) for p in args.pads.split(",")]:
        dev = DeviceTableau(T, n, m, m, ld_extra=pad)
        for v in variants:
            for bpc in [int(x) for x in args.bpcs.split(",")]:
                L.smx_tune_set(v, bpc)
                tr, vec, nt = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
                L.smx_tune_get(None, None, None, ctypes.byref(tr), ctypes.byref(vec), ctypes.byref(nt))
                s = dev.stream
                with torch.cuda.stream(s):
                    for _ in range(3):
                        dev.forced(1, 2)
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev0.record(s)
                    for _ in range(args.iters):
                        dev.forced(1, 2)
                    ev1.record(s)
                s.synchronize()
                ms = ev0.elapsed_time(ev1) / args.iters
                print(json.dumps({"what": "update_forced", "pad": pad, "ld": dev.ld, "variant": v,
                                  "u": tr.value, "vec": vec.value, "nt": nt.value, "bpc": bpc,
                                  "ms": ms, "gbs": bytes_pp / ms / 1e6}), flush=True)
        dev.close()
        del dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
