"""VALU instructions per element-pivot of the block sweep, from the committed SQ counter passes.

SQ_INSTS_VALU counts wave64 instructions per dispatch; the sources sweep a 16384x16384 tableau
(R = C = 16384) with P pivots per launch, so lane-instructions per element-pivot =
SQ_INSTS_VALU * 64 / (R * C * P).  bench.py reads the result (profiles/valu_instr.json) to price
the sweep against the fp64 VALU issue rate beside the HBM roofline.

Two kinds of source:
  * summaries written by tools/sweep_pmc.py (rounds 2-3: `*_pmc_summary.json`, several SQ passes
    merged, so the fp64 share of the VALU stream is known);
  * raw rocprofv3 `--pmc` passes (`*_counter_collection.csv`, round 4 on): every dispatch of a
    `k_blk_sweep<P, ...>` kernel with the given P, its SQ_INSTS_VALU averaged over dispatches.
usage: python tools/valu_instr.py > profiles/valu_instr.json"""
import csv
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUMMARIES = ["profiles/r02d/sweep8_pmc_summary.json",
             "profiles/r03/sweep10_pmc_summary.json",
             "profiles/r03c/sweep12_pmc_summary.json"]
# (counter CSV, pivots per sweep of the dispatches to read, what the pass was)
PASSES = [("profiles/r05l/sq20/run_counter_collection.csv", 20,
           "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES, bench.py --steps 20 --warmup 5 (round 5): "
           "every k_blk_sweep<20, 5> dispatch")]
SIZE = 16384
_SWEEP = re.compile(r"k_blk_sweep<(\d+)[,>]")


def counter_per_dispatch(path, counter, pivots):
    """{dispatch id: value} of `counter` over the k_blk_sweep<pivots, ...> dispatches of a
    rocprofv3 counter-collection CSV (values of one dispatch summed, should a pass split them)."""
    out = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            m = _SWEEP.search(r["Kernel_Name"])
            if m is None or int(m.group(1)) != pivots or r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            out[d] = out.get(d, 0.0) + float(r["Counter_Value"])
    return out


def main():
    out = {}
    for rel in SUMMARIES:
        with open(os.path.join(REPO, rel)) as fh:
            d = json.load(fh)
        P = int(_SWEEP.search(d["kernels"][0]).group(1))
        c = d["counters"]
        valu = c["SQ_INSTS_VALU"]["mean_per_dispatch"]
        out[f"{SIZE}x{SIZE}/k_blk_sweep<{P}>"] = {
            "instr_per_element_pivot": valu * 64.0 / (SIZE * SIZE * P),
            "wave_instr_per_launch": valu,
            "f64_fma_mul_add_share": sum(c[k]["mean_per_dispatch"] for k in (
                "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")
                if k in c) / valu,
            "source": rel}
    for rel, P, what in PASSES:
        per = counter_per_dispatch(os.path.join(REPO, rel), "SQ_INSTS_VALU", P)
        if not per:
            raise SystemExit(f"{rel}: no k_blk_sweep<{P}> dispatch")
        valu = sum(per.values()) / len(per)
        out[f"{SIZE}x{SIZE}/k_blk_sweep<{P}>"] = {
            "instr_per_element_pivot": valu * 64.0 / (SIZE * SIZE * P),
            "wave_instr_per_launch": valu,
            "dispatches": sorted(per),
            "source": f"{rel} ({what})"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
