"""VALU instructions per element-pivot of the block sweep, from the committed SQ counter summaries.

SQ_INSTS_VALU counts wave64 instructions per dispatch; tools/sweep_pmc.py sweeps a 16384x16384
tableau (R = C = 16384) with P pivots per launch, so lane-instructions per element-pivot =
SQ_INSTS_VALU * 64 / (R * C * P).  bench.py reads the result (profiles/valu_instr.json) to price
the sweep against the fp64 VALU issue rate beside the HBM roofline.
usage: python tools/valu_instr.py > profiles/valu_instr.json"""
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["profiles/r02d/sweep8_pmc_summary.json",
           "profiles/r03/sweep10_pmc_summary.json",
           "profiles/r03c/sweep12_pmc_summary.json"]
SIZE = 16384


def main():
    out = {}
    for rel in SOURCES:
        with open(os.path.join(REPO, rel)) as fh:
            d = json.load(fh)
        P = int(re.search(r"k_blk_sweep<(\d+)", d["kernels"][0]).group(1))
        c = d["counters"]
        valu = c["SQ_INSTS_VALU"]["mean_per_dispatch"]
        out[f"{SIZE}x{SIZE}/k_blk_sweep<{P}>"] = {
            "instr_per_element_pivot": valu * 64.0 / (SIZE * SIZE * P),
            "wave_instr_per_launch": valu,
            "f64_fma_mul_add_share": sum(c[k]["mean_per_dispatch"] for k in (
                "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")
                if k in c) / valu,
            "source": rel}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
