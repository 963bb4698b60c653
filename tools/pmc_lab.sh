#!/bin/bash
# SQ counters of the lab sweep (tools/sweep_lab, variant 1) beside the production flag-form kernel
# (tools/sweep_prod_probe), each pass its own rocprofv3 run under a time limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_lab
export TMPDIR=/tmp
export STEPS_LOGDIR=$OUT
mkdir -p "$OUT"
cd /tmp || exit 1
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
PB="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_LDS GRBM_GUI_ACTIVE"
"$ROOT/tools/gpu_steps.sh" \
  "labA|60|timeout -s KILL 50 rocprofv3 --pmc $PA -d $OUT/labA -o run --output-format csv -- $ROOT/tools/sweep_lab 16384 10 3 7 1 > $OUT/labA.out" \
  "labB|60|timeout -s KILL 50 rocprofv3 --pmc $PB -d $OUT/labB -o run --output-format csv -- $ROOT/tools/sweep_lab 16384 10 3 7 1 > $OUT/labB.out" \
  "prA|90|timeout -s KILL 80 rocprofv3 --pmc $PA -d $OUT/prA -o run --output-format csv -- $ROOT/tools/sweep_prod_probe 16384 3 7 > $OUT/prA.out" \
  "prB|90|timeout -s KILL 80 rocprofv3 --pmc $PB -d $OUT/prB -o run --output-format csv -- $ROOT/tools/sweep_prod_probe 16384 3 7 > $OUT/prB.out"
