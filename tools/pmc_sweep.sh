#!/bin/bash
# Counter evidence for the block sweep (run on the GPU box from the repo root):
#   kernel-trace stats + separate rocprofv3 --pmc passes (SQ instruction / cycle counters, HBM
#   bytes) over tools/sweep_pmc.py.  Counters not listed by `rocprofv3 -L` on this box are dropped
#   from their pass.  Each rocprofv3 call is its own step under a time limit (tools/gpu_steps.sh).
# usage: tools/pmc_sweep.sh TAG [sweep_pmc.py args...]
set -o pipefail
TAG=${1:-r02}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
export TMPDIR=/tmp
export STEPS_LOGDIR=$OUT
mkdir -p "$OUT"
D="python3 $ROOT/tools/sweep_pmc.py $*"
cd /tmp || exit 1
timeout -k 10 90 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "rocprofv3 -L failed" >> "$OUT/counters.txt"
have() {   # the subset of the given counters this box lists
  local out=""
  for c in "$@"; do grep -qw "$c" "$OUT/counters.txt" && out="$out $c"; done
  echo $out
}
PA=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT)
PB=$(have SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_LDS GRBM_GUI_ACTIVE)
PC=$(have SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MISC)
echo "passes: A=[$PA] B=[$PB] C=[$PC]" | tee "$OUT/passes.txt"
STEPS=("stats|240|rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $D > $OUT/stats_driver.log 2>&1"
       "fetch|180|rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $D > $OUT/fetch_driver.log 2>&1"
       "write|180|rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $D > $OUT/write_driver.log 2>&1")
[ -n "$PA" ] && STEPS+=("pa|180|rocprofv3 --pmc $PA -d $OUT/pa -o run --output-format csv -- $D > $OUT/pa_driver.log 2>&1")
[ -n "$PB" ] && STEPS+=("pb|180|rocprofv3 --pmc $PB -d $OUT/pb -o run --output-format csv -- $D > $OUT/pb_driver.log 2>&1")
[ -n "$PC" ] && STEPS+=("pc|180|rocprofv3 --pmc $PC -d $OUT/pc -o run --output-format csv -- $D > $OUT/pc_driver.log 2>&1")
"$ROOT/tools/gpu_steps.sh" "${STEPS[@]}"
