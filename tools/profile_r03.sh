#!/bin/bash
# Round-3 rocprofv3 evidence (run on the GPU box from the repo root): kernel-trace stats of the
# driver's bench line at 16384^2 (--steps 20: two blocks of 10) and of --steps 200, two separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) over the --steps 20 line (the roofline's traffic:
# tools/pmc_traffic.py), then the SQ counter passes of k_blk_sweep<10> (tools/pmc_sweep.sh).
# Every rocprofv3 call is its own step under a time limit.
set -o pipefail
TAG=${1:-r03a}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
export TMPDIR=/tmp
export STEPS_LOGDIR=$OUT
mkdir -p "$OUT"
B="python3 $ROOT/bench.py --no-cpu-baseline"
cd /tmp || exit 1
"$ROOT/tools/gpu_steps.sh" \
  "s20|300|rocprofv3 --kernel-trace --stats -d $OUT/s20 -o run --output-format csv -- $B --steps 20 --warmup 5 > $OUT/bench20.log 2>&1" \
  "s200|300|rocprofv3 --kernel-trace --stats -d $OUT/s200 -o run --output-format csv -- $B --steps 200 --warmup 10 > $OUT/bench200.log 2>&1" \
  "f20|300|rocprofv3 --pmc FETCH_SIZE -d $OUT/f20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" \
  "w20|300|rocprofv3 --pmc WRITE_SIZE -d $OUT/w20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" || exit $?
[ "${SKIP_SQ:-0}" = 1 ] || "$ROOT/tools/pmc_sweep.sh" "${TAG}_sq10" --pivots 10 --k 40
