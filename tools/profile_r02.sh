#!/bin/bash
# Round-2 rocprofv3 evidence (run on the GPU box from the repo root): kernel-trace stats of the
# bench line at 16384^2 (--steps 200: blocks of 12 and 11; --steps 20: two blocks of 10) and
# 1024^2, two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for each 16384^2 form (the
# roofline's traffic: tools/pmc_traffic.py), then SQ counter passes of k_blk_sweep<12>
# (tools/pmc_sweep.sh).  Every rocprofv3 call is its own step under a time limit.
set -o pipefail
TAG=${1:-r02p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
export TMPDIR=/tmp
export STEPS_LOGDIR=$OUT
mkdir -p "$OUT"
B="python3 $ROOT/bench.py --no-cpu-baseline"
cd /tmp || exit 1
"$ROOT/tools/gpu_steps.sh" \
  "s200|300|rocprofv3 --kernel-trace --stats -d $OUT/s200 -o run --output-format csv -- $B --steps 200 --warmup 10 > $OUT/bench200.log 2>&1" \
  "s20|300|rocprofv3 --kernel-trace --stats -d $OUT/s20 -o run --output-format csv -- $B --steps 20 --warmup 5 > $OUT/bench20.log 2>&1" \
  "s1k|300|rocprofv3 --kernel-trace --stats -d $OUT/s1k -o run --output-format csv -- $B --rows 1024 --cols 1024 --steps 1000 --warmup 10 > $OUT/bench1k.log 2>&1" \
  "f200|300|rocprofv3 --pmc FETCH_SIZE -d $OUT/f200 -o run --output-format csv -- $B --steps 48 --warmup 8 > /dev/null 2>&1" \
  "w200|300|rocprofv3 --pmc WRITE_SIZE -d $OUT/w200 -o run --output-format csv -- $B --steps 48 --warmup 8 > /dev/null 2>&1" \
  "f20|300|rocprofv3 --pmc FETCH_SIZE -d $OUT/f20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" \
  "w20|300|rocprofv3 --pmc WRITE_SIZE -d $OUT/w20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" || exit $?
# SKIP_SQ=1: kernel-trace and traffic passes only (the SQ passes depend on the sweep's code alone)
[ "${SKIP_SQ:-0}" = 1 ] || "$ROOT/tools/pmc_sweep.sh" "${TAG}_sq12" --pivots 12 --k 48
