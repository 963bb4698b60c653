#!/bin/bash
# Round-4 rocprofv3 evidence (GPU box, repo root): kernel-trace stats of the driver's bench line
# (16384^2, --steps 20) and two PMC passes (FETCH_SIZE, WRITE_SIZE) over it; then the same for
# config 5 (65536 x 32768 degenerate LP, one GPU, 24 pivots = two sweeps of 12) so its bench line
# carries measured traffic.  Every rocprofv3 call is its own step under a time limit.
set -o pipefail
TAG=${1:-r04}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
export TMPDIR=/tmp
export STEPS_LOGDIR=$OUT
mkdir -p "$OUT"
B="python3 $ROOT/bench.py --no-cpu-baseline"
C5="$B --rows 65536 --cols 32768 --kind degenerate"
cd /tmp || exit 1
"$ROOT/tools/gpu_steps.sh" \
  "s20|300|rocprofv3 --kernel-trace --stats -d $OUT/s20 -o run --output-format csv -- $B --steps 20 --warmup 5 > $OUT/bench20.log 2>&1" \
  "f20|300|rocprofv3 --pmc FETCH_SIZE -d $OUT/f20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" \
  "w20|300|rocprofv3 --pmc WRITE_SIZE -d $OUT/w20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" \
  "c5s|400|rocprofv3 --kernel-trace --stats -d $OUT/c5s -o run --output-format csv -- $C5 --steps 24 --warmup 0 > $OUT/config5.log 2>&1" \
  "c5f|400|rocprofv3 --pmc FETCH_SIZE -d $OUT/c5f -o run --output-format csv -- $C5 --steps 24 --warmup 0 > /dev/null 2>&1" \
  "c5w|400|rocprofv3 --pmc WRITE_SIZE -d $OUT/c5w -o run --output-format csv -- $C5 --steps 24 --warmup 0 > /dev/null 2>&1"
