#!/bin/bash
# rocprofv3 evidence for the bench kernel (run on the GPU box from the repo root):
#   kernel-trace stats of bench.py at 16384^2 (the bench line: block sweeps + planner, and the
#   one-pivot k_update line) and 1024^2 (BASELINE config 2, the LDS-resident loop), and two
#   separate PMC passes (FETCH_SIZE, WRITE_SIZE) at 16384^2 for the roofline "traffic"
#   (tools/pmc_traffic.py ... "16384x16384/k_blk_sweep<8>" profiles/pmc_traffic.json k_blk_sweep).
# Every rocprofv3 call is its own step under a time limit (tools/gpu_steps.sh).
# usage: tools/profile_round.sh TAG
set -o pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
export TMPDIR=/tmp
export STEPS_LOGDIR=$ROOT/gpurun_out
mkdir -p "$OUT"
B="python3 $ROOT/bench.py --no-cpu-baseline"
cd /tmp || exit 1
"$ROOT/tools/gpu_steps.sh" \
  "stats16k|300|rocprofv3 --kernel-trace --stats -d $OUT/stats16k -o run --output-format csv -- $B --steps 100 --warmup 10 > $OUT/bench16k.log 2>&1" \
  "stats1k|300|rocprofv3 --kernel-trace --stats -d $OUT/stats1k -o run --output-format csv -- $B --rows 1024 --cols 1024 --steps 1000 --warmup 10 > $OUT/bench1k.log 2>&1" \
  "pmcf|300|rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B --steps 32 --warmup 8 > /dev/null 2>&1" \
  "pmcw|300|rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B --steps 32 --warmup 8 > /dev/null 2>&1"
