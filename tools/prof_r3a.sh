set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3a -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_r3a_bench.json 2>&1 || exit $?
cd $R && timeout -k 10 60 tools/sweep_lab 16384 10 5 7 0159 > gpurun_out/lab4.jsonl
