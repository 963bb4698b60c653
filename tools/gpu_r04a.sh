set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04a
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/run_configs.py 2,3 > $O/configs_2_3.jsonl
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg3 -o run -- python -u $R/tools/run_configs.py 3 > $O/prof_cfg3.log 2>&1
