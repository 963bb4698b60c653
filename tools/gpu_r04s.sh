# round 4: 20 pivots per sweep for 1-4 GiB tables -- block suite (bit-exact through the default
# policy at 16384^2), smoke, the driver's line, then rocprofv3 kernel stats and FETCH / WRITE
# passes of the --steps 20 line (k_blk_sweep<20, 5>)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_block_pipe.py tests/test_gpu_configs.py tests/test_gpu_block_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || exit $?
export TMPDIR=/tmp
export STEPS_LOGDIR=$O/prof
B="python3 $R/bench.py --no-cpu-baseline"
cd /tmp || exit 1
"$R/tools/gpu_steps.sh" \
  "s20|300|rocprofv3 --kernel-trace --stats -d $O/prof/s20 -o run --output-format csv -- $B --steps 20 --warmup 5 > $O/prof/bench20.log 2>&1" \
  "f20|300|rocprofv3 --pmc FETCH_SIZE -d $O/prof/f20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1" \
  "w20|300|rocprofv3 --pmc WRITE_SIZE -d $O/prof/w20 -o run --output-format csv -- $B --steps 20 --warmup 5 > /dev/null 2>&1"
