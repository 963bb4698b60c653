# round 4: planner (records first; row-pass column load before the step's stores): block /
# sharded / multi / int suites, planner traces old vs new, driver line, P sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_block_sharded.py tests/test_gpu_multi.py tests/test_intzero.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for b in trace_planner_old trace_planner_p1b trace_planner_p1c; do
  timeout -k 10 120 tools/$b 16384 10 3 > $O/${b}_P10.jsonl || exit $?
  timeout -k 10 120 tools/$b 16384 20 2 > $O/${b}_P20.jsonl || exit $?
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
timeout -k 10 600 python -u tools/block_bench.py --sizes 16384 --pivots 12,16,20 --form 0 --k 120 > $O/block_bench_16384.jsonl 2> $O/block_bench.err
