# round 4: records-first planner prefetch (no LDS window), captured multi-device chain, 256 planner
# workgroups at 65536 rows -- block / sharded / multi / int suites, planner traces old vs new,
# multi-device host cost eager vs graph, driver line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_block_sharded.py tests/test_gpu_multi.py tests/test_intzero.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for b in trace_planner_old trace_planner_p1b; do
  timeout -k 10 120 tools/$b 16384 10 3 > $O/${b}_P10.jsonl || exit $?
  timeout -k 10 120 tools/$b 16384 20 2 > $O/${b}_P20.jsonl || exit $?
done
timeout -k 10 300 python -u tools/mshard_host_cost.py > $O/mshard_host_cost.jsonl 2> $O/mshard_host_cost.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err
