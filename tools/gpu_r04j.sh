# round 4: planner back to the round-3 body (+256 workgroups on tall tables), single-launch copy
# exchange for same-device ranks -- suites, multi-device host cost, driver line, config 5
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_block_sharded.py tests/test_gpu_multi.py tests/test_intzero.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mshard_host_cost.py > $O/mshard_host_cost.jsonl 2> $O/mshard_host_cost.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
timeout -k 10 600 python -u bench.py --rows 65536 --cols 32768 --kind degenerate --steps 200 --warmup 10 --no-cpu-baseline > $O/config5_degenerate.json 2> $O/config5_degenerate.err
