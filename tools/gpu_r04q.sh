# round 4: one host thread per device for the RCCL multi-device chain -- full GPU suite, smoke,
# host cost (copy exchange 1-8 ranks, RCCL world 1), driver line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/mshard_host_cost.py --ranks 1 --exchange rccl > $O/mshard_host_cost_rccl.jsonl 2> $O/mshard.err || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err
