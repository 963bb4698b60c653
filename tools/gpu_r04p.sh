# round 4 final build: full GPU suite, smoke, the driver's bench line, config 2 and the resident
# anatomy at 1024^2 (the overlapped loop as committed)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
timeout -k 10 600 python -u tools/run_configs.py 2,3 > $O/configs_2_3.jsonl 2> $O/configs.err || exit $?
timeout -k 10 300 python -u tools/resident_bench.py --sizes 1024 --wgs 0 --overlap 1 --k 400 --trace > $O/resident_1024_trace.jsonl 2> $O/resident.err
