# round 4: resident overlap with the automatic width policy -- resident / parity suites, smoke,
# the loop's anatomy old vs new at 1024^2, config 2 (run_configs: 1024^2 seeds, forced update)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_surface.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/resident_bench.py --sizes 1024 --wgs 0 --overlap 0,1 --k 400 --trace > $O/resident_1024_trace.jsonl 2> $O/resident.err || exit $?
timeout -k 10 300 python -u tools/run_configs.py 2 > $O/configs_2.jsonl 2> $O/configs_2.err
