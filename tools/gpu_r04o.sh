# round 4: resident overlap with the candidate rows published by the non-polling waves inside E2 -- resident / int
# suites, anatomy at 1024^2, config 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_intzero.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/resident_bench.py --sizes 1024 --wgs 0 --overlap 0,1 --k 400 --trace > $O/resident_1024_trace.jsonl 2> $O/resident.err || exit $?
timeout -k 10 300 python -u tools/run_configs.py 2 > $O/configs_2.jsonl 2> $O/configs_2.err
