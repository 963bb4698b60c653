# round 4: the overlapped LDS-resident loop (bulk update under the next hand-off) -- resident
# suite (both loops vs the oracle), then config 2 (1024^2, seeds 0..4) per-pivot time old vs new
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_intzero.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/resident_bench.py --sizes 1024 --wgs 0 --overlap 0,1 --seeds 0,1,2,3,4 --k 1000 > $O/resident_1024.jsonl 2> $O/resident_1024.err || exit $?
timeout -k 10 300 python -u tools/resident_bench.py --sizes 512,1536 --wgs 0 --overlap 0,1 --k 600 > $O/resident_sizes.jsonl 2>> $O/resident_1024.err
