# round 4: large-P sweep layouts -- block GPU tests, then per-pivot cost vs P and layout
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 300 --timeout-method thread > $O/pytest_block.txt 2>&1
echo "pytest rc=$?" >> $O/pytest_block.txt
timeout -k 10 600 python -u tools/block_bench.py --sizes 16384 --pivots 10,12,16,20,24 --form 4,5 --k 120 > $O/block_bench_16384.jsonl 2> $O/block_bench.err
timeout -k 10 300 python -u tools/block_bench.py --sizes 8192 --pivots 12,16,20,24 --form 0 --k 120 > $O/block_bench_8192.jsonl 2>> $O/block_bench.err
