# round 4 re-entry: full GPU suite + smoke on the form-5 build, the default bench line, then
# per-pivot cost vs P and sweep layout (form 4 registers / 5 LDS) at 16384^2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 600 python -u tools/block_bench.py --sizes 16384 --pivots 10,12,16,20,24 --form 4,5 --k 120 > $O/block_bench_16384.jsonl 2> $O/block_bench.err
