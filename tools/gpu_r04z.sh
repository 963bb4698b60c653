# round 4 final build evidence: full GPU suite, smoke, the driver's bench line, then the rocprofv3
# kernel stats and PMC traffic passes (tools/profile_r04.sh: 16384^2 --steps 20 and config 5)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
bash tools/profile_r04.sh r04z
