# round 4, last build: the full GPU suite and smoke (the driver's round-end tiers)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04u
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/sq20 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/sq20.log 2>&1
