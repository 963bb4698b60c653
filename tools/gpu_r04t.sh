# round 4: SQ_INSTS_VALU pass over the driver's line (k_blk_sweep<20, 5>) for the two-term bound
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/sq20 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/sq20.log 2>&1
