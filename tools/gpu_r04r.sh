# round 4: form-5 sweep grid at 6 / 7 / 8 blocks per CU (occupancy 7 by SGPRs at P = 16-20, 6 by
# LDS at 24) -- per-pivot cost at 16384^2 and 16 / 20 pivots per sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04r
mkdir -p $O
cd $R
for b in 6 7 8; do
  timeout -k 10 300 python -u tools/block_bench.py --sizes 16384 --pivots 16,20 --form 5 --k 120 --bpc $b > $O/block_bench_form5_bpc$b.jsonl 2>> $O/block_bench.err || exit $?
done
timeout -k 10 300 python -u tools/block_bench.py --sizes 16384 --pivots 10,12 --form 4 --k 120 > $O/block_bench_form4_default.jsonl 2>> $O/block_bench.err
