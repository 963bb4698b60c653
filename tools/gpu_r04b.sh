# sweep_lab2: large-P sweep variants (16384^2), bpc 5 and 8
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
for P in 10 12 16 20 24; do
  timeout -k 10 120 tools/sweep_lab2 16384 $P 5 5 0123456 >> $O/lab2.jsonl
  timeout -k 10 120 tools/sweep_lab2 16384 $P 5 8 0346 >> $O/lab2.jsonl
done
