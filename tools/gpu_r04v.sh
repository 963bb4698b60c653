# round 4 final build: three driver-shaped bench lines back to back on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench20_repeats.jsonl 2>> $O/bench.err || exit $?
done
