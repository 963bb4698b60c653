# round 4: planner operand prefetch (P1) and the LDS column window (P3) -- bit-exactness of the
# block path, planner traces old / P1 / P1+P3 on one box, per-pivot cost vs P, driver line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R



for b in trace_planner_old trace_planner_p1 trace_planner_win; do
  timeout -k 10 120 tools/$b 16384 10 3 > $O/${b}_P10.jsonl || exit $?
  timeout -k 10 120 tools/$b 16384 20 2 > $O/${b}_P20.jsonl || exit $?
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
timeout -k 10 600 python -u tools/block_bench.py --sizes 16384 --pivots 12,16,20 --form 0 --k 120 > $O/block_bench_16384.jsonl 2> $O/block_bench.err
timeout -k 10 300 python -u tools/mshard_host_cost.py > $O/mshard_host_cost.jsonl 2> $O/mshard_host_cost.err
timeout -k 10 600 python -u bench.py --rows 65536 --cols 32768 --kind degenerate --steps 200 --warmup 10 --no-cpu-baseline > $O/config5_degenerate.json 2> $O/config5_degenerate.err
