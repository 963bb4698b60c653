#!/bin/bash
# One GPU session on the box, as named recipes run in order (each its own step under its own time
# limit, tools/gpu_steps.sh: a fault / abort / time-out ends the session there; a failing test does
# not).  Replaces the round-4 one-off tools/gpu_r04*.sh scripts.
#   usage (from the repo root, e.g. through gpurun):  tools/gpu_round.sh TAG RECIPE...
# Output under gpurun_out/TAG/ (one <recipe>.log each, steps.log).  Recipes (ARGS: spaces as ',',
# a literal comma as '+', e.g. `py=tools/mshard_host_cost.py,--ranks,1+2+4+8`):
#   pytest                 the full `pytest -m gpu` suite (the driver's round-end tier)
#   pytest=FILES           those test files (comma separated) with -m gpu
#   smoke                  __graft_entry__.smoke()
#   bench20 / bench200     bench.py --steps 20 --warmup 5 (the driver's line) / --steps 200 --warmup 20
#   benchN=ARGS            bench.py with ARGS (`benchN=--size,8192,--steps,200` -> benchN.log)
#   stats20 / stats200     rocprofv3 --kernel-trace --stats of bench20 / bench200 (no cpu baseline)
#   statsN=ARGS            rocprofv3 --kernel-trace --stats of bench.py ARGS (-> gpurun_out/TAG/N_statsN/)
#   fetch20 / write20      rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench20
#   sq20 / clock200        rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES of bench20; GRBM_GUI_ACTIVE
#                          GRBM_COUNT SQ_INSTS_VALU SQ_BUSY_CYCLES of bench200 (the clock per sweep)
#   clock20                the same counters over the driver's bench20 line (the timed sweep's clock)
#   paths=ARGS             tools/sweep_paths.py ARGS on the diagnostic build (libsmx_diag.so)
#   pmcpaths=ARGS          rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
#                          GRBM_GUI_ACTIVE of tools/sweep_paths.py ARGS (product build; per sweep)
#   sweeps=ARGS            tools/sweep_paths.py ARGS on the product build (timings only)
#   sweepslib=LIB,ARGS     tools/sweep_paths.py ARGS on another build of libsmx (SMX_LIB=LIB: an A/B)
#   blockbench=ARGS        tools/block_bench.py ARGS
#   blockbenchlib=LIB,ARGS tools/block_bench.py ARGS on another build of libsmx (SMX_LIB=LIB)
#   configs=ARGS           tools/run_configs.py ARGS
#   py=SCRIPT,ARGS         python3 SCRIPT ARGS (a tools/ probe)
#   run=PROGRAM,ARGS       a built tools/ probe (e.g. `run=tools/cumask_probe`)
#   pmcrun=C1:C2..,PROGRAM,ARGS  one rocprofv3 --pmc pass (counters ':'-separated) over a built probe
#   pmcpy=C1:C2..,SCRIPT,ARGS    the same over a python script (python3 SCRIPT ARGS)
# A recipe may carry its own time limit: `paths=...@300` (seconds; default per recipe below).
set -o pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
export STEPS_LOGDIR=$O
B="python3 $R/bench.py --no-cpu-baseline"
STEPS=()
n=0
for spec in "$@"; do
  n=$((n + 1))
  lim=""
  if [[ "$spec" == *@* ]]; then lim="${spec##*@}"; spec="${spec%@*}"; fi
  name="${spec%%=*}"
  arg=""
  [[ "$spec" == *=* ]] && arg="${spec#*=}"
  arg="${arg//,/ }"
  arg="${arg//+/,}"
  tag="${n}_${name}"
  case "$name" in
    pytest)
      if [ -n "$arg" ]; then files=""; for f in $arg; do files="$files $R/$f"; done
      else files="$R/tests"; fi
      cmd="cd $R && python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread"
      d=900 ;;
    smoke) cmd="cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'"; d=180 ;;
    bench20) cmd="cd $R && python -u bench.py --gpus 1 --steps 20 --warmup 5"; d=300 ;;
    bench200) cmd="cd $R && python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"; d=300 ;;
    benchN) cmd="cd $R && python -u bench.py $arg"; d=400 ;;
    stats20) cmd="cd /tmp && rocprofv3 --kernel-trace --stats -d $O/stats20 -o run --output-format csv -- $B --steps 20 --warmup 5"; d=300 ;;
    statsN) cmd="cd /tmp && rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- $B $arg"; d=300 ;;
    stats200) cmd="cd /tmp && rocprofv3 --kernel-trace --stats -d $O/stats200 -o run --output-format csv -- $B --steps 200 --warmup 20"; d=300 ;;
    fetch20) cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch20 -o run --output-format csv -- $B --steps 20 --warmup 5"; d=300 ;;
    write20) cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write20 -o run --output-format csv -- $B --steps 20 --warmup 5"; d=300 ;;
    sq20) cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/sq20 -o run --output-format csv -- $B --steps 20 --warmup 5"; d=300 ;;
    clock20) cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/clock20 -o run --output-format csv -- $B --steps 20 --warmup 5 --sustained 0"; d=300 ;;
    clock200) cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/clock200 -o run --output-format csv -- $B --steps 200 --warmup 20"; d=300 ;;
    pmcpaths) cmd="cd /tmp && timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/$tag -o run --output-format csv -- python3 $R/tools/sweep_paths.py $arg"; d=300 ;;
    paths) cmd="cd $R && SMX_LIB=libsmx_diag.so python -u tools/sweep_paths.py $arg"; d=300 ;;
    sweeps) cmd="cd $R && python -u tools/sweep_paths.py $arg"; d=300 ;;
    sweepslib) lib="${arg%% *}"; cmd="cd $R && SMX_LIB=$lib python -u tools/sweep_paths.py ${arg#* }"; d=300 ;;
    blockbench) cmd="cd $R && python -u tools/block_bench.py $arg"; d=400 ;;
    blockbenchlib) lib="${arg%% *}"; cmd="cd $R && SMX_LIB=$lib python -u tools/block_bench.py ${arg#* }"; d=400 ;;
    configs) cmd="cd $R && python -u tools/run_configs.py $arg"; d=600 ;;
    py) cmd="cd $R && python -u $arg"; d=300 ;;
    run) cmd="cd $R && $arg"; d=300 ;;
    pmcpy) ctrs="${arg%% *}"; cmd="cd /tmp && timeout -s KILL 240 rocprofv3 --pmc ${ctrs//:/ } -d $O/$tag -o run --output-format csv -- python3 $R/${arg#* }"; d=280 ;;
    pmcrun) ctrs="${arg%% *}"; cmd="cd /tmp && timeout -s KILL 60 rocprofv3 --pmc ${ctrs//:/ } -d $O/$tag -o run --output-format csv -- $R/${arg#* }"; d=90 ;;
    *) echo "unknown recipe $name"; exit 2 ;;
  esac
  STEPS+=("$tag|${lim:-$d}|$cmd")
done
"$R/tools/gpu_steps.sh" "${STEPS[@]}"
