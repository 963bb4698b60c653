#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the first step whose exit
# status signals a fault, abort, segfault or time-out (124/134/137/139 or >128), and keep going
# past ordinary failures (exit 1: a failing test) so later measurements still happen.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc"; exit $rc; fi
done
exit 0
