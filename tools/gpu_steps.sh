#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the first step whose exit
# status signals a fault, abort, segfault or time-out (124/134/137/139 or >128), and keep going
# past ordinary failures (exit 1: a failing test) so later measurements still happen.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
LOG=${STEPS_LOGDIR:-gpurun_out}
mkdir -p "$LOG"
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a "$LOG/steps.log"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$LOG/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc after $(( $(date +%s) - start ))s" | tee -a "$LOG/steps.log"
  tail -5 "$LOG/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc"; exit $rc; fi
done
exit 0
