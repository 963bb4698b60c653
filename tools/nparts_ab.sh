#!/bin/bash
# Planner workgroup-count A/B on the production block path (SMX_NPARTS_MAX), alternating.
# usage: tools/nparts_ab.sh OUT.jsonl "0 16 32" [sizes] [pivots] [reps]
set -o pipefail
OUT=$1; SETS=${2:-"0 16 32"}; SIZES=${3:-16384}; PIVS=${4:-10,12}; REPS=${5:-2}
: > "$OUT"
for rep in $(seq 1 "$REPS"); do
  for g in $SETS; do
    SMX_NPARTS_MAX=$g timeout -k 10 150 python3 tools/block_bench.py --sizes "$SIZES" --pivots "$PIVS" --k 96 \
      | sed "s/^{/{\"nparts_max\": $g, \"rep\": $rep, /" >> "$OUT" || exit $?
  done
done
