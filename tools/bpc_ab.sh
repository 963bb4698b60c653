#!/bin/bash
# Sweep blocks-per-CU A/B on the production block path (SMX_BLK_BPC), alternating settings.
# usage: tools/bpc_ab.sh OUT.jsonl "0 5 6 7 8" [sizes] [pivots] [reps]
set -o pipefail
OUT=$1; SETS=${2:-"0 5 6 7 8"}; SIZES=${3:-16384}; PIVS=${4:-10,12}; REPS=${5:-2}
: > "$OUT"
for rep in $(seq 1 "$REPS"); do
  for b in $SETS; do
    SMX_BLK_BPC=$b timeout -k 10 150 python3 tools/block_bench.py --sizes "$SIZES" --pivots "$PIVS" --k 96 \
      | sed "s/^{/{\"bpc_env\": $b, \"rep\": $rep, /" >> "$OUT" || exit $?
  done
done
