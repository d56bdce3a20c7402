#!/bin/bash
# Interleaved decode A/B (dev tool, GPU): tools/decode_ab.py under two environments.
#   tools/ab_decode.sh <tag> "<env A>" "<env B>" [rounds]   -> gpurun_out/<tag>/dab.txt
set -euo pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/dab.txt"
for i in $(seq 1 "$R"); do
  for e in "$A" "$B"; do
    echo "== $e" >> "$OUT/dab.txt"
    env $e timeout -k 10 300 python -u tools/decode_ab.py >> "$OUT/dab.txt" 2>&1
  done
done
cat "$OUT/dab.txt"
