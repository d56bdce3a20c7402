#!/bin/bash
# Interleaved A/B of the bench train step under two environment settings (dev tool, GPU):
#   tools/ab_env.sh <tag> "<env A>" "<env B>" [rounds]
# e.g. tools/ab_env.sh pre "TT2_G7_PRE=0" "TT2_G7_PRE=1" 3   -> gpurun_out/<tag>/ab.txt
set -euo pipefail
TAG=$1; A=$2; B=$3; R=${4:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/ab.txt"
for i in $(seq 1 "$R"); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode \
      > "$OUT/run.json" 2> "$OUT/run.err"
    echo "$e $(python -c "import json;d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")" \
      >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
