#!/bin/bash
# A/B two environment settings of the cfg2 training step on one box (run via gpurun):
#   tools/ab_env.sh "TT2_LN_CHAIN=0" "TT2_LN_CHAIN=1" [rounds]
# Alternates A and B `rounds` times (bench.py, training step only) and prints ms/step.
set -euo pipefail
A=$1; B=$2; R=${3:-3}
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-decode --no-ragged"
for i in $(seq "$R"); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    ms=$(env $E timeout -k 10 300 python3 bench.py $ARGS 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "$v ($E) $ms"
  done
done
