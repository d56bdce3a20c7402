#!/bin/bash
# A/B two environment settings of the decode legs (cfg3, cfg5) of bench.py on one box:
#   tools/ab_decode.sh "TT2_CAPTURE_MODE=global" "TT2_CAPTURE_MODE=thread_local" [rounds]
set -euo pipefail
A=$1; B=$2; R=${3:-2}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-ragged"
for i in $(seq "$R"); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    r=$(env $E timeout -k 10 300 python3 bench.py $ARGS 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["decode"]["ms_per_frame_step"], d["decode_longform"]["ms_per_frame_step"])')
    echo "$v ($E) train/decode/longform ms: $r"
  done
done
