#!/bin/bash
# training-step A/B on one box: alternate library builds (TT2_LIB) over bench.py --profile-run
set -e
for r in 1 2 3; do
  for lib in "$@"; do
    v=$(TT2_LIB=abl/$lib timeout -k 10 240 python3 -u bench.py --steps 30 --warmup 5 --profile-run 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$lib $v"
  done
done
