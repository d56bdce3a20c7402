#!/bin/bash
# decode A/B on one box: alternate library builds (TT2_LIB) over the cfg3 decode bench
set -e
mkdir -p gpurun_out/decab
for r in 1 2 3; do
  for lib in "$@"; do
    v=$(TT2_LIB=abl/$lib timeout -k 10 200 python3 -u tools/decode_bench_only.py --no-longform 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['decode']['value'])")
    echo "$lib $v"
  done
done
