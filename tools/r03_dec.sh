#!/bin/bash
# decode checks after a decode-step change: decode tests, cfg3/cfg5 timing, decode profile
set -euo pipefail
OUT=gpurun_out/${1:-r03dec2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_kernels.py -x -q \
  --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
echo "tests ok"
timeout -k 10 300 python -u tools/decode_bench_only.py > "$OUT/dec.json" 2> "$OUT/dec.err"
echo "bench ok"
