#!/bin/bash
# Round-3 DP checks on one GPU: the DP / decode GPU tests, the 2-rank gloo rehearsal of
# bench.py's own launcher, and the 1-rank in-graph RCCL step vs the plain step.
set -euo pipefail
OUT=gpurun_out/${1:-r03dp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dist2.py tests/test_gpu_decode.py \
  -x -v --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
echo "tests ok"
TT2_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 \
  > "$OUT/gloo2.json" 2> "$OUT/gloo2.err"
echo "gloo2 ok"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-decode --no-cpu-baseline --no-ragged \
  > "$OUT/plain.json" 2> "$OUT/plain.err"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-decode --no-cpu-baseline --no-ragged --force-dp \
  > "$OUT/forcedp.json" 2> "$OUT/forcedp.err"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-decode --no-cpu-baseline --no-ragged \
  > "$OUT/plain2.json" 2> "$OUT/plain2.err"
echo "bench ok"
