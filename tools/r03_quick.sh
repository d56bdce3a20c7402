#!/bin/bash
# quick A/B pass: GEMM + full-size tests, a training-only bench line, timed-step profile
set -euo pipefail
TAG=${1:-r03q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_norm.py tests/test_gpu_gemm.py tests/test_gpu_fullsize.py tests/test_gpu_model.py \
  tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
echo "tests ok"
timeout -k 10 300 python -u bench.py --steps 30 --no-decode --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err"
echo "prof ok"
