#!/bin/bash
# Quick GPU pass for a kernel change: the suites that exercise GEMM split-K, BatchNorm and the
# bitwise graph-vs-eager step, then the default bench line and the timed-step kernel profile.
set -euo pipefail
TAG=${1:-r03u}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_norm.py tests/test_gpu_fullsize.py tests/test_gpu_blocks.py \
  tests/test_gpu_model.py tests/test_gpu_dist.py > "$OUT/gpu_tests.log" 2>&1
echo "tests ok"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err"
echo "prof ok"
