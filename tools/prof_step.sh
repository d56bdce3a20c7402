#!/bin/bash
# rocprofv3 kernel trace of bench.py's timed training steps (tools/summarize_step.py turns
# it into profiles/<tag>_step_kernels.md), then the per-shape GEMM census.
set -euo pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err"
echo "prof ok"
if [ "${2:-}" = census ]; then
  timeout -k 10 300 python3 tools/gemm_census.py > "$OUT/census.txt" 2>&1
  echo "census ok"
fi
