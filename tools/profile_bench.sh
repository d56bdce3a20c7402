#!/bin/bash
# Profile bench.py on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats  (per-kernel durations)
#   2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass)
# Outputs under gpurun_out/prof_<tag>/; tools/summarize_prof.py turns them into profiles/.
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-decode"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py $ARGS > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 bench.py $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 bench.py $ARGS > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
echo done
