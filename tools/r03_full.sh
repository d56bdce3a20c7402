#!/bin/bash
# Full GPU pass: GPU test suite, smoke, default bench line, timed-step kernel profile.
set -euo pipefail
TAG=${1:-r03v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
echo "tests ok"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err"
echo "prof ok"
