#!/bin/bash
# pos.alpha conditioning A/B (fused vs separate BatchNorm statistics), then bench + step profile.
set -euo pipefail
OUT=gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_syncbn.py > "$OUT/gpu_tests.log" 2>&1
echo "tests ok"
timeout -k 10 400 python -u tools/alpha_check.py > "$OUT/alpha_new.txt" 2>&1
echo "alpha new ok"
TT2_BN_OLD=1 timeout -k 10 400 python -u tools/alpha_check.py > "$OUT/alpha_old.txt" 2>&1
echo "alpha old ok"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err"
echo "prof ok"
