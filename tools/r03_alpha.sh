#!/bin/bash
# pos.alpha gradient error A/B (fused vs separate BatchNorm statistics, both against a float64
# oracle), then bench with each and the timed-step profile.
set -uo pipefail
OUT=gpurun_out/r03t
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/alpha_check.py > "$OUT/alpha_new.txt" 2>&1 || exit 1
echo "alpha new ok"
TT2_BN_OLD=1 timeout -k 10 400 python -u tools/alpha_check.py > "$OUT/alpha_old.txt" 2>&1 || exit 1
echo "alpha old ok"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo "bench ok"
TT2_BN_OLD=1 timeout -k 10 600 python -u bench.py > "$OUT/bench_bnold.json" 2> "$OUT/bench_bnold.err" || exit 1
echo "bench bnold ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err" || exit 1
echo "prof ok"
