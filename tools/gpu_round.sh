#!/bin/bash
# One GPU-box pass (run via gpurun from the repo root): GPU tests, smoke, bench, rocprof
# kernel-trace stats of the bench step.  Every GPU step has its own time limit; the
# steps are chained so that the first failure ends the call.
#   tools/gpu_round.sh <tag> [tests|bench|prof|pmc|mfma|dpmc ...]   (default: tests bench prof)
set -euo pipefail
TAG=${1:-r02}
shift || true
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      ;;
    bench)
      timeout -k 10 420 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode \
        > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
      ;;
    pmc)   # HBM bytes of the bench step's kernels (FETCH_SIZE and WRITE_SIZE cannot share a pass)
      ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-decode"
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
        python3 bench.py $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
        python3 bench.py $ARGS > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
      ;;
    mfma)  # matrix-pipe busy cycles per kernel (tools/summarize_mfma.py)
      timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/mfma" -o run \
        --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-decode --no-cpu-baseline --no-ragged \
        > "$OUT/bench_mfma.json" 2> "$OUT/bench_mfma.err"
      ;;
    dpmc)  # the same for one cfg3 decode run
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/dtr/fetch" -o run --output-format csv -- \
        python3 tools/decode_traffic.py --out="$OUT/dtr" > "$OUT/dtr_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/dtr/write" -o run --output-format csv -- \
        python3 tools/decode_traffic.py --out="$OUT/dtr" > "$OUT/dtr_write.log" 2>&1
      ;;
    lpmc)  # and for one cfg5 long-form run
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/ltr/fetch" -o run --output-format csv -- \
        python3 tools/decode_traffic.py --longform --out="$OUT/ltr" > "$OUT/ltr_fetch.log" 2>&1
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/ltr/write" -o run --output-format csv -- \
        python3 tools/decode_traffic.py --longform --out="$OUT/ltr" > "$OUT/ltr_write.log" 2>&1
      ;;
    dpt)   # the DP / SyncBN / norm / full-length parity tests of round 4
      timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_syncbn.py tests/test_gpu_norm.py \
        tests/test_gpu_overlap.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_metrics.py -x -v --timeout 300 --timeout-method thread > "$OUT/dpt_tests.log" 2>&1
      ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
