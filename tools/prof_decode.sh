#!/bin/bash
# cfg3 decode step: kernel trace of the graph-replayed loop + FETCH / WRITE PMC passes of the
# eager loop (tools/summarize_decode_step.py <tag> gpurun_out/<tag>).
set -euo pipefail
OUT=gpurun_out/${1:-r03dec}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
  python3 tools/decode_prof.py > "$OUT/kt.log" 2>&1
echo "kt ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/dtr/fetch" -o run --output-format csv -- \
  python3 tools/decode_traffic.py > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/dtr/write" -o run --output-format csv -- \
  python3 tools/decode_traffic.py > "$OUT/write.log" 2>&1
echo "pmc ok"
