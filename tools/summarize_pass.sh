#!/bin/bash
# Summarise a tools/gpu_pass.sh evidence pass ON THE GPU BOX (CPU-only scripts), copy the
# profiles/<tag>_* summaries into gpurun_out/<tag>/prof/ (gpurun merges back only gpurun_out/,
# at most 64 MiB) and delete the raw rocprofv3 CSVs they came from:
#   tools/summarize_pass.sh <tag>
TAG=$1
OUT=gpurun_out/$TAG
[ -f "$OUT/bench_step.json" ] && cp "$OUT/bench_step.json" "$OUT/bench_kt.json"
[ -d "$OUT/kt" ] && python tools/summarize_step.py "$TAG" "$OUT" > "$OUT/sum_step.log" 2>&1
[ -d "$OUT/kt" ] && python tools/step_gaps.py "$TAG" "$OUT" > "$OUT/sum_gaps.log" 2>&1
[ -d "$OUT/kt" ] && python tools/summarize_prof.py "$TAG" > "$OUT/sum_prof.log" 2>&1
[ -d "$OUT/mfma" ] && python tools/summarize_mfma.py "$OUT/mfma/run_counter_collection.csv" \
  "profiles/${TAG}_mfma_busy.json" > "$OUT/sum_mfma.log" 2>&1
[ -d "$OUT/dtr" ] && python tools/summarize_decode_traffic.py "$OUT/dtr" "$TAG" > "$OUT/sum_dtr.log" 2>&1
[ -d "$OUT/ltr" ] && python tools/summarize_decode_traffic.py "$OUT/ltr" "$TAG" > "$OUT/sum_ltr.log" 2>&1
if [ -d "$OUT/dk" ]; then
  mkdir -p "$OUT/decsum" && ln -sfn "$PWD/$OUT/dk" "$OUT/decsum/kt" && ln -sfn "$PWD/$OUT/dtr" "$OUT/decsum/dtr"
  python tools/summarize_decode_step.py "$TAG" "$OUT/decsum" > "$OUT/sum_decstep.log" 2>&1
  [ -f "$OUT/dk/run_kernel_stats.csv" ] && cp "$OUT/dk/run_kernel_stats.csv" "profiles/${TAG}_decode_kernel_stats.csv"
  rm -rf "$OUT/decsum"
fi
mkdir -p "$OUT/prof"
cp profiles/${TAG}_* "$OUT/prof/" 2>/dev/null
# the raw traces and counter dumps stay on the box
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*agent_info.csv" \) -delete
du -sh "$OUT"
ls "$OUT/prof"
