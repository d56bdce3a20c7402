#!/bin/bash
# v7 in-kernel timelines (tools/gemm_stamps.hip) for the step's main shapes
set -euo pipefail
OUT=gpurun_out/${1:-stamps}
mkdir -p "$OUT"
S=./tools/bin/gemm_stamps
for shape in "12800 512 512 0 0 14 1" "12800 2048 512 0 0 14 1" "12800 512 2048 0 0 14 1" "12800 1536 512 0 0 14 1" \
             "12800 512 512 0 1 14 1" ; do
  TT2_BIAS=1 timeout -k 5 60 $S $shape >> "$OUT/stamps.txt" 2>&1
done
echo ok
