#!/bin/bash
# v7 loader-wave count A/B: GEMM tests on the variant, then GEMM shapes and the bench step for each build
set -e
OUT=gpurun_out/lw; mkdir -p $OUT
TT2_LIB=abl/lw8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > $OUT/tests_lw8.log 2>&1
for lib in lw4 lw8 lw4 lw8; do
  TT2_LIB=abl/$lib.so timeout -k 10 240 python3 -u tools/gemm_time.py >> $OUT/gemm_$lib.txt 2>&1
done
bash tools/step_ab.sh lw4.so lw8.so > $OUT/step.txt 2>&1
cat $OUT/step.txt
