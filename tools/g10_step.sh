#!/bin/bash
# v10 auto routing on/off in the bench step (interleaved), then the GEMM tests on the default build
set -e
OUT=gpurun_out/g10s; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm10.py tests/test_gpu_gemm.py tests/test_gpu_fullsize.py > $OUT/tests.log 2>&1
bash tools/step_ab.sh noauto.so auto.so > $OUT/step.txt 2>&1
cat $OUT/step.txt
