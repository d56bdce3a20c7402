#!/bin/bash
# v10 A/B (forced variant 16 vs auto; step with the v10 route built on / off via TT2_G10_AUTO): correctness tests, per-shape auto vs variant 16, then the bench step with v10 auto on/off
set -e
OUT=gpurun_out/g10; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm10.py > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -u tools/v9_ab.py 16 > $OUT/shapes.txt 2>&1
bash tools/step_ab.sh base.so g10a.so > $OUT/step.txt 2>&1
cat $OUT/step.txt
