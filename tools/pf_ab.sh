#!/bin/bash
# A/B of the v7 A-operand L2 prefetch: GEMM shapes and the bench step, prefetch off vs on.
set -e
mkdir -p gpurun_out/pf
for pf in 0 1; do
  TT2_G7_PF=$pf timeout -k 10 240 python3 -u tools/gemm_time.py > gpurun_out/pf/gemm_$pf.txt 2>&1
  TT2_G7_PF=$pf timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --profile-run > gpurun_out/pf/bench_$pf.json 2> gpurun_out/pf/bench_$pf.err
done
for pf in 0 1; do echo "== pf=$pf"; cat gpurun_out/pf/gemm_$pf.txt; tail -1 gpurun_out/pf/bench_$pf.json | cut -c1-200; done
