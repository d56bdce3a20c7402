#!/bin/bash
# SQ counter passes for one GEMM shape / variant: bash tools/gemm_pmc.sh TAG m n k ta tb var [splits]
set -euo pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/gemm_pmc/$TAG
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/gemm_one.py "$@" 5 > $OUT/p$i.txt 2>&1
done
timeout -k 10 60 python3 tools/gemm_one.py "$@" 1 20 > $OUT/time.txt 2>&1
echo ok
