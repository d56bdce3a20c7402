#!/bin/bash
# SQ counter passes over tools/attn_bench.py (variant given as $1, default 0).
set -euo pipefail
export TMPDIR=/tmp
V=${1:-0}
OUT=gpurun_out/attn_pmc
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/attn_bench.py $V > $OUT/p$i.txt 2>&1
done
echo ok
