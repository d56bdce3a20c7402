#!/bin/bash
# attention kernels: timing, then PMC passes (one rocprofv3 run per counter set)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/attn
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/attn_bench.py > $OUT/bench.txt 2>&1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python3 tools/attn_bench.py 1 > $OUT/pmc$i.log 2>&1
done
echo done
