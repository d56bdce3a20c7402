#!/bin/bash
# Timing-only ablations of the v3 attention kernels (results are garbage by design):
# builds libtt2 variants with TT2_ABL_* defines and runs tools/attn_bench.py on each.
#   bash tools/attn_ablate.sh          (on the GPU box, from the repo root)
set -euo pipefail
PKG=transformer-tacotron2_amd
OUT=gpurun_out/abl
mkdir -p $OUT
python3 $PKG/build_lib.py > /dev/null
OBJS=$(ls $PKG/build/*.o | grep -v attention)
for v in BASE NOEXP L2HOT NOSYNC; do
  D=""; [ $v != BASE ] && D="-DTT2_ABL_$v"
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc -mllvm -amdgpu-mfma-vgpr-form=1 $D \
    -c $PKG/csrc/attention.hip -o $OUT/attn_$v.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$v.so $OBJS $OUT/attn_$v.o
  echo "== $v"
  TT2_LIB=$OUT/lib_$v.so timeout -k 10 120 python3 tools/attn_bench.py 0
done
