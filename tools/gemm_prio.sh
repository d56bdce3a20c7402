#!/bin/bash
# A/B: v2 GEMM with s_setprio(1) around its MFMA cluster (TT2_G2_PRIO) vs without.
set -euo pipefail
PKG=transformer-tacotron2_amd
OUT=gpurun_out/prio
mkdir -p $OUT
python3 $PKG/build_lib.py > /dev/null
OBJS=$(ls $PKG/build/*.o | grep -v gemm.hip)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc -DTT2_G2_PRIO -c $PKG/csrc/gemm.hip -o $OUT/gemm_prio.o
hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_prio.so $OBJS $OUT/gemm_prio.o
for s in "12800 512 2048 0 0 2 1" "12800 2048 512 0 0 2 1" "12800 512 2048 0 1 2 1" "2048 512 12800 1 1 2 8"; do
  timeout -k 10 60 python3 tools/gemm_one.py $s 20 | grep TF
  TT2_LIB=$OUT/lib_prio.so timeout -k 10 60 python3 tools/gemm_one.py $s 20 | sed 's/^/prio /' | grep TF
done
