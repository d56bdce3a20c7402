#!/bin/bash
# attention A/B on one box: alternate library builds (TT2_LIB) over tools/attn_bench.py
for r in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    TT2_LIB=abl/$lib timeout -k 10 120 python3 -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
  done
done
