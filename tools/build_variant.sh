#!/bin/bash
# Build abl/<name>.so: the current objects with gemm.hip recompiled under extra -D flags
# (dev tool for interleaved A/B via TT2_LIB).   tools/build_variant.sh <name> -DFOO=1 ...
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/transformer-tacotron2_amd
python "$PKG/build_lib.py" > /dev/null
mkdir -p "$ROOT/abl"
TMP=$(mktemp -d)
OBJS=()
for o in "$PKG"/build/*.o; do
  if [[ $(basename "$o") == gemm.hip.o || $(basename "$o") == gemm.o ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$PKG/csrc" \
      -Wno-unused-result "$@" -c "$PKG/csrc/gemm.hip" -o "$TMP/gemm.o"
    OBJS+=("$TMP/gemm.o")
  else
    OBJS+=("$o")
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abl/$NAME.so" "${OBJS[@]}"
rm -rf "$TMP"
echo "abl/$NAME.so"
