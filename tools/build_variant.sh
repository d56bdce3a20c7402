#!/bin/bash
# Build abl/<name>.so: the current objects with one source (gemm.hip, or $VAR_SRC.hip) recompiled
# under extra -D flags (dev tool for interleaved A/B via TT2_LIB).
#   [VAR_SRC=norm] tools/build_variant.sh <name> -DFOO=1 ...
set -euo pipefail
NAME=$1; shift
SRC=${VAR_SRC:-gemm}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/transformer-tacotron2_amd
python "$PKG/build_lib.py" > /dev/null
mkdir -p "$ROOT/abl"
TMP=$(mktemp -d)
OBJS=()
for o in "$PKG"/build/*.o; do
  if [[ $(basename "$o") == $SRC.hip.o || $(basename "$o") == $SRC.cpp.o || $(basename "$o") == $SRC.o ]]; then
    SRCF="$PKG/csrc/$SRC.hip"; [ -f "$SRCF" ] || SRCF="$PKG/csrc/$SRC.cpp"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$PKG/csrc" \
      -Wno-unused-result "$@" -c "$SRCF" -o "$TMP/$SRC.o"
    OBJS+=("$TMP/$SRC.o")
  else
    OBJS+=("$o")
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abl/$NAME.so" "${OBJS[@]}"
rm -rf "$TMP"
echo "abl/$NAME.so"
