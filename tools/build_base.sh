#!/bin/bash
# Build tools/bin/libtt2_base.so: the current objects with one csrc file taken from a git
# revision (dev tool for interleaved A/B via TT2_LIB).   tools/build_base.sh <rev> [file ...]
set -euo pipefail
REV=$1; shift
FILES=${*:-gemm.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/transformer-tacotron2_amd
TMP=$(mktemp -d)
python "$PKG/build_lib.py" > /dev/null
OBJS=()
for o in "$PKG"/build/*.o; do
  f=$(basename "$o" .o)
  if [[ " $FILES " == *" $f "* ]]; then
    git -C "$ROOT" show "$REV:transformer-tacotron2_amd/csrc/$f" > "$TMP/$f"
    [[ -n "${SED:-}" ]] && sed -i "$SED" "$TMP/$f"   # optional ablation edit, e.g. SED='s/st8nt(/st8(/g'
    true
    extra=()
    [[ $f == attention.hip ]] && extra=(-mllvm -amdgpu-mfma-vgpr-form=1)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$PKG/csrc" \
      -Wno-unused-result "${extra[@]}" -c "$TMP/$f" -o "$TMP/$f.o"
    OBJS+=("$TMP/$f.o")
  else
    OBJS+=("$o")
  fi
done
mkdir -p "$ROOT/tools/bin"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/bin/libtt2_base.so" "${OBJS[@]}"
rm -rf "$TMP"
echo "tools/bin/libtt2_base.so: $FILES from $REV"
