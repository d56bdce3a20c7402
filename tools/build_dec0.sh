#!/bin/bash
# abl/dec0.so: the current library with decode.hip as of commit $1 (default 060e3a0, before the
# round-4 decode attention changes) -- decode A/B via TT2_LIB (tools/dec_ab.sh dec0.so ...)
set -euo pipefail
REV=${1:-060e3a0}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$ROOT/transformer-tacotron2_amd
python "$P/build_lib.py" > /dev/null
TMP=$(mktemp -d)
git -C "$ROOT" show "$REV:transformer-tacotron2_amd/csrc/decode.hip" > "$P/csrc/_dec0.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$P/csrc" -Wno-unused-result \
  -c "$P/csrc/_dec0.hip" -o "$TMP/dec0.o" || { rm -f "$P/csrc/_dec0.hip"; exit 1; }
rm -f "$P/csrc/_dec0.hip"
mkdir -p "$ROOT/abl"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abl/dec0.so" $(ls "$P"/build/*.o | grep -v decode.hip.o) "$TMP/dec0.o"
rm -rf "$TMP"
echo abl/dec0.so
