#!/bin/bash
# abl/<name>.so: the current library with one source file as of commit <rev> (dev tool for
# interleaved A/B via TT2_LIB).   tools/build_old.sh <name> <rev> <csrc file, e.g. norm.hip>
set -euo pipefail
NAME=$1; REV=$2; FILE=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$ROOT/transformer-tacotron2_amd
python "$P/build_lib.py" > /dev/null
TMP=$(mktemp -d)
git -C "$ROOT" show "$REV:transformer-tacotron2_amd/csrc/$FILE" > "$P/csrc/_old_$FILE"
# the file's per-file flags from build_lib.py (attention.hip: MFMA results in arch VGPRs), so the
# A/B differs in the source only
EXTRA=$(cd "$P" && python -c "import build_lib; print(' '.join(build_lib.EXTRA.get('$FILE', [])))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$P/csrc" -Wno-unused-result \
  $EXTRA -c "$P/csrc/_old_$FILE" -o "$TMP/old.o" || { rm -f "$P/csrc/_old_$FILE"; exit 1; }
rm -f "$P/csrc/_old_$FILE"
mkdir -p "$ROOT/abl"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abl/$NAME.so" $(ls "$P"/build/*.o | grep -v "/$FILE.o") "$TMP/old.o"
rm -rf "$TMP"
echo "abl/$NAME.so"
