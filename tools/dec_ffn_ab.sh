#!/bin/bash
# cfg3 / cfg5 decode with the one-launch FFN (TT2_DEC_SCHEDULE=4) against the default three-launch
# FFN (0), interleaved, same box (GPU; run from the repo root).
# usage: tools/dec_ffn_ab.sh OUTDIR [ROUNDS]
set -o pipefail
out=${1:?outdir}; rounds=${2:-2}
mkdir -p "$out"
for i in $(seq 1 "$rounds"); do
  for sch in 4 0; do
    TT2_DEC_SCHEDULE=$sch timeout -k 10 300 python tools/decode_bench_only.py > "$out/dec_s${sch}_$i.json" 2> "$out/dec_s${sch}_$i.err" || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('schedule', sys.argv[2], 'cfg3', d['decode']['value'], d['decode']['ms_per_frame_step'], 'cfg5', d['longform']['value'], d['longform'].get('ms_per_frame_step'))" "$out/dec_s${sch}_$i.json" $sch | tee -a "$out/ab.txt"
  done
done
