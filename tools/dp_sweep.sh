#!/bin/bash
# DP-path overhead vs gradient bucket size on one GPU (1-rank RCCL group, segmented graph):
#   tools/dp_sweep.sh "25 50 100 256"
set -euo pipefail
for mb in ${1:-25 50 100 256}; do
  ms=$(TT2_BUCKET_MB=$mb timeout -k 10 300 python3 bench.py --force-dp --steps 20 --no-decode --no-cpu-baseline --no-ragged 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
  echo "bucket ${mb} MB: $ms ms/step"
done
ms=$(timeout -k 10 300 python3 bench.py --steps 20 --no-decode --no-cpu-baseline --no-ragged 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
echo "no DP: $ms ms/step"
