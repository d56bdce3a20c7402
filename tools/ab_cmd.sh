set -e
mkdir -p gpurun_out/g8b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g8b/tests.log 2>&1
for i in 1 2; do
  for L in tools/bin/libtt2_base.so transformer-tacotron2_amd/tt2/libtt2.so; do
    TT2_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-decode --no-ragged > gpurun_out/g8b/b.json 2>> gpurun_out/g8b/err.txt
    python -c "import json;d=json.loads(open('gpurun_out/g8b/b.json').read().strip().splitlines()[-1]);print('$L', d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> gpurun_out/g8b/ab.txt
  done
done
