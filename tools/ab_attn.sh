set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in 0 1; do
TT2_ATTN_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/v$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode > gpurun_out/ab/v$v.json 2> gpurun_out/ab/v$v.err
done
