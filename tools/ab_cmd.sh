set -e
mkdir -p gpurun_out/bn2
export TMPDIR=/tmp
for L in base new; do
  LIB=tools/bin/libtt2_base.so; [ $L = new ] && LIB=transformer-tacotron2_amd/tt2/libtt2.so
  TT2_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bn2/$L -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode --no-ragged > gpurun_out/bn2/$L.json 2> gpurun_out/bn2/$L.err
done
