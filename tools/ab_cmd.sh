set -e
mkdir -p gpurun_out/dln
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_kernels.py tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dln/tests.log 2>&1
timeout -k 10 300 python -u tools/decode_ab.py > gpurun_out/dln/ab.txt 2>&1
DEC_B=64 DEC_DT=f16 timeout -k 10 300 python -u tools/decode_ab.py > gpurun_out/dln/ab64.txt 2>&1
