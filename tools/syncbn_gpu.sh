set -e
mkdir -p gpurun_out/sbn
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_syncbn.py tests/test_gpu_dist.py > gpurun_out/sbn/tests.log 2>&1
