mkdir -p gpurun_out/diag1
timeout -k 10 300 env TT2_ENC_OVERLAP=0 python -u -m pytest tests/test_gpu_dist.py -x -v -k "captured_rccl or dp_graph" --timeout 200 --timeout-method thread > gpurun_out/diag1/enc0.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v -k "captured_rccl or dp_graph" --timeout 200 --timeout-method thread > gpurun_out/diag1/enc1.log 2>&1
