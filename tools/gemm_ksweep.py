"""K sweep of the v7 GEMM at the step's row count (dev tool, GPU): time per launch vs K
for N = 512 / 1536 / 2048, no epilogue and bias epilogue, to split fixed cost from the
per-K-step cost.   python tools/gemm_ksweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

m = 12800
for n in (512, 2048):
    for k in (64, 128, 256, 512, 1024, 2048):
        A = torch.randn(m, k, device="cuda").bfloat16()
        B = torch.randn(n, k, device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        bias = torch.randn(n, device="cuda")
        t0 = timeit(lambda: ops.gemm(A, B, C, m, n, k, k, k, n))
        t1 = timeit(lambda: ops.gemm(A, B, C, m, n, k, k, k, n, bias=bias))
        print(f"{m}x{n}x{k}: none {t0 * 1e6:6.1f} us | bias {t1 * 1e6:6.1f} us | {2.0 * m * n * k / t1 / 1e12:6.0f} TF",
              flush=True)
