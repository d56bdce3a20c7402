"""Post-net conv as an implicit GEMM vs the plain GEMM of the same size (dev tool, GPU):
what the loaders' conv tracking costs.   python tools/gemm_conv.py [variant]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_fixed import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

var = int(sys.argv[1]) if len(sys.argv) > 1 else 0
KW = 5
for B, T, cin, cout in ((16, 800, 512, 512), (16, 800, 80, 512), (16, 800, 512, 80), (16, 128, 512, 512)):
    M = B * T
    K = KW * cin
    X = torch.randn(M, cin, device="cuda").bfloat16()
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(cout, K, device="cuda").bfloat16()
    Y = torch.empty(M, cout, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(cout, device="cuda")
    tc = timeit(lambda: ops.gemm(X, W, Y, M, cout, K, cin, K, cout, bias=bias, a_conv=(T, cin, 2), variant=var))
    tp = timeit(lambda: ops.gemm(A, W, Y, M, cout, K, K, K, cout, bias=bias, variant=var))
    print(f"conv {cin}->{cout} (M {M}, K {K}): implicit {tc * 1e6:6.1f} us | plain GEMM {tp * 1e6:6.1f} us",
          flush=True)
