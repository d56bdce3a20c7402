"""Epilogue cost of the v7 GEMM (dev tool, GPU): the same GEMM with no epilogue operands,
bias only, bias + bf16 residual, bias + residual + relu gate."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

for m, n, k in [(12800, 512, 512), (12800, 512, 2048), (12800, 2048, 512), (2048, 512, 512)]:
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = torch.randn(n, k, device="cuda").bfloat16()
    C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    R = torch.randn(m, n, device="cuda").bfloat16()
    G = torch.randn(m, n, device="cuda").bfloat16()
    bias = torch.randn(n, device="cuda")
    row = []
    for name, kw in [("none", {}), ("bias", dict(bias=bias)), ("bias+res", dict(bias=bias, res=R, ldr=n)),
                     ("bias+res+gate", dict(bias=bias, res=R, ldr=n, gate=G, ldg=n))]:
        t = timeit(lambda: ops.gemm(A, B, C, m, n, k, k, k, n, **kw))
        row.append(f"{name} {t * 1e6:6.1f}")
    print(f"{m}x{n}x{k}: " + " | ".join(row), flush=True)
