"""GEMM epilogue cost on the FFN1 shape (dev tool, GPU): same GEMM, epilogue
options added one at a time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402

m, n, k = 12800, 2048, 512
A = torch.randn(m, k, device="cuda").bfloat16()
B = torch.randn(n, k, device="cuda").bfloat16()
bias = torch.randn(n, device="cuda")
G = torch.randn(m, n, device="cuda").bfloat16()
C16 = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
C32 = torch.empty(m, n, device="cuda", dtype=torch.float32)
seed = torch.tensor([5], dtype=torch.int32, device="cuda")
fl = 2.0 * m * n * k
cases = [
    ("f32 out", dict(c=C32)),
    ("bf16 out", dict(c=C16)),
    ("+bias", dict(c=C16, bias=bias)),
    ("+bias+relu", dict(c=C16, bias=bias, act=ACT_RELU)),
    ("+bias+relu+drop", dict(c=C16, bias=bias, act=ACT_RELU, drop=ops.Drop(seed, 3, 0.1))),
    ("gate", dict(c=C16, gate=G, ldg=n, gate_scale=1.1)),
    ("gate (B^T)", dict(c=C16, gate=G, ldg=n, gate_scale=1.1, tb=True)),
    ("res", dict(c=C16, res=G, ldr=n)),
]
for name, kw in cases:
    c = kw.pop("c")
    tb = kw.pop("tb", False)
    Bm = B.t().contiguous() if tb else B
    t = timeit(lambda: ops.gemm(A, Bm, c, m, n, k, k, Bm.shape[1], n, trans_b=tb, **kw))
    print(f"{name:18s} {t * 1e6:7.1f} us {fl / t / 1e12:6.0f} TF", flush=True)
