"""Weight-gradient GEMM shapes of the decoder (K = 12800 tokens, both operands M/N-
contiguous) with and without the fused bias-gradient row sums (a_ksum) (dev tool, GPU).
    python tools/gemm_wgrad.py [variant]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_fixed import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

var = int(sys.argv[1]) if len(sys.argv) > 1 else 0
K = 12800
ws = ops.Workspace()
for m, n in ((512, 512), (1536, 512), (2048, 512), (512, 2048)):
    dY = torch.randn(K, m, device="cuda").bfloat16()
    X = torch.randn(K, n, device="cuda").bfloat16()
    dW = torch.empty(m, n, device="cuda")
    ks = torch.empty(m, device="cuda")
    row = []
    for sp in (1, 2, 4):
        for use_ks in (False, True):
            kw = dict(trans_a=True, trans_b=True, splits=sp, ws=ws, variant=var)
            if use_ks:
                kw["a_ksum"] = ks
            t = timeit(lambda: ops.gemm(dY, X, dW, m, n, K, m, n, n, **kw), iters=10)
            row.append(f"s{sp}{'+ks' if use_ks else ''} {t * 1e6:6.1f}")
    print(f"{m}x{n}x{K}: " + " | ".join(row), flush=True)
