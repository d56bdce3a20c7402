"""LayerNorm backward A/B on the decoder shape (dev tool, GPU): M=12800, C=512, bf16,
dropout + dbias, timed with events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

for m in (12800, 2048):
    C = 512
    x, br, dy = (torch.randn(m, C, device="cuda").bfloat16() for _ in range(3))
    gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    mean, rstd = torch.zeros(m, device="cuda"), torch.ones(m, device="cuda")
    dx, dbr = torch.empty_like(x), torch.empty_like(x)
    dg, db, dbias = (torch.empty(C, device="cuda") for _ in range(3))
    seed = torch.tensor([3], dtype=torch.int32, device="cuda")
    drop = ops.Drop(seed, 9, float(os.environ.get("TT2_P", "0.1")))
    t = timeit(lambda: ops.layernorm_bwd(dy, x, br, gamma, mean, rstd, dx, dbr, dg, db, m, drop=drop, dbias=dbias))
    y = torch.empty_like(x)
    t2 = timeit(lambda: ops.layernorm_fwd(x, br, gamma, beta, y, mean, rstd, m, drop=drop))
    print(f"M={m}: bwd {t * 1e6:.1f} us  fwd {t2 * 1e6:.1f} us", flush=True)
