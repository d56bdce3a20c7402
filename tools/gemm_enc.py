"""Encoder-shape GEMMs (M = 2048 tokens) per kernel variant (dev tool, GPU): where the
256 x 128 v7 tiles leave most CUs idle.   python tools/gemm_enc.py [variants...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402


def timeit(fn, iters=50):
    """Per-call device time of fn from a graph of `iters` calls (no host launch cost)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters) * 1e-3

SHAPES = [  # name, m, n, k, trans_b
    ("qkv fwd", 2048, 1536, 512, False), ("o fwd", 2048, 512, 512, False), ("ffn1 fwd", 2048, 2048, 512, False),
    ("ffn2 fwd", 2048, 512, 2048, False), ("mkv fwd", 2048, 6144, 512, False),
    ("qkv dgrad", 2048, 512, 1536, True), ("o dgrad", 2048, 512, 512, True), ("ffn1 dgrad", 2048, 512, 2048, True),
    ("ffn2 dgrad", 2048, 2048, 512, True), ("dec o fwd", 12800, 512, 512, False),
    ("pre fc1", 12800, 256, 80, False), ("pre fc2", 12800, 256, 256, False), ("pre proj", 12800, 512, 256, False),
    ("fc2 dgrad", 12800, 256, 256, True), ("proj dgrad", 12800, 256, 512, True),
]
if os.environ.get("ONLY_NEW"):
    SHAPES = SHAPES[-5:]
variants = [int(v) for v in sys.argv[1:]] or [2, 13]
ws = ops.Workspace() if hasattr(ops, "Workspace") else None
for name, m, n, k, tb in SHAPES:
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16()
    C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(n, device="cuda")
    row = []
    for v in variants:
        for sp in (1, 2, 4):
            if sp > 1 and k < 1024:
                continue
            kw = dict(trans_b=tb, variant=v, splits=sp)
            if sp > 1:
                kw["ws"] = ws
            if not tb:
                kw["bias"] = bias
            try:
                t = timeit(lambda: ops.gemm(A, B, C, m, n, k, k, B.shape[1], n, **kw), iters=50)
                row.append(f"v{v}/s{sp} {t * 1e6:6.1f}us")
            except Exception as e:  # noqa: BLE001
                row.append(f"v{v}/s{sp} n/a")
    print(f"{name:11s} {m}x{n}x{k}: " + " | ".join(row), flush=True)
