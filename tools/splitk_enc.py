"""Split-K on the encoder's long-K 2048-row products (dev tool, GPU): the auto plan (v8, no split)
against v7 / v2 with split-K factors (slabs + the fixed-order reduce launch), us per launch."""
import os, sys
sys.path.insert(0, "/root/repo/tools")
import torch
from gemm_ab import graph_of, time_graph, ops
ws = ops.Workspace()
for (m, n, k, tb, conv) in [(2048, 512, 2048, False, None), (2048, 512, 2560, False, (128, 512, 2)), (2048, 512, 2048, True, None), (2048, 512, 1536, True, None)]:
    lda = k if conv is None else conv[1]
    A = torch.randn(m, lda, device="cuda").bfloat16()
    B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16() / k ** 0.5
    bias = torch.randn(n, device="cuda")
    out = []
    for var, sp in ((0, 1), (13, 1), (13, 2), (13, 4), (13, 8), (2, 4), (2, 8)):
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        g = graph_of(lambda: ops.gemm(A, B, C, m, n, k, lda, B.shape[1], n, trans_b=tb, a_conv=conv, bias=bias, splits=sp, ws=ws, variant=var))
        t = min(time_graph(g) for _ in range(3))
        out.append(f"v{var}/sp{sp} {t*1e6:.1f}")
        del g
    print(f"{m}x{n}x{k} tb={tb} conv={conv is not None}: " + " | ".join(out), flush=True)
