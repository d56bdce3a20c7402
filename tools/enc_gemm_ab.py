"""The encoder's 2048-row GEMMs (B = 16 x 128 tokens) under each kernel the planner could give
them (dev tool, GPU): v8 (64 x 64 tiles, no split-K; the auto plan when v7 would run <= 64
tiles) against v7 with split-K 2..8 (slabs + a reduce launch that applies the epilogue), each
as 10 launches replayed from a hipGraph; outputs checked against the auto plan's.

    python tools/enc_gemm_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402

SHAPES = [  # name, m, n, k, trans_b (dgrad), a_conv
    ("enc conv fwd", 2048, 512, 2560, False, (128, 512, 2)),
    ("enc ffn2 fwd", 2048, 512, 2048, False, None),
    ("enc o fwd", 2048, 512, 512, False, None),
    ("enc ffn1 dgrad", 2048, 512, 2048, True, None),
    ("enc qkv dgrad", 2048, 512, 1536, True, None),
    ("enc conv dgrad", 2048, 512, 2560, False, (128, 512, 2)),
]


def main():
    torch.manual_seed(0)
    ws = ops.Workspace()
    for name, m, n, k, tb, conv in SHAPES:
        lda = k if conv is None else conv[1]
        a = (torch.randn(m, lda, device="cuda") * 0.5).bfloat16()
        b = (torch.randn(k, n, device="cuda") * 0.05).bfloat16() if tb else \
            (torch.randn(n, k, device="cuda") * 0.05).bfloat16()
        bias = torch.randn(n, device="cuda") * 0.1
        ref = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        ldb = n if tb else k
        kw = dict(trans_b=tb, a_conv=conv, ws=ws) | ({} if tb else dict(bias=bias))
        res = []
        for var, sp in [(0, 1), (13, 2), (13, 4), (13, 5), (13, 8)]:
            out = torch.empty_like(ref)
            fn = lambda: ops.gemm(a, b, out, m, n, k, lda, ldb, n, variant=var, splits=sp, **kw)  # noqa: E731
            g = graph_of(fn)
            t = min(time_graph(g) for _ in range(3))
            del g
            if var == 0:
                ref.copy_(out)
                err = 0.0
            else:
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
            res.append(f"{'auto' if var == 0 else f'v7 sp{sp}'} {t * 1e6:6.1f} us (err {err:.1e})")
        print(f"{name:16s} " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
