"""Encoder-shape GEMMs (M = 2048): each plan / split-K factor timed as 10 whole tt2_gemm calls
(main kernel + split-K reduce) replayed from a hipGraph, best of 3, output checked against the
first arm (dev tool, GPU).

    python tools/enc_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from v9_ab import graph_of, time_graph, ops, ACT_RELU  # noqa: E402

SHAPES = [  # name, m, n, k, trans_b, epilogue
    ("ffn2 fwd", 2048, 512, 2048, False, "b"),
    ("ffn1 dgrad", 2048, 512, 2048, True, "res"),
    ("qkv dgrad", 2048, 512, 1536, True, "res"),
    ("o fwd", 2048, 512, 512, False, "b"),
    ("ffn1 fwd", 2048, 2048, 512, False, "brd"),
    ("ffn2 dgrad", 2048, 2048, 512, True, "gate"),
    ("qkv fwd", 2048, 1536, 512, False, "b"),
]
ARMS = [(0, 1), (15, 1), (13, 1), (13, 2), (13, 4), (13, 8)]


def main():
    torch.manual_seed(0)
    seed = torch.tensor([99], dtype=torch.int32, device="cuda")
    ws = ops.Workspace()
    for name, m, n, k, tb, epi in SHAPES:
        A = torch.randn(m, k, device="cuda").bfloat16()
        B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16() / k ** 0.5
        X = torch.randn(m, n, device="cuda").bfloat16()
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(n, device="cuda")
        if "r" in epi and epi != "res":
            kw["act"] = ACT_RELU
        if "d" in epi:
            kw["drop"] = ops.Drop(seed, 5, 0.1)
        if epi == "gate":
            kw.update(gate=X.relu(), ldg=n, gate_scale=1.1)
        if epi == "res":
            kw.update(res=X, ldr=n)
        ref = None
        line = f"{name:11s} {m}x{n}x{k}:"
        for var, sp in ARMS:
            C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
            fn = (lambda C=C, var=var, sp=sp: ops.gemm(A, B, C, m, n, k, k, B.shape[1], n, trans_b=tb, variant=var,
                                                       splits=sp, ws=ws, **kw))
            try:
                g = graph_of(fn)
            except Exception as ex:   # an arm this request cannot take
                line += f" | v{var}s{sp} n/a"
                continue
            t = min(time_graph(g) for _ in range(3))
            if ref is None:
                ref = C.double()
            err = ((C.double() - ref).norm() / ref.norm()).item()
            line += f" | v{var}s{sp} {t * 1e6:5.1f}us{'' if err < 1e-2 else ' BAD%.0e' % err}"
            del g
        print(line, flush=True)


if __name__ == "__main__":
    main()
