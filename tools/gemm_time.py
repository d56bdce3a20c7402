"""Times the training step's GEMM shapes under the auto plan (dev tool, GPU): 10 launches
replayed from a hipGraph, best of 3 rounds; prints us and TF/s per shape and a checksum so two
builds / settings can be compared (`TT2_G7_PF=0|1 python tools/gemm_time.py`).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import SHAPES, graph_of, time_graph, ops, ACT_RELU  # noqa: E402


def main():
    torch.manual_seed(0)
    seed = torch.tensor([99], dtype=torch.int32, device="cuda")
    for name, m, n, k, tb, epi, conv in SHAPES:
        lda = k if conv is None else conv[1]
        A = torch.randn(m, lda, device="cuda").bfloat16()
        B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16() / k ** 0.5
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(n, device="cuda")
        if "r" in epi and epi != "res":
            kw["act"] = ACT_RELU
        if "d" in epi:
            kw["drop"] = ops.Drop(seed, 5, 0.1)
        X = torch.randn(m, n, device="cuda").bfloat16()
        if epi == "gate":
            kw.update(gate=X.relu(), ldg=n, gate_scale=1.1)
        if epi == "res":
            kw.update(res=X, ldr=n)
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        g = graph_of(lambda: ops.gemm(A, B, C, m, n, k, lda, B.shape[1], n, trans_b=tb, a_conv=conv, **kw))
        t = min(time_graph(g) for _ in range(3))
        print(f"{name:22s} {m}x{n}x{k}: {t * 1e6:7.1f} us {2.0 * m * n * k / t / 1e12:6.0f} TF  "
              f"sum {C.double().sum().item():.6e}", flush=True)
        del g


if __name__ == "__main__":
    main()
