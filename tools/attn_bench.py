"""The training step's attention launches on their own (dev tool, GPU): decoder causal
self-attention (B=16, H=8, 800 x 800), cross-attention (800 queries x 128 keys) and encoder
self-attention (128 x 128), forward and backward, bf16, each as 10 launches replayed from a
hipGraph (best of 3); prints us, TFLOP/s (causal counted half) and a checksum.

    python tools/attn_bench.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402

B, H, D = 16, 8, 64
CASES = [("dec self causal", 800, 800, True), ("cross", 800, 128, False), ("enc self", 128, 128, False)]


def main():
    torch.manual_seed(0)
    for name, tq, tk, causal in CASES:
        d = H * D
        qkv = (torch.randn(B * tq, 3 * d, device="cuda") * 0.5).bfloat16()
        kv = (torch.randn(B * tk, 2 * d, device="cuda") * 0.5).bfloat16()
        q, k, v = (qkv, qkv[:, d:], qkv[:, 2 * d:]) if tq == tk else (qkv, kv, kv[:, d:])
        qld, kld = 3 * d, (3 * d if tq == tk else 2 * d)
        out = torch.empty(B * tq, d, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H, tq, device="cuda")
        klen = torch.full((B,), tk, dtype=torch.int32, device="cuda")
        fwd = lambda: ops.attn_fwd(q, k, v, out, lse, qld, kld, kld, d, B, H, tq, tk, klen, causal, 0.125)  # noqa
        g = graph_of(fwd)
        tf = min(time_graph(g) for _ in range(3))
        del g
        dout = (torch.randn(B * tq, d, device="cuda") * 0.1).bfloat16()
        dq = torch.empty(B * tq, d, device="cuda", dtype=torch.bfloat16)
        dk = torch.empty(B * tk, d, device="cuda", dtype=torch.bfloat16)
        dv = torch.empty(B * tk, d, device="cuda", dtype=torch.bfloat16)
        delta = torch.empty(B * H, max(tq, tk), device="cuda")
        bwd = lambda: ops.attn_bwd(q, k, v, out, dout, lse, delta, dq, dk, dv, qld, kld, kld, d, d, d, d, d,  # noqa
                                   B, H, tq, tk, klen, causal, 0.125)
        g = graph_of(bwd)
        tb = min(time_graph(g) for _ in range(3))
        del g
        fl = 4.0 * B * H * tq * tk * D * (0.5 if causal else 1.0)
        print(f"{name:16s} fwd {tf * 1e6:6.1f} us {fl / tf / 1e12:5.0f} TF | bwd {tb * 1e6:6.1f} us "
              f"{2.5 * fl / tb / 1e12:5.0f} TF | sum {out.float().sum().item():.5e} {dq.float().sum().item():.5e}",
              flush=True)


if __name__ == "__main__":
    main()
