"""Attention kernel micro-benchmark on the GPU (dev tool).

Times tt2_attn_fwd / tt2_attn_bwd at the three attention shapes of the bench
workload (B=16, H=8, text 128, mel 800) for each kernel variant and prints
achieved TFLOP/s (causal FLOPs counted over the visible triangle only).

    python tools/attn_bench.py [variants...]      (default: 1 2 3)
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


B, H, D = 16, 8, 64
SHAPES = [  # name, Tq, Tk, causal, packed
    ("enc self", 128, 128, False, True),
    ("dec self", 800, 800, True, True),
    ("cross", 800, 128, False, False),
]


def run(variant):
    ops.ATTN_VARIANT = variant
    g = torch.Generator(device="cuda").manual_seed(0)
    HD = H * D
    for name, Tq, Tk, causal, packed in SHAPES:
        if packed:
            qkv = torch.randn(B * Tq, 3 * HD, device="cuda", generator=g).bfloat16()
            q, k, v = qkv[:, :HD], qkv[:, HD:2 * HD], qkv[:, 2 * HD:]
            lq = lk = lv = 3 * HD
        else:
            q = torch.randn(B * Tq, HD, device="cuda", generator=g).bfloat16()
            kv = torch.randn(B * Tk, 2 * HD, device="cuda", generator=g).bfloat16()
            k, v = kv[:, :HD], kv[:, HD:]
            lq, lk, lv = HD, 2 * HD, 2 * HD
        klen = torch.full((B,), Tk, dtype=torch.int32, device="cuda")
        out = torch.empty(B * Tq, HD, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(B * H, Tq, device="cuda")
        dout = torch.randn(B * Tq, HD, device="cuda", generator=g).bfloat16()
        delta = torch.empty(B * H, Tq, device="cuda")
        dq = torch.empty(B * Tq, HD, dtype=torch.bfloat16, device="cuda")
        dkv = torch.empty(B * Tk, 2 * HD, dtype=torch.bfloat16, device="cuda")
        scale = 1.0 / math.sqrt(D)

        def fwd():
            ops.attn_fwd(q, k, v, out, lse, lq, lk, lv, HD, B, H, Tq, Tk, klen, causal, scale)

        def bwd():
            ops.attn_bwd(q, k, v, out, dout, lse, delta, dq, dkv[:, :HD], dkv[:, HD:], lq, lk, lv, HD, HD, HD,
                         2 * HD, 2 * HD, B, H, Tq, Tk, klen, causal, scale)

        pairs = B * H * (Tq * (Tq + 1) / 2 if causal else Tq * Tk)
        tf = timeit(fwd)
        fwd()
        tb = timeit(bwd)
        print(f"v{variant} {name:9s} fwd {tf * 1e6:7.1f} us {4 * pairs * D / tf / 1e12:6.1f} TF | "
              f"bwd {tb * 1e6:7.1f} us {10 * pairs * D / tb / 1e12:6.1f} TF", flush=True)


if __name__ == "__main__":
    for v in [int(x) for x in sys.argv[1:]] or [1, 2, 3]:
        run(v)
