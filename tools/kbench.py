"""Kernel micro-benchmarks on the GPU (dev tool): tt2 GEMM vs torch.matmul."""
import os
import sys
import time

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


def gemm_bench():
    shapes = [  # (name, m, n, k, ta, tb, splits)
        ("ffn1 fwd", 12800, 2048, 512, False, False, 1),
        ("ffn2 fwd", 12800, 512, 2048, False, False, 1),
        ("qkv fwd", 12800, 1536, 512, False, False, 1),
        ("ffn2 dgrad", 12800, 2048, 512, False, True, 1),
        ("ffn1 wgrad", 2048, 512, 12800, True, True, 4),
        ("o wgrad", 512, 512, 12800, True, True, 16),
        ("sq 4096", 4096, 4096, 4096, False, False, 1),
    ]
    for name, m, n, k, ta, tb, sp in shapes:
        A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
        B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, trans_a=ta, trans_b=tb, splits=sp))
        Am = A.t() if ta else A
        Bm = B if tb else B.t()
        tr = timeit(lambda: torch.matmul(Am, Bm))
        fl = 2.0 * m * n * k
        print(f"{name:12s} m={m} n={n} k={k}: tt2 {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF | torch {tr*1e6:8.1f} us "
              f"{fl/tr/1e12:7.1f} TF", flush=True)


if __name__ == "__main__":
    gemm_bench()
