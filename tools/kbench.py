"""Kernel micro-benchmarks on the GPU (dev tool): tt2 GEMM variants vs torch.matmul."""
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


SHAPES = [  # (name, m, n, k, ta, tb, splits, a_conv)
    ("ffn1 fwd", 12800, 2048, 512, False, False, 1, None),
    ("ffn2 fwd", 12800, 512, 2048, False, False, 1, None),
    ("qkv fwd", 12800, 1536, 512, False, False, 1, None),
    ("o fwd", 12800, 512, 512, False, False, 1, None),
    ("conv fwd", 12800, 512, 2560, False, False, 1, (800, 512, 2)),
    ("ffn2 dgrad", 12800, 2048, 512, False, True, 1, None),
    ("ffn1 dgrad", 12800, 512, 2048, False, True, 1, None),
    ("ffn1 wgrad", 2048, 512, 12800, True, True, 4, None),
    ("o wgrad", 512, 512, 12800, True, True, 16, None),
    ("sq 4096", 4096, 4096, 4096, False, False, 1, None),
]


def gemm_bench(variants):
    for name, m, n, k, ta, tb, sp, conv in SHAPES:
        lda = (m if ta else k) if conv is None else conv[1]
        A = torch.randn((k, m) if ta else (m, lda if conv else k), device="cuda").bfloat16()
        B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * m * n * k
        res = []
        for v in variants:
            t = timeit(lambda: ops.gemm(A, B, C, m, n, k, lda, B.shape[1], n, trans_a=ta, trans_b=tb, splits=sp,
                                        a_conv=conv, variant=v))
            res.append(f"v{v} {fl / t / 1e12:6.1f}")
        tr = None
        if conv is None:
            Am = A.t() if ta else A
            Bm = B if tb else B.t()
            tr = timeit(lambda: torch.matmul(Am, Bm))
        print(f"{name:12s} {m}x{n}x{k}: " + " | ".join(res) +
              (f" | torch {fl / tr / 1e12:6.1f} TF" if tr else ""), flush=True)


if __name__ == "__main__":
    vs = [int(x) for x in sys.argv[1:]] or [2, 13]
    gemm_bench(vs)
