"""Time GEMM shapes in both operand layouts (dev tool, GPU): each as 10 launches replayed from a
hipGraph (best of 3), f32 C as the weight gradients write it.

    python tools/gemm_one.py m n k [splits ...]

For every split factor: the weight-gradient layout (trans_a, trans_b: both operands token-major,
as dY and X sit in memory) and the NT layout (both K-contiguous, as after an explicit transpose).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402


def main():
    m, n, k = (int(x) for x in sys.argv[1:4])
    splits = [int(x) for x in sys.argv[4:]] or [1]
    torch.manual_seed(0)
    ws = ops.Workspace()
    for ta in (1, 0):
        A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
        B = torch.randn((k, n) if ta else (n, k), device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda")
        for sp in splits:
            fn = lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, trans_a=bool(ta),  # noqa: E731
                                  trans_b=bool(ta), splits=sp, ws=ws)
            t = min(time_graph(graph_of(fn)) for _ in range(3))
            print(f"{m}x{n}x{k} {'TT (token-major)' if ta else 'NT (K-contig.) '} splits {sp}: {t * 1e6:8.1f} us "
                  f"{2.0 * m * n * k / t / 1e12:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
