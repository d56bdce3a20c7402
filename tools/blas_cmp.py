"""The training step's GEMM shapes: libtt2's auto plan (no epilogue) against torch.matmul
(hipBLASLt) on the same bf16 operands, each as 10 launches replayed from a hipGraph, best of 3
(dev tool, GPU; a yardstick for the v7 tiles, not part of the product)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402

SHAPES = [(12800, 2048, 512), (12800, 1536, 512), (12800, 512, 512), (12800, 512, 2048), (2048, 6144, 512),
          (2048, 2048, 512), (2048, 512, 2048), (4096, 4096, 4096), (8192, 8192, 8192)]
# `enc`: the encoder chain's 2048-row products (forward QKV / o / FFN1 / FFN2 / pre-net conv as a plain
# K = 2560 GEMM, and the dgrads' M x N x K: o, qkv, FFN1)
ENC_SHAPES = [(2048, 1536, 512), (2048, 512, 512), (2048, 2048, 512), (2048, 512, 2048), (2048, 512, 2560),
              (2048, 512, 1536)]


def main():
    torch.manual_seed(0)
    for m, n, k in (ENC_SHAPES if "enc" in sys.argv[1:] else SHAPES):
        A = torch.randn(m, k, device="cuda").bfloat16()
        B = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        C2 = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        g1 = graph_of(lambda: ops.gemm(A, B, C, m, n, k, k, k, n))
        g2 = graph_of(lambda: torch.mm(A, B.t(), out=C2))
        t1 = min(time_graph(g1) for _ in range(3))
        t2 = min(time_graph(g2) for _ in range(3))
        f = 2.0 * m * n * k
        err = ((C.float() - C2.float()).norm() / C2.float().norm()).item()
        print(f"{m}x{n}x{k}: tt2 {t1 * 1e6:7.1f} us {f / t1 / 1e12:6.0f} TF | hipBLASLt {t2 * 1e6:7.1f} us "
              f"{f / t2 / 1e12:6.0f} TF | ratio {t2 / t1:.2f} | diff {err:.1e}", flush=True)
        del g1, g2


if __name__ == "__main__":
    main()
