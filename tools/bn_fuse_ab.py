"""Cost of the fused BatchNorm statistics epilogues (dev tool, GPU): the post-net conv
(12800 x 512 x 2560, 256 x 128 kernel) and the encoder pre-net conv (2048 x 512 x 2560, 64 x 64
kernel) plain, with col_stats (forward moments) and with bn_bwd (backward sums, tanh / ReLU,
dropout); 10 launches replayed from a hipGraph, best of 3.

    python tools/bn_fuse_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402
from tt2._lib import ACT_RELU, ACT_TANH  # noqa: E402


def main():
    torch.manual_seed(0)
    for m, T, act in ((12800, 800, ACT_TANH), (2048, 128, ACT_RELU)):
        c, K = 512, 5
        k = K * c
        x = torch.randn(m, c, device="cuda").bfloat16()
        w = (torch.randn(c, k, device="cuda") / k ** 0.5).bfloat16()
        b = torch.randn(c, device="cuda") * 0.1
        y = torch.empty(m, c, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(y)
        conv = (T, c, 2)
        rows = ops.gemm_stats_rows(x, w, out, m, c, k, c, k, c, bias=b, a_conv=conv)
        st = torch.empty(2 * ((m + rows - 1) // rows) * c, device="cuda")
        g, be = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
        mean, rstd = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
        seed = torch.tensor([3], dtype=torch.int32, device="cuda")
        bnb = ops.bn_bwd_args(y, g, be, mean, rstd, m, c, act, ops.Drop(seed, 40, 0.5), (st, rows))
        forms = {"plain": lambda: ops.gemm(x, w, out, m, c, k, c, k, c, bias=b, a_conv=conv),
                 "col_stats": lambda: ops.gemm(x, w, out, m, c, k, c, k, c, bias=b, a_conv=conv, col_stats=st),
                 "bn_bwd": lambda: ops.gemm(x, w, out, m, c, k, c, k, c, a_conv=conv, bn_bwd=bnb)}
        for name, fn in forms.items():
            t = min(time_graph(graph_of(fn)) for _ in range(3))
            print(f"{m}x{c}x{k} ({rows}-row chunks) {name:10s} {t * 1e6:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
