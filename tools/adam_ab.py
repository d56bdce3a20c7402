"""The fused Adam update over the model's 52.99M parameters (dev tool, GPU): 10 launches replayed
from a hipGraph, best of 3, with HBM GB/s at 30 B per parameter (p, m, v read + written, g read,
bf16 shadow written).  TT2_LIB=abl/<variant>.so compares builds.

    python tools/adam_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402


def main():
    n = 52986691 // 16 * 16
    p = torch.randn(n, device="cuda") * 0.02
    g = torch.randn(n, device="cuda") * 1e-3
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    sh = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    step = torch.zeros(1, dtype=torch.int32, device="cuda")
    ws = ops.Workspace()
    parts = torch.full((64,), 1e-3, device="cuda")
    fn = lambda: ops.adam_step(p, g, m, v, sh, step, n, 1e-3, ws=ws, norm_parts=parts)  # noqa: E731
    t = min(time_graph(graph_of(fn)) for _ in range(3))
    print(f"lib {os.environ.get('TT2_LIB', 'default')}: adam {n} params {t * 1e6:.1f} us "
          f"{30.0 * n / t / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
