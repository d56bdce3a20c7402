"""v8 (forced variant 15) time against K at M = 2048, N = 512 (dev tool, GPU; TT2_LIB picks the build):
the slope is the in-kernel cost of a 64-deep K step, the intercept the fixed cost of a tile.

    python tools/g8_ksweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402

m, n = 2048, 512
res = []
for k in (256, 512, 1024, 2048, 4096, 8192):
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    g = graph_of(lambda: ops.gemm(A, B, C, m, n, k, k, k, n, variant=15))
    t = min(time_graph(g) for _ in range(3))
    res.append((k, t * 1e6))
    del g
ks = [k for k, _ in res]
ts = [t for _, t in res]
kbar, tbar = sum(ks) / len(ks), sum(ts) / len(ts)
slope = sum((k - kbar) * (t - tbar) for k, t in res) / sum((k - kbar) ** 2 for k in ks)
print(f"lib {os.environ.get('TT2_LIB', 'default')}: " + " ".join(f"K{k} {t:.1f}" for k, t in res) +
      f" | {slope * 64 * 1e3:.0f} ns per 64-deep step ({slope * 64 * 2.4e3:.0f} cycles at 2.4 GHz), "
      f"intercept {tbar - slope * kbar:.1f} us")
