"""GEMM time inside a graph chain (dev tool, GPU): each configuration is captured 20x back
to back in a torch CUDA graph and replayed, so host launch cost is excluded (the eager
timers in gemm_sweep.py are host-bound below ~12 us).

    python tools/gemm_graph.py "m,n,k,ta,tb;..." "variants" "splits"
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from decode_kern import graph_time  # noqa: E402
from tt2 import ops  # noqa: E402


def main(shapes, variants, splits):
    for sh in shapes.split(";"):
        m, n, k, ta, tb = (int(x) for x in sh.split(","))
        A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
        B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.float32 if ta else torch.bfloat16)
        fl = 2.0 * m * n * k
        ws = ops.Workspace()
        for v in (int(x) for x in variants.split(",")):
            row = []
            for sp in (int(x) for x in splits.split(",")):
                kw = dict(trans_a=bool(ta), trans_b=bool(tb), variant=v, splits=sp, ws=ws)
                try:
                    ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, **kw)
                    t = graph_time(lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, **kw)) * 1e-6
                    row.append(f"sp{sp:<2d} {t * 1e6:6.1f} {fl / t / 1e12:5.0f}TF")
                except Exception as e:  # noqa: BLE001
                    row.append(f"sp{sp:<2d} err {str(e)[:30]}")
            print(f"{m}x{n}x{k} ta{ta} tb{tb} v{v:<2d} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:4])
