"""Sweep GEMM variants x split-K counts on a few shapes (dev tool, GPU).

    python tools/gemm_sweep.py "m,n,k,ta,tb;..." "variants" "splits"
e.g. python tools/gemm_sweep.py "512,512,12800,1,1" "2,5,7" "8,16,32"

Prints the time with the split-K reduce and the main kernel alone (main_only).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402


def main(shapes, variants, splits):
    for sh in shapes.split(";"):
        m, n, k, ta, tb = (int(x) for x in sh.split(","))
        A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
        B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
        C = torch.empty(m, n, device="cuda", dtype=torch.float32 if ta else torch.bfloat16)
        fl = 2.0 * m * n * k
        for v in (int(x) for x in variants.split(",")):
            row = []
            for sp in (int(x) for x in splits.split(",")):
                kw = dict(trans_a=bool(ta), trans_b=bool(tb), variant=v, splits=sp)
                try:
                    t = timeit(lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, **kw))
                    tm = timeit(lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, main_only=True, **kw))
                    row.append(f"sp{sp:<2d} {t * 1e6:6.1f} ({tm * 1e6:5.1f}) {fl / t / 1e12:4.0f}TF")
                except Exception as e:  # noqa: BLE001
                    row.append(f"sp{sp:<2d} err {str(e)[:30]}")
            print(f"{m}x{n}x{k} ta{ta} tb{tb} v{v:<2d} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:4])
