"""Run one GEMM shape repeatedly (dev tool, for rocprofv3 counter passes).

    python tools/gemm_one.py m n k ta tb variant [splits] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

m, n, k, ta, tb, var = (int(x) for x in sys.argv[1:7])
sp = int(sys.argv[7]) if len(sys.argv) > 7 else 1
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 20
A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
t = timeit(lambda: ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, trans_a=bool(ta), trans_b=bool(tb),
                            variant=var, splits=sp), iters=reps)
print(f"{m}x{n}x{k} ta{ta} tb{tb} v{var} sp{sp}: {t * 1e6:.1f} us {2.0 * m * n * k / t / 1e12:.0f} TF")
