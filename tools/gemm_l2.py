"""GEMM operand-source experiment (dev tool, GPU): the same launch with normal
operands vs leading dimension 0 (every row aliases row 0, so all operand reads
are L2 hits).  Separates operand-fetch latency/bandwidth beyond L2 from the
in-CU pipeline limit.

    python tools/gemm_l2.py "m,n,k,ta,tb,var,splits;..."
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from tt2 import ops  # noqa: E402

for sh in sys.argv[1].split(";"):
    m, n, k, ta, tb, var, sp = (int(x) for x in sh.split(","))
    A = torch.randn((k, m) if ta else (m, k), device="cuda").bfloat16()
    B = torch.randn((k, n) if tb else (n, k), device="cuda").bfloat16()
    C = torch.empty(m, n, device="cuda", dtype=torch.float32 if ta else torch.bfloat16)
    fl = 2.0 * m * n * k
    out = []
    for la, lb, tag in ((A.shape[1], B.shape[1], "normal"), (0, B.shape[1], "A-L2"), (A.shape[1], 0, "B-L2"),
                        (0, 0, "both-L2")):
        t = timeit(lambda: ops.gemm(A, B, C, m, n, k, la, lb, n, trans_a=bool(ta), trans_b=bool(tb), variant=var,
                                    splits=sp, main_only=True))
        out.append(f"{tag} {t * 1e6:6.1f}us {fl / t / 1e12:4.0f}TF")
    print(f"{m}x{n}x{k} ta{ta} tb{tb} v{var} sp{sp}: " + " | ".join(out), flush=True)
