"""The training step's LayerNorm / BatchNorm passes on their own (dev tool, GPU): the decoder's
LayerNorm forward and backward (12800 x 512, residual branch, dropout) and the post-net's BatchNorm forward
and backward (12800 x 512, tanh, dropout), each as 10 launches replayed from a hipGraph (best
of 3), plus a checksum so two builds (TT2_LIB=...) can be compared bit for bit.

    TT2_LIB=abl/norm0.so python tools/norm_ab.py ; python tools/norm_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402
from tt2._lib import ACT_TANH  # noqa: E402


def main():
    torch.manual_seed(0)
    M, C = 12800, 512
    seed = torch.tensor([7], dtype=torch.int32, device="cuda")
    drop = ops.Drop(seed, 3, 0.1) if hasattr(ops, "Drop") else ops.NO_DROP
    x = torch.randn(M, C, device="cuda").bfloat16()
    br = torch.randn(M, C, device="cuda").bfloat16()
    dy = torch.randn(M, C, device="cuda").bfloat16()
    g, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    y = torch.empty(M, C, device="cuda").bfloat16()
    ops.layernorm_fwd(x, br, g, b, y, mean, rstd, M, drop=drop)
    dx, dbr = torch.empty_like(x), torch.empty_like(x)
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ws = ops.Workspace()
    ln = lambda: ops.layernorm_bwd(dy, x, br, g, mean, rstd, dx, dbr, dg, db, M, drop=drop, ws=ws)  # noqa: E731
    t_ln = min(time_graph(graph_of(ln)) for _ in range(3))
    lnf = lambda: ops.layernorm_fwd(x, br, g, b, y, mean, rstd, M, drop=drop)  # noqa: E731
    t_lnf = min(time_graph(graph_of(lnf)) for _ in range(3))
    bm, br_ = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    out = torch.empty_like(x)
    bnf = lambda: ops.batchnorm_fwd(x, g, b, bm, br_, rm, rv, out, M, C, ACT_TANH, True, drop=drop, ws=ws)  # noqa
    t_bnf = min(time_graph(graph_of(bnf)) for _ in range(3))
    dyb, dgb, dbb = torch.empty_like(x), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    bnb = lambda: ops.batchnorm_bwd(x, dy, g, b, bm, br_, dyb, dgb, dbb, M, C, ACT_TANH, drop=drop, ws=ws)  # noqa
    t_bnb = min(time_graph(graph_of(bnb)) for _ in range(3))
    torch.cuda.synchronize()
    cs = [t.float().sum().item() for t in (dx, dbr, dg, db, out, bm, br_, dyb, dgb, dbb)]
    print(f"lib {os.environ.get('TT2_LIB', 'default')}: ln_fwd {t_lnf * 1e6:.2f} us | ln_bwd {t_ln * 1e6:.2f} us | "
          f"bn_fwd {t_bnf * 1e6:.2f} us | "
          f"bn_bwd {t_bnb * 1e6:.2f} us | checksums {' '.join(f'{v:.9e}' for v in cs)}", flush=True)


if __name__ == "__main__":
    main()
