"""BatchNorm backward of the fused-finalize apply against the separate finalize + apply (dev
tool, GPU): run once per library (TT2_LIB) and compare the saved outputs.

    TT2_LIB=abl/bnf0.so python tools/bn_fin_check.py save gpurun_out/bn_old.pt
    python tools/bn_fin_check.py cmp gpurun_out/bn_old.pt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402


def run():
    torch.manual_seed(3)
    M, c = 700, 512
    y = torch.randn(M, c, device="cuda").bfloat16()
    dout = torch.randn(M, c, device="cuda").bfloat16()
    gamma, beta = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1
    mean, rstd = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    out = torch.empty(M, c, dtype=y.dtype, device="cuda")
    ops.batchnorm_fwd(y, gamma, beta, mean, rstd, torch.zeros(c, device="cuda"), torch.ones(c, device="cuda"), out,
                      M, c, 2, True)
    dy = torch.empty(M, c, dtype=y.dtype, device="cuda")
    dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ops.batchnorm_bwd(y, dout, gamma, beta, mean, rstd, dy, dg, db, M, c, 2)
    torch.cuda.synchronize()
    return {"out": out.cpu(), "mean": mean.cpu(), "rstd": rstd.cpu(), "dy": dy.cpu(), "dg": dg.cpu(), "db": db.cpu()}


if __name__ == "__main__":
    r = run()
    if sys.argv[1] == "save":
        torch.save(r, sys.argv[2])
    else:
        o = torch.load(sys.argv[2])
        for k in r:
            a, b = r[k].float(), o[k].float()
            n = (a != b).sum().item()
            print(f"{k}: {n} of {a.numel()} differ, max abs {((a - b).abs().max().item()):.3g}")
