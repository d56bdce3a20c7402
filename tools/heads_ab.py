"""The mel + stop head GEMM (12800 x 81 x 512, f32 out, ld 96) in several launch forms (dev
tool, GPU): as the engine launches it, with N padded to 88 / 96 (zero weight rows and bias),
on the 128 x 128 v2 kernel, and split-K; 10 launches replayed from a hipGraph (best of 5), and
the first 81 columns compared with the engine form.

    python tools/heads_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph, ops  # noqa: E402


def main():
    torch.manual_seed(0)
    M, N, K, LD = 12800, 81, 512, 96
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda")
    ws = ops.Workspace()
    ref = torch.zeros(M, LD, device="cuda")
    ops.gemm(x, w, ref, M, N, K, K, K, LD, bias=b, ws=ws)
    torch.cuda.synchronize()
    forms = {}
    for npad in (88, 96):
        wp = torch.zeros(npad, K, device="cuda").bfloat16()
        wp[:N] = w
        bp = torch.zeros(npad, device="cuda")
        bp[:N] = b
        forms[f"N={npad} padded"] = (lambda wp=wp, bp=bp, npad=npad, out=torch.zeros(M, LD, device="cuda"):
                                     (ops.gemm(x, wp, out, M, npad, K, K, K, LD, bias=bp, ws=ws), out)[1])
    forms["engine (N=81)"] = lambda out=torch.zeros(M, LD, device="cuda"): (
        ops.gemm(x, w, out, M, N, K, K, K, LD, bias=b, ws=ws), out)[1]
    forms["v2 128x128"] = lambda out=torch.zeros(M, LD, device="cuda"): (
        ops.gemm(x, w, out, M, N, K, K, K, LD, bias=b, ws=ws, variant=2), out)[1]
    for sp in (2, 4):
        forms[f"split-K {sp}"] = (lambda sp=sp, out=torch.zeros(M, LD, device="cuda"):
                                  (ops.gemm(x, w, out, M, N, K, K, K, LD, bias=b, ws=ws, splits=sp), out)[1])
    for name, fn in forms.items():
        out = fn()
        torch.cuda.synchronize()
        err = (out[:, :N] - ref[:, :N]).abs().max().item()
        same = torch.equal(out[:, :N], ref[:, :N])
        t = min(time_graph(graph_of(fn)) for _ in range(3))
        print(f"{name:16s} {t * 1e6:7.2f} us  bit-identical {same}  max|diff| {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
