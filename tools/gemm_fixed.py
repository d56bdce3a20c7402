"""Where a decoder-shape v7 GEMM spends its time (dev tool, GPU): graph-replayed time of
M = 12800 products over K (fixed part vs per-K-step part) and per epilogue option.
    python tools/gemm_fixed.py [variant]      (default 13 = v7)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402


def timeit(fn, iters=40):
    """Per-call device time of fn from a graph of `iters` calls (no host launch cost)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters) * 1e-3


def main():
    var = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    M = 12800
    seed = torch.tensor([1234], dtype=torch.int32, device="cuda")
    drop = ops.Drop(seed, 3, 0.1)
    for n in (512, 2048):
        A = torch.randn(M, 2048, device="cuda").bfloat16()
        B = torch.randn(n, 2048, device="cuda").bfloat16()
        C = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        R = torch.randn(M, n, device="cuda").bfloat16()
        bias = torch.randn(n, device="cuda")
        row = []
        for k in (64, 128, 256, 512, 1024, 2048):
            t = timeit(lambda: ops.gemm(A, B, C, M, n, k, 2048, 2048, n, variant=var), iters=40)
            row.append(f"K{k} {t * 1e6:5.1f}")
        print(f"N={n} plain: " + " | ".join(row), flush=True)
        epis = {"plain": {}, "bias": dict(bias=bias), "bias+res": dict(bias=bias, res=R, ldr=n),
                "bias+res+drop": dict(bias=bias, res=R, ldr=n, drop=drop),
                "bias+relu+drop": dict(bias=bias, act=1, drop=drop)}
        row = []
        for name, kw in epis.items():
            t = timeit(lambda: ops.gemm(A, B, C, M, n, 512, 2048, 2048, n, variant=var, **kw), iters=40)
            row.append(f"{name} {t * 1e6:5.1f}")
        print(f"N={n} K=512: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
