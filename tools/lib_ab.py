"""Library-vs-library A/B of the v7 / grouped-v7 GEMMs on the training step's shapes (dev tool, GPU).

Each run uses the libtt2 that TT2_LIB names (tt2._lib), times every shape as 10 launches replayed
from a hipGraph, and saves the outputs; `compare` checks two runs' outputs bit for bit.

    TT2_LIB=abl/old.so python tools/lib_ab.py run gpurun_out/x/old.pt
    python tools/lib_ab.py run gpurun_out/x/new.pt
    python tools/lib_ab.py compare gpurun_out/x/old.pt gpurun_out/x/new.pt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402

# name, m, n, k, trans_a, trans_b, epilogue, a_conv, variant (13: v7 forced, 0: auto)
SHAPES = [
    ("o fwd bias", 12800, 512, 512, False, False, "b", None, 0),
    ("qkv fwd bias", 12800, 1536, 512, False, False, "b", None, 0),
    ("ffn1 fwd v7 b+relu+drop", 12800, 2048, 512, False, False, "brd", None, 13),
    ("ffn2 fwd bias", 12800, 512, 2048, False, False, "b", None, 0),
    ("o dgrad res", 12800, 512, 512, False, True, "res", None, 0),
    ("ffn2 dgrad gate", 12800, 2048, 512, False, True, "gate", None, 0),
    ("ffn1 dgrad res", 12800, 512, 2048, False, True, "res", None, 0),
    ("qkv dgrad", 12800, 512, 1536, False, True, "", None, 0),
    ("conv fwd bias", 12800, 512, 2560, False, False, "b", (800, 512, 2), 0),
    ("wgrad 512x2048 K12800", 512, 2048, 12800, True, True, "ks", None, 0),
    ("wgrad 2048x512 K12800", 2048, 512, 12800, True, True, "ks", None, 0),
    ("wgrad 1536x512 K12800", 1536, 512, 12800, True, True, "ks", None, 0),
    ("sq 4096", 4096, 4096, 4096, False, False, "", None, 13),
]


def run(out_path):
    torch.manual_seed(0)
    seed = torch.tensor([99], dtype=torch.int32, device="cuda")
    outs = {}
    for name, m, n, k, ta, tb, epi, conv, var in SHAPES:
        if ta:     # A given as [k, m] (token-major dY), B as [k, n]
            A = torch.randn(k, m, device="cuda").bfloat16()
            lda = m
        else:
            lda = k if conv is None else conv[1]
            A = torch.randn(m, lda, device="cuda").bfloat16()
        B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16() / k ** 0.5
        X = torch.randn(m, n, device="cuda").bfloat16()
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(n, device="cuda")
        if "r" in epi and epi != "res":
            kw["act"] = ACT_RELU
        if "d" in epi:
            kw["drop"] = ops.Drop(seed, 5, 0.1)
        if epi == "gate":
            kw.update(gate=X.relu(), ldg=n, gate_scale=1.1)
        if epi == "res":
            kw.update(res=X, ldr=n)
        ks = None
        if epi == "ks":
            ks = torch.zeros(m, device="cuda")
            kw["a_ksum"] = ks
        dt = torch.float32 if ta else torch.bfloat16
        Cm = torch.empty(m, n, device="cuda", dtype=dt)
        fn = (lambda: ops.gemm(A, B, Cm, m, n, k, lda, B.shape[1], n, trans_a=ta, trans_b=tb, a_conv=conv,
                               variant=var, **kw))
        g = graph_of(fn)
        ts = [time_graph(g) for _ in range(3)]
        fn()
        torch.cuda.synchronize()
        outs[name] = (Cm.clone(), ks.clone() if ks is not None else None)
        t = min(ts)
        print(f"{name:26s} {m}x{n}x{k}: {t * 1e6:7.1f} us {2.0 * m * n * k / t / 1e12:6.0f} TF", flush=True)
        del g
    torch.save({k: v for k, v in outs.items()}, out_path)


def compare(a, b):
    x, y = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for k in x:
        for u, v in zip(x[k], y[k]):
            if u is None:
                continue
            if not torch.equal(u, v):
                bad += 1
                print(f"DIFF {k}: max {(u.double() - v.double()).abs().max().item():.3e}")
    print("bit-identical" if bad == 0 else f"{bad} outputs differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
