"""A/B of the GEMM kernels on the training step's shapes (dev tool, GPU): auto plan vs a forced
variant, each timed as 10 launches replayed from a hipGraph (no host gaps), interleaved rounds,
and the forced variant's output checked against the auto plan's.

    python tools/gemm_ab.py [variant=16] [enc]  (enc: the encoder's 2048-row shapes; also the graph_of /
    time_graph helpers of the other A/B tools)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402

SHAPES = [  # name, m, n, k, trans_b, epilogue, a_conv
    ("ffn1 fwd b+relu+drop", 12800, 2048, 512, False, "brd", None),
    ("ffn2 dgrad gate", 12800, 2048, 512, True, "gate", None),
    ("qkv fwd bias", 12800, 1536, 512, False, "b", None),
    ("mkv fwd bias", 2048, 6144, 512, False, "b", None),
    ("o fwd bias", 12800, 512, 512, False, "b", None),
    ("ffn2 fwd bias", 12800, 512, 2048, False, "b", None),
    ("ffn1 dgrad res", 12800, 512, 2048, True, "res", None),
    ("conv fwd bias", 12800, 512, 2560, False, "b", (800, 512, 2)),
    ("sq 4096", 4096, 4096, 4096, False, "", None),
    ("sq 8192", 8192, 8192, 8192, False, "", None),
]


def graph_of(fn, n=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s, capture_error_mode=ops.CAPTURE_MODE):
        for _ in range(n):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    return g


def time_graph(g, n=10, reps=5):
    g.replay()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        g.replay()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) * 1e-3 / (reps * n)


ENC_SHAPES = [  # the encoder's 2048-row products (`enc`)
    ("enc qkv fwd bias", 2048, 1536, 512, False, "b", None),
    ("enc ffn1 fwd b+relu+drop", 2048, 2048, 512, False, "brd", None),
    ("enc ffn2 fwd bias", 2048, 512, 2048, False, "b", None),
    ("enc o fwd bias", 2048, 512, 512, False, "b", None),
    ("enc ffn2 dgrad gate", 2048, 2048, 512, True, "gate", None),
    ("enc ffn1 dgrad res", 2048, 512, 2048, True, "res", None),
    ("enc qkv dgrad", 2048, 512, 1536, True, "", None),
    ("enc conv fwd bias", 2048, 512, 2560, False, "b", (128, 512, 2)),
]


def main(variant=16, enc=False):
    torch.manual_seed(0)
    seed = torch.tensor([99], dtype=torch.int32, device="cuda")
    for name, m, n, k, tb, epi, conv in (ENC_SHAPES if enc else SHAPES):
        lda = k if conv is None else conv[1]
        A = torch.randn(m, lda, device="cuda").bfloat16()
        B = (torch.randn(k, n, device="cuda") if tb else torch.randn(n, k, device="cuda")).bfloat16() / k ** 0.5
        bias = torch.randn(n, device="cuda")
        X = torch.randn(m, n, device="cuda").bfloat16()
        kw = {}
        if "b" in epi:
            kw["bias"] = bias
        if "r" in epi and epi != "res":
            kw["act"] = ACT_RELU
        if "d" in epi:
            kw["drop"] = ops.Drop(seed, 5, 0.1)
        if epi == "gate":
            kw.update(gate=X.relu(), ldg=n, gate_scale=1.1)
        if epi == "res":
            kw.update(res=X, ldr=n)
        outs = {}
        graphs = {}
        for v in (0, variant):
            C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
            fn = (lambda C=C, v=v: ops.gemm(A, B, C, m, n, k, lda, B.shape[1], n, trans_b=tb, a_conv=conv, variant=v,
                                            **kw))
            graphs[v] = graph_of(fn)
            outs[v] = C
        ts = {0: [], variant: []}
        for _ in range(3):   # interleaved rounds
            for v in (0, variant):
                ts[v].append(time_graph(graphs[v]))
        err = ((outs[variant].double() - outs[0].double()).norm() / outs[0].double().norm()).item()
        fl = 2.0 * m * n * k
        t0, t1 = min(ts[0]), min(ts[variant])
        print(f"{name:22s} {m}x{n}x{k}: auto {t0 * 1e6:7.1f} us {fl / t0 / 1e12:6.0f} TF | v{variant} "
              f"{t1 * 1e6:7.1f} us {fl / t1 / 1e12:6.0f} TF | x{t0 / t1:.2f} | rel diff {err:.1e}", flush=True)
        del graphs


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:] if a != "enc"], enc="enc" in sys.argv[1:])
