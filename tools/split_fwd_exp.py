"""Experiment (GPU, dev): does running the decoder stack's forward as two concurrent half-batch
streams inside one hipGraph beat the full-batch single-stream schedule?  Timing only (dropout
off, eval BN irrelevant: the decoder layers have no BN).

    python tools/split_fwd_exp.py
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def dec_layers(e, A, b0, b1):
    c = e.cfg
    Ty, Tx = A.Ty, A.Tx
    d, F, H = c.d_model, c.d_ffn, c.n_heads
    r0, r1 = b0 * Ty, b1 * Ty
    n = r1 - r0
    B = b1 - b0
    R = lambda name: A[name][r0:r1]  # noqa: E731
    scale = 1.0 / math.sqrt(c.head_dim)
    x = R("dx0")
    mkv = A["mkv"][b0 * Tx:b1 * Tx]
    kvld = c.n_dec * 2 * d
    ml, tl = A["mel_len"][b0:b1], A["text_len"][b0:b1]
    for l in range(c.n_dec):
        p = f"dec{l}."
        qkv = R(f"dqkv{l}")
        e._lin(x, e.W(p + "qkv.w"), qkv, n, 3 * d, d, bias=e.P(p + "qkv.b"))
        ops.attn_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], R(f"datt{l}"), A[f"dlse{l}"][b0 * H:b1 * H], 3 * d, 3 * d,
                     3 * d, d, B, H, Ty, Ty, ml, True, scale)
        e._lin(R(f"datt{l}"), e.W(p + "o.w"), R(f"do{l}"), n, d, d, bias=e.P(p + "o.b"))
        ops.layernorm_fwd(x, R(f"do{l}"), e.P(p + "ln1.g"), e.P(p + "ln1.b"), R(f"dh1{l}"),
                          A[f"dln1m{l}"][r0:r1], A[f"dln1r{l}"][r0:r1], n, c.ln_eps)
        h1 = R(f"dh1{l}")
        e._lin(h1, e.W(p + "cq.w"), R(f"dcq{l}"), n, d, d, bias=e.P(p + "cq.b"))
        ko = 2 * d * l
        ops.attn_fwd(R(f"dcq{l}"), mkv[:, ko:], mkv[:, ko + d:], R(f"dcatt{l}"), A[f"dclse{l}"][b0 * H:b1 * H], d,
                     kvld, kvld, d, B, H, Ty, Tx, tl, False, scale)
        e._lin(R(f"dcatt{l}"), e.W(p + "co.w"), R(f"dco{l}"), n, d, d, bias=e.P(p + "co.b"))
        ops.layernorm_fwd(h1, R(f"dco{l}"), e.P(p + "ln2.g"), e.P(p + "ln2.b"), R(f"dh2{l}"),
                          A[f"dln2m{l}"][r0:r1], A[f"dln2r{l}"][r0:r1], n, c.ln_eps)
        h2 = R(f"dh2{l}")
        e._lin(h2, e.W(p + "ffn1.w"), R(f"df1{l}"), n, F, d, bias=e.P(p + "ffn1.b"), act=ACT_RELU)
        e._lin(R(f"df1{l}"), e.W(p + "ffn2.w"), R(f"df2{l}"), n, d, F, bias=e.P(p + "ffn2.b"))
        ops.layernorm_fwd(h2, R(f"df2{l}"), e.P(p + "ln3.g"), e.P(p + "ln3.b"), R(f"dx{l + 1}"),
                          A[f"dln3m{l}"][r0:r1], A[f"dln3r{l}"][r0:r1], n, c.ln_eps)
        x = R(f"dx{l + 1}")


def timed(g, reps=20):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    model.eval()
    e = model.engine
    text, tl, mel, ml = bench.synth_batch(0)
    A = model._stage(text, tl, mel, ml)
    e.forward(A)      # materialises the arena
    torch.cuda.synchronize()
    B = A.B
    cur = torch.cuda.current_stream()
    res = {}
    ws0 = e.ws
    wss = [ops.Workspace() for _ in range(4)]
    for w in wss:   # sized outside the capture
        w.get(64 << 20)
    for name, parts, stagger in (("full", 1, False), ("split2", 2, False), ("split2-stagger", 2, True),
                                 ("split4", 4, False)):
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream()
        side = [torch.cuda.Stream() for _ in range(parts)]
        s0.wait_stream(cur)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s0, capture_error_mode=ops.CAPTURE_MODE):
            if parts == 1:
                dec_layers(e, A, 0, B)
            else:
                for i, s in enumerate(side):
                    s.wait_stream(s0)
                    e.ws = wss[i]            # each stream its own split-K workspace
                    with torch.cuda.stream(s):
                        if stagger and i > 0:   # delay the later halves by one small GEMM
                            e._lin(A["dx0"][:128], e.W("dec0.o.w"), A["do0"][:128], 128, 512, 512)
                        dec_layers(e, A, B * i // parts, B * (i + 1) // parts)
                for s in side:
                    s0.wait_stream(s)
        cur.wait_stream(s0)
        e.ws = ws0
        res[name] = timed(g)
        print(f"{name:16s} {res[name]:.3f} ms", flush=True)
    print({k: round(v / res['full'], 3) for k, v in res.items()})


if __name__ == "__main__":
    main()
