"""The decode attention launch piece by piece (dev tool, GPU): cfg3 shapes (B = 32, 8 heads,
128 encoder keys, self-attention at t), each form captured 50 times back to back in a graph
and replayed (tools/decode_kern.py's timing), so us/launch includes the launch boundary.

    python tools/dec_attn_ab.py [t]

Forms, as csrc/decoder.cpp launches them: self-attention (+ the fused output projection),
cross-attention plain, + output projection, + query projection, + the LayerNorm-combine
prologue (the decode step's cross launch), and the same with the stop check.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from decode_kern import graph_time, ops  # noqa: E402


def main(t=400):
    dev, bf = "cuda", torch.bfloat16
    B, d, H, Tx, Tm = 32, 512, 8, 128, 800
    r = lambda *s, dt=bf: (torch.randn(s, device=dev) * 0.1).to(dt)  # noqa: E731
    tp = torch.full((1,), t, dtype=torch.int32, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    stop = torch.full((B,), 2 ** 31 - 1, dtype=torch.int32, device=dev)
    cache = r(B, Tm, 2 * d)
    mkv = r(B * Tx, 6 * 2 * d)
    kvld = 12 * d
    tl = torch.full((B,), Tx, dtype=torch.int32, device=dev)
    wq, wo = r(d, d), r(d, d)
    bq = torch.zeros(d, device=dev)
    part = torch.randn(H, B, d, device=dev) * 0.1
    lb, lg, lbe = torch.zeros(d, device=dev), torch.ones(d, device=dev), torch.zeros(d, device=dev)
    lout = r(B, d)
    x = r(B, d)
    q3 = r(B, 3 * d)
    att = r(B, d)
    slab = torch.empty(H, B, d, device=dev)
    res = {}
    self_kw = dict(t_ptr=tp)
    res[f"self t={t}"] = graph_time(lambda: ops.attn_decode(
        q3, cache, cache[:, :, d:], att, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm, **self_kw))
    res[f"self t={t} +o"] = graph_time(lambda: ops.attn_decode(
        q3, cache, cache[:, :, d:], None, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm,
        wo=wo, wo_ld=d, slab=slab, **self_kw))
    res[f"self t={t} +o +stop"] = graph_time(lambda: ops.attn_decode(
        q3, cache, cache[:, :, d:], None, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm,
        wo=wo, wo_ld=d, slab=slab, stop_len=stop, step=step, **self_kw))

    def cross(o=False, q=False, ln=False, st=False):
        kw = dict(key_len=tl)
        if o:
            kw.update(wo=wo, wo_ld=d, slab=slab)
        if q:
            kw.update(wq=wq, wq_ld=d, bq=bq)
        if ln:
            kw.update(ln=(part, lb, lg, lbe, lout, 1e-5))
        if st:
            kw.update(stop_len=stop, step=step)
        return lambda: ops.attn_decode(x, mkv, mkv[:, d:], None if o else att, d, Tx * kvld, kvld, Tx * kvld, kvld, d,
                                       B, H, Tx, **kw)
    res["cross"] = graph_time(cross())
    res["cross +o"] = graph_time(cross(o=True))
    res["cross +o +q"] = graph_time(cross(o=True, q=True))
    res["cross +o +q +ln"] = graph_time(cross(o=True, q=True, ln=True))
    res["cross +o +q +ln +stop (the step's launch)"] = graph_time(cross(o=True, q=True, ln=True, st=True))
    res["ln_combine 8 slabs"] = graph_time(lambda: ops.ln_combine(x, part, 8, lb, lg, lbe, lout, B, 1e-5))
    for k, v in res.items():
        print(f"{v:7.2f} us  {k}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400)
