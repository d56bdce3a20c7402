"""Per-kernel cost of the decode step (dev tool, GPU).

Each decode-step kernel is captured 50 times back to back into a torch CUDA graph
and replayed; us/launch = steady-state cost of that kernel inside a graph chain,
boundary included (compare tools/launch_floor.hip for the empty-kernel floor).

    python tools/decode_kern.py [t]      # t: self-attention keys (default 400)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402

N = 50


def graph_time(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * N)


def main(t=400):
    dev, bf = "cuda", torch.bfloat16
    B, d, F, H, Tx, Tm = 32, 512, 2048, 8, 128, 800
    r = lambda *s, dt=bf: (torch.randn(s, device=dev) * 0.1).to(dt)  # noqa: E731
    x, br, y = r(B, d), r(B, d), r(B, d)
    g, b = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    tp = torch.full((1,), t, dtype=torch.int32, device=dev)
    cache = r(B, Tm, 2 * d)
    mkv = r(B * Tx, 6 * 2 * d)
    tl = torch.full((B,), Tx, dtype=torch.int32, device=dev)
    res = {}
    res["torch add_ (32x512)"] = graph_time(lambda: x.add_(0))
    res["ln_fwd 32 rows"] = graph_time(lambda: ops.layernorm_fwd(x, br, g, b, y, None, None, B))
    pe = torch.randn(Tm, d, device=dev)
    al = torch.ones(1, device=dev)
    res["posenc_fwd (t_ptr)"] = graph_time(lambda: ops.posenc_fwd(x, al, pe, y, B, 1, t_ptr=tp))
    for (n, k, kw, name) in [(256, 80, dict(act=ACT_RELU), "prenet fc1 256x80"),
                             (256, 256, dict(act=ACT_RELU), "prenet fc2 256x256"),
                             (512, 256, {}, "prenet proj 512x256"),
                             (1536, 512, dict(kv=(cache, tp, d, Tm * 2 * d, 2 * d)), "qkv 1536x512 +kv"),
                             (512, 512, {}, "o 512x512"),
                             (512, 512, dict(a_ln=(br, g, b, y, 1e-5)), "cq 512x512 +ln"),
                             (2048, 512, dict(act=ACT_RELU), "ffn1 2048x512"),
                             (512, 2048, {}, "ffn2 512x2048"),
                             (81, 512, dict(ldo=96), "heads 81x512")]:
        a = r(B, k)
        w = r(n, k)
        ldo = kw.pop("ldo", n)
        out = torch.empty(B, ldo, device=dev, dtype=torch.float32 if name.startswith("heads") else bf)
        bias = torch.zeros(n, device=dev)
        res[name] = graph_time(lambda: ops.gemm(a, w, out, B, n, k, k, k, ldo, bias=bias, **kw))
    q = r(B, 3 * d)
    att = r(B, d)
    res[f"attn_decode self t={t}"] = graph_time(lambda: ops.attn_decode(
        q, cache, cache[:, :, d:], att, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm, t_ptr=tp))
    cq = r(B, d)
    kvld = 12 * d
    res["attn_decode cross 128"] = graph_time(lambda: ops.attn_decode(
        cq, mkv, mkv[:, d:], att, d, Tx * kvld, kvld, Tx * kvld, kvld, d, B, H, Tx, key_len=tl))
    heads = torch.zeros(B, 96, device=dev)
    mel_seq = torch.zeros(B, Tm, 80, device=dev)
    stop = torch.zeros(B, Tm, device=dev)
    prev = r(B, 80)
    t2 = torch.zeros(1, dtype=torch.int32, device=dev)
    res["decode_emit"] = graph_time(lambda: ops.decode_emit(heads, 96, B, 80, Tm, mel_seq, stop, prev, t2))
    for k, v in res.items():
        print(f"{v:7.2f} us  {k}", flush=True)


def gemm_shapes(spec):
    """python tools/decode_kern.py gemm "32,512,512;32,512,128;..." -> us per skinny launch"""
    for sh in spec.split(";"):
        m, n, k = (int(v) for v in sh.split(","))
        a = torch.randn(m, k, device="cuda").bfloat16()
        w = torch.randn(n, k, device="cuda").bfloat16()
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        t = graph_time(lambda: ops.gemm(a, w, out, m, n, k, k, k, n, variant=3))
        kb = (16 + m) * k * 2 / 1024
        print(f"{t:7.2f} us  skinny m{m} n{n} k{k}  ({(n + 15) // 16} WGs, {kb:.0f} KB per WG)", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "gemm":
        gemm_shapes(sys.argv[2])
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 400)
