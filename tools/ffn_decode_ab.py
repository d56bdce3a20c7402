"""The decode step's FFN sublayer: one tt2_ffn_decode launch vs the three launches it replaces
(skinny FFN1 + skinny FFN2 split-K slabs + tt2_ln_combine), cfg3 / cfg5 shapes, 6 layers of
distinct weights per graph replay (dev tool, GPU; TT2_LIB picks the library build).  Also the
fused kernel's per-work-group phase stamps (tt2_ffn_decode_stamps), in us after the first
work group's entry: median and max over the work groups of each phase point.

    python tools/ffn_decode_ab.py [m] [bf16|f16]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_of, time_graph  # noqa: E402
from tt2 import ops  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dtype = torch.float16 if len(sys.argv) > 2 and sys.argv[2] == "f16" else torch.bfloat16
d, f, L = 512, 2048, 6
g = torch.Generator(device="cuda").manual_seed(0)
rn = lambda *sh: torch.randn(*sh, generator=g, device="cuda")  # noqa: E731
layers = [(rn(f, d).mul(d ** -0.5).to(dtype), rn(f) * 0.1, rn(d, f).mul(f ** -0.5).to(dtype), rn(d) * 0.1,
           rn(d) * 0.1 + 1, rn(d) * 0.1) for _ in range(L)]
x = rn(m, d).to(dtype)
hid = torch.zeros(m, f, dtype=dtype, device="cuda")
slab = torch.zeros(8 * m * d, device="cuda")
y = torch.zeros(m, d, dtype=dtype, device="cuda")
sync = torch.zeros(2048, dtype=torch.int32, device="cuda")
dummy = torch.empty(m, d, dtype=dtype, device="cuda")


class WS:
    def get(self, nbytes):
        return slab


def three():
    for (w1, b1, w2, b2, ga, be) in layers:
        ops.gemm(x, w1, hid, m, f, d, d, d, f, bias=b1, act=1)
        ops.gemm(hid, w2, dummy, m, d, f, f, f, d, splits=8, main_only=True, ws=WS())
        ops.ln_combine(x, slab, 8, b2, ga, be, y, m)


def one():
    for (w1, b1, w2, b2, ga, be) in layers:
        ops.ffn_decode(x, w1, b1, w2, b2, ga, be, hid, slab, sync, y, m)


res = {}
for name, fn in (("three", three), ("one", one), ("three", three), ("one", one)):
    gr = graph_of(fn, 4)
    t = time_graph(gr, 4 * L, 20)
    res.setdefault(name, []).append(t * 1e6)
print(f"m={m} {dtype}: three launches {' '.join(f'{v:.2f}' for v in res['three'])} us/layer, "
      f"one launch {' '.join(f'{v:.2f}' for v in res['one'])} us/layer")
assert int(sync.abs().sum()) == 0, "sync not re-armed"
stamps = torch.zeros(256, 8, dtype=torch.int64, device="cuda")
for _ in range(3):
    w1, b1, w2, b2, ga, be = layers[0]
    ops.ffn_decode(x, w1, b1, w2, b2, ga, be, hid, slab, sync, y, m, stamps=stamps)
    torch.cuda.synchronize()
st = stamps.cpu().double()
t0 = st[:, 0].min()
names = ["entry", "hid stored", "hid counted", "slice ready", "slab stored", "slab counted", "rows ready", "exit"]
prod = torch.arange(256) % 32 < 16
nrow = (m + 3) // 4
for k, nm in enumerate(names):
    sel = st[:, k]
    if k in (1, 2):
        sel = sel[prod]
    if k == 6:
        sel = sel[:nrow]
    v = (sel - t0) / 100.0   # 100 MHz wall clock -> us
    print(f"  {nm:13s} median {v.median().item():6.2f} us  max {v.max().item():6.2f} us")
