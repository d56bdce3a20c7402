"""Per-shape GEMM census of one bench train step (dev tool, GPU).

Runs one eager step of the bench workload with the launch probe on, re-times
every recorded tt2_gemm launch back-to-back (10 reps), and prints the launches
grouped by (m, n, k, layout, splits, conv) with achieved TFLOP/s.

    python tools/gemm_census.py [variant]
"""
import ctypes as C
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2._lib import check, lib, stream_ptr  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def main(variant=None):
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    eng = model.engine
    with torch.no_grad():
        g = torch.Generator(device="cuda").manual_seed(0)
        for name, (off, shape, n) in eng.lay.slots.items():
            v = eng.P(name)
            if len(shape) >= 2:
                v.copy_(torch.randn(shape, generator=g, device="cuda") / (n // shape[0]) ** 0.5)
        eng.sync_shadow()
    model.configure_optimizer(lr=1.0, warmup=4000.0, clip_norm=1.0)
    model.train()
    text, tl, mel, ml = bench.synth_batch(0)
    model.train_step(text, tl, mel, ml)
    ops.PROBE = probe = ops.LaunchProbe()
    model.train_step(text, tl, mel, ml)
    ops.PROBE = None
    torch.cuda.synchronize()
    L = lib()
    groups = defaultdict(lambda: [0, 0.0, 0.0])
    total = 0.0
    for key, flops, _, _, _, saved in probe.rec:
        if saved is None:
            continue
        grouped = key[0] == "gemm_grouped"
        if variant is not None and not grouped:
            saved[0].kernel_variant = int(variant)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            if grouped:
                check(L.tt2_gemm_grouped(saved, len(saved), stream_ptr()), "gemm_grouped")
            else:
                check(L.tt2_gemm(C.byref(saved[0]), stream_ptr()), "gemm")
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) * 1e-3 / 10
        g0 = saved[0]
        conv = any(g.a_conv_t > 0 or g.b_conv_t > 0 for g in saved)
        epi = ("b" if g0.bias else "") + ("r" if g0.res else "") + ("g" if g0.gate else "") + \
              ("a%d" % g0.act if g0.act else "") + ("d" if g0.drop_thr else "") + ("G%d" % len(saved) if grouped else "")
        k = (g0.m, g0.n, g0.k, g0.trans_a, g0.trans_b, g0.splits, conv, epi, g0.dtype_out)
        grp = groups[k]
        grp[0] += 1
        grp[1] += t
        grp[2] += flops
        total += t
    print(f"{'m':>6} {'n':>6} {'k':>6} ta tb sp conv epi     out  cnt   us/launch   TF   ms total")
    for k, (c, t, f) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        m, n, kk, ta, tb, sp, conv, epi, do = k
        print(f"{m:6d} {n:6d} {kk:6d} {ta:2d} {tb:2d} {sp:2d} {int(conv):4d} {epi:6s} {'bf16' if do else 'f32 ':4s} "
              f"{c:4d} {t / c * 1e6:9.1f} {f / t / 1e12:6.0f} {t * 1e3:8.3f}")
    print(f"total {total * 1e3:.3f} ms over {sum(v[0] for v in groups.values())} launches")


if __name__ == "__main__":
    main(*sys.argv[1:])
