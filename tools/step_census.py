"""Per-shape GEMM census INSIDE the graph-replayed training step (dev tool, GPU): the step
is captured with the launch probe armed for every GEMM, replayed, and each launch's own
wall-clock span (tt2_probe_span_ms) read back, so every figure is the launch as the timed
steps run it.  Also prints the launch's work groups (how well it fills 256 CUs).

    python tools/step_census.py
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2._lib import lib  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def groups_of(g, plan):
    if plan == 15:
        return ((g.m + 63) // 64) * ((g.n + 63) // 64)
    return ((g.m + 255) // 256) * ((g.n + 127) // 128) * max(1, g.splits)


def main(reps=5):
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    model.configure_optimizer(lr=1e-4, warmup=4000.0, clip_norm=1.0)
    model.train()
    text, tl, mel, ml = bench.synth_batch(0)
    for _ in range(2):
        model.train_step(text, tl, mel, ml)
    torch.cuda.synchronize()
    eng = model.engine
    B, Tx, Ty = text.shape[0], text.shape[1], mel.shape[1]
    A = eng.arena(B, Tx, Ty)
    eng.stage_inputs(A, text, tl.to(torch.int32), mel, ml.to(torch.int32))
    lib().tt2_probe_arm()     # allocates the span pool outside the capture
    lib().tt2_probe_reset()
    ops.PROBE = probe = ops.LaunchProbe()
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    nbt = dict(eng.nbt)
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode=ops.CAPTURE_MODE):
            model._step_body(A)
    finally:
        ops.PROBE = None
        eng.nbt = nbt
    torch.cuda.current_stream().wait_stream(s)
    L = lib()
    per = [0.0] * len(probe.rec)
    for _ in range(reps):
        g.replay()
        torch.cuda.synchronize()
        for i, r in enumerate(probe.rec):
            per[i] += L.tt2_probe_span_ms(r[2]) * 1e-3 / reps
    rows = defaultdict(lambda: [0, 0.0, 0.0, 0])
    order = []
    for (key, flops, slot, _, _, saved), t in zip(probe.rec, per):
        g0 = saved[0]
        grouped = key[0] == "gemm_grouped"
        epi = ("b" if g0.bias else "") + ("r" if g0.res else "") + ("g" if g0.gate else "") + \
              ("a%d" % g0.act if g0.act else "") + ("d" if g0.drop_thr else "") + ("G%d" % len(saved) if grouped else "")
        conv = any(x.a_conv_t > 0 or x.b_conv_t > 0 for x in saved)
        wg = sum(groups_of(x, key[1]) for x in saved)
        k = (g0.m, g0.n, g0.k, g0.trans_a, g0.trans_b, g0.splits, int(conv), epi, key[1])
        if k not in rows:
            order.append(k)
        d = rows[k]
        d[0] += 1
        d[1] += t
        d[2] += flops
        d[3] = wg
    tot = sum(v[1] for v in rows.values())
    print(f"{'m':>6} {'n':>6} {'k':>6} ta tb sp conv epi      plan  WGs  cnt  us/launch    TF  ms/step")
    for k, (c, t, f, wg) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        m, n, kk, ta, tb, sp, conv, epi, plan = k
        print(f"{m:6d} {n:6d} {kk:6d} {ta:2d} {tb:2d} {sp:2d} {conv:4d} {epi:8s} {plan:4d} {wg:4d} {c:4d} "
              f"{t / c * 1e6:10.1f} {f / t / 1e12:5.0f} {t * 1e3:8.3f}")
    print(f"total {tot * 1e3:.3f} ms/step of GEMM main kernels over {sum(v[0] for v in rows.values())} launches")
    probe.close()


if __name__ == "__main__":
    main()
