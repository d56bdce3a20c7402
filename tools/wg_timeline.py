"""Work-group timeline of the GEMM launches inside the graph-replayed training step (dev tool,
GPU): from the launch probe's per-work-group span records, per launch shape: the kernel span,
the spread of work-group starts (dispatch ramp), the median / max work-group duration and how
long the last work groups run past the median end (tail).

    python tools/wg_timeline.py
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
from tt2._lib import lib  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def main():
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    model.configure_optimizer(lr=1e-4, warmup=4000.0, clip_norm=1.0)
    model.train()
    text, tl, mel, ml = bench.synth_batch(0)
    for _ in range(2):
        model.train_step(text, tl, mel, ml)
    torch.cuda.synchronize()
    eng = model.engine
    A = eng.arena(text.shape[0], text.shape[1], mel.shape[1])
    eng.stage_inputs(A, text, tl.to(torch.int32), mel, ml.to(torch.int32))
    L = lib()
    L.tt2_probe_arm()
    L.tt2_probe_reset()
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
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    khz = 100000.0   # MI355X wall clock: 100 MHz
    buf = (C.c_uint64 * 16384)()
    rows = defaultdict(list)
    for key, flops, slot, _, _, saved in probe.rec:
        n = L.tt2_probe_span_records(slot, buf, 8192)
        if n <= 0:
            continue
        st = sorted(buf[2 * i] for i in range(n))
        en = sorted(buf[2 * i + 1] for i in range(n))
        du = sorted(buf[2 * i + 1] - buf[2 * i] for i in range(n))
        t0 = st[0]
        us = lambda t: t / khz * 1e3   # noqa: E731
        g0 = saved[0]
        k = (g0.m, g0.n, g0.k, g0.trans_a, g0.trans_b, len(saved), key[1])
        rows[k].append((n, us(en[-1] - t0), us(st[-1] - t0), us(du[n // 2]), us(du[-1]), us(en[-1] - en[n // 2]),
                        us(st[min(n - 1, 255)] - t0)))
    print(f"{'m':>6} {'n':>5} {'k':>6} ta tb np plan  WGs  span  ramp256 ramp_all  wg_med  wg_max  tail")
    for k, v in sorted(rows.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
        c = len(v)
        avg = [sum(x[i] for x in v) / c for i in range(7)]
        m, n, kk, ta, tb, npb, plan = k
        print(f"{m:6d} {n:5d} {kk:6d} {ta:2d} {tb:2d} {npb:2d} {plan:4d} {int(avg[0]):4d} {avg[1]:6.1f} {avg[6]:7.1f} "
              f"{avg[2]:8.1f} {avg[3]:7.1f} {avg[4]:7.1f} {avg[5]:5.1f}   x{c}")
    probe.close()


if __name__ == "__main__":
    main()
