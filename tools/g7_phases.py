"""Cycle budget of the v7 / v10 GEMM tiles INSIDE the graph-replayed training step (dev tool, GPU).

Needs the in-step phase build of libtt2 (tools/build_variant.sh phase -DTT2_PHASE=1, then
TT2_LIB=abl/phase.so): every v7 / grouped-v7 / v10 work group then writes, into its launch-probe
record, s_memtime stamps of its first MFMA wave (gemm.hip, TT2_SPAN_W = 32 slots): entry, the start
of K steps 0..11 and the end of their MFMA issue, the end of the K loop, the C image written, the
work group's barrier, the C stores issued, and (last wave) the stores drained.  The step is captured
with the probe armed for every GEMM (as tools/step_census.py), replayed, and each launch's records
are read back.  Per launch shape (median over work groups, mean over launches):

  pro   entry -> K step 0 starts (lane setup, first copies landing, first barrier)
  mfma  K loop: cycles from a step's start to the end of its MFMA issue (fragment reads + MFMAs)
  wait  K loop: cycles from there to the next step's start (lgkmcnt drain + the step barrier,
        i.e. waiting for the loaders' copies of the next stage)
  img   epilogue values -> LDS C image;  bar: the work group's barrier before the store
  st    C store issue;  drain: stores issued -> the last wave's stores complete
  clk   cycles per wall-clock us (the shader clock the work group ran at)

    TT2_LIB=abl/phase.so python tools/g7_phases.py [--json out.json]
"""
import ctypes as C
import json
import os
import statistics
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

W = 32


def wg_phases(r, nkt):
    """One work group's record (W u64) -> dict of phase cycles, or None if incomplete."""
    if r[0] == 0 or r[1] < r[0] or r[2] == 0 or r[31] == 0 or r[3] == 0:
        return None
    st = min(nkt, 12)
    mf = [r[4 + 2 * t] - r[3 + 2 * t] for t in range(st)]
    nxt = [r[3 + 2 * (t + 1)] for t in range(st - 1)] + [r[27] if nkt <= 12 else 0]
    wt = [nxt[t] - r[4 + 2 * t] for t in range(st) if nxt[t]]
    kend = r[27]
    img = r[28] - r[27] if r[28] and r[27] else 0
    bar = r[29] - r[28] if r[29] and r[28] else 0
    stv = r[30] - (r[29] or r[27]) if r[30] else 0
    drain = r[31] - r[30] if r[30] else r[31] - kend
    wall_us = (r[1] - r[0]) / 100.0   # 100 MHz wall clock
    cyc = r[31] - r[2]
    return {"pro": r[3] - r[2], "mfma": sum(mf) / len(mf), "wait": sum(wt) / max(1, len(wt)),
            "kloop": kend - r[3], "img": img, "bar": bar, "st": stv, "drain": drain, "total": cyc,
            "clk": cyc / wall_us if wall_us > 0 else 0.0, "wall_us": wall_us}


def main():
    L = lib()
    if L.tt2_probe_span_width() != W:
        raise SystemExit("needs the phase build: tools/build_variant.sh phase -DTT2_PHASE=1; TT2_LIB=abl/phase.so")
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
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    buf = (C.c_uint64 * (W * 8192))()
    rows = defaultdict(list)
    for key, flops, slot, _, _, saved in probe.rec:
        plan = key[1]
        if plan not in (13, 16):
            continue
        n = L.tt2_probe_span_records(slot, buf, 8192)
        if n <= 0:
            continue
        g0 = saved[0]
        ksplit = g0.k if g0.splits <= 1 else ((g0.k + g0.splits - 1) // g0.splits + 63) // 64 * 64
        nkt = (ksplit + 63) // 64
        ph = [p for p in (wg_phases(buf[W * i:W * (i + 1)], nkt) for i in range(n)) if p]
        if not ph:
            continue
        med = {k: statistics.median(p[k] for p in ph) for k in ph[0]}
        k = (key[0], plan, g0.m, g0.n, g0.k, g0.trans_a, g0.trans_b, len(saved), g0.splits, nkt)
        rows[k].append((n, med, flops))
    out = []
    hdr = (f"{'kind':8s} {'plan':>4} {'m':>6} {'n':>5} {'k':>6} ta tb np sp nkt  WGs x  "
           f"{'pro':>6} {'mfma':>6} {'wait':>6} {'kloop':>7} {'img':>6} {'bar':>6} {'st':>6} {'drain':>6} "
           f"{'total':>7} {'clk':>5} {'wg_us':>6}")
    print(hdr)
    for k, v in sorted(rows.items(), key=lambda kv: -sum(x[1]["wall_us"] * x[0] for x in kv[1])):
        c = len(v)
        avg = {f: sum(x[1][f] for x in v) / c for f in v[0][1]}
        kind, plan, m, n, kk, ta, tb, npb, sp, nkt = k
        print(f"{kind[:8]:8s} {plan:4d} {m:6d} {n:5d} {kk:6d} {ta:2d} {tb:2d} {npb:2d} {sp:2d} {nkt:3d} "
              f"{int(sum(x[0] for x in v) / c):4d} {c:2d}  {avg['pro']:6.0f} {avg['mfma']:6.0f} {avg['wait']:6.0f} "
              f"{avg['kloop']:7.0f} {avg['img']:6.0f} {avg['bar']:6.0f} {avg['st']:6.0f} {avg['drain']:6.0f} "
              f"{avg['total']:7.0f} {avg['clk']:5.0f} {avg['wall_us']:6.2f}")
        out.append({"kind": kind, "plan": plan, "m": m, "n": n, "k": kk, "trans_a": ta, "trans_b": tb,
                    "problems": npb, "splits": sp, "k_steps": nkt, "launches": c, "median_wg": avg})
    probe.close()
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
