"""bench.py -- mel frames/s of the Transformer-TTS training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset), this process starts the
N rank processes itself (fresh interpreters; it makes no GPU call of its own), waits for
them and forwards rank 0's JSON line; it exits non-zero if any rank fails, and a line
whose n_gpus differs from N is never printed.

Workload (BASELINE.json configs[1], the metric's single-GPU config): one
training step = forward + loss + backward + (RCCL gradient all-reduce when
N > 1) + fused Adam/clip, bf16 compute with f32 master weights, B = 16
utterances per GPU of LJSpeech shape (phoneme 128, mel 800 x 80), synthetic
seeded data (seed 0 + rank), random-init weights of the 52.99M-parameter
architecture.  Weak scaling: every rank trains its own 16 utterances.

Rank 0 prints ONE JSON line: value = all ranks' frames / max-over-ranks time;
roofline = the dominant kernel (bf16 forward GEMM) measured with HIP events
around each launch in an instrumented step right after the timed region;
cpu_baseline = the CPU oracle's training step on a bounded sample of the same
workload on this box's host cores (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# TT2_PKG (dev): the directory holding the tt2 host package, for A/B of host-schedule versions
sys.path.insert(0, os.environ.get("TT2_PKG") or os.path.join(ROOT, "transformer-tacotron2_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B_PER_GPU, TX, TY, NMEL = 16, 128, 800, 80
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
METRIC = "mel frames/sec (train step) at 1/2/4/8 GPUs; decode frames/sec b=32"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_batch(rank: int, B: int = B_PER_GPU, dev="cuda"):
    g = torch.Generator().manual_seed(0 + rank)
    text = torch.randint(1, 80, (B, TX), generator=g)
    mel = torch.randn(B, TY, NMEL, generator=g)
    tl = torch.full((B,), TX, dtype=torch.int32)
    ml = torch.full((B,), TY, dtype=torch.int32)
    return text.to(dev), tl.to(dev), mel.to(dev), ml.to(dev)


def ragged_batch(rank: int, B: int = B_PER_GPU, dev="cuda"):
    """cfg2's ragged variant: per-utterance lengths ~ U[0.5, 1] x max, seeded,
    padded to the same [B, 128] / [B, 800] shape (pad ids 0, zero mel frames)."""
    g = torch.Generator().manual_seed(1000 + rank)
    text, _, mel, _ = synth_batch(rank, B, dev="cpu")
    tl = (TX * (0.5 + 0.5 * torch.rand(B, generator=g))).round().clamp(1, TX).to(torch.int32)
    ml = (TY * (0.5 + 0.5 * torch.rand(B, generator=g))).round().clamp(1, TY).to(torch.int32)
    for b in range(B):
        text[b, tl[b]:] = 0
        mel[b, ml[b]:] = 0
    return text.to(dev), tl.to(dev), mel.to(dev), ml.to(dev)


def ragged_bench(step_fn, rank: int, steps: int, bufs=None):
    """Times the same captured step on the ragged cfg2 batch; value counts valid frames only
    (padding is computed and masked, as the boundary specifies).  bufs: the step's input tensors
    (model.input_buffers), which then hold the ragged batch for the timed steps."""
    text, tl, mel, ml = ragged_batch(rank)
    if bufs is not None:
        for dst, src in zip(bufs, (text, tl, mel, ml)):
            dst.copy_(src)
        text, tl, mel, ml = bufs
    for _ in range(2):
        step_fn(text, tl, mel, ml)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step_fn(text, tl, mel, ml)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    valid = int(ml.sum().item())
    return {"value": round(valid * steps / dt, 1), "unit": "frames/s (valid frames)",
            "padded_frames_per_s": round(B_PER_GPU * TY * steps / dt, 1),
            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "loss": round(loss[0].item(), 5),
            "config": {"workload": "cfg2 ragged variant: lengths ~ U[0.5,1] x max (seed 1000+rank), "
                                   "padded to 128 / 800", "valid_frames": valid,
                       "valid_text": int(tl.sum().item())}}


def cpu_baseline(budget_s: float = 20.0):
    """The CPU oracle (pure PyTorch fp32) training step on a bounded sample
    (B=2 utterances of the same 128/800 shape), timed on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic
    cores = len(os.sched_getaffinity(0))
    # the GPU box's CPU share is 16 threads per GPU (OMP_NUM_THREADS): sweep up to it
    cap = min(16, cores, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    model = init_deterministic(TransformerTTSOracle(OracleConfig()), 0).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    text, tl, mel, ml = [t.cpu() for t in synth_batch(0, B=2, dev="cpu")]
    tl, ml = tl.long(), ml.long()

    def step(i):
        model.set_seed(i)
        opt.zero_grad()
        out = model(text, tl, mel, ml)
        loss, _ = model.loss(out[:3], mel, ml)
        loss.backward()
        opt.step()

    # thread sweep: one timed step at each smaller count, then the bounded sample at the best
    sweep = {}
    step(0)
    for th in sorted({max(1, cap // 4), max(1, cap // 2)} - {cap}):
        torch.set_num_threads(th)
        t0 = time.perf_counter()
        step(1)
        sweep[th] = round(2 * TY / (time.perf_counter() - t0), 2)
    torch.set_num_threads(cap)
    step(0)
    n, t0 = 0, time.perf_counter()
    while True:
        step(n + 1)
        n += 1
        if time.perf_counter() - t0 > budget_s / 2 or n >= 8:
            break
    dt = (time.perf_counter() - t0) / n
    sweep[cap] = round(2 * TY / dt, 2)
    threads = max(sweep, key=sweep.get)
    # cfg1: one LJSpeech-size utterance (100 phonemes -> 400 frames), eval forward
    model.eval()
    g = torch.Generator().manual_seed(0)
    t1 = torch.randint(1, 80, (1, 100), generator=g)
    m1 = torch.randn(1, 400, NMEL, generator=g)
    l1, lm1 = torch.tensor([100]), torch.tensor([400])
    with torch.no_grad():
        model(t1, l1, m1, lm1)
        c0 = time.perf_counter()
        for _ in range(5):
            model(t1, l1, m1, lm1)
        dc = (time.perf_counter() - c0) / 5
    return {"value": sweep[threads], "unit": "frames/s", "cores": threads, "kind": "port",
            "thread_sweep": {str(k): v for k, v in sorted(sweep.items())},
            "sample": f"CPU oracle fp32 train step (fwd+loss+bwd+Adam), B=2 x (128 phonemes, 800x80 mel), "
                      f"{n} timed steps at {cap} threads after 1 warm-up (one step at each smaller count); "
                      f"{cores} cores visible, the box's CPU share is {cap} threads",
            "cfg1_forward": {"value": round(400 / dc, 1), "unit": "frames/s",
                             "sample": "CPU oracle fp32 eval forward, B=1, 100 phonemes -> 400 frames, 5 runs"}}


def gpu_cfg1(model):
    """cfg1 on the GPU engine (bf16 eval forward, eager launches) for comparison."""
    g = torch.Generator().manual_seed(0)
    t1 = torch.randint(1, 80, (1, 100), generator=g).cuda()
    m1 = torch.randn(1, 400, NMEL, generator=g).cuda()
    l1, lm1 = torch.tensor([100]).cuda(), torch.tensor([400]).cuda()
    was = model.engine.training
    model.eval()
    model(t1, l1, m1, lm1)
    torch.cuda.synchronize()
    c0 = time.perf_counter()
    for _ in range(20):
        model(t1, l1, m1, lm1)
    torch.cuda.synchronize()
    dc = (time.perf_counter() - c0) / 20
    model.train(was)
    return {"value": round(400 / dc, 1), "unit": "frames/s", "ms": round(dc * 1e3, 3),
            "sample": "bf16 eval forward on the GPU, B=1, 100 phonemes -> 400 frames, eager launches"}


DEC_B, DEC_T = 32, 800
# algorithmic HBM bytes of one forced 800-frame decode at B=32:
# bf16 weights read per step + self-KV cache reads (sum over t) + cross-KV reads per step
DEC_BYTES = 2.019e11


def decode_bench(model, reps: int = 3):
    """cfg3: AR decode B=32, 128 phonemes, forced 800 frames, bf16, hipGraph step."""
    from tt2.infer import Decoder
    g = torch.Generator().manual_seed(1)
    text = torch.randint(1, 80, (DEC_B, TX), generator=g).cuda()
    tl = torch.full((DEC_B,), TX, dtype=torch.int32, device="cuda")
    was = model.engine.training
    model.eval()
    dec = Decoder(model.engine, DEC_B, TX, DEC_T)
    dec.encode(text, tl)
    dec.capture(None)              # forced length: the stop head never ends the loop
    dec.reset()
    dec.decode_loop(16)            # warm
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dec.encode(text, tl)
        dec.reset()
        dec.decode_loop(DEC_T, stop_threshold=None)
        mel, _ = dec.postnet(DEC_T, None)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    model.train(was)
    dt = min(times)
    return {"value": round(DEC_B * DEC_T / dt, 1), "unit": "frames/s", "ms_per_run": round(dt * 1e3, 2),
            "ms_per_frame_step": round(dt / DEC_T * 1e3, 4),
            "config": {"workload": "AR decode: encoder + 800 forced hipGraph decode steps + post-net", "batch": DEC_B,
                       "text_len": TX, "frames": DEC_T, "dtype": "bf16"},
            "roofline": {"bound": "hbm", "achieved": round(DEC_BYTES / dt / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(DEC_BYTES / dt / 8e12, 4), **decode_traffic("decode"),
                         "note": "whole-run algorithmic bytes / wall time (latency-bound: a chain of "
                                 f"{DECODE_LAUNCHES} dependent kernels per step)"}}


DECODE_LAUNCHES = 46   # kernels per decode step (csrc/decoder.cpp step_launches: 7 per layer + 4)


def decode_traffic(kind: str):
    """PMC HBM bytes of one decode run: kind "decode" (cfg3) or "longform" (cfg5), from the
    latest profiles/*_<kind>_traffic.json (tools/decode_traffic.py + summarize_decode_traffic.py)."""
    prof = os.path.join(ROOT, "profiles")
    suffix = f"_{kind}_traffic.json"
    files = sorted(f for f in os.listdir(prof) if f.endswith(suffix)) if os.path.isdir(prof) else []
    if not files:
        return {"traffic": None}
    t = json.load(open(os.path.join(prof, files[-1])))
    return {"traffic": round(t["hbm_bytes_per_run"]), "traffic_unit": "B per run",
            "traffic_over_algorithmic": round(t["traffic_over_algorithmic"], 3),
            "traffic_source": "profiles/" + files[-1]}


def gemm_kernel_name(plan: int, ta: int, tb: int) -> str:
    """rocprofv3's (demangled) name of the kernel tt2_gemm_plan selected."""
    t = lambda b: "true" if b else "false"  # noqa: E731
    ak, bk = t(not ta), t(not tb)
    if plan == 2:
        return f"gemm2_kernel<{ak}, {bk}>"
    if plan == 3:
        return "gemm_skinny_kernel"
    if plan == 13:   # (the third argument: the fused-statistics epilogue, 0 = none)
        return f"gemm7_kernel<{ak}, {bk}, 0>"
    if plan == 15:
        return f"gemm8_kernel<{bk}, 0>"
    if plan == 16:
        return "gemm10_kernel"
    if plan == 17:
        return "gemm11_kernel"
    if plan == 1:
        return "gemm_kernel"
    return f"gemm plan {plan}"


def graph_probe(model, text, tl, mel, ml, reps: int = 5, serial: bool = False):
    """Per-launch GEMM times inside GRAPH-REPLAYED steps: the training step is captured once
    more with libtt2's launch probe armed for every GEMM (under capture each v7 / v8 kernel
    records only its own wall-clock span; nothing is added to the graph), replayed `reps`
    times, and each replay's spans read back.  Returns {key: [launches/step, flops, seconds,
    bytes]} averaged over the replays (and, as acc["_wgs"], the work groups of each grouped
    launch: {key: [per launch]}), or None if a probed launch recorded no span.
    serial: the engine's side stream (overlapped weight gradients, encoder forward) is the
    capture stream itself, so the step's launches run one after another in issue order, as
    rocprofv3's kernel trace serialises them: each span is then the kernel's own duration,
    not its duration while another stream holds part of the chip."""
    from tt2 import ops
    eng = model.engine
    B, Tx, Ty = text.shape[0], text.shape[1], mel.shape[1]
    A = eng.arena(B, Tx, Ty)
    eng.stage_inputs(A, text, tl.to(torch.int32), mel, ml.to(torch.int32))
    probe = ops.LaunchProbe()
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    nbt = dict(eng.nbt)
    side = eng._side
    if serial:
        eng._side = s
        if eng._side_ws is None:
            eng._side_ws = ops.Workspace()
    ops.PROBE = probe
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode=ops.CAPTURE_MODE):
            model._step_body(A)
    finally:
        ops.PROBE = None
        eng.nbt = nbt
        eng._side = side
    torch.cuda.current_stream().wait_stream(s)
    acc: dict = {}
    try:
        for _ in range(reps):
            g.replay()
            try:
                summ = probe.summary(span=True)
            except RuntimeError as ex:   # a probe the runtime could not record in the graph
                log(f"[bench] graph probe unavailable ({ex}); eager-step timing only")
                return None
            for k, v in summ.items():
                d = acc.setdefault(k, [0, 0.0, 0.0, 0.0])
                for i in range(4):
                    d[i] += v[i] / reps
    finally:
        probe.close()
        del g
    acc["_wgs"] = dict(probe.wgs)     # per grouped call: its work groups
    acc["_disp"] = dict(probe.disp)   # per call: its kernel dispatches (capped grouped grids: several)
    return acc


def roofline(model, text, tl, mel, ml, replay: bool = True):
    """Live per-launch timing of the dominant kernel family: its launches inside graph-replayed
    training steps, each timed by the kernel's own wall-clock span (graph_probe; no event or
    node added to the graph), with the eager step's dispatch events and a back-to-back
    re-launch beside it."""
    from tt2 import ops
    # rank 0 only: the DP gradient hook must not fire (its all-reduces would have no peers)
    eng = model.engine
    hook, eng.grad_ready_hook = eng.grad_ready_hook, None
    ops.PROBE = probe = ops.LaunchProbe()
    try:
        model.train_step(text, tl, mel, ml)
        summ = probe.summary()
        gsum = graph_probe(model, text, tl, mel, ml) if text is not None else None
        gser = graph_probe(model, text, tl, mel, ml, serial=True) if gsum else None
    finally:
        ops.PROBE = None
        eng.grad_ready_hook = hook
        if hasattr(probe, "close"):
            probe.close()
    # dominant = the GEMM variant with the most device time
    key, (n_calls, flops, secs, abytes) = max(summ.items(), key=lambda kv: kv[1][2])
    wgs_ser = (gser or {}).pop("_wgs", {})
    disp_calls = (gser or {}).pop("_disp", None) or dict(getattr(probe, "disp", {}))
    for d in (gsum, gser):
        if d:
            d.pop("_wgs", None)
            d.pop("_disp", None)
    # counted per kernel DISPATCH, as rocprofv3 counts them: a grouped call whose grid is capped
    # (the side stream's weight gradients) goes out as several consecutive launches
    ndisp = {k: sum(v) for k, v in disp_calls.items()}
    n = ndisp.get(key, n_calls)
    eager_us = secs / n * 1e6
    gk, gs = (gsum or {}).get(key), (gser or {}).get(key)
    conc = None
    if gk:
        # beside it: the same launches in the timed step's own schedule, where the side stream's
        # weight-gradient GEMMs hold part of the chip while the main stream's kernels run
        conc = {"avg_launch_us": round(gk[2] / n * 1e6, 2),
                "frac": round(gk[1] / gk[2] / 1e12 / PEAK_BF16_TFLOPS, 4),
                "all_gemms_ms_per_step": round(sum(v[2] for v in gsum.values()) * 1e3, 3)}
    if gs:
        # the launches inside the replayed step graph with the streams serialised in issue
        # order, as rocprofv3's kernel trace runs them (its average agrees, profiles/*_step_kernels.md)
        secs = gs[2] * n_calls / gs[0]
        timing = ("in-step kernel spans (tt2_probe_span_ms: device wall clock, first workgroup start to last "
                  "wave end) of the launches inside graph-replayed training steps, streams serialised in "
                  "issue order as under rocprofv3, mean of 5 replays")
    elif gk:
        secs = gk[2] * n_calls / gk[0]
        timing = ("in-step kernel spans (tt2_probe_span_ms) of the launches inside graph-replayed training "
                  "steps, mean of 5 replays")
    else:
        timing = "in-step kernel dispatch events (tt2_probe_arm: the kernel's own dispatch records them), eager step"
    # beside it, for reference only: the eager step's dispatch events (each carries the
    # event's completion signal and host-gap clocks, reads high) and a back-to-back replay
    # of the same launches (warm caches, no step context).
    replay = probe.replay_time(key) if replay else None
    allg = gser if gs else (gsum if gk else summ)
    tot_t = sum(v[2] for v in allg.values())
    tot_f = sum(v[1] for v in allg.values())
    achieved = flops / secs / 1e12
    share = None
    if wgs_ser.get(key):   # mean share of the 256 CUs one dispatch's work groups can hold
        share = sum(d * min(w / d, 256) for w, d in zip(wgs_ser[key], disp_calls[key])) / (256 * n)
    kname = gemm_kernel_name(*key[1:4])
    if key[0] == "gemm_grouped":
        kname = kname.replace("gemm7_kernel", "gemm7g_kernel").replace(", 0>", ">")
    traffic, tsrc = None, None
    prof = os.path.join(ROOT, "profiles")
    tfiles = sorted(f for f in os.listdir(prof) if f.endswith("_traffic.json")
                    and not f.endswith(("_decode_traffic.json", "_longform_traffic.json"))) if os.path.isdir(prof) else []
    if tfiles:
        t = json.load(open(os.path.join(prof, tfiles[-1])))
        if t.get("kernel", "") == kname:
            traffic, tsrc = round(t["hbm_bytes_per_launch"]), "profiles/" + tfiles[-1]
    busy, bsrc = None, None   # SQ_VALU_MFMA_BUSY_CYCLES pass (tools/summarize_mfma.py)
    bfiles = sorted(f for f in os.listdir(prof) if f.endswith("_mfma_busy.json")) if os.path.isdir(prof) else []
    if bfiles:
        for name, v in json.load(open(os.path.join(prof, bfiles[-1])))["kernels"].items():
            if kname + "(" in name:
                busy, bsrc = round(v["busy_fraction"], 4), "profiles/" + bfiles[-1]
    return {
        "kernel": kname,
        "bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic, "traffic_source": tsrc,
        "mfma_busy_under_profiler": busy, "mfma_busy_source": bsrc,
        "algo_bytes_per_launch": round(abytes / n), "launches_per_step": n, "flops_per_launch": flops / n,
        "avg_launch_us": round(secs / n * 1e6, 2), "timing": timing,
        "eager_dispatch_avg_launch_us": round(eager_us, 2),
        # (per call: the back-to-back replay launches a grouped call's items as one grid)
        "replay_avg_launch_us": round(replay / n_calls * 1e6, 2) if replay is not None else None,
        "concurrent": conc,
        # a grouped launch on the side stream runs a capped grid (<= 128 work groups while the
        # dgrad chain holds the rest): the share of the 256 CUs its work groups can occupy, and
        # the fraction of that share's MFMA peak
        "cu_share": round(share, 3) if share else None,
        "frac_of_cu_share": round(achieved / PEAK_BF16_TFLOPS / share, 4) if share else None,
        "all_gemms": {"launches": sum(ndisp.get(k, round(v[0])) for k, v in allg.items()),
                      "ms_per_step": round(tot_t * 1e3, 3), "tflops": round(tot_f / tot_t / 1e12, 1)},
        # the four GEMM variants with the most in-step device time, same timing as above
        "top_gemms": [{"kernel": (gemm_kernel_name(*k[1:4]).replace("gemm7_kernel", "gemm7g_kernel").replace(", 0>", ">")
                                  if k[0] == "gemm_grouped" else gemm_kernel_name(*k[1:4])),
                       "launches": ndisp.get(k, round(v[0])),
                       "avg_launch_us": round(v[2] / ndisp.get(k, v[0]) * 1e6, 2),
                       "algo_mb_per_step": round(v[3] / 1e6, 1),
                       "frac": round(v[1] / v[2] / 1e12 / PEAK_BF16_TFLOPS, 4)}
                      for k, v in sorted(allg.items(), key=lambda kv: -kv[1][2])[:4]],
    }


LF_B, LF_T = 64, 2000
LF_W_BYTES = 4.45e7                          # decode-step weights read per step
LF_CROSS_BYTES = 6 * TX * 2 * 512 * 2        # one utterance's cross K/V per step (6 layers)
LF_KEY_BYTES = 6 * 2 * 512 * 2               # one utterance's self K/V per cached position


def longform_algo_bytes(lens, n_steps: int) -> float:
    """Algorithmic HBM bytes of a long-form run: the weights once per step, plus, for each
    utterance while it is still running (frames t < len_b), its cross K/V and its t + 1 cached
    self K/V rows.  Finished utterances read no keys (their attention exits), so they count 0."""
    L = lens.double()
    return n_steps * LF_W_BYTES + float((L * LF_CROSS_BYTES + LF_KEY_BYTES * L * (L + 1) / 2).sum())


def longform_bench(model):
    """cfg5: long-form AR decode in fp16, B=64, 128 phonemes, T_max=2000, stop-token early exit:
    stop logits injected at seeded per-utterance lengths ~ U[1000, 2000] (random weights give a
    meaningless stop head); the device tracks each utterance's stop and skips its attention
    afterwards, the host polls every 32 frames.  frames/s = sum of lengths / wall time."""
    from tt2.infer import Decoder
    g = torch.Generator().manual_seed(5)
    text = torch.randint(1, 80, (LF_B, TX), generator=g).cuda()
    tl = torch.full((LF_B,), TX, dtype=torch.int32, device="cuda")
    lens = torch.randint(1000, LF_T + 1, (LF_B,), generator=g)
    was = model.engine.training
    model.eval()
    dec = Decoder(model.engine, LF_B, TX, LF_T, dtype=torch.float16)
    dec.inject_stop(lens)
    dec.encode(text, tl)
    dec.capture(0.5)
    torch.cuda.synchronize()

    def one_run():
        t0 = time.perf_counter()
        dec.encode(text, tl)
        dec.reset()
        n = dec.decode_loop(LF_T, stop_threshold=0.5)
        _, out_len = dec.postnet(n, 0.5)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, n, out_len

    one_run()   # untimed: first-touch of the 2000-step KV cache and workspaces
    runs = [one_run() for _ in range(2)]
    dt = sum(r[0] for r in runs) / len(runs)
    n, out_len = runs[-1][1], runs[-1][2]
    model.train(was)
    frames = int(out_len.sum())
    if not torch.equal(out_len.cpu(), lens):
        raise RuntimeError("long-form: the injected stops did not end the utterances")
    algo = longform_algo_bytes(lens, n)
    return {"value": round(frames / dt, 1), "unit": "frames/s", "ms_per_run": round(dt * 1e3, 2),
            "runs_ms": [round(r[0] * 1e3, 2) for r in runs], "steps_run": n, "frames": frames,
            "ms_per_frame_step": round(dt / n * 1e3, 4),
            "config": {"workload": "long-form AR decode: encoder + hipGraph decode steps until every utterance "
                                   "has stopped (stop logits injected at its length) + post-net", "batch": LF_B,
                       "text_len": TX, "t_max": LF_T, "lengths": "U[1000, 2000] seeded",
                       "dtype": "fp16 decode step (f16 weights, KV cache, cross K/V; bf16 encoder / post-net)"},
            "roofline": {"bound": "hbm", "achieved": round(algo / dt / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(algo / dt / 8e12, 4), **decode_traffic("longform"),
                         "algo_bytes": algo, "note": "weights per step + running utterances' KV bytes only"}}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (torchrun's env contract: RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR/PORT), wait for all of them, forward rank 0's JSON line.
    Any rank failing ends the others and the launch (non-zero exit)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    log(f"[bench] launched {n} ranks (pids {[p.pid for p in procs]}), rendezvous 127.0.0.1:{port}")
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p for p in procs if p.poll() not in (None, 0)]
        if bad:
            rc = bad[0].returncode
            log(f"[bench] rank process {procs.index(bad[0])} exited with {rc}; stopping the others")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    out = procs[0].stdout.read()
    codes = [p.wait() for p in procs]
    if rc == 0 and any(codes):
        rc = next(c for c in codes if c)
    if rc != 0:
        return rc if rc > 0 else 1
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if not lines:
        log("[bench] rank 0 printed no JSON line")
        return 1
    rec = json.loads(lines[-1])
    if rec.get("n_gpus") != n:
        log(f"[bench] rank 0 reported n_gpus={rec.get('n_gpus')} for a {n}-GPU launch; not printing it")
        return 1
    print(lines[-1], flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--pipeline", action="store_true",
                    help="pipelined optimizer: each step's Adam at the start of the next step, beside the encoder "
                         "(identical updates; measured neutral, DESIGN.md section 0.3)")
    ap.add_argument("--no-pipeline", action="store_true", help="(the default) each step's Adam at its end")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the cfg3 / cfg5 decode measurements")
    ap.add_argument("--no-longform", action="store_true", help="skip the cfg5 long-form decode measurement")
    ap.add_argument("--no-ragged", action="store_true", help="skip the cfg2 ragged-length variant")
    ap.add_argument("--profile-run", action="store_true", help="the run a rocprofv3 kernel trace is taken of: "
                    "training step only (no ragged / decode / CPU legs, no back-to-back probe replays)")
    ap.add_argument("--force-dp", action="store_true", help="dev: run the DP path (bucketed RCCL all-reduce "
                    "inside the step graph) even at world size 1")
    ap.add_argument("--dp-standin", action="store_true", help="dev: the DP path at world size 1 with each bucket's "
                    "all-reduce replaced by a kernel with an N-rank ring all-reduce's CU footprint, HBM bytes and "
                    "duration (tt2.dist.StandinGradSync; TT2_DP_STANDIN_N / _GBPS / _WG)")
    args = ap.parse_args()
    if args.dp_standin:
        args.force_dp = True
    if args.profile_run:
        args.no_ragged = args.no_decode = args.no_longform = args.no_cpu_baseline = True
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))    # before anything touches the GPU

    from tt2.config import TTSConfig
    from tt2.dist import StandinGradSync, attach, broadcast_params, init_from_env, rccl_env
    from tt2.model import TransformerTTS

    rank, world, local = init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a dp{world} run "
                         f"for a {args.gpus}-GPU request")
    torch.cuda.set_device(local % torch.cuda.device_count())   # ranks > GPUs: a 1-GPU gloo rehearsal
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    # random init of the architecture (seeded), then the standard Transformer-TTS Adam/Noam setup
    eng = model.engine
    with torch.no_grad():
        g = torch.Generator(device="cuda").manual_seed(0)
        for name, (off, shape, n) in eng.lay.slots.items():
            v = eng.P(name)
            if len(shape) >= 2:
                fan_in = n // shape[0]
                v.copy_(torch.randn(shape, generator=g, device="cuda") / fan_in ** 0.5)
            elif not (name.endswith(".g") or name.endswith("alpha")):
                v.zero_()
        eng.sync_shadow()
    model.configure_optimizer(lr=1.0, warmup=4000.0, clip_norm=1.0)
    sync = None
    if world > 1 or args.force_dp:
        if world == 1:   # dev check of the DP path on one GPU: a 1-rank RCCL group
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", rank=0, world_size=1)
        broadcast_params(model)
        if args.dp_standin and world > 1:
            raise SystemExit("bench: --dp-standin rehearses the exchange on ONE rank")
        sync = attach(model, bucket_bytes=int(float(os.environ.get("TT2_BUCKET_MB", "25")) * (1 << 20)),
                      sync_cls=StandinGradSync if args.dp_standin else None)
    model.train()
    # pipelined optimizer: each step's Adam runs at the start of the next step beside the encoder
    # forward (identical updates); the last step's Adam is flushed INSIDE the timed region
    pipelined = args.pipeline and not args.no_pipeline
    model.pipeline_optimizer(pipelined)
    text, tl, mel, ml = synth_batch(rank)
    sync_fn = sync.finish if sync is not None else None

    log(f"[bench] rank {rank}/{world}: warm-up {args.warmup} eager steps")
    for _ in range(max(1, args.warmup)):
        model.train_step(text, tl, mel, ml, sync_grads=sync_fn)
    torch.cuda.synchronize()
    if args.no_graph:
        def run(*batch):
            return model.train_step(*batch, sync_grads=sync_fn)
    else:
        run = model.capture_train_step(B_PER_GPU, TX, TY, sync_grads=sync_fn)
        for _ in range(2):
            run(text, tl, mel, ml)

    # the batch sits in the step's own input tensors (model.input_buffers: the static inputs the
    # graph reads; a data loader writes each batch there), so a step is the replay alone
    bufs = model.input_buffers(B_PER_GPU, TX, TY)
    for dst, src in zip(bufs, (text, tl, mel, ml)):
        dst.copy_(src)

    def step():
        return run(*bufs)
    torch.cuda.synchronize()
    log(f"[bench] timing {args.steps} steps")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    model.flush_optimizer()   # the K-th step's Adam (pipelined): K full steps inside the window
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    lval = loss[0].item()
    frames = world * B_PER_GPU * TY * args.steps
    value = frames / dt
    log(f"[bench] {dt / args.steps * 1e3:.2f} ms/step, loss {lval:.4f}")
    comm = None
    if sync is not None:   # every rank: the bucketed exchange alone (outside the timed region)
        comm = {"sync": "rccl in-graph (libtt2 communicator, comm stream inside the step graph)" if sync.in_graph
                else "segmented (torch.distributed between graph segments)",
                "backend": dist.get_backend(), "bucket_mb": round((sync.buckets[0][1] - sync.buckets[0][0]) * 4 / 2**20, 2),
                "rccl_env": rccl_env(), "allreduce_alone": sync.bench_allreduce()}
        if args.dp_standin:
            comm["sync"] = "stand-in (one rank; per bucket a kernel with an N-rank ring all-reduce's footprint)"
            comm["standin"] = sync.params()
        log(f"[bench] all-reduce alone: {comm['allreduce_alone']}")

    rag = None
    if rank == 0 and world == 1 and not args.no_ragged:
        log("[bench] cfg2 ragged variant")
        rag = ragged_bench(run, rank, max(5, args.steps // 2), bufs)
        log(f"[bench] ragged {rag['value']:.0f} valid frames/s ({rag['ms_per_step']} ms/step)")
    rl = roofline(model, text, tl, mel, ml, replay=not args.profile_run) if rank == 0 else None
    dec = None
    if rank == 0 and world == 1 and not args.no_decode:
        log("[bench] decode (cfg3)")
        dec = decode_bench(model)
        log(f"[bench] decode {dec['value']:.0f} frames/s ({dec['ms_per_frame_step']} ms/step)")
    lf = None
    if rank == 0 and world == 1 and not args.no_decode and not args.no_longform:
        log("[bench] long-form decode (cfg5)")
        lf = longform_bench(model)
        log(f"[bench] long-form {lf['value']:.0f} frames/s ({lf['steps_run']} steps)")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("[bench] cpu baseline (oracle on host cores)")
        cpu = cpu_baseline()
        cpu["cfg1_forward"]["gpu"] = gpu_cfg1(model)
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": ("train step (fwd+loss+bwd+STAND-IN grad exchange+Adam), LJSpeech-shape synthetic "
                                    "batch" if args.dp_standin else
                                    "train step (fwd+loss+bwd+grad all-reduce+Adam), LJSpeech-shape synthetic batch"
                                    if sync is not None else
                                    "train step (fwd+loss+bwd+Adam; one rank: no gradient exchange), "
                                    "LJSpeech-shape synthetic batch"),
                       "global_batch": world * B_PER_GPU, "per_gpu_batch": B_PER_GPU, "seq_len": TY,
                       "text_len": TX, "n_mels": NMEL, "params": model.n_params(), "parallelism": f"dp{world}",
                       "graph": not args.no_graph,
                       "optimizer": ("pipelined: step N's Adam runs at the start of step N+1 beside the encoder "
                                     "forward (identical updates); step K's Adam is flushed inside the timed window")
                       if pipelined else "Adam at the end of each step"},
            "loss": round(lval, 5),
            "grad_exchange": comm,
            "roofline": rl,
            "train_ragged": rag,
            "cpu_baseline": cpu,
            "decode": dec,
            "decode_longform": lf,
        }
        print(json.dumps(out), flush=True)
    if sync is not None:
        sync.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
