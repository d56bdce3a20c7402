"""When each GEMM launch of the graph-replayed training step runs, from the launch probe's
per-work-group wall-clock spans (dev tool, GPU).  Unlike a rocprofv3 kernel trace, which
serialises the dispatches it times, the spans are recorded by the kernels themselves inside
an unprofiled replay, so kernels of the overlapped backward's side stream show where they
really run against the main stream's.

    python tools/overlap_timeline.py [--from-ms X] [--pipeline] [--standin]

--standin: the DP step rehearsed on one GPU (tt2.dist.StandinGradSync on a 1-rank nccl group: each
bucket's all-reduce replaced by a kernel with an N-rank ring all-reduce's footprint), whose
per-bucket spans are printed with the GEMMs' (kind "standin").
"""
import ctypes as C
import os
import sys

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
    frm = float(sys.argv[sys.argv.index("--from-ms") + 1]) if "--from-ms" in sys.argv else 0.0
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    model.configure_optimizer(lr=1e-4, warmup=4000.0, clip_norm=1.0)
    model.train()
    if "--pipeline" in sys.argv:   # the bench's mode: the deferred Adam in the forward
        model.pipeline_optimizer(True)
    text, tl, mel, ml = bench.synth_batch(0)
    sync = None
    if "--standin" in sys.argv:
        import torch.distributed as dist
        from tt2.dist import StandinGradSync, attach
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1)
        sync = attach(model, sync_cls=StandinGradSync)
    fin = sync.finish if sync is not None else None
    for _ in range(2):
        model.train_step(text, tl, mel, ml, sync_grads=fin)
    torch.cuda.synchronize()
    eng = model.engine
    A = eng.arena(text.shape[0], text.shape[1], mel.shape[1])
    eng.stage_inputs(A, text, tl.to(torch.int32), mel, ml.to(torch.int32))
    L = lib()
    W = L.tt2_probe_span_width()
    L.tt2_probe_arm()
    L.tt2_probe_reset()
    ops.PROBE = probe = ops.LaunchProbe()
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    nbt = dict(eng.nbt)
    if sync is not None:
        sync.rec = torch.zeros(len(sync.buckets), 2 * sync.wgs, dtype=torch.int64, device="cuda")
        sync.reset()
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode=ops.CAPTURE_MODE):
            model._step_body(A, sync_grads=fin)
    finally:
        ops.PROBE = None
        eng.nbt = nbt
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    buf = (C.c_uint64 * (W * 16384))()
    spans = []
    for i, (key, flops, slot, _, _, saved) in enumerate(probe.rec):
        n = L.tt2_probe_span_records(slot, buf, 16384)
        if n <= 0:
            continue
        st = min(buf[W * j] for j in range(n))
        en = max(buf[W * j + 1] for j in range(n))
        g0 = saved[0]
        spans.append((st, en, i, key[0], key[1], g0.m, g0.n, g0.k, len(saved), n))
    if sync is not None:
        rec = sync.rec.cpu()
        for bi, (lo, hi) in enumerate(sync.buckets):
            r = rec[bi].view(-1, 2)
            if int(r[:, 0].min()) > 0:
                spans.append((int(r[:, 0].min()), int(r[:, 1].max()), -1, "standin", 0, lo, hi - lo, 0, 1,
                              sync.wgs))
    t0 = min(x[0] for x in spans)
    us = lambda t: (t - t0) / 100.0   # noqa: E731  100 MHz wall clock
    print(f"{'start_us':>9} {'end_us':>9} {'dur':>7} issue kind      plan     m     n      k np  WGs")
    for st, en, i, kind, plan, m, n, k, npb, wg in sorted(spans):
        if us(st) / 1e3 < frm:
            continue
        print(f"{us(st):9.1f} {us(en):9.1f} {us(en) - us(st):7.1f} {i:5d} {kind[:9]:9s} {plan:4d} {m:6d} {n:5d} {k:6d} "
              f"{npb:2d} {wg:4d}")
    probe.close()
    if sync is not None:
        sync.close()
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
