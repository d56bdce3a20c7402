"""Capture probe for the SyncBatchNorm + encoder-forward-overlap segfault (round 4, r04j:
hipStreamEndCapture segfaulted in tests/test_gpu_dist.py::test_buckets_final_in_captured_rccl_step_cfg2
[sync_bn=True] while the encoder forward ran on the side stream).

One configuration per process (a segfault ends the process, and the GPU call after it):
    python tools/capture_probe.py --kind rccl|record --shape small|cfg2 [--snap] [--no-syncbn]
        [--enc-syncbn 0|1]
Prints the capture's join status and "PROBE OK <args>" after two replays (with --snap: every
bucket and BatchNorm exchange final, as in the test)."""
from __future__ import annotations

import argparse
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    faulthandler.enable()
    os.environ.setdefault("TT2_CAPTURE_TRACE", "1")
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="rccl", choices=["rccl", "record"])
    ap.add_argument("--shape", default="cfg2", choices=["small", "cfg2"])
    ap.add_argument("--snap", action="store_true")
    ap.add_argument("--no-syncbn", action="store_true")
    ap.add_argument("--enc-syncbn", type=int, default=1)
    a = ap.parse_args()
    from tt2.config import TTSConfig
    from tt2.dist import attach
    from tt2.model import TransformerTTS
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl" if a.kind == "rccl" else "gloo", rank=0, world_size=1)
    if a.shape == "cfg2":
        B, Tx, Ty = 16, 128, 800
    else:
        B, Tx, Ty = 2, 24, 48
    g = torch.Generator().manual_seed(4)
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.full((B,), Tx, dtype=torch.int32).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.full((B,), Ty, dtype=torch.int32).cuda()
    torch.manual_seed(0)
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
    m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
    m.engine.enc_overlap_syncbn = bool(a.enc_syncbn)
    kw = {}
    if a.kind == "record":
        from _dp_recording import RecordingBn, RecordingSync
        kw = dict(sync_cls=RecordingSync, bn_cls=RecordingBn)
    sync = attach(m, kind="rccl", sync_bn=not a.no_syncbn, **kw)
    snap = None
    if a.snap:
        from test_gpu_dist import InGraphSnap
        snap = InGraphSnap(sync, m.engine.bn_sync)
    for _ in range(2):
        m.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    t0 = time.time()
    run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    print(f"captured in {time.time() - t0:.2f} s", flush=True)
    for _ in range(2):
        if snap is not None:
            snap.buf.fill_(float("nan"))
        run(text, tl, mel, ml)
        if snap is not None:
            assert snap.bad() == [], "captured: a bucket or exchange was not final"
    torch.cuda.synchronize()
    sync.close()
    dist.destroy_process_group()
    print("PROBE OK", " ".join(sys.argv[1:]), flush=True)


if __name__ == "__main__":
    main()
