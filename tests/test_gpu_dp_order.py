"""Two ranks run the PRODUCTION N > 1 step schedule and must issue the same collectives in the
same order (cfg4 readiness).

The schedule bench.py runs at N > 1 with the nccl backend is RcclGradSync's one-graph capture:
bucket all-reduces handed to the comm stream from the overlapped backward's side stream, the
encoder forward on the side stream beside the decoder's first block, and with SyncBatchNorm 16
BatchNorm exchanges per step on the same comm stream.  An N-rank replay is deadlock-free only if
every rank's graph holds the same collective sequence on the communicator.  librccl refuses two
ranks on one device, so the ranks here share the one GPU with gloo as the control channel and the
recording syncs of tests/_dp_recording.py in place of RCCL (same class, same attach(), same
capture path; in eager steps they really exchange the buckets over gloo).

Per rank, on its OWN ragged cfg2 shard (B = 16, 128 phonemes, 800 frames, dropout on), with and
without SyncBatchNorm:
* the eager steps and the captured step log the same (kind, offsets / size, issuing stream)
  sequence, and rank 1's sequences equal rank 0's (tt2.dist.compare_issue_logs over
  all_gather_object);
* every bucket is handed over from the side stream, once, in reverse layout order; with
  SyncBatchNorm 16 exchanges per step, all issued from the main stream (the capture's origin:
  the encoder pre-net runs there, its layers on the side stream, engine.forward);
* without SyncBatchNorm the eager overlapped step's reduced gradient equals the mean of the two
  shards' standalone gradients (<= 1e-6 relative) and is bitwise equal on both ranks;
* negative control: rank 1 holding one bucket's hand-off back behind the next one is flagged.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(r, B=16, Tx=128, Ty=800):
    g = torch.Generator().manual_seed(31 + r)
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.randint(Tx // 2, Tx + 1, (B,), generator=g)
    mel = torch.randn(B, Ty, 80, generator=g)
    ml = torch.randint(Ty // 2, Ty + 1, (B,), generator=g)
    tl[0], ml[0] = Tx, Ty
    for b in range(B):
        text[b, tl[b]:] = 0
        mel[b, ml[b]:] = 0
    return [t.cuda() for t in (text, tl, mel, ml)]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TT2_DIST_BACKEND="gloo")
    sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import torch.distributed as dist
        from _dp_recording import RecordingBn, RecordingSync
        from tt2.config import TTSConfig
        from tt2.dist import attach, compare_issue_logs, init_from_env
        from tt2.model import TransformerTTS
        torch.cuda.set_device(0)
        init_from_env()
        shards = [_shard(r) for r in range(world)]
        B, Tx, Ty = 16, 128, 800
        res = {}
        for sync_bn in (False, True):
            torch.manual_seed(0)
            m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16, seed=5).train()
            e = m.engine
            with torch.no_grad():
                g = torch.Generator(device="cuda").manual_seed(0)
                for name, (off, shape, n) in e.lay.slots.items():
                    if len(shape) >= 2:
                        e.P(name).copy_(torch.randn(shape, generator=g, device="cuda") / (n // shape[0]) ** 0.5)
                e.sync_shadow()
            m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
            assert e.wgrad_overlap and e.enc_overlap   # the production defaults
            P0 = e.params.clone()
            G = None
            if not sync_bn:
                def standalone(shard):
                    e.seed.fill_(5)
                    A = m._stage(*shard)
                    e.forward(A)
                    e.loss(A)
                    e.backward(A)
                    return e.grads.clone()
                G = [standalone(s) for s in shards]
            sync = attach(m, bucket_bytes=25 << 20, sync_bn=sync_bn, sync_cls=RecordingSync, bn_cls=RecordingBn)
            assert type(sync) is RecordingSync and sync.in_graph and len(sync.buckets) >= 8
            logs = {}
            with torch.no_grad():
                e.params.copy_(P0)
                e.sync_shadow()
                e.seed.fill_(5)
            for step in range(2):
                sync.log = []
                m.train_step(*shards[rank], sync_grads=sync.finish)
                torch.cuda.synchronize()
                logs[f"eager{step}"] = list(sync.log)
                if step == 0 and G is not None:
                    red = e.grads.clone()
                    ref = (G[0] + G[1]) / 2
                    res["rel"] = ((red.double() - ref.double()).norm() / ref.double().norm()).item()
                    res["own"] = ((G[rank].double() / 2 - red.double()).norm() / red.double().norm()).item()
                    h = [None] * world
                    dist.all_gather_object(h, red.sum(dtype=torch.float64).item())
                    res["red_sums"] = h
            sync.log = []
            run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
            logs["captured"] = list(sync.log)
            run(*shards[rank])
            torch.cuda.synchronize()
            # negative control: rank 1 holds bucket 1's hand-off back behind bucket 2
            if rank == 1:
                sync.hold = 1
            sync.log = []
            m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
            logs["held"] = list(sync.log)
            sync.hold = None
            allg = [None] * world
            dist.all_gather_object(allg, logs)
            mism = {k: compare_issue_logs([a[k] for a in allg]) for k in logs}
            res[f"bn{int(sync_bn)}"] = dict(logs=logs, mism=mism, buckets=list(sync.buckets))
            sync.close()
            del run, m
            torch.cuda.empty_cache()
        q.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:   # report, then fail the rank
        import traceback
        q.put((rank, dict(error=repr(ex), tb=traceback.format_exc())))
        raise


def test_production_schedule_issue_order_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=540) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        assert "error" not in v, (r, v.get("tb"))
    for p in ps:
        assert p.exitcode == 0
    for r in range(world):
        v = out[r]
        assert v["rel"] <= 1e-6, v["rel"]             # reduced = mean of the shards' gradients
        assert v["own"] > 1e-3                        # the shards differ
        assert v["red_sums"][0] == v["red_sums"][1]
        for bn in (0, 1):
            rec = v[f"bn{bn}"]
            logs, mism, buckets = rec["logs"], rec["mism"], [tuple(b) for b in rec["buckets"]]
            for k in ("eager0", "eager1", "captured"):
                assert mism[k] == [], (bn, k, mism[k])
                assert logs[k] == logs["eager0"], (bn, k)       # captured == eager sequence
            seq = logs["captured"]
            bk = [x for x in seq if x[0] == "bucket"]
            assert [(x[1], x[2]) for x in bk] == buckets          # each bucket once, reverse layout order
            assert all(x[3] == "side" for x in bk)                # from the overlapped backward
            bns = [x for x in seq if x[0] == "bn"]
            if bn:
                assert len(bns) == 16, len(bns)
                assert all(x[2] == "main" for x in bns)           # the comm stream forks from the origin only
            else:
                assert bns == []
            assert len(mism["held"]) == 1 and mism["held"][0][0] == 1, mism["held"]   # the control is caught
