"""Two ranks, DIFFERENT shards, the engine's own data-parallel step.

Both ranks share the one visible GPU and exchange over gloo (RCCL refuses two ranks on
one device), so the exchange is the segmented path: the captured step is cut at bucket
boundaries and torch.distributed all-reduces the finished buckets between segment replays.
Each rank runs ``attach()`` + ``capture_train_step(sync_grads=...)`` on its own shard.
Checks:
* the reduced gradient on every rank equals the mean of the two shards' standalone
  single-rank gradients (same weights, same dropout seed) to 1e-6 relative;
* after the captured step's Adam update the parameters are bitwise equal on both ranks,
  and so are the reduced gradients.
"""
import hashlib
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(r, B=3, Tx=24, Ty=56):
    g = torch.Generator().manual_seed(11 + r)
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.tensor([Tx, Tx - 5 - r, Tx - 9])
    mel = torch.randn(B, Ty, 80, generator=g)
    ml = torch.tensor([Ty, Ty - 13 + r, Ty - 20])
    for b in range(B):
        text[b, tl[b]:] = 0
        mel[b, ml[b]:] = 0
    return [t.cuda() for t in (text, tl, mel, ml)]


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TT2_DIST_BACKEND="gloo")
    sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
    try:
        import torch.distributed as dist
        from tt2.config import TTSConfig
        from tt2.dist import GradSync, attach, init_from_env
        from tt2.model import TransformerTTS
        torch.cuda.set_device(0)
        init_from_env()
        assert dist.get_world_size() == world
        m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
        e = m.engine
        with torch.no_grad():
            g = torch.Generator(device="cuda").manual_seed(0)
            for name, (off, shape, n) in e.lay.slots.items():
                if len(shape) >= 2:
                    e.P(name).copy_(torch.randn(shape, generator=g, device="cuda") / (n // shape[0]) ** 0.5)
            e.sync_shadow()
        m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
        shards = [_shard(r) for r in range(world)]
        B, Tx, Ty = shards[0][0].shape[0], shards[0][0].shape[1], shards[0][2].shape[1]
        P0, S0 = e.params.clone(), e.stats.clone()
        SEED = 5

        def standalone(shard):
            e.seed.fill_(SEED)
            A = m._stage(*shard)
            e.forward(A)
            e.loss(A)
            e.backward(A)
            return e.grads.clone()

        G = [standalone(s) for s in shards]          # grad_scale 1, no hook
        sync = attach(m, bucket_bytes=4 << 20)       # gloo -> segmented GradSync, grad_scale 1/2
        assert type(sync) is GradSync and len(sync.buckets) > 3
        for _ in range(2):                           # eager DP warm-up (sizes workspaces)
            m.train_step(*shards[rank], sync_grads=sync.finish)
        run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
        segs, g2 = m._graphs[(B, Tx, Ty)]
        assert g2 is not None and len(segs) > 2
        with torch.no_grad():                        # back to the standalone starting point
            e.params.copy_(P0)
            e.stats.copy_(S0)
            e.sync_shadow()
            e.exp_avg.zero_()
            e.exp_avg_sq.zero_()
            e.step_t.zero_()
            e.seed.fill_(SEED)
        run(*shards[rank])
        torch.cuda.synchronize()
        red = e.grads.clone()
        ref = (G[0] + G[1]) / 2
        rel = ((red.double() - ref.double()).norm() / ref.double().norm()).item()
        moved = (e.params - P0).abs().max().item()
        q.put((rank, dict(rel=rel, moved=moved, params=_digest(e.params), grads=_digest(red),
                          own_vs_ref=((G[rank].double() / 2 - red.double()).norm() / red.double().norm()).item())))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:   # report, then fail the rank
        q.put((rank, dict(error=repr(ex))))
        raise


def test_two_rank_engine_dp_step_on_different_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=240) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        assert "error" not in v, (r, v)
    for p in ps:
        assert p.exitcode == 0
    for r, v in out.items():
        assert v["rel"] <= 1e-6, (r, v)
        assert v["own_vs_ref"] > 1e-3, (r, v)     # the shards differ: the exchange did something
        assert v["moved"] > 0.0
    assert out[0]["grads"] == out[1]["grads"]
    assert out[0]["params"] == out[1]["params"]
