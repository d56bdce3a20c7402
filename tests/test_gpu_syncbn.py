"""SyncBatchNorm (SURVEY.md:219, optional; tt2_batchnorm_{fwd,bwd}_{stats,apply}, tt2/dist.py BnSync).

* kernels: two ranks simulated in one process (each rank's exchange adds the other rank's
  recorded slots, which is what the SUM all-reduce of zero-padded slots does): every rank's
  output, statistics, running statistics and input gradient equal plain BatchNorm over the
  concatenated rows; the ranks' dgamma / dbeta are their own sums and add up to the full ones;
* engine: two ranks (gloo, both on the one GPU, eager steps) on different shards with
  SyncBN: the data-parallel gradient equals the single-rank gradient of the concatenated
  batch, where per-replica statistics do not; a captured step with the gloo exchange is
  refused.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


class SimSync:
    """One simulated rank: exchange() records this rank's slots and adds the other ranks'."""

    def __init__(self, world, rank, others=()):
        self.world, self.rank, self.others = world, rank, list(others)
        self.buf = torch.zeros((3 * world + 2) * 2048 + 4, device="cuda")
        self.sent = None

    def buffer(self, nbytes):
        return self.buf[:(nbytes + 3) // 4]

    def exchange(self, slots):
        self.sent = slots.clone()
        for o in self.others:
            slots += o


def _bn_fwd(y, gamma, beta, m, c, act, rm, rv, sync=None):
    mean, rstd = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    out = torch.empty(m, c, dtype=y.dtype, device="cuda")
    ops.batchnorm_fwd(y, gamma, beta, mean, rstd, rm, rv, out, m, c, act, True, sync=sync)
    return out, mean, rstd


def _bn_bwd(y, dout, gamma, beta, mean, rstd, m, c, act, sync=None):
    dy = torch.empty(m, c, dtype=y.dtype, device="cuda")
    dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ops.batchnorm_bwd(y, dout, gamma, beta, mean, rstd, dy, dg, db, m, c, act, sync=sync)
    return dy, dg, db


@pytest.mark.parametrize("c,act,Ms", [(512, 1, (640, 640)), (80, 0, (640, 640)), (512, 2, (640, 640)),
                                      (512, 2, (640, 213)), (80, 1, (96, 1201))])
def test_syncbn_kernels_match_full_batch(c, act, Ms):
    """Ms: each rank's row count (ranks padded to different lengths hold different counts;
    the exchange carries them and weights each rank by its rows)."""
    torch.manual_seed(c + act + Ms[1])
    W = 2
    y = [(torch.randn(Ms[r], c, device="cuda") * 1.7 + 0.3 * r + 2.0) for r in range(W)]
    dout = [torch.randn(Ms[r], c, device="cuda") for r in range(W)]
    gamma, beta = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1
    rm0, rv0 = torch.randn(c, device="cuda") * 0.1, torch.rand(c, device="cuda") + 0.5
    # the full batch, plain BatchNorm
    rmf, rvf = rm0.clone(), rv0.clone()
    yf, df = torch.cat(y), torch.cat(dout)
    of, mf, sf = _bn_fwd(yf, gamma, beta, sum(Ms), c, act, rmf, rvf)
    dyf, dgf, dbf = _bn_bwd(yf, df, gamma, beta, mf, sf, sum(Ms), c, act)
    # rank 1's slots first (its own outputs are not used), then each rank with the other's
    pre = SimSync(W, 1)
    _bn_fwd(y[1], gamma, beta, Ms[1], c, act, rm0.clone(), rv0.clone(), pre)
    s0 = SimSync(W, 0, [pre.sent])
    rm_0, rv_0 = rm0.clone(), rv0.clone()
    o0, m0, r0 = _bn_fwd(y[0], gamma, beta, Ms[0], c, act, rm_0, rv_0, s0)
    s1 = SimSync(W, 1, [s0.sent])
    rm_1, rv_1 = rm0.clone(), rv0.clone()
    o1, m1, r1 = _bn_fwd(y[1], gamma, beta, Ms[1], c, act, rm_1, rv_1, s1)
    assert torch.equal(m0, m1) and torch.equal(r0, r1)          # same slots, same order: same statistics
    assert torch.equal(rm_0, rm_1) and torch.equal(rv_0, rv_1)
    assert rel(m0, mf) < 1e-6 and rel(r0, sf) < 1e-6
    assert rel(rm_0, rmf) < 1e-6 and rel(rv_0, rvf) < 1e-6
    assert rel(torch.cat([o0, o1]), of) < 1e-6
    # backward
    preb = SimSync(W, 1)
    _bn_bwd(y[1], dout[1], gamma, beta, m1, r1, Ms[1], c, act, preb)
    b0 = SimSync(W, 0, [preb.sent])
    dy0, dg0, db0 = _bn_bwd(y[0], dout[0], gamma, beta, m0, r0, Ms[0], c, act, b0)
    b1 = SimSync(W, 1, [b0.sent])
    dy1, dg1, db1 = _bn_bwd(y[1], dout[1], gamma, beta, m1, r1, Ms[1], c, act, b1)
    assert rel(torch.cat([dy0, dy1]), dyf) < 1e-5
    assert rel(dg0 + dg1, dgf) < 1e-5 and rel(db0 + db1, dbf) < 1e-5
    # dgamma / dbeta are each rank's own sums (the gradient all-reduce adds them)
    _, dg0s, db0s = _bn_bwd(y[0], dout[0], gamma, beta, m0, r0, Ms[0], c, act)
    assert torch.equal(dg0, dg0s) and torch.equal(db0, db0s)
    # per-replica statistics differ from the full batch's (the shards were shifted apart)
    _, ml, _ = _bn_fwd(y[0], gamma, beta, Ms[0], c, act, rm0.clone(), rv0.clone())
    assert rel(ml, mf) > 1e-2


def test_syncbn_world1_matches_plain():
    torch.manual_seed(3)
    M, c = 700, 512
    y = torch.randn(M, c, device="cuda").bfloat16()
    dout = torch.randn(M, c, device="cuda").bfloat16()
    gamma, beta = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1
    o, m, r = _bn_fwd(y, gamma, beta, M, c, 2, torch.zeros(c, device="cuda"), torch.ones(c, device="cuda"))
    so, sm, sr = _bn_fwd(y, gamma, beta, M, c, 2, torch.zeros(c, device="cuda"), torch.ones(c, device="cuda"),
                         SimSync(1, 0))
    assert rel(sm, m) < 1e-6 and rel(sr, r) < 1e-6
    assert (so.float() - o.float()).abs().max().item() <= 2 ** -7 * o.float().abs().max().item()
    dy, dg, db = _bn_bwd(y, dout, gamma, beta, m, r, M, c, 2)
    sdy, sdg, sdb = _bn_bwd(y, dout, gamma, beta, m, r, M, c, 2, SimSync(1, 0))
    assert torch.equal(sdg, dg) and torch.equal(sdb, db)
    assert torch.equal(sdy, dy)


def test_syncbn_rejects_bad_rank():
    M, c = 64, 512
    y = torch.randn(M, c, device="cuda")
    s = SimSync(2, 0)
    s.rank = 2
    with pytest.raises(RuntimeError, match="sync_rank"):
        _bn_fwd(y, torch.ones(c, device="cuda"), torch.zeros(c, device="cuda"), M, c, 0,
                torch.zeros(c, device="cuda"), torch.ones(c, device="cuda"), s)


# ------------------------------------------------------------------ two ranks, engine


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(r, B=3, Tx=24, Ty=56):
    g = torch.Generator().manual_seed(31 + r)
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.tensor([Tx, Tx - 5 - r, Tx - 9][:B])
    mel = torch.randn(B, Ty, 80, generator=g) * (1.0 + r) + 0.5 * r   # shards with different statistics
    ml = torch.tensor([Ty, Ty - 13, Ty - 20][:B])                      # equal valid frames per rank
    for b in range(B):
        text[b, tl[b]:] = 0
        mel[b, ml[b]:] = 0
    return [t.cuda() for t in (text, tl, mel, ml)]


def _rank(rank, world, port, q, Bs=(3, 3)):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TT2_DIST_BACKEND="gloo")
    sys.path.insert(0, os.path.join(ROOT, "transformer-tacotron2_amd"))
    try:
        import torch.distributed as dist
        from tt2.config import TTSConfig
        from tt2.dist import attach, init_from_env
        from tt2.model import TransformerTTS
        torch.cuda.set_device(0)
        init_from_env()
        m = TransformerTTS(TTSConfig(), dtype=torch.float32).train()
        e = m.engine
        e.dropout_enabled = False      # hashed masks index rows: a shard's rows are not the batch's rows
        with torch.no_grad():
            g = torch.Generator(device="cuda").manual_seed(0)
            for name, (off, shape, n) in e.lay.slots.items():
                if len(shape) >= 2:
                    e.P(name).copy_(torch.randn(shape, generator=g, device="cuda") / (n // shape[0]) ** 0.5)
            e.sync_shadow()
        shards = [_shard(r, B=Bs[r]) for r in range(world)]
        full = [torch.cat([s[i] for s in shards]) for i in range(4)]
        S0 = e.stats.clone()

        def step(batch):
            e.stats.copy_(S0)
            A = m._stage(*batch)
            e.forward(A)
            e.loss(A)
            e.backward(A)

        step(full)
        G_full, S_full = e.grads.clone(), e.stats.clone()
        G = []
        for s in shards:
            step(s)
            G.append(e.grads.clone())
        sync = attach(m, bucket_bytes=4 << 20, sync_bn=True)
        assert e.bn_sync is not None and not e.bn_sync.in_graph
        step(shards[rank])
        sync.finish()
        torch.cuda.synchronize()
        red, S_sync = e.grads.clone(), e.stats.clone()
        refused = False
        try:
            m.capture_train_step(*shards[0][0].shape, shards[0][2].shape[1], sync_grads=sync.finish)
        except RuntimeError as ex:
            refused = "SyncBatchNorm" in str(ex)
        nrm = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
        q.put((rank, dict(sync=nrm(red, G_full), replica=nrm((G[0] + G[1]) / 2, G_full),
                          stats=nrm(S_sync, S_full), refused=refused)))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:   # report, then fail the rank
        q.put((rank, dict(error=repr(ex))))
        raise


@pytest.mark.parametrize("Bs", [(3, 3), (3, 1)])
def test_two_rank_syncbn_equals_full_batch(Bs):
    """Bs: utterances per rank.  (3, 1): the ranks' BatchNorms hold 3x56 and 1x56 decoder rows
    (3x24 / 1x24 encoder rows); the exchanged row counts weight them, so the running statistics
    are the concatenated batch's.  The DP gradient is a mean over ranks of per-rank losses and
    equals the concatenated batch's only when the ranks hold equal batches (3, 3)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, Bs)) for r in range(world)]
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
        if Bs[0] == Bs[1]:
            assert v["sync"] < 1e-4, (r, v)           # SyncBN DP gradient = the concatenated batch's
            assert v["replica"] > 20 * v["sync"], (r, v)   # per-replica statistics are not
        assert v["stats"] < 1e-5, (r, v)          # running statistics of the whole batch
        assert v["refused"], (r, v)
