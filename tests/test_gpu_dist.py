"""Data-parallel train step on the GPU with a 1-rank RCCL group, both exchange paths:
'rccl' (libtt2's communicator; the bucket all-reduces forked onto a comm stream INSIDE
the one captured step graph) and 'segmented' (torch.distributed all-reduces between graph
segments cut at bucket boundaries).  With one rank the all-reduce is the identity, so
either DP step must reproduce the single-graph step bit for bit."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.dist import GradSync, RcclGradSync, attach  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_group():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        yield
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


def _model():
    torch.manual_seed(0)
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16)
    m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
    return m.train()


@pytest.mark.parametrize("kind", ["rccl", "segmented"])
def test_dp_graph_matches_single_graph(nccl_group, kind):
    g = torch.Generator().manual_seed(3)
    B, Tx, Ty = 2, 24, 48
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([24, 17]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([48, 30]).cuda()
    ref, dp = _model(), _model()
    sync = attach(dp, kind=kind)
    assert len(sync.buckets) > 2 and sync.in_graph == (kind == "rccl")
    for _ in range(2):   # eager warm-up (sizes workspaces)
        ref.train_step(text, tl, mel, ml)
        dp.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    run_ref = ref.capture_train_step(B, Tx, Ty)
    run_dp = dp.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    segs, g2 = dp._graphs[(B, Tx, Ty)]
    if kind == "rccl":
        assert g2 is None and len(segs) == 1          # one graph: all-reduces captured inside
    else:
        assert g2 is not None and len(segs) > 2      # cut at bucket boundaries
    for _ in range(3):
        la = run_ref(text, tl, mel, ml).clone()
        lb = run_dp(text, tl, mel, ml).clone()
        assert torch.equal(la, lb)
    torch.cuda.synchronize()
    assert torch.equal(ref.engine.params, dp.engine.params)
    sync.close()


class _Snap:
    """GradSync that snapshots each bucket on the compute stream at the moment its
    all-reduce is launched (what RCCL would read) and, in finish(), compares every snapshot
    with the final gradients.  A kernel that writes into a bucket after it was handed to
    RCCL -- a missing or misplaced grad_ready call, or a deferred LayerNorm finalize landing
    in an already-launched bucket -- shows up as a mismatch even on one rank, where the
    all-reduce itself is the identity."""

    def _init_snap(self):
        self.snaps, self.bad, self.steps = [], [], 0

    def _launch(self, lo, hi):
        self.snaps.append((lo, hi, self.flat[lo:hi].clone()))
        super()._launch(lo, hi)

    def finish(self):
        super().finish()
        assert sorted((lo, hi) for lo, hi, _ in self.snaps) == sorted(self.buckets)
        for lo, hi, s in self.snaps:
            if not torch.equal(s, self.flat[lo:hi]):
                self.bad.append((lo, hi))
        self.snaps = []
        self.steps += 1


class SnapshotSync(_Snap, GradSync):
    def __init__(self, *a, **kw):
        GradSync.__init__(self, *a, **kw)
        self._init_snap()


class RcclSnapshotSync(_Snap, RcclGradSync):
    """The same check for the in-graph path, eagerly (its launch points are the same hook
    calls; inside a capture the comm stream is ordered by the same stream waits)."""

    def __init__(self, *a, **kw):
        RcclGradSync.__init__(self, *a, **kw)
        self._init_snap()


@pytest.mark.parametrize("bucket_mb,cls", [(4, SnapshotSync), (25, SnapshotSync), (25, RcclSnapshotSync)])
def test_buckets_final_when_launched_cfg2(nccl_group, bucket_mb, cls):
    """At the cfg2 shape (B = 16, 128 phonemes, 800 frames, dropout on): every gradient
    bucket is final when its all-reduce is launched, eagerly (hook during the backward)
    and in the segmented captured step (launches between graph segments)."""
    g = torch.Generator().manual_seed(4)
    B, Tx, Ty = 16, 128, 800
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.full((B,), Tx, dtype=torch.int32).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.full((B,), Ty, dtype=torch.int32).cuda()
    m = _model()
    eng = m.engine
    sync = cls(eng.grads, bucket_mb << 20)
    eng.grad_scale = 1.0 / sync.world
    eng.grad_ready_hook = sync.ready
    assert len(sync.buckets) >= 3
    for _ in range(2):
        m.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    torch.cuda.synchronize()
    assert sync.steps == 2 and sync.bad == [], f"eager: buckets written after launch {sync.bad}"
    if cls is RcclSnapshotSync:
        sync.close()
        return
    run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    for _ in range(2):
        run(text, tl, mel, ml)
    torch.cuda.synchronize()
    assert sync.steps == 4 and sync.bad == [], f"captured: buckets written after launch {sync.bad}"


def test_syncbn_rccl_exchange_in_graph_one_rank(nccl_group):
    """SyncBatchNorm over libtt2's RCCL communicator (attach(sync_bn=True), nccl): the 16
    BatchNorm exchanges per step are captured in the one step graph with the bucket
    all-reduces; with one rank the exchange is the identity, so the step follows the plain
    one up to the slot's f32 rounding of M2 (no host sync anywhere: replays only)."""
    g = torch.Generator().manual_seed(4)
    B, Tx, Ty = 2, 24, 48
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([24, 19]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([48, 33]).cuda()
    ref, dp = _model(), _model()
    sync = attach(dp, kind="rccl", sync_bn=True)
    assert dp.engine.bn_sync is not None and dp.engine.bn_sync.in_graph
    for _ in range(2):
        ref.train_step(text, tl, mel, ml)
        dp.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    run_ref = ref.capture_train_step(B, Tx, Ty)
    run_dp = dp.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    segs, g2 = dp._graphs[(B, Tx, Ty)]
    assert g2 is None and len(segs) == 1
    for _ in range(3):
        la = run_ref(text, tl, mel, ml).clone()
        lb = run_dp(text, tl, mel, ml).clone()
        assert ((la - lb).abs() <= 1e-3 * la.abs() + 1e-5).all(), (la, lb)
    torch.cuda.synchronize()
    d = (ref.engine.params - dp.engine.params).abs().max().item()
    assert d < 1e-3, d
    assert torch.allclose(ref.engine.stats, dp.engine.stats, rtol=1e-3, atol=1e-5)
    sync.close()
