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
from tt2.dist import GradSync, attach  # noqa: E402
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

    def _launch(self, lo, hi, after=None):
        if after is not None:   # the snapshot is taken on the stream the bucket is final on
            torch.cuda.current_stream().wait_event(after)
        self.snaps.append((lo, hi, self.flat[lo:hi].clone()))
        super()._launch(lo, hi, after)

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


@pytest.mark.parametrize("bucket_mb,cls", [(4, SnapshotSync), (25, SnapshotSync)])
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
    run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    for _ in range(2):
        run(text, tl, mel, ml)
    torch.cuda.synchronize()
    assert sync.steps == 4 and sync.bad == [], f"captured: buckets written after launch {sync.bad}"


class InGraphSnap:
    """Bucket finality INSIDE the captured one-graph DP step (RcclGradSync, the path bench.py
    runs at N > 1).  RcclGradSync.snap_hook copies each bucket on the comm stream right after
    its all-reduce is issued, so the copies are captured with the step and replay in the
    comm stream's order; after a replay every copy must equal the final gradients bit for
    bit (one rank: the all-reduce is the identity).  A kernel of the compute stream that
    writes into a bucket after the bucket was forked to RCCL changes the final gradients
    but not the copy.  SyncBatchNorm exchanges (BnSync on the same comm stream) are checked
    the same way: the slots as the stats kernel left them on the compute stream (copied
    before the fork) against the slots after the comm stream's all-reduce."""

    def __init__(self, sync, bn=None, n_bn=64):
        self.sync = sync
        self.buf = torch.zeros_like(sync.flat)
        sync.snap_hook = self._bucket
        self.bn = bn
        if bn is not None:
            self.pre = torch.zeros(n_bn, bn._buf.numel(), device=bn._buf.device)
            self.post = torch.zeros_like(self.pre)
            self.n = [0, 0]
            bn.snap_hook = self._bn_post
            ex = bn.exchange

            def exchange(slots):
                k = self.n[0] % n_bn
                self.pre[k, :slots.numel()].copy_(slots)
                self.n[0] += 1
                ex(slots)
            bn.exchange = exchange

    def _bucket(self, lo, hi):
        self.buf[lo:hi].copy_(self.sync.flat[lo:hi])

    def _bn_post(self, slots):
        k = self.n[1] % self.pre.shape[0]
        self.post[k, :slots.numel()].copy_(slots)
        self.n[1] += 1

    def bad(self):
        torch.cuda.synchronize()
        out = [(lo, hi) for lo, hi in self.sync.buckets if not torch.equal(self.buf[lo:hi], self.sync.flat[lo:hi])]
        if self.bn is not None:
            n = min(self.n[1], self.pre.shape[0])
            out += [("bn", k) for k in range(n) if not torch.equal(self.pre[k], self.post[k])]
        return out


def _cfg2_batch(seed=4):
    g = torch.Generator().manual_seed(seed)
    B, Tx, Ty = 16, 128, 800
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.full((B,), Tx, dtype=torch.int32).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.full((B,), Ty, dtype=torch.int32).cuda()
    return B, Tx, Ty, text, tl, mel, ml


@pytest.mark.parametrize("sync_bn", [False, True])
def test_buckets_final_in_captured_rccl_step_cfg2(nccl_group, sync_bn):
    """cfg2 (B = 16, 128 phonemes, 800 frames, dropout on), the RCCL in-graph path that
    bench.py runs at N = 8: inside the ONE captured step graph every bucket is final when the
    comm stream's all-reduce runs, over two replays, with and without SyncBatchNorm (whose
    16 exchanges per step share the comm stream)."""
    B, Tx, Ty, text, tl, mel, ml = _cfg2_batch()
    m = _model()
    sync = attach(m, kind="rccl", sync_bn=sync_bn)
    assert sync.in_graph and len(sync.buckets) >= 3
    snap = InGraphSnap(sync, m.engine.bn_sync)
    for _ in range(2):
        m.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    assert snap.bad() == [], "eager"
    run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    segs, g2 = m._graphs[(B, Tx, Ty)]
    assert g2 is None and len(segs) == 1
    for _ in range(2):
        snap.buf.fill_(float("nan"))      # a bucket the graph does not copy stays NaN: unequal
        run(text, tl, mel, ml)
        assert snap.bad() == [], "captured"
    if sync_bn:
        assert snap.n[0] == snap.n[1] and snap.n[0] >= 2 * 16
    sync.close()
    assert m.engine.bn_sync is None and m.engine.grad_ready_hook is None   # detached on close


class IssueSnap:
    """Each bucket copied on the stream that issues its all-reduce, at the moment of issue: in
    that stream's order, before any later kernel of it (the compute stream, or the overlapped
    backward's side stream, which issues every bucket hook).  Unlike the comm-stream copy,
    whose moment races with the issuing stream's next kernels, this sees a bucket handed over
    before it is final deterministically, so it serves the negative control."""

    def __init__(self, sync):
        self.sync = sync
        self.buf = torch.zeros_like(sync.flat)
        ready = sync.ready

        def hooked(off):
            for i in range(sync.next, len(sync.buckets)):
                lo, hi = sync.buckets[i]
                if lo >= off:
                    self.buf[lo:hi].copy_(sync.flat[lo:hi])
            ready(off)
        sync.ready = hooked

    def bad(self):
        torch.cuda.synchronize()
        return [(lo, hi) for lo, hi in self.sync.buckets if not torch.equal(self.buf[lo:hi], self.sync.flat[lo:hi])]


@pytest.mark.parametrize("overlap,layers", [(False, False), (True, False), (True, True)])
def test_misplaced_grad_ready_is_caught(nccl_group, overlap, layers):
    """Negative control for the checks above: the engine's bucket hook shifted so every bucket
    is handed to RCCL early -- 2M elements (8 MB of gradients) with fixed 25 MB buckets, 4M (more
    than a layer) with layer-aligned ones -- before it is final.  The captured step must then show
    buckets whose final gradients differ from what the issuing stream copied at the hand-off, with
    the in-place and with the overlapped (side-stream) weight gradients; the correctly placed hook
    shows none (IssueSnap agrees with InGraphSnap's positive check)."""
    B, Tx, Ty, text, tl, mel, ml = _cfg2_batch()
    for shift, want_bad in (((4 if layers else 2) << 20, True), (0, False)):
        m = _model()
        m.engine.wgrad_overlap = overlap
        sync = attach(m, kind="rccl", layer_buckets=layers)
        ready = sync.ready
        sync.ready = lambda off, r=ready, s=shift: r(max(0, off - s))   # the captured step hooks it too
        snap = IssueSnap(sync)
        m.engine.grad_ready_hook = sync.ready
        for _ in range(2):
            m.train_step(text, tl, mel, ml, sync_grads=sync.finish)
        run = m.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
        run(text, tl, mel, ml)
        bad = snap.bad()
        if want_bad:
            assert len(bad) >= 1, "an early bucket hand-off went unnoticed"
        else:
            assert bad == [], bad
        sync.close()


def test_syncbn_rccl_exchange_in_graph_one_rank(nccl_group):
    """SyncBatchNorm over libtt2's RCCL communicator (attach(sync_bn=True), nccl): the 16
    BatchNorm exchanges per step are captured in the one step graph with the bucket
    all-reduces, on the comm stream; with one rank the exchange (which runs: BnSync does not
    skip it at world 1 on RCCL) is the identity on raw column sums, and the apply gets the same
    1/N, so the step equals the plain one bit for bit: losses, parameters and running
    statistics (no host sync anywhere: replays only)."""
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
        assert torch.equal(la, lb), (la, lb)
    torch.cuda.synchronize()
    assert torch.equal(ref.engine.params, dp.engine.params)
    assert torch.equal(ref.engine.stats, dp.engine.stats)
    sync.close()


def test_comm_standin_kernel():
    """tt2_comm_standin (the DP stand-in's per-bucket kernel): copies `bytes` from src into the
    scratch buffer, leaves src unchanged, and every work group holds its CU for the requested time
    (its {start, end} wall-clock record spans at least that)."""
    import ctypes as C
    from tt2._lib import check, lib
    torch.manual_seed(5)
    src = torch.randn(1 << 20, device="cuda")
    keep = src.clone()
    scratch = torch.zeros(1 << 20, device="cuda")
    rec = torch.zeros(2 * 32, dtype=torch.int64, device="cuda")
    nbytes, secs = 3 << 20, 200e-6
    check(lib().tt2_comm_standin(C.c_void_p(src.data_ptr()), C.c_void_p(scratch.data_ptr()), nbytes, secs, 32,
                                 C.c_void_p(rec.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream)),
          "tt2_comm_standin")
    torch.cuda.synchronize()
    assert torch.equal(src, keep)
    n = nbytes // 4
    assert torch.equal(scratch[:n], src[:n]) and scratch[n:].abs().sum().item() == 0
    r = rec.view(32, 2).cpu()
    assert (r[:, 0] > 0).all()
    assert ((r[:, 1] - r[:, 0]) >= int(0.95 * secs * 1e8)).all()   # 100 MHz wall clock
    assert lib().tt2_comm_standin(C.c_void_p(src.data_ptr()), C.c_void_p(scratch.data_ptr()), 16, 2.0, 32,
                                  None, None) != 0   # > 1 s refused


def test_standin_dp_step_matches_single_graph(nccl_group):
    """The DP schedule with the stand-in transport (bench.py --dp-standin): each bucket handed to
    the comm stream inside the one captured step runs the stand-in kernel instead of an all-reduce;
    the gradients are untouched, so the captured DP step reproduces the plain single-graph step bit
    for bit, and every bucket's stand-in ran in each replay (span records)."""
    from tt2.dist import StandinGradSync
    g = torch.Generator().manual_seed(3)
    B, Tx, Ty = 2, 24, 48
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([24, 17]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([48, 30]).cuda()
    ref, dp = _model(), _model()
    sync = attach(dp, sync_cls=StandinGradSync, bucket_bytes=4 << 20)
    assert isinstance(sync, StandinGradSync) and sync.in_graph and len(sync.buckets) > 2
    for _ in range(2):
        ref.train_step(text, tl, mel, ml)
        dp.train_step(text, tl, mel, ml, sync_grads=sync.finish)
    sync.rec = torch.zeros(len(sync.buckets), 2 * sync.wgs, dtype=torch.int64, device="cuda")
    run_ref = ref.capture_train_step(B, Tx, Ty)
    run_dp = dp.capture_train_step(B, Tx, Ty, sync_grads=sync.finish)
    for _ in range(2):
        sync.rec.zero_()
        la = run_ref(text, tl, mel, ml).clone()
        lb = run_dp(text, tl, mel, ml).clone()
        assert torch.equal(la, lb)
        torch.cuda.synchronize()
        assert (sync.rec.view(len(sync.buckets), -1, 2)[:, :, 0] > 0).all()
    assert torch.equal(ref.engine.params, dp.engine.params)
    sync.close()
