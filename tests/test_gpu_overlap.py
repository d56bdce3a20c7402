"""The overlapped bf16 backward (engine.wgrad_overlap: every weight-gradient GEMM queued as a job
on a side stream that runs beside the encoder backward, per-layer dY buffers, the layer's last
LayerNorm finalize deferred into its job, clip-norm partials per finished gradient range) against
the in-place schedule it replaces, and its two kernel-level pieces: the grid-capped grouped GEMM
(tt2_gemm_grouped_ex) and the range-partitioned clip norm (tt2_sumsq_parts + adam norm_parts)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2._lib import lib  # noqa: E402
from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def _model(overlap, **knobs):
    torch.manual_seed(0)
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16, seed=5)
    with torch.no_grad():
        for name, (off, shape, n) in m.engine.lay.slots.items():
            if len(shape) >= 2:
                m.engine.P(name).normal_(0, 0.02)
        m.engine.sync_shadow()
    m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
    m.engine.wgrad_overlap = overlap
    for k, v in knobs.items():
        setattr(m.engine, k, v)
    return m.train()


def _batch(B=3, Tx=40, Ty=96, seed=2):
    g = torch.Generator().manual_seed(seed)
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([Tx, Tx - 7, Tx - 19][:B]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([Ty, Ty - 30, Ty - 51][:B]).cuda()
    return text, tl, mel, ml


def _grads(m, b):
    e = m.engine
    m._sync_shadow()
    A = m._stage(*b)
    e.forward(A)
    e.loss(A)
    e.backward(A)
    torch.cuda.synchronize()
    return e.grads.clone()


@pytest.mark.parametrize("knobs", [{"enc_overlap": 0}, {"enc_overlap": 1},
                                   {"enc_overlap": 2, "side_start": 2},
                                   {"side_groups": 64, "side_split": 2}])
def test_overlapped_backward_gradients_bitwise(knobs):
    """Same kernels, same split factors (side_split 1), same order per stream: the gradients of
    the overlapped backward (with the encoder forward beside the decoder's first block, or not)
    equal the in-place schedule's bit for bit; with a capped grid (the same tiles) too; with
    side_split 2 the weight gradients take twice the split-K slabs, so those are compared at f32
    rounding."""
    b = _batch()
    ref = _grads(_model(False, enc_overlap=0), b)
    got = _grads(_model(True, **knobs), b)
    if knobs.get("side_split", 1) == 1:
        assert torch.equal(ref, got)
    else:
        assert ((got - ref).norm() / ref.norm()).item() < 1e-5


def test_overlapped_backward_bitwise_cfg2():
    """The production bf16 schedule at the cfg2 shape (B = 16, 128 phonemes, 800 frames, ragged
    lengths, dropout on, default side-grid caps and split factors): the overlapped backward with
    the encoder forward on the side stream writes the same gradients as the in-place schedule
    (which test_gpu_bf16_parity pins to the oracle), bit for bit, and a captured step of each
    schedule leaves the same parameters."""
    g = torch.Generator().manual_seed(12)
    B, Tx, Ty = 16, 128, 800
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.randint(Tx // 2, Tx + 1, (B,), generator=g)
    mel = torch.randn(B, Ty, 80, generator=g)
    ml = torch.randint(Ty // 2, Ty + 1, (B,), generator=g)
    tl[3], ml[5] = Tx, Ty
    for i in range(B):
        text[i, tl[i]:] = 0
        mel[i, ml[i]:] = 0
    b = [t.cuda() for t in (text, tl, mel, ml)]
    ref_m, ov_m = _model(False, enc_overlap=0), _model(True)
    assert ov_m.engine.enc_overlap and ov_m.engine.side_groups == 0 and ov_m.engine.side_split == 1
    ref, got = _grads(ref_m, b), _grads(ov_m, b)
    wo = _grads(_model(True, enc_overlap=0), b)     # the weight-gradient overlap alone
    twice = _grads(_model(False, enc_overlap=0), b)   # the in-place schedule against itself
    lay = ref_m.engine.lay

    def diff(x):
        out = []
        for name in lay.slots:
            u, v = lay.view(ref, name), lay.view(x, name)
            if not torch.equal(u, v):
                out.append((name, float((u - v).abs().max()), float(u.abs().max())))
        return out
    assert diff(twice) == [], ("in-place schedule not reproducible", diff(twice)[:8])
    assert diff(wo) == [], ("overlapped backward", diff(wo)[:8])
    assert diff(got) == [], ("overlapped backward + encoder forward overlap", diff(got)[:8])
    for m in (ref_m, ov_m):
        m.train_step(*b)
    runs = [m.capture_train_step(B, Tx, Ty) for m in (ref_m, ov_m)]
    for _ in range(2):
        la, lb = (r(*b).clone() for r in runs)
        assert torch.equal(la, lb)
    torch.cuda.synchronize()
    assert torch.equal(ref_m.engine.params, ov_m.engine.params)
    assert torch.equal(ref_m.engine.exp_avg_sq, ov_m.engine.exp_avg_sq)


def test_overlapped_step_clip_norm_and_graph():
    """A train step with the overlap: the clip norm's partial sums are taken over the same
    gradient ranges as in the in-place schedule (on the side stream as each range becomes final,
    there in the optimizer), so the parameters equal the in-place step's bit for bit (clipping
    active: lr and clip chosen so the norm exceeds it); the captured overlapped step equals its
    own eager step bit for bit."""
    b = _batch()
    a, o = _model(False), _model(True)
    for m in (a, o):
        m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1e-3)
    for _ in range(2):
        a.train_step(*b)
        o.train_step(*b)
    torch.cuda.synchronize()
    assert torch.equal(o.engine.params, a.engine.params)
    assert torch.equal(o.engine.exp_avg_sq, a.engine.exp_avg_sq)
    # eager vs captured, both overlapped, from the same state
    e1, e2 = _model(True), _model(True)
    for m in (e1, e2):
        m.train_step(*b)
    run = e2.capture_train_step(b[0].shape[0], b[0].shape[1], b[2].shape[1])
    for _ in range(2):
        l1 = e1.train_step(*b).clone()
        l2 = run(*b).clone()
        assert torch.equal(l1, l2)
    torch.cuda.synchronize()
    assert torch.equal(e1.engine.params, e2.engine.params)


@pytest.mark.parametrize("cap", [8, 64, 200])
def test_grouped_gemm_grid_cap_bitwise(cap):
    """tt2_gemm_grouped_ex with at most `cap` work groups at a time (consecutive launches of
    256 x 128 items, some split-K) writes the same bits as one launch of every item."""
    torch.manual_seed(1)
    K = 3000
    probs = []
    for mo, no in ((512, 2048), (1536, 512), (88, 512)):
        dy = torch.randn(K, mo, device="cuda").bfloat16()
        x = torch.randn(K, no, device="cuda").bfloat16()
        probs.append((dy, x, mo, no))

    def run(max_groups):
        outs, reqs = [], []
        for dy, x, mo, no in probs:
            c = torch.empty(mo, no, device="cuda")
            ks = torch.empty(mo, device="cuda")
            outs.append((c, ks))
            reqs.append(dict(a=dy, b=x, c=c, m=mo, n=no, k=K, lda=mo, ldb=no, ldc=no, trans_a=True, trans_b=True,
                             a_ksum=ks, splits=3))
        ops.gemm_grouped(reqs, max_groups=max_groups)
        torch.cuda.synchronize()
        return outs

    ref, got = run(0), run(cap)
    for (c0, k0), (c1, k1) in zip(ref, got):
        assert torch.equal(c0, c1) and torch.equal(k0, k1)
    dy, x, mo, no = probs[0]
    want = dy.float().t() @ x.float()
    assert ((ref[0][0] - want).norm() / want.norm()).item() < 1e-5


def test_sumsq_parts_and_adam_norm_parts():
    torch.manual_seed(2)
    n = 1 << 20
    g = torch.randn(n, device="cuda") * 0.01
    cuts = [0, 4096, 70000, 500000, n]
    parts = torch.zeros(32 * (len(cuts) - 1), device="cuda")
    for k in range(len(cuts) - 1):
        ops.sumsq_parts(g[cuts[k]:cuts[k + 1]], parts[32 * k:], 32)
    torch.cuda.synchronize()
    ref = (g.double() ** 2).sum().item()
    assert abs(parts.double().sum().item() - ref) / ref < 1e-5
    # adam with precomputed partials == adam with its own norm pass (to f32 summation order)
    outs = []
    for use in (False, True):
        p = torch.ones(n, device="cuda")
        m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        step = torch.zeros(1, dtype=torch.int32, device="cuda")
        ops.adam_step(p, g, m, v, None, step, n, 1e-3, clip_norm=0.5, noam=False,
                      norm_parts=parts if use else None)
        outs.append(p)
    torch.cuda.synchronize()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-6
    assert lib().tt2_sumsq_parts(C.c_void_p(g.data_ptr()), n, C.c_void_p(parts.data_ptr()), 0, None) != 0


@pytest.mark.parametrize("enc_overlap", [1, 2])
@pytest.mark.parametrize("graph", [False, True])
def test_pipelined_optimizer_bitwise(graph, enc_overlap):
    """The pipelined optimizer (each step's Adam deferred to the start of the next forward, the
    encoder's share on the side stream ahead of the encoder): 3 steps + flush equal 3 plain
    steps bit for bit (parameters, Adam moments, step counter, dropout seed), eager, and with
    the captured step (one eager step, then two replays).  enc_overlap 2 issues the decoder's
    part first, so the main stream's conv weight flip follows the side stream's encoder-conv
    update closely: the flip must wait for that update, or the encoder conv
    gradients are taken against stale weights."""
    b = _batch()
    a, p = _model(True, enc_overlap=enc_overlap), _model(True, enc_overlap=enc_overlap)
    p.pipeline_optimizer(True)
    la = [a.train_step(*b).clone() for _ in range(3)]
    if graph:
        lp = [p.train_step(*b).clone()]
        run = p.capture_train_step(b[0].shape[0], b[0].shape[1], b[2].shape[1])
        lp += [run(*b).clone() for _ in range(2)]
    else:
        lp = [p.train_step(*b).clone() for _ in range(3)]
    p.flush_optimizer()
    torch.cuda.synchronize()
    for x, y in zip(la, lp):
        assert torch.equal(x, y)
    ea, ep = a.engine, p.engine
    assert torch.equal(ea.params, ep.params) and torch.equal(ea.exp_avg, ep.exp_avg)
    assert torch.equal(ea.exp_avg_sq, ep.exp_avg_sq) and torch.equal(ea.shadow, ep.shadow)
    assert ea.step_t.item() == ep.step_t.item() == 3 and ea.seed.item() == ep.seed.item()
    p.flush_optimizer()   # nothing pending: a no-op
    torch.cuda.synchronize()
    assert torch.equal(ea.params, ep.params)


def test_pipelined_optimizer_flush_between_replays(tmp_path):
    """The pipelined optimizer with a captured step and eager flushes in between:
    replay, save_checkpoint (flushes the pending Adam), replay, replay equals four plain steps
    bit for bit -- the replay after the flush must not apply that update again, its device gate
    is consumed.  Then load_checkpoint (a plain model's state after 2 steps) into a pipelined
    model with an update pending, and two replays: equal to the plain model's steps 3-4, so the
    stale pending update was dropped."""
    b = _batch()
    B, Tx, Ty = b[0].shape[0], b[0].shape[1], b[2].shape[1]
    a, p = _model(True), _model(True)
    p.pipeline_optimizer(True)
    la = []
    for i in range(4):
        la.append(a.train_step(*b).clone())
        if i == 1:
            a.save_checkpoint(str(tmp_path / "plain2.pt"))
    lp = [p.train_step(*b).clone()]
    run = p.capture_train_step(B, Tx, Ty)
    lp.append(run(*b).clone())
    p.save_checkpoint(str(tmp_path / "pipe2.pt"))     # flush: update 2 applied eagerly
    lp += [run(*b).clone() for _ in range(2)]
    p.flush_optimizer()
    torch.cuda.synchronize()
    for x, y in zip(la, lp):
        assert torch.equal(x, y)
    ea, ep = a.engine, p.engine
    assert torch.equal(ea.params, ep.params) and torch.equal(ea.exp_avg, ep.exp_avg)
    assert torch.equal(ea.exp_avg_sq, ep.exp_avg_sq) and torch.equal(ea.shadow, ep.shadow)
    assert ea.step_t.item() == ep.step_t.item() == 4 and ea.seed.item() == ep.seed.item()
    # load over a pending update
    q = _model(True)
    q.pipeline_optimizer(True)
    q.train_step(*b)
    runq = q.capture_train_step(B, Tx, Ty)
    runq(*b)                                           # update 2 of q's own run pending
    q.load_checkpoint(str(tmp_path / "plain2.pt"))
    lq = [runq(*b).clone() for _ in range(2)]
    q.flush_optimizer()
    torch.cuda.synchronize()
    assert torch.equal(lq[0], la[2]) and torch.equal(lq[1], la[3])
    eq = q.engine
    assert torch.equal(ea.params, eq.params) and torch.equal(ea.exp_avg_sq, eq.exp_avg_sq)
    assert eq.step_t.item() == 4


def test_overlapped_forward_one_layer_decoder():
    """The bf16 overlapped forward with n_dec = 1: the decoder generator then yields
    once, and there is no part-1 memory K/V projection; the forward and the gradients equal the
    in-place schedule's bit for bit."""
    def mk(overlap):
        torch.manual_seed(0)
        m = TransformerTTS(TTSConfig(n_enc=2, n_dec=1), dtype=torch.bfloat16, seed=5)
        m.configure_optimizer(lr=1e-3, warmup=10.0, clip_norm=1.0)
        m.engine.wgrad_overlap = overlap
        m.engine.enc_overlap = 1 if overlap else 0
        return m.train()
    b = _batch()
    ref, got = _grads(mk(False), b), _grads(mk(True), b)
    assert torch.equal(ref, got)
    m = mk(True)
    loss = [m.train_step(*b).clone() for _ in range(2)]
    assert all(torch.isfinite(x).all() for x in loss)
