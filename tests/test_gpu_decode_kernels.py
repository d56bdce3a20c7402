"""Decode-step kernels vs float64 torch references (GPU): the skinny-M GEMM over every
K regime (one pass per wave slice and multi-pass), its LayerNorm prologue, KV-cache
scatter, positional-encoding and frame-emit epilogues, and the decode attention over a
KV cache at short and long key counts."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bf(shape, gen, scale=1.0):
    return (torch.randn(shape, generator=gen) * scale).bfloat16().cuda()


@pytest.mark.parametrize("m", [1, 17, 32])
@pytest.mark.parametrize("n,k", [(81, 512), (256, 80), (256, 256), (1536, 512), (512, 2048), (40, 1000),
                                 (24, 2104), (16, 8)])
def test_skinny_gemm_k_regimes(m, n, k):
    g = torch.Generator().manual_seed(m * 7 + k)
    A, W = _bf((m, k), g), _bf((n, k), g)
    bias = torch.randn(n, generator=g).cuda()
    C = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, W, C, m, n, k, k, k, n, bias=bias, variant=3)
    ref = A.double() @ W.double().t() + bias.double()
    assert rel(C, ref) < 1e-2


def test_skinny_ln_prologue_and_kv_scatter():
    g = torch.Generator().manual_seed(11)
    m, n, k, Tm = 29, 1536, 512, 40
    x, br = _bf((m, k), g), _bf((m, k), g)
    gam, bet = torch.randn(k, generator=g).cuda(), torch.randn(k, generator=g).cuda()
    W = _bf((n, k), g, 0.05)
    h = torch.empty(m, k, dtype=torch.bfloat16, device="cuda")
    C = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    cache = torch.zeros(m, Tm, 1024, dtype=torch.bfloat16, device="cuda")
    t = torch.tensor([13], dtype=torch.int32, device="cuda")
    ops.gemm(x, W, C, m, n, k, k, k, n, a_ln=(br, gam, bet, h, 1e-5), kv=(cache, t, 512, Tm * 1024, 1024),
             variant=3)
    hr = F.layer_norm(x.double() + br.double(), (k,), gam.double(), bet.double(), 1e-5)
    assert rel(h, hr) < 1e-2
    ref = h.double() @ W.double().t()
    assert rel(C, ref) < 1e-2
    assert torch.equal(cache[:, 13], C[:, 512:])
    assert cache[:, :13].abs().sum().item() == 0 and cache[:, 14:].abs().sum().item() == 0


def test_skinny_pe_epilogue():
    g = torch.Generator().manual_seed(3)
    m, n, k = 32, 512, 256
    A, W = _bf((m, k), g), _bf((n, k), g, 0.1)
    bias = torch.randn(n, generator=g).cuda()
    pe = torch.randn(50, n, generator=g).cuda()
    alpha = torch.tensor([0.7], device="cuda")
    t = torch.tensor([21], dtype=torch.int32, device="cuda")
    C = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, W, C, m, n, k, k, k, n, bias=bias, pe=(pe, alpha, t), variant=3)
    ref = A.double() @ W.double().t() + bias.double() + 0.7 * pe[21].double()
    assert rel(C, ref) < 1e-2


def test_skinny_emit_advances_step():
    """Three heads GEMMs with the emit epilogue (t_max = 2): frames land at t = 0, 1, the
    previous-frame buffer holds the last one, the seed advances, the arrival counter is
    re-armed; the third call (t = t_max) writes no frame and the counter and seed saturate."""
    g = torch.Generator().manual_seed(5)
    m, n, k, nm, Tm = 32, 81, 512, 80, 2
    W = _bf((n, k), g, 0.1)
    bias = torch.randn(n, generator=g).cuda()
    mel = torch.zeros(m, Tm, nm, device="cuda")
    stop = torch.zeros(m, Tm, device="cuda")
    prev = torch.zeros(m, nm, dtype=torch.bfloat16, device="cuda")
    t = torch.zeros(1, dtype=torch.int32, device="cuda")
    seed = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    done = torch.zeros(1, dtype=torch.int32, device="cuda")
    heads = torch.empty(m, 96, device="cuda")
    outs = []
    for step in range(3):
        A = _bf((m, k), g)
        ops.gemm(A, W, heads, m, n, k, k, k, 96, bias=bias, emit=(mel, stop, prev, t, seed, done, nm, Tm),
                 variant=3)
        ref = A.double() @ W.double().t() + bias.double()
        outs.append(ref)
        assert rel(heads[:, :n], ref) < 1e-5
        assert t.item() == min(step + 1, Tm) and seed.item() == 7 + min(step + 1, Tm) and done.item() == 0
    for s in range(Tm):
        assert rel(mel[:, s], outs[s][:, :nm]) < 1e-5
        assert rel(stop[:, s], outs[s][:, nm]) < 1e-5
    assert rel(prev, outs[Tm - 1][:, :nm]) < 1e-2   # step 2 (t = Tm) writes no frame


@pytest.mark.parametrize("k,sp", [(512, 4), (2048, 8), (2048, 16), (512, 2)])
def test_skinny_split_slabs_ln_combine(k, sp):
    """Split-K slabs of the skinny kernel folded by tt2_ln_combine = LN(x + bias + X W^T)."""
    g = torch.Generator().manual_seed(k + sp)
    m, n = 32, 512
    A, W = _bf((m, k), g), _bf((n, k), g, 0.05)
    x = _bf((m, n), g)
    bias, gam, bet = (torch.randn(n, generator=g).cuda() for _ in range(3))
    slab = torch.full((sp * m * n,), float("nan"), device="cuda")

    class WS:
        def get(self, nbytes):
            assert nbytes <= slab.numel() * 4
            return slab

    dummy = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, W, dummy, m, n, k, k, k, n, splits=sp, main_only=True, ws=WS(), variant=3)
    part = A.double() @ W.double().t()
    assert rel(slab.view(sp, m, n).sum(0), part) < 1e-5
    y = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    ops.ln_combine(x, slab, sp, bias, gam, bet, y, m)
    ref = F.layer_norm(x.double() + bias.double() + part, (n,), gam.double(), bet.double(), 1e-5)
    assert rel(y, ref) < 1e-2


def _attn_ref(q, K, V, nk, scale):
    B, H = q.shape[0], q.shape[1] // 64
    out = torch.zeros(B, H * 64, dtype=torch.float64)
    for b in range(B):
        n = int(nk[b])
        if n == 0:
            continue
        for h in range(H):
            qq = q[b, h * 64:(h + 1) * 64].double().cpu()
            kk = K[b, :n, h * 64:(h + 1) * 64].double().cpu()
            vv = V[b, :n, h * 64:(h + 1) * 64].double().cpu()
            p = torch.softmax(kk @ qq * scale, 0)
            out[b, h * 64:(h + 1) * 64] = p @ vv
    return out


@pytest.mark.parametrize("t", [0, 6, 33, 257, 1999])
def test_attn_decode_self_cache(t):
    g = torch.Generator().manual_seed(t)
    B, H, d, Tm = 4, 8, 512, 2000
    qkv = _bf((B, 3 * d), g)
    cache = _bf((B, Tm, 2 * d), g)
    tp = torch.tensor([t], dtype=torch.int32, device="cuda")
    out = torch.empty(B, d, dtype=torch.bfloat16, device="cuda")
    ops.attn_decode(qkv, cache, cache[:, :, d:], out, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm,
                    t_ptr=tp, scale=0.125)
    ref = _attn_ref(qkv[:, :d], cache[:, :, :d], cache[:, :, d:], [t + 1] * B, 0.125)
    assert rel(out, ref) < 1e-2


def test_attn_decode_cross_ragged():
    g = torch.Generator().manual_seed(9)
    B, H, d, Tx = 5, 8, 512, 128
    q = _bf((B, d), g)
    mem = _bf((B, Tx, 2 * d), g)
    kl = torch.tensor([128, 1, 0, 77, 9], dtype=torch.int32, device="cuda")
    out = torch.empty(B, d, dtype=torch.bfloat16, device="cuda")
    ops.attn_decode(q, mem, mem[:, :, d:], out, d, Tx * 2 * d, 2 * d, Tx * 2 * d, 2 * d, d, B, H, Tx, key_len=kl,
                    scale=1 / math.sqrt(64))
    ref = _attn_ref(q, mem[:, :, :d], mem[:, :, d:], kl.tolist(), 0.125)
    assert rel(out, ref) < 1e-2
    assert out[2].float().abs().sum().item() == 0   # no keys -> zeros, never NaN


@pytest.mark.parametrize("dtype,H", [(torch.bfloat16, 8), (torch.float16, 8), (torch.bfloat16, 4)])
def test_attn_decode_fused_oproj(dtype, H):
    """The output projection fused into the decode attention launch: one f32 slab per
    head, slab[h, b] = o[b, h] W_o[:, h]^T; the sum over heads is o W_o^T (float64 ref).
    A finished utterance (stop_len) writes zero slabs.  H = 4 (W_o is [256, 256]): the waves
    past the 4 row blocks prefetch nothing (no read past the end of W_o)."""
    g = torch.Generator().manual_seed(11)
    B, d, Tm, t = 6, 64 * H, 300, 140
    mk = (lambda sh: _bf(sh, g)) if dtype == torch.bfloat16 else (lambda sh: _h(sh, g))
    qkv, cache = mk((B, 3 * d)), mk((B, Tm, 2 * d))
    wo = (torch.randn(d, d, generator=g) / math.sqrt(d)).to(dtype).cuda()
    tp = torch.tensor([t], dtype=torch.int32, device="cuda")
    stop = torch.tensor([1000, 1000, 50, 1000, 141, 1000], dtype=torch.int32, device="cuda")
    out = torch.empty(B, d, dtype=dtype, device="cuda")
    slab = torch.full((H, B, d), float("nan"), device="cuda")
    args = (qkv, cache, cache[:, :, d:], None, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, H, Tm)
    ops.attn_decode(*args, t_ptr=tp, scale=0.125, stop_len=stop, wo=wo, wo_ld=d, slab=slab)
    ref_o = _attn_ref(qkv[:, :d], cache[:, :, :d], cache[:, :, d:], [t + 1] * B, 0.125)
    done = (stop.cpu() <= t)
    ref_o[done] = 0.0
    w = wo.double().cpu()
    ref = torch.stack([ref_o[:, h * 64:(h + 1) * 64] @ w[:, h * 64:(h + 1) * 64].t() for h in range(H)])
    assert torch.isfinite(slab).all()
    assert rel(slab, ref) < 1e-2
    assert slab[:, 2].abs().sum().item() == 0
    assert rel(slab.sum(0), ref_o @ w.t()) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_attn_decode_fused_qproj(dtype):
    """The cross-attention query projection fused into the decode attention launch (with the
    output projection): q = x W_q^T + b_q per head in f32, then attention over ragged memory
    keys, then the per-head output slabs (float64 reference)."""
    g = torch.Generator().manual_seed(12)
    B, H, d, Tx = 5, 8, 512, 128
    mk = (lambda sh, sc=1.0: _bf(sh, g, sc)) if dtype == torch.bfloat16 else (lambda sh, sc=1.0: _h(sh, g, sc))
    x, mem = mk((B, d)), mk((B, Tx, 2 * d))
    wq, wo = mk((d, d), 1 / math.sqrt(d)), mk((d, d), 1 / math.sqrt(d))
    bq = torch.randn(d, generator=g).cuda()
    kl = torch.tensor([128, 1, 0, 77, 9], dtype=torch.int32, device="cuda")
    slab = torch.full((H, B, d), float("nan"), device="cuda")
    ops.attn_decode(x, mem, mem[:, :, d:], None, d, Tx * 2 * d, 2 * d, Tx * 2 * d, 2 * d, d, B, H, Tx, key_len=kl,
                    scale=0.125, wo=wo, wo_ld=d, slab=slab, wq=wq, wq_ld=d, bq=bq)
    q = x.double().cpu() @ wq.double().cpu().t() + bq.double().cpu()
    ref_o = _attn_ref(q, mem[:, :, :d], mem[:, :, d:], kl.tolist(), 0.125)
    w = wo.double().cpu()
    ref = torch.stack([ref_o[:, h * 64:(h + 1) * 64] @ w[:, h * 64:(h + 1) * 64].t() for h in range(H)])
    assert torch.isfinite(slab).all()
    assert rel(slab, ref) < 1e-2
    assert slab[:, 2].abs().sum().item() == 0   # no keys -> zero output, never NaN


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_attn_decode_fused_ln_prologue(dtype):
    """The self-attention sublayer's residual combine + LayerNorm inside the cross-attention
    launch (the decode step's fused schedule): bitwise the same row as tt2_ln_combine followed by
    the fused query projection on that row, written to ln_out by head 0; a finished utterance
    (stop_len) still gets its row."""
    g = torch.Generator().manual_seed(21)
    B, H, d, Tx = 6, 8, 512, 128
    mk = (lambda sh, sc=1.0: _bf(sh, g, sc)) if dtype == torch.bfloat16 else (lambda sh, sc=1.0: _h(sh, g, sc))
    x, mem = mk((B, d)), mk((B, Tx, 2 * d))
    wq, wo = mk((d, d), 1 / math.sqrt(d)), mk((d, d), 1 / math.sqrt(d))
    bq = torch.randn(d, generator=g).cuda()
    part = (torch.randn(H, B, d, generator=g) * 0.3).cuda()
    lb, lg, lbe = (torch.randn(d, generator=g).cuda() for _ in range(3))
    kl = torch.tensor([128, 5, 77, 128, 9, 64], dtype=torch.int32, device="cuda")
    step = torch.tensor([3], dtype=torch.int32, device="cuda")
    stop = torch.tensor([100, 100, 2, 100, 100, 100], dtype=torch.int32, device="cuda")   # row 2 finished
    h1 = torch.empty(B, d, dtype=dtype, device="cuda")
    ops.ln_combine(x, part, H, lb, lg, lbe, h1, B)
    slab_ref = torch.full((H, B, d), float("nan"), device="cuda")
    ops.attn_decode(h1, mem, mem[:, :, d:], None, d, Tx * 2 * d, 2 * d, Tx * 2 * d, 2 * d, d, B, H, Tx, key_len=kl,
                    scale=0.125, wo=wo, wo_ld=d, slab=slab_ref, wq=wq, wq_ld=d, bq=bq, stop_len=stop, step=step)
    out = torch.full((B, d), float("nan"), device="cuda").to(dtype)
    slab = torch.full((H, B, d), float("nan"), device="cuda")
    ops.attn_decode(x, mem, mem[:, :, d:], None, d, Tx * 2 * d, 2 * d, Tx * 2 * d, 2 * d, d, B, H, Tx, key_len=kl,
                    scale=0.125, wo=wo, wo_ld=d, slab=slab, wq=wq, wq_ld=d, bq=bq, stop_len=stop, step=step,
                    ln=(part, lb, lg, lbe, out, 1e-5))
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), h1.view(torch.int16))      # every row, the finished one too
    assert torch.equal(slab, slab_ref)
    assert slab[:, 2].abs().sum().item() == 0


def _h(shape, gen, scale=1.0):
    return (torch.randn(shape, generator=gen) * scale).half().cuda()


@pytest.mark.parametrize("m,n,k", [(32, 1536, 512), (64, 512, 2048), (17, 81, 512), (64, 256, 80)])
def test_skinny_gemm_fp16(m, n, k):
    g = torch.Generator().manual_seed(n + k)
    A, W = _h((m, k), g), _h((n, k), g, 0.1)
    bias = torch.randn(n, generator=g).cuda()
    C = torch.empty(m, n, dtype=torch.float16, device="cuda")
    ops.gemm(A, W, C, m, n, k, k, k, n, bias=bias, variant=3)
    assert rel(C, A.double() @ W.double().t() + bias.double()) < 2e-3


def test_fp16_kv_scatter_attention_ln_combine():
    g = torch.Generator().manual_seed(13)
    B, d, Tm, t = 48, 512, 64, 20
    x = _h((B, d), g)
    W = _h((3 * d, d), g, 0.05)
    qkv = torch.empty(B, 3 * d, dtype=torch.float16, device="cuda")
    cache = _h((B, Tm, 2 * d), g)
    tp = torch.tensor([t], dtype=torch.int32, device="cuda")
    ops.gemm(x, W, qkv, B, 3 * d, d, d, d, 3 * d, kv=(cache, tp, d, Tm * 2 * d, 2 * d), variant=3)
    assert torch.equal(cache[:, t], qkv[:, d:])
    out = torch.empty(B, d, dtype=torch.float16, device="cuda")
    ops.attn_decode(qkv, cache, cache[:, :, d:], out, 3 * d, Tm * 2 * d, 2 * d, Tm * 2 * d, 2 * d, d, B, 8, Tm,
                    t_ptr=tp, scale=0.125)
    ref = _attn_ref(qkv[:, :d], cache[:, :, :d], cache[:, :, d:], [t + 1] * B, 0.125)
    assert rel(out, ref) < 2e-3
    slab = torch.randn(4 * B * d, device="cuda")
    bias, gam, bet = (torch.randn(d, generator=g).cuda() for _ in range(3))
    y = torch.empty(B, d, dtype=torch.float16, device="cuda")
    ops.ln_combine(x, slab, 4, bias, gam, bet, y, B)
    s = x.double() + bias.double() + slab.view(4, B, d).double().sum(0)
    assert rel(y, F.layer_norm(s, (d,), gam.double(), bet.double(), 1e-5)) < 2e-3


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m", [1, 17, 32, 40, 64])
def test_ffn_decode_one_launch_equals_three(dtype, m):
    """tt2_ffn_decode (the FFN sublayer in one launch of 256 work groups ordered by device
    counters) writes bit for bit what the three launches it replaces write: the skinny FFN1
    with relu (hidden), the skinny FFN2 split-K slabs (8, raw f32) and tt2_ln_combine (y).
    Three calls in a row on NEW inputs into the same hidden / slab buffers (a reader that hit a
    stale cache line of the previous call would differ); the counters are re-armed after every
    call, no phase timed out, and y is LN(x + b2 + relu(x W1^T + b1) W2^T) against float64."""
    g = torch.Generator().manual_seed(100 + m)
    d, f = 512, 2048
    mk = (lambda sh, sc=1.0: _bf(sh, g, sc)) if dtype == torch.bfloat16 else (lambda sh, sc=1.0: _h(sh, g, sc))
    w1, w2 = mk((f, d), 1 / math.sqrt(d)), mk((d, f), 1 / math.sqrt(f))
    b1, b2, gam, bet = (torch.randn(n, generator=g).cuda() * 0.1 for n in (f, d, d, d))
    sync = torch.zeros(2048, dtype=torch.int32, device="cuda")
    hid = torch.full((m, f), float("nan"), device="cuda").to(dtype)
    slab = torch.full((8 * m * d,), float("nan"), device="cuda")
    for _ in range(3):
        x = mk((m, d))
        # reference: the three launches of the split schedule
        h_ref = torch.empty(m, f, dtype=dtype, device="cuda")
        ops.gemm(x, w1, h_ref, m, f, d, d, d, f, bias=b1, act=1, variant=3)
        slab_ref = torch.full((8 * m * d,), float("nan"), device="cuda")

        class WS:
            def get(self, nbytes):
                assert nbytes <= slab_ref.numel() * 4
                return slab_ref

        dummy = torch.empty(m, d, dtype=dtype, device="cuda")
        ops.gemm(h_ref, w2, dummy, m, d, f, f, f, d, splits=8, main_only=True, ws=WS(), variant=3)
        y_ref = torch.empty(m, d, dtype=dtype, device="cuda")
        ops.ln_combine(x, slab_ref, 8, b2, gam, bet, y_ref, m)
        y = torch.full((m, d), float("nan"), device="cuda").to(dtype)
        ops.ffn_decode(x, w1, b1, w2, b2, gam, bet, hid, slab, sync, y, m)
        torch.cuda.synchronize()
        assert int(sync.abs().sum()) == 0, sync.tolist()
        assert torch.equal(hid.view(torch.int16), h_ref.view(torch.int16))
        assert torch.equal(slab, slab_ref)
        assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
    hd = torch.relu(x.double() @ w1.double().t() + b1.double())
    ref = F.layer_norm(x.double() + b2.double() + hd @ w2.double().t(), (d,), gam.double(), bet.double(), 1e-5)
    assert rel(y, ref) < 2e-2


def test_ffn_decode_rejects_unsupported_shapes():
    """m > 64, d_ffn != 2048 or f32: TT2_E_INVALID before any launch (the decoder then keeps the
    three-launch FFN)."""
    g = torch.Generator().manual_seed(5)
    d = 512
    for m, f, dtype in ((65, 2048, torch.bfloat16), (8, 1024, torch.bfloat16), (8, 2048, torch.float32)):
        x = torch.randn(m, d, generator=g).cuda().to(dtype)
        w1, w2 = torch.zeros(f, d, device="cuda", dtype=dtype), torch.zeros(d, f, device="cuda", dtype=dtype)
        v = torch.zeros(f, device="cuda")
        hid = torch.zeros(m, f, device="cuda", dtype=dtype)
        slab = torch.zeros(8 * m * d, device="cuda")
        sync = torch.zeros(2048, dtype=torch.int32, device="cuda")
        with pytest.raises(RuntimeError, match="tt2_ffn_decode"):
            ops.ffn_decode(x, w1, v, w2, v[:d], v[:d], v[:d], hid, slab, sync, x.clone(), m)
