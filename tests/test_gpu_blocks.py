"""Block-level C ABI (include/tt2_capi.h tt2_*_fwd / _bwd) against float64
references built from the oracle's blocks (oracle/tt2_oracle.py: MHA pinned to
nn.MultiheadAttention, hash dropout, tts_loss) and torch autograd.  Every call goes
through ctypes, the way a non-Python host binds the library.

Tolerances: exact-f32 mode (TT2_DT_F32: f32-input MFMA) 2e-4 relative L2 on every output
and gradient; bf16 mode 3e-2 (bf16 activations / weights, f32 accumulation)."""
import ctypes as C
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from tt2 import _lib  # noqa: E402
from tt2_oracle import MHA, dropout_keep, tts_loss  # noqa: E402

D, H, FF = 512, 8, 2048
TOL = {torch.float32: 2e-4, torch.bfloat16: 3e-2}


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def P(t):
    return None if t is None else t.data_ptr()


def S():
    return torch.cuda.current_stream().cuda_stream


def L():
    return _lib.lib()


def desc(dtype, **kw):
    d = _lib.Desc()
    d.d_model, d.n_heads, d.d_ffn = D, H, FF
    d.dtype = _lib.DT_BF16 if dtype == torch.bfloat16 else _lib.DT_F32
    d.eps, d.momentum, d.pos_weight, d.grad_scale = 1e-5, 0.1, 5.0, 1.0
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def buf(nbytes):
    return torch.zeros(max(int(nbytes), 1), dtype=torch.uint8, device="cuda")


def call(name, *args):
    _lib.check(getattr(L(), name)(*args), name)


def seed_t(v):
    return torch.tensor([v], dtype=torch.int32, device="cuda")


def keep_mask(seed, site, shape, p):
    n = math.prod(shape)
    return torch.from_numpy(dropout_keep(seed, site, n, p)).reshape(shape).double() / (1.0 - p)


def rnd(shape, g, scale=1.0):
    return torch.randn(shape, generator=g, dtype=torch.float64) * scale


def dev(t, dtype):
    return t.to(dtype).cuda().contiguous()


# ----------------------------------------------------------------- attention sublayer
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cross", [False, True])
def test_attn_block(dtype, cross):
    g = torch.Generator().manual_seed(3 + cross)
    B, Tq, Tk = 3, 40, (29 if cross else 40)
    p_drop, site, seed = 0.1, 81, 12345
    klen = torch.tensor([Tk, 0 if cross else 17, Tk - 5], dtype=torch.int32)
    x = rnd((B, Tq, D), g)
    mem = rnd((B, Tk, D), g) if cross else None
    w_in, b_in = rnd((3 * D, D), g, D ** -0.5), rnd((3 * D,), g, 0.1)
    w_out, b_out = rnd((D, D), g, D ** -0.5), rnd((D,), g, 0.1)
    ln_g, ln_b = 1 + rnd((D,), g, 0.1), rnd((D,), g, 0.1)
    dy = rnd((B, Tq, D), g)
    # device copies (bf16 mode: the reference runs on the same rounded values)
    xs = [x, mem, w_in, w_out, dy]
    if dtype == torch.bfloat16:
        x, mem, w_in, w_out, dy = [None if t is None else t.bfloat16().double() for t in xs]
    d = desc(dtype, batch=B, tq=Tq, tk=Tk, causal=int(not cross), cross=int(cross), training=1, dropout=p_drop,
             site=site)
    sd = seed_t(seed)
    kl = klen.cuda()
    d.seed, d.k_len = sd.data_ptr(), kl.data_ptr()
    X, M = dev(x, dtype), (dev(mem, dtype) if cross else None)
    Wi, Wo = dev(w_in, dtype), dev(w_out, dtype)
    bi, bo, lg, lb = (t.float().cuda() for t in (b_in, b_out, ln_g, ln_b))
    Y = torch.empty(B * Tq, D, dtype=dtype, device="cuda")
    saved = buf(L().tt2_attn_block_saved_size(C.byref(d)))
    ws = buf(L().tt2_attn_block_workspace_size(C.byref(d)))
    call("tt2_attn_block_fwd", C.byref(d), P(X), P(M), P(Wi), P(bi), P(Wo), P(bo), P(lg), P(lb), P(Y), P(saved),
         P(ws), ws.numel(), S())
    dX = torch.empty_like(X)
    dM = torch.empty_like(M) if cross else None
    dWi, dbi = torch.empty(3 * D, D, device="cuda"), torch.empty(3 * D, device="cuda")
    dWo, dbo = torch.empty(D, D, device="cuda"), torch.empty(D, device="cuda")
    dlg, dlb = torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    call("tt2_attn_block_bwd", C.byref(d), P(X), P(M), P(Wi), P(Wo), P(lg), P(lb), P(saved), P(dev(dy, dtype)),
         P(dX), P(dM), P(dWi), P(dbi), P(dWo), P(dbo), P(dlg), P(dlb), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    # reference: the oracle's MHA (f32 scores by construction, so the whole reference runs in f32 on the CPU)
    mha = MHA(D, H)
    with torch.no_grad():
        mha.in_proj_weight.copy_(w_in)
        mha.in_proj_bias.copy_(b_in)
        mha.out_proj.weight.copy_(w_out)
        mha.out_proj.bias.copy_(b_out)
    xr = x.float().requires_grad_()
    mr = mem.float().requires_grad_() if cross else xr
    lgr, lbr = ln_g.float().requires_grad_(), ln_b.float().requires_grad_()
    o, _ = mha(xr, mr, key_len=klen.long(), causal=not cross)
    o = o * keep_mask(seed, site, (B, Tq, D), p_drop).float()
    y = F.layer_norm(xr + o, (D,), lgr, lbr, 1e-5)
    y.backward(dy.float())
    tol = TOL[dtype]
    assert rel(Y.view(B, Tq, D), y.detach()) < tol
    assert rel(dX.view(B, Tq, D), xr.grad) < tol
    if cross:
        assert rel(dM.view(B, Tk, D), mr.grad) < tol
    assert rel(dWi, mha.in_proj_weight.grad) < tol
    assert rel(dbi, mha.in_proj_bias.grad) < tol
    assert rel(dWo, mha.out_proj.weight.grad) < tol
    assert rel(dbo, mha.out_proj.bias.grad) < tol
    assert rel(dlg, lgr.grad) < tol and rel(dlb, lbr.grad) < tol


# ------------------------------------------------------------------------ FFN sublayer
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ffn_block(dtype):
    g = torch.Generator().manual_seed(5)
    B, T, site, seed, p = 2, 72, 82, 99, 0.1
    x = rnd((B * T, D), g)
    w1, b1 = rnd((FF, D), g, D ** -0.5), rnd((FF,), g, 0.1)
    w2, b2 = rnd((D, FF), g, FF ** -0.5), rnd((D,), g, 0.1)
    ln_g, ln_b = 1 + rnd((D,), g, 0.1), rnd((D,), g, 0.1)
    dy = rnd((B * T, D), g)
    if dtype == torch.bfloat16:
        x, w1, w2, dy = (t.bfloat16().double() for t in (x, w1, w2, dy))
    d = desc(dtype, batch=B, tq=T, training=1, dropout=p, site=site)
    sd = seed_t(seed)
    d.seed = sd.data_ptr()
    X, W1, W2 = dev(x, dtype), dev(w1, dtype), dev(w2, dtype)
    B1, B2, lg, lb = (t.float().cuda() for t in (b1, b2, ln_g, ln_b))
    Y = torch.empty_like(X)
    saved = buf(L().tt2_ffn_saved_size(C.byref(d)))
    ws = buf(L().tt2_ffn_workspace_size(C.byref(d)))
    call("tt2_ffn_fwd", C.byref(d), P(X), P(W1), P(B1), P(W2), P(B2), P(lg), P(lb), P(Y), P(saved), P(ws),
         ws.numel(), S())
    dX = torch.empty_like(X)
    g1, gb1, g2, gb2 = (torch.empty(s, device="cuda") for s in ((FF, D), (FF,), (D, FF), (D,)))
    gg, gb = torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    call("tt2_ffn_bwd", C.byref(d), P(X), P(W1), P(W2), P(lg), P(lb), P(saved), P(dev(dy, dtype)), P(dX), P(g1),
         P(gb1), P(g2), P(gb2), P(gg), P(gb), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    xr = x.clone().requires_grad_()
    ps = [t.clone().requires_grad_() for t in (w1, b1, w2, b2, ln_g, ln_b)]
    h = F.relu(F.linear(xr, ps[0], ps[1])) * keep_mask(seed, site, (B * T, FF), p)
    f = F.linear(h, ps[2], ps[3]) * keep_mask(seed, site + 1, (B * T, D), p)
    y = F.layer_norm(xr + f, (D,), ps[4], ps[5], 1e-5)
    y.backward(dy)
    tol = TOL[dtype]
    assert rel(Y, y.detach()) < tol
    assert rel(dX, xr.grad) < tol
    for got, ref in zip((g1, gb1, g2, gb2, gg, gb), ps):
        assert rel(got, ref.grad) < tol


# --------------------------------------------------------------- linear / add + LN
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_and_add_ln(dtype):
    g = torch.Generator().manual_seed(6)
    B, T, ci, co = 2, 50, 80, 256
    x, w, b, dy = rnd((B * T, ci), g), rnd((co, ci), g, ci ** -0.5), rnd((co,), g), rnd((B * T, co), g)
    if dtype == torch.bfloat16:
        x, w, dy = (t.bfloat16().double() for t in (x, w, dy))
    d = desc(dtype, batch=B, tq=T, c_in=ci, c_out=co)
    X, W, Bb = dev(x, dtype), dev(w, dtype), b.float().cuda()
    Y = torch.empty(B * T, co, dtype=dtype, device="cuda")
    ws = buf(L().tt2_linear_workspace_size(C.byref(d)))
    call("tt2_linear_fwd", C.byref(d), P(X), P(W), P(Bb), P(Y), P(ws), ws.numel(), S())
    dX, dW, db = torch.empty_like(X), torch.empty(co, ci, device="cuda"), torch.empty(co, device="cuda")
    call("tt2_linear_bwd", C.byref(d), P(X), P(W), P(dev(dy, dtype)), P(dX), P(dW), P(db), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel(Y, F.linear(x, w, b)) < tol
    assert rel(dX, dy @ w) < tol and rel(dW, dy.t() @ x) < tol and rel(db, dy.sum(0)) < tol
    # add + LN with dropout on the branch
    site, seed, p = 80, 7, 0.1
    xa, br, gy = rnd((B * T, D), g), rnd((B * T, D), g), rnd((B * T, D), g)
    lg, lb = 1 + rnd((D,), g, 0.1), rnd((D,), g, 0.1)
    if dtype == torch.bfloat16:
        xa, br, gy = (t.bfloat16().double() for t in (xa, br, gy))
    d = desc(dtype, batch=B, tq=T, training=1, dropout=p, site=site)
    sd = seed_t(seed)
    d.seed = sd.data_ptr()
    XA, BR = dev(xa, dtype), dev(br, dtype)
    G_, B_ = lg.float().cuda(), lb.float().cuda()
    Y = torch.empty_like(XA)
    saved = buf(L().tt2_add_ln_saved_size(C.byref(d)))
    call("tt2_add_ln_fwd", C.byref(d), P(XA), P(BR), P(G_), P(B_), P(Y), P(saved), S())
    ws = buf(L().tt2_add_ln_workspace_size(C.byref(d)))
    dX, dB = torch.empty_like(XA), torch.empty_like(BR)
    dg, dbb = torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    call("tt2_add_ln_bwd", C.byref(d), P(XA), P(BR), P(G_), P(saved), P(dev(gy, dtype)), P(dX), P(dB), P(dg),
         P(dbb), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    xr, brr = xa.clone().requires_grad_(), br.clone().requires_grad_()
    lgr, lbr = lg.clone().requires_grad_(), lb.clone().requires_grad_()
    y = F.layer_norm(xr + brr * keep_mask(seed, site, (B * T, D), p), (D,), lgr, lbr, 1e-5)
    y.backward(gy)
    assert rel(Y, y.detach()) < tol
    assert rel(dX, xr.grad) < tol and rel(dB, brr.grad) < tol
    assert rel(dg, lgr.grad) < tol and rel(dbb, lbr.grad) < tol


# ------------------------------------------------------------ conv1d + BN + act
@pytest.mark.parametrize("dtype,T,act,res", [(torch.float32, 48, 2, False), (torch.bfloat16, 80, 1, False),
                                             (torch.float32, 48, 0, True)])
def test_conv1d_bn_act(dtype, T, act, res):
    g = torch.Generator().manual_seed(7 + act)
    B, ci, co, K, site, seed, p = 2, 80, 512, 5, 112, 3, 0.5
    if res:
        ci, co = 512, 80
    x = rnd((B, T, ci), g)
    w_ref, b = rnd((co, ci, K), g, (ci * K) ** -0.5), rnd((co,), g, 0.1)
    bn_g, bn_b = 1 + rnd((co,), g, 0.1), rnd((co,), g, 0.1)
    r = rnd((B, T, co), g) if res else None
    dout = rnd((B, T, co), g)
    if dtype == torch.bfloat16:
        x, w_ref, dout = (t.bfloat16().double() for t in (x, w_ref, dout))
    d = desc(dtype, batch=B, tq=T, c_in=ci, c_out=co, kernel=K, act=act, training=1, dropout=p, site=site)
    sd = seed_t(seed)
    d.seed = sd.data_ptr()
    X, Wr = dev(x, dtype), dev(w_ref, dtype)
    Wp = torch.empty_like(Wr)
    call("tt2_conv_weight_pack", P(Wr), P(Wp), co, ci, K, d.dtype, S())
    Bb, G_, Be = b.float().cuda(), bn_g.float().cuda(), bn_b.float().cuda()
    rm, rv = torch.zeros(co, device="cuda"), torch.ones(co, device="cuda")
    R = r.float().cuda() if res else None
    out = torch.empty(B * T, co, dtype=dtype, device="cuda")
    saved = buf(L().tt2_conv1d_bn_act_saved_size(C.byref(d)))
    ws = buf(L().tt2_conv1d_bn_act_workspace_size(C.byref(d)))
    call("tt2_conv1d_bn_act_fwd", C.byref(d), P(X), P(Wp), P(Bb), P(G_), P(Be), P(rm), P(rv), P(R),
         _lib.DT_F32, P(out), P(saved), P(ws), ws.numel(), S())
    dX = torch.empty_like(X)
    dW, db = torch.empty(co, K * ci, device="cuda"), torch.empty(co, device="cuda")
    dg, dbb = torch.empty(co, device="cuda"), torch.empty(co, device="cuda")
    call("tt2_conv1d_bn_act_bwd", C.byref(d), P(X), P(Wp), P(G_), P(Be), P(saved), P(dev(dout, dtype)), P(dX),
         P(dW), P(db), P(dg), P(dbb), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    xr = x.clone().requires_grad_()
    wr, br, gr, ber = (t.clone().requires_grad_() for t in (w_ref, b, bn_g, bn_b))
    y = F.conv1d(xr.transpose(1, 2), wr, br, padding=(K - 1) // 2)
    mean, var = y.mean((0, 2)), y.var((0, 2), unbiased=False)
    z = (y - mean[None, :, None]) / torch.sqrt(var[None, :, None] + 1e-5) * gr[None, :, None] + ber[None, :, None]
    z = {0: z, 1: F.relu(z), 2: torch.tanh(z)}[act].transpose(1, 2)
    z = z * keep_mask(seed, site, (B, T, co), p)
    if res:
        z = z + r
    z.backward(dout)
    tol = TOL[dtype]
    assert rel(out.view(B, T, co), z.detach()) < tol
    assert rel(dX.view(B, T, ci), xr.grad) < tol
    assert rel(dW.view(co, K, ci).permute(0, 2, 1), wr.grad) < tol
    assert rel(dg, gr.grad) < tol and rel(dbb, ber.grad) < tol
    # a conv bias in front of training-mode BN gets an analytically zero gradient
    assert db.abs().max().item() < (1e-3 if dtype == torch.float32 else 0.5)
    assert rel(rm, 0.1 * mean.detach()) < tol
    assert rel(rv, 0.9 + 0.1 * y.detach().var((0, 2), unbiased=True)) < tol * (10 if dtype != torch.float32 else 1)


# ------------------------------------------------------------------ heads + loss
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_heads_and_loss(dtype):
    g = torch.Generator().manual_seed(8)
    B, T, NM, LD = 3, 40, 80, 96
    x = rnd((B * T, D), g)
    w, b = rnd((NM + 1, D), g, D ** -0.5), rnd((NM + 1,), g, 0.1)
    if dtype == torch.bfloat16:
        x, w = (t.bfloat16().double() for t in (x, w))
    mel_len = torch.tensor([T, 23, 31], dtype=torch.int32)
    d = desc(dtype, batch=B, tq=T, n_mels=NM, heads_ld=LD)
    ml = mel_len.cuda()
    d.mel_len = ml.data_ptr()
    X, W, Bb = dev(x, dtype), dev(w, dtype), b.float().cuda()
    heads = torch.zeros(B * T, LD, device="cuda")
    ws = buf(L().tt2_heads_workspace_size(C.byref(d)))
    call("tt2_heads_fwd", C.byref(d), P(X), P(W), P(Bb), P(heads), P(ws), ws.numel(), S())
    target = rnd((B, T, NM), g)
    after = heads[:, :NM].double().cpu() + rnd((B * T, NM), g, 0.1)
    Af, Tg = after.float().cuda(), target.float().cuda()
    lws = buf(L().tt2_loss_block_workspace_size(C.byref(d)))
    lf, lb = torch.zeros(4, device="cuda"), torch.zeros(4, device="cuda")
    call("tt2_loss_fwd", C.byref(d), P(heads), P(Af), P(Tg), P(lf), P(lws), lws.numel(), S())
    gh = torch.zeros(B * T, LD, device="cuda")
    ga = torch.empty(B * T, NM, dtype=dtype, device="cuda")
    call("tt2_loss_bwd", C.byref(d), P(heads), P(Af), P(Tg), P(lb), P(gh), P(ga), P(lws), lws.numel(), S())
    dX, dW, db = torch.empty_like(X), torch.empty(NM + 1, D, device="cuda"), torch.empty(NM + 1, device="cuda")
    call("tt2_heads_bwd", C.byref(d), P(X), P(W), P(gh), P(dX), P(dW), P(db), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    # reference: heads = x W^T + b; loss via the oracle's tts_loss
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    hd = F.linear(xr, wr, br)
    bef, stop = hd[:, :NM].view(B, T, NM), hd[:, NM].view(B, T)
    aft = after.view(B, T, NM).clone().requires_grad_()
    total, parts = tts_loss(bef, aft, stop, target, mel_len.long(), 5.0)
    total.backward()
    tol = TOL[dtype]
    assert rel(heads[:, :NM + 1], hd.detach()) < tol
    ref4 = torch.tensor([total.item(), parts["mel_before"].item(), parts["mel_after"].item(), parts["stop"].item()]) \
        if isinstance(parts, dict) else None
    if ref4 is not None:
        assert rel(lf.cpu(), ref4) < 1e-4
    assert torch.equal(lf, lb)
    assert rel(ga.view(B, T, NM), aft.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    assert rel(dX, xr.grad) < tol and rel(dW, wr.grad) < tol and rel(db, br.grad) < tol


# ----------------------------------------------------------- DP bucket all-reduce
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_allreduce_bucket_one_rank(dtype):
    """tt2_comm_* + tt2_allreduce_bucket on a 1-rank RCCL communicator: the SUM is the
    identity, in place, on the caller's stream (multi-rank runs: tt2/dist.py's RCCL path)."""
    Lb = L()
    uid = (C.c_char * 128)()
    call("tt2_comm_unique_id", uid)
    comm = C.c_void_p()
    call("tt2_comm_init", C.byref(comm), 1, uid, 0)
    try:
        x = torch.randn(1 << 20, device="cuda").to(dtype)
        ref = x.clone()
        call("tt2_allreduce_bucket", P(x), x.numel(), _lib.DT_F32 if dtype == torch.float32 else _lib.DT_BF16,
             comm, S())
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        assert Lb.tt2_allreduce_bucket(P(x), 4, 7, comm, S()) != 0   # bad dtype is an error, not a launch
    finally:
        call("tt2_comm_destroy", comm)
