"""Fused residual + dropout + LayerNorm forward/backward vs float64 torch (GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2_oracle import dropout_keep  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("m", [1, 37, 2048, 5000])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_fwd_bwd_dbias(dtype, m, p):
    C = 512
    g = torch.Generator().manual_seed(m + int(p * 10))
    x = torch.randn(m, C, generator=g)
    br = torch.randn(m, C, generator=g)
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(m, C, generator=g)
    xd, brd, dyd = x.to(dtype).cuda(), br.to(dtype).cuda(), dy.to(dtype).cuda()
    seed = torch.tensor([99], dtype=torch.int32).cuda()
    drop = ops.Drop(seed, 17, p)
    y = torch.empty(m, C, dtype=dtype, device="cuda")
    mean = torch.empty(m, device="cuda")
    rstd = torch.empty(m, device="cuda")
    ops.layernorm_fwd(xd, brd, gamma.cuda(), beta.cuda(), y, mean, rstd, m, drop=drop)

    keep = torch.from_numpy(dropout_keep(99, 17, m * C, p)).view(m, C).double() if p > 0 else torch.ones(m, C,
                                                                                                           dtype=torch.float64)
    xr = x.to(dtype).double()
    brr = br.to(dtype).double().requires_grad_(True)
    s = xr.requires_grad_(True) + brr * keep / (1 - p)
    yr = torch.nn.functional.layer_norm(s, (C,), gamma.double().requires_grad_(True),
                                        beta.double().requires_grad_(True), eps=1e-5)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(y, yr) < tol
    yr.backward(dy.to(dtype).double())

    dx = torch.empty(m, C, dtype=dtype, device="cuda")
    dbr = torch.empty(m, C, dtype=dtype, device="cuda")
    dgamma = torch.full((C,), 0.5, device="cuda")
    dbeta = torch.zeros(C, device="cuda")
    dbias = torch.full((C,), 0.25, device="cuda")
    ops.layernorm_bwd(dyd, xd, brd, gamma.cuda(), mean, rstd, dx, dbr, dgamma, dbeta, m, drop=drop, dbias=dbias)
    tol_b = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(dx, xr.grad) < tol_b
    assert rel(dbr, brr.grad) < tol_b
    # grads overwrite (grad_beta 0) the destinations
    ref_g = (dy.to(dtype).double() * (s - s.mean(1, keepdim=True)) /
             (s.var(1, unbiased=False, keepdim=True) + 1e-5).sqrt()).sum(0)
    assert rel(dgamma, ref_g.detach()) < tol_b
    assert rel(dbeta, dy.to(dtype).double().sum(0)) < tol_b
    assert rel(dbias, brr.grad.sum(0)) < tol_b


@pytest.mark.parametrize("m1,m2", [(12800, 12800), (2048, 12800), (12800, 37), (5, 2048)])
def test_layernorm_bwd_chained_finalize(m1, m2):
    """A deferred LayerNorm backward (defer=True) completed inside the next one's launch
    (prev=) or by layernorm_bwd_finalize equals the immediate finalize (f32 sums in another
    fixed order: 1e-5), and a grad_beta accumulation is carried through the chain."""
    C = 512
    g = torch.Generator().manual_seed(m1 + m2)
    calls = []
    for m in (m1, m2):
        x, br, dy = (torch.randn(m, C, generator=g).bfloat16().cuda() for _ in range(3))
        gamma = (1 + 0.1 * torch.randn(C, generator=g)).cuda()
        beta = torch.zeros(C, device="cuda")
        y = torch.empty_like(x)
        mean, rstd = torch.empty(m, device="cuda"), torch.empty(m, device="cuda")
        ops.layernorm_fwd(x, br, gamma, beta, y, mean, rstd, m)
        calls.append((dy, x, br, gamma, mean, rstd, m))

    def run(mode):
        outs = []
        parts = [torch.empty(ops.layernorm_bwd_workspace_size(1 << 30, C), dtype=torch.uint8, device="cuda")
                 for _ in range(2)]
        prev = None
        for i, (dy, x, br, gamma, mean, rstd, m) in enumerate(calls):
            dx, dbr = torch.empty_like(x), torch.empty_like(x)
            dg, db, dbias = (torch.full((C,), 0.5, device="cuda") for _ in range(3))
            kw = {}
            if mode != "plain" and i == 0:
                kw = dict(part=parts[0], defer=True)
            a = ops.layernorm_bwd(dy, x, br, gamma, mean, rstd, dx, dbr, dg, db, m, dbias=dbias,
                                  prev=prev if mode == "chain" else None, **kw)
            if mode == "standalone" and i == 0:
                ops.layernorm_bwd_finalize(a)
            if mode == "grouped" and i == 0:   # completed in a (here empty) grouped GEMM's reduce launch
                ops.gemm_grouped([], fin=a)
            prev = a
            outs.append((dx, dbr, dg, db, dbias))
        torch.cuda.synchronize()
        return outs

    ref, chain, alone, grouped = run("plain"), run("chain"), run("standalone"), run("grouped")
    for got in (chain, alone, grouped):
        for (rx, rb, rg, rbe, rbi), (gx, gb, gg, gbe, gbi) in zip(ref, got):
            assert torch.equal(rx, gx) and torch.equal(rb, gb)
            for r, v in ((rg, gg), (rbe, gbe), (rbi, gbi)):
                assert rel(v, r) < 1e-5
    # chained and standalone completions share one summation order: bitwise equal
    for a_, b_, c_ in zip(chain[0][2:], alone[0][2:], grouped[0][2:]):
        assert torch.equal(a_, b_) and torch.equal(a_, c_)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("m,c,act,res", [(1000, 512, 1, False), (333, 80, 0, True), (64, 512, 2, False),
                                         (12800, 80, 2, True), (12800, 512, 1, False), (12800, 512, 2, False)])
def test_batchnorm_train_fwd_bwd(dtype, m, c, act, res):
    """Training-mode BatchNorm1d over rows + act + dropout (+ residual): forward, running
    statistics and backward vs float64 torch, up to cfg2's 12800 post-net rows (B = 16 x 800
    frames; C = 80 is the last post-net layer with the residual, C = 512 the tanh layers);
    repeated calls give bitwise the same statistics and gradients."""
    g = torch.Generator().manual_seed(m + c + act)
    y = (torch.randn(m, c, generator=g) * 3 + 1.5)
    gamma = 1 + 0.1 * torch.randn(c, generator=g)
    beta = 0.1 * torch.randn(c, generator=g)
    dout = torch.randn(m, c, generator=g)
    r = torch.randn(m, 96, generator=g) if res else None
    p = 0.2
    seed = torch.tensor([7], dtype=torch.int32).cuda()
    drop = ops.Drop(seed, 33, p)
    yd, dd = y.to(dtype).cuda(), dout.to(dtype).cuda()
    mean = torch.empty(c, device="cuda")
    rstd = torch.empty(c, device="cuda")
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    out = torch.empty(m, c, dtype=dtype, device="cuda")
    ops.batchnorm_fwd(yd, gamma.cuda(), beta.cuda(), mean, rstd, rm, rv, out, m, c, act, True, drop=drop,
                      res=r.cuda() if res else None, res_ld=96)
    keep = torch.from_numpy(dropout_keep(7, 33, m * c, p)).view(m, c).double()
    yr = y.to(dtype).double().requires_grad_(True)
    gr, br = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    z = torch.nn.functional.batch_norm(yr, None, None, gr, br, training=True, eps=1e-5)
    z = z.relu() if act == 1 else (z.tanh() if act == 2 else z)
    o = z * keep / (1 - p)
    if res:
        o = o + r[:, :c].double()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(out, o) < tol
    yv = y.to(dtype).double()
    assert rel(rm, 0.1 * yv.mean(0)) < 1e-5
    assert rel(rv, 0.9 + 0.1 * yv.var(0, unbiased=True)) < 1e-5
    o.backward(dout.to(dtype).double())
    dy = torch.empty(m, c, dtype=dtype, device="cuda")
    dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ops.batchnorm_bwd(yd, dd, gamma.cuda(), beta.cuda(), mean, rstd, dy, dg, db, m, c, act, drop=drop)
    tol_b = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(dy, yr.grad) < tol_b
    assert rel(dg, gr.grad) < tol_b
    assert rel(db, br.grad) < tol_b
    for _ in range(2):   # fixed reduction order: repeated calls are bitwise identical
        m2, r2, o2 = torch.empty_like(mean), torch.empty_like(rstd), torch.empty_like(out)
        ops.batchnorm_fwd(yd, gamma.cuda(), beta.cuda(), m2, r2, torch.zeros(c, device="cuda"),
                          torch.ones(c, device="cuda"), o2, m, c, act, True, drop=drop,
                          res=r.cuda() if res else None, res_ld=96)
        dy2, dg2, db2 = torch.empty_like(dy), torch.empty_like(dg), torch.empty_like(db)
        ops.batchnorm_bwd(yd, dd, gamma.cuda(), beta.cuda(), m2, r2, dy2, dg2, db2, m, c, act, drop=drop)
        assert torch.equal(m2, mean) and torch.equal(r2, rstd) and torch.equal(o2, out)
        assert torch.equal(dy2, dy) and torch.equal(dg2, dg) and torch.equal(db2, db)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cout,cin", [(512, 512), (80, 512), (512, 80), (100, 70)])
def test_conv_weight_flip(dtype, cout, cin):
    """wd[ci][tap'][co] = w[co][K-1-tap'][ci] (the conv dgrad weight, internal [Cout][tap][Cin])."""
    from tt2 import ops
    K = 5
    w = torch.randn(cout, K, cin, device="cuda").to(dtype)
    wd = torch.empty(cin, K * cout, device="cuda", dtype=dtype)
    ops.conv_weight_flip(w, wd, cout, cin, K)
    ref = w.flip(1).permute(2, 1, 0).reshape(cin, K * cout)
    assert torch.equal(wd, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_weight_flip_batch(dtype):
    """All conv layers' flips in one launch == the per-layer flip (ragged channel counts and
    kernel widths, so jobs span different work-item ranges)."""
    from tt2 import ops
    shapes = [(512, 512, 5), (80, 512, 5), (512, 80, 5), (100, 70, 3), (64, 64, 1)]
    jobs = []
    for cout, cin, K in shapes:
        w = torch.randn(cout, K, cin, device="cuda").to(dtype)
        jobs.append((w, torch.empty(cin, K * cout, device="cuda", dtype=dtype), cout, cin, K))
    ops.conv_weight_flip_batch(jobs)
    for w, wd, cout, cin, K in jobs:
        assert torch.equal(wd, w.flip(1).permute(2, 1, 0).reshape(cin, K * cout))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c,t_offset", [(512, 0), (512, 3), (36, 0)])
def test_posenc_fwd(dtype, c, t_offset):
    """out = drop(x + alpha * pe[t % T + t_offset]) (8-wide path for C % 8 == 0, scalar else)."""
    from tt2 import ops
    B, T = 3, 37
    m = B * T
    x = torch.randn(m, c, device="cuda").to(dtype)
    pe = torch.randn(T + 8, c, device="cuda")
    alpha = torch.tensor([1.7], device="cuda")
    out = torch.empty_like(x)
    seed = torch.tensor([5], dtype=torch.int32, device="cuda")
    ops.posenc_fwd(x, alpha, pe, out, m, T, drop=ops.Drop(seed, 9, 0.2), t_offset=t_offset)
    rows = torch.arange(m, device="cuda") % T + t_offset
    ref = x.double() + 1.7 * pe.double()[rows]
    keep = torch.from_numpy(dropout_keep(5, 9, m * c, 0.2)).view(m, c).cuda()
    ref = ref * keep / 0.8
    assert rel(out, ref) < (1e-6 if dtype == torch.float32 else 8e-3)
