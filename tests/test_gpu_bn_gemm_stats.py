"""BatchNorm statistics fused into the producing conv GEMM (tt2_gemm col_stats / bn_bwd +
tt2_bn_args stats_rows, GPU), on both kernels that carry them (64-row chunks on the 64 x 64
kernel, 256-row chunks on the 256 x 128 one; tt2_gemm_stats_rows says which): the chunk
statistics against float64 of the stored bf16 output, the BatchNorm forward / backward from them
against the BatchNorm's own statistics pass, and the requests the fusion refuses
(tests/test_gpu_norm.py covers the BatchNorm kernels themselves)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU, ACT_TANH, TT2Error  # noqa: E402


def _conv(m, cin, cout, T, g):
    """a post-net conv as the engine issues it: implicit im2col over T-frame utterances"""
    K, pad = 5, 2
    x = torch.randn(m, cin, generator=g).bfloat16().cuda()
    w = (torch.randn(cout, K * cin, generator=g) / (K * cin) ** 0.5).bfloat16().cuda()
    b = (0.1 * torch.randn(cout, generator=g)).cuda()
    return x, w, b, (T, cin, pad), K * cin


@pytest.mark.parametrize("m,cin,cout,T,rows", [(12800, 512, 512, 800, 256), (12800, 80, 512, 800, 256),
                                               (12500, 512, 512, 125, 256), (3 * 96, 512, 256, 96, 64),
                                               (1000, 512, 128, 125, 64), (2048, 512, 512, 128, 64)])
def test_gemm_col_stats(m, cin, cout, T, rows):
    g = torch.Generator().manual_seed(m + cin)
    x, w, b, conv, k = _conv(m, cin, cout, T, g)
    y = torch.empty(m, cout, dtype=torch.bfloat16, device="cuda")
    assert ops.gemm_stats_rows(x, w, y, m, cout, k, cin, k, cout, bias=b, a_conv=conv) == rows
    R = (m + rows - 1) // rows
    st = torch.full((2 * R * cout,), float("nan"), device="cuda")
    ops.gemm(x, w, y, m, cout, k, cin, k, cout, bias=b, a_conv=conv, col_stats=st)
    y_ref = torch.empty_like(y)   # the same kernel (the auto plan) without the statistics
    ops.gemm(x, w, y_ref, m, cout, k, cin, k, cout, bias=b, a_conv=conv)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)          # the statistics do not change what is stored
    yd = y.double().cpu()
    st = st.view(R, 2, cout).double().cpu()
    for r in range(R):
        blk = yd[r * rows:(r + 1) * rows]
        mu = blk.mean(0)
        m2 = ((blk - mu) ** 2).sum(0)
        assert torch.allclose(st[r, 0], mu, rtol=1e-5, atol=1e-6), (r, (st[r, 0] - mu).abs().max())
        assert torch.allclose(st[r, 1], m2, rtol=1e-4, atol=1e-4 * blk.shape[0]), (r, (st[r, 1] - m2).abs().max())


@pytest.mark.parametrize("m,T", [(12800, 800), (1000, 125), (2048, 128)])
def test_batchnorm_fwd_from_gemm_stats(m, T):
    cin = cout = 512
    g = torch.Generator().manual_seed(7 + m)
    x, w, b, conv, k = _conv(m, cin, cout, T, g)
    y = torch.empty(m, cout, dtype=torch.bfloat16, device="cuda")
    rows = ops.gemm_stats_rows(x, w, y, m, cout, k, cin, k, cout, bias=b, a_conv=conv)
    R = (m + rows - 1) // rows
    st = torch.empty(2 * R * cout, device="cuda")
    ops.gemm(x, w, y, m, cout, k, cin, k, cout, bias=b, a_conv=conv, col_stats=st)
    gamma = (1 + 0.1 * torch.randn(cout, generator=g)).cuda()
    beta = (0.1 * torch.randn(cout, generator=g)).cuda()
    seed = torch.tensor([5], dtype=torch.int32, device="cuda")
    drop = ops.Drop(seed, 40, 0.5)
    outs = []
    for stats in ((st, rows), None):
        mean, rstd = torch.empty(cout, device="cuda"), torch.empty(cout, device="cuda")
        rm, rv = torch.zeros(cout, device="cuda"), torch.ones(cout, device="cuda")
        out = torch.empty_like(y)
        ops.batchnorm_fwd(y, gamma, beta, mean, rstd, rm, rv, out, m, cout, ACT_TANH, True, drop=drop,
                          ws=ops.Workspace(), stats=stats)
        outs.append((mean, rstd, rm, rv, out))
    torch.cuda.synchronize()
    (mf, rf, rmf, rvf, of), (ms, rs, rms, rvs, os_) = outs
    yd = y.double()
    assert torch.allclose(mf.double(), yd.mean(0), rtol=1e-6, atol=1e-6)
    assert torch.allclose(rf.double(), 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5), rtol=1e-5)
    for a, b_ in ((mf, ms), (rf, rs), (rmf, rms), (rvf, rvs)):
        assert torch.allclose(a, b_, rtol=1e-5, atol=1e-7), (a - b_).abs().max()
    # the same statistics to f32 rounding: the outputs (|out| < 2 after tanh and the 1 / (1 - p)
    # dropout scale) agree to a bf16 step or two
    assert (of.float() - os_.float()).abs().max().item() <= 2 ** -6


def test_col_stats_refused():
    g = torch.Generator().manual_seed(3)
    m, cin, cout, T = 12800, 512, 512, 800
    x, w, b, conv, k = _conv(m, cin, cout, T, g)
    st = torch.empty(2 * 200 * cout, device="cuda")
    with pytest.raises(TT2Error):   # split-K
        ops.gemm(x, w, torch.empty(m, cout, dtype=torch.bfloat16, device="cuda"), m, cout, k, cin, k, cout,
                 a_conv=conv, splits=2, col_stats=st, ws=ops.Workspace())
    with pytest.raises(TT2Error):   # f32 C
        ops.gemm(x, w, torch.empty(m, cout, device="cuda"), m, cout, k, cin, k, cout, a_conv=conv, col_stats=st)
    w2 = torch.zeros(576, k, dtype=torch.bfloat16, device="cuda")
    y2 = torch.empty(m, 576, dtype=torch.bfloat16, device="cuda")
    assert ops.gemm_stats_rows(x, w2, y2, m, 576, k, cin, k, 576, a_conv=conv) == 0
    with pytest.raises(TT2Error):   # the 256 x 128 kernel with n % 128 != 0
        ops.gemm(x, w2, y2, m, 576, k, cin, k, 576, a_conv=conv, col_stats=st)


@pytest.mark.parametrize("m,T,p,act", [(12800, 800, 0.5, ACT_TANH), (1000, 125, 0.0, ACT_TANH),
                                       (2048, 128, 0.5, ACT_RELU)])
def test_batchnorm_bwd_from_gemm_sums(m, T, p, act):
    """the post-net / pre-net backward's pairing: the conv dgrad that produces a BatchNorm's dout
    also leaves its column sums (tt2_gemm bn_bwd), and the BatchNorm backward skips its own pass"""
    c = 512
    g = torch.Generator().manual_seed(11 + m)
    dyn, wf, _, conv, k = _conv(m, c, c, T, g)          # the next layer's dy and flipped weights
    y = (torch.randn(m, c, generator=g) * 2 + 0.3).bfloat16().cuda()   # this layer's conv output
    gamma = (1 + 0.1 * torch.randn(c, generator=g)).cuda()
    beta = (0.1 * torch.randn(c, generator=g)).cuda()
    mean = y.float().mean(0)
    rstd = 1 / torch.sqrt(y.float().var(0, unbiased=False) + 1e-5)
    seed = torch.tensor([9], dtype=torch.int32, device="cuda")
    drop = ops.Drop(seed, 41, p)
    dout = torch.empty(m, c, dtype=torch.bfloat16, device="cuda")
    rows = ops.gemm_stats_rows(dyn, wf, dout, m, c, k, c, k, c, a_conv=conv)
    R = (m + rows - 1) // rows
    sums = torch.full((2 * R * c,), float("nan"), device="cuda")
    bnb = ops.bn_bwd_args(y, gamma, beta, mean, rstd, m, c, act, drop, (sums, rows))
    ops.gemm(dyn, wf, dout, m, c, k, c, k, c, a_conv=conv, bn_bwd=bnb)
    dout_ref = torch.empty_like(dout)
    ops.gemm(dyn, wf, dout_ref, m, c, k, c, k, c, a_conv=conv)
    res = []
    for stats in ((sums, rows), None):
        dy = torch.empty_like(y)
        dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
        ops.batchnorm_bwd(y, dout, gamma, beta, mean, rstd, dy, dg, db, m, c, act, drop=drop,
                          ws=ops.Workspace(), stats=stats)
        res.append((dy, dg, db))
    torch.cuda.synchronize()
    assert torch.equal(dout, dout_ref)
    # float64 column sums of the same per-element terms
    keep = torch.ones(m, c, dtype=torch.float64)
    if p > 0:
        from tt2_oracle import dropout_keep
        keep = torch.from_numpy(dropout_keep(9, 41, m * c, p)).view(m, c).double() / (1 - p)
    xh = (y.double().cpu() - mean.double().cpu()) * rstd.double().cpu()
    u = xh * gamma.double().cpu() + beta.double().cpu()
    if act == ACT_TANH:
        z = torch.tanh(u)
        dp = dout.double().cpu() * keep * (1 - z * z)
    else:
        dp = dout.double().cpu() * keep * (u > 0).double()
    s = sums.view(R, 2, c).double().cpu().sum(0)
    assert torch.allclose(s[0], dp.sum(0), rtol=1e-4, atol=1e-3), (s[0] - dp.sum(0)).abs().max()
    assert torch.allclose(s[1], (dp * xh).sum(0), rtol=1e-4, atol=1e-3), (s[1] - (dp * xh).sum(0)).abs().max()
    (dyf, dgf, dbf), (dys, dgs, dbs) = res
    assert torch.allclose(dgf, dgs, rtol=1e-4, atol=1e-3) and torch.allclose(dbf, dbs, rtol=1e-4, atol=1e-3)
    assert (dyf.float() - dys.float()).abs().max().item() <= 2e-2 * dys.float().abs().max().item()
