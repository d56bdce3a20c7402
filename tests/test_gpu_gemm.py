"""GEMM kernel numerics vs a float64 torch reference (GPU)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2_oracle import dropout_keep  # noqa: E402


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _mk(shape, dtype, gen):
    return torch.randn(shape, generator=gen, dtype=torch.float32).to(dtype).cuda()


VARIANTS = [(torch.float32, 1), (torch.bfloat16, 1), (torch.bfloat16, 2), (torch.bfloat16, 13),
            (torch.bfloat16, 14), (torch.bfloat16, 15)]


@pytest.mark.parametrize("dtype,variant", VARIANTS)
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("mnk", [(200, 136, 72), (128, 128, 32), (40, 264, 520), (256, 384, 1000), (96, 80, 46),
                                 (600, 520, 1000)])
def test_gemm_layouts(dtype, variant, ta, tb, mnk):
    m, n, k = mnk
    if (ta and m % 8) or (tb and n % 8) or (not ta and k % 8) or (not tb and k % 8):
        pytest.skip("inner dims must keep 16-B aligned rows")
    g = torch.Generator().manual_seed(m * 7 + n * 3 + k + ta * 2 + tb)
    A = _mk((k, m) if ta else (m, k), dtype, g)
    B = _mk((k, n) if tb else (n, k), dtype, g)
    C = torch.empty(m, n, dtype=torch.float32, device="cuda")
    ops.gemm(A, B, C, m, n, k, A.shape[1], B.shape[1], n, trans_a=ta, trans_b=tb, variant=variant)
    Am = (A.t() if ta else A).double()
    Bm = (B.t() if tb else B).double()
    ref = Am @ Bm.t()
    tol = 1e-5 if dtype == torch.float32 else 1e-5  # inputs are exact in both; f32 accumulation
    assert rel(C, ref) < tol


@pytest.mark.parametrize("dtype,variant", VARIANTS)
@pytest.mark.parametrize("n", [200, 81])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_epilogue(dtype, variant, n, splits):
    """Fused epilogue (bias, residual, ReLU, gate, dropout), applied in the kernel or
    in the split-K reduce."""
    m, k = 300, 96 * splits
    g = torch.Generator().manual_seed(1)
    A, B = _mk((m, k), dtype, g), _mk((n, k), dtype, g)
    bias = torch.randn(n, generator=g).cuda()
    R = _mk((m, n), dtype, g)
    G = _mk((m, n), dtype, g).relu()
    seed = torch.tensor([1234], dtype=torch.int32).cuda()
    out = torch.empty(m, n, dtype=dtype, device="cuda")
    ops.gemm(A, B, out, m, n, k, k, k, n, bias=bias, res=R, ldr=n, act=ops._lib.ACT_RELU, gate=G, ldg=n,
             gate_scale=1.7, alpha=0.5, drop=ops.Drop(seed, 77, 0.3), variant=variant, splits=splits)
    ref = 0.5 * (A.double() @ B.double().t()) + bias.double() + R.double()
    ref = ref.relu() * (G.double() != 0) * 1.7
    keep = torch.from_numpy(dropout_keep(1234, 77, m * n, 0.3)).view(m, n).cuda()
    ref = ref * keep / 0.7
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert rel(out, ref) < tol


@pytest.mark.parametrize("variant", [0, 13, 14])
@pytest.mark.parametrize("k", [64, 128, 192, 520])
@pytest.mark.parametrize("tile_op", ["res", "gate", "none"])
def test_gemm_epilogue_staged(variant, k, tile_op):
    """v7 with the loader waves hashing the dropout bits and staging the residual / gate
    tile in LDS (K steps 1, 2, 3 and 9: every stage hand-off of the staged image), ragged
    M and N edges."""
    m, n = 520, 264
    g = torch.Generator().manual_seed(k + len(tile_op))
    A, B = _mk((m, k), torch.bfloat16, g), _mk((n, k), torch.bfloat16, g)
    bias = torch.randn(n, generator=g).cuda()
    X = _mk((m, n), torch.bfloat16, g)
    seed = torch.tensor([99], dtype=torch.int32).cuda()
    out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    kw = dict(res=X, ldr=n) if tile_op == "res" else (dict(gate=X.relu(), ldg=n, gate_scale=1.3)
                                                     if tile_op == "gate" else {})
    ops.gemm(A, B, out, m, n, k, k, k, n, bias=bias, act=ops._lib.ACT_RELU, drop=ops.Drop(seed, 5, 0.25),
             variant=variant, **kw)
    ref = A.double() @ B.double().t() + bias.double()
    if tile_op == "res":
        ref = ref + X.double()
    ref = ref.relu()
    if tile_op == "gate":
        ref = ref * (X.double().relu() != 0) * 1.3
    keep = torch.from_numpy(dropout_keep(99, 5, m * n, 0.25)).view(m, n).cuda()
    ref = ref * keep / 0.75
    assert rel(out, ref) < 8e-3


@pytest.mark.parametrize("dtype,variant", VARIANTS)
def test_gemm_splitk_tanh_beta(dtype, variant):
    m, n, k = 160, 96, 1000
    g = torch.Generator().manual_seed(2)
    A, B = _mk((k, m), dtype, g), _mk((k, n), dtype, g)
    C0 = torch.randn(m, n, generator=g).cuda()
    C = C0.clone()
    ops.gemm(A, B, C, m, n, k, m, n, n, trans_a=True, trans_b=True, beta=1.0, alpha=0.01, act=ops._lib.ACT_TANH,
             splits=7, variant=variant)
    ref = torch.tanh(0.01 * (A.double().t() @ B.double())) + C0.double()
    assert rel(C, ref) < 1e-5


@pytest.mark.parametrize("dtype,variant", VARIANTS)
@pytest.mark.parametrize("cin,cout", [(80, 136), (64, 80)])
@pytest.mark.parametrize("T", [37, 100])
def test_conv_implicit_gemm(dtype, variant, cin, cout, T):
    """Conv1d(k5, pad2) fwd / dgrad / wgrad as implicit GEMMs, channels-last (T >= 64
    and C >= 64 also run the v7 loaders' conv tracking)."""
    Bsz, KS, pad = 3, 5, 2
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(Bsz, T, cin, generator=g)
    w = torch.randn(cout, cin, KS, generator=g) / math.sqrt(cin * KS)
    dy = torch.randn(Bsz, T, cout, generator=g)
    xd, dyd = x.to(dtype).cuda(), dy.to(dtype).cuda()
    wp = w.permute(0, 2, 1).contiguous().to(dtype).cuda()          # [Cout][tap][Cin]
    wflip = w.flip(2).permute(1, 2, 0).contiguous().to(dtype).cuda()  # [Cin][tap'][Cout]
    M = Bsz * T
    y = torch.empty(M, cout, device="cuda")
    ops.gemm(xd, wp, y, M, cout, KS * cin, cin, KS * cin, cout, a_conv=(T, cin, pad), variant=variant)
    xr = x.to(dtype).double()
    wr = w.to(dtype).double()
    dyr = dy.to(dtype).double()
    ref = F.conv1d(xr.transpose(1, 2), wr, padding=pad).transpose(1, 2).reshape(M, cout)
    assert rel(y, ref) < 1e-5
    y2 = torch.empty(M, cout, device="cuda")
    ops.gemm(xd, wp, y2, M, cout, KS * cin, cin, KS * cin, cout, a_conv=(T, cin, pad), variant=variant, splits=2)
    assert rel(y2, ref) < 1e-5
    # dgrad
    dx = torch.empty(M, cin, device="cuda")
    ops.gemm(dyd, wflip, dx, M, cin, KS * cout, cout, KS * cout, cin, a_conv=(T, cout, pad), variant=variant)
    xq = xr.clone().requires_grad_(True)
    yq = F.conv1d(xq.transpose(1, 2), wr.clone().requires_grad_(True), padding=pad)
    (yq * dyr.transpose(1, 2)).sum().backward()
    assert rel(dx, xq.grad.reshape(M, cin)) < 1e-5
    # wgrad: dW[co][tap][ci] = sum_m dy[m,co] x(m + tap - pad, ci)
    dw = torch.empty(cout, KS * cin, device="cuda")
    ops.gemm(dyd, xd, dw, cout, KS * cin, M, cout, cin, KS * cin, trans_a=True, trans_b=True,
             b_conv=(T, cin, pad), splits=3, variant=variant)
    wq = wr.clone().requires_grad_(True)
    yq = F.conv1d(xr.transpose(1, 2), wq, padding=pad)
    (yq * dyr.transpose(1, 2)).sum().backward()
    ref_w = wq.grad.permute(0, 2, 1).reshape(cout, KS * cin)
    assert rel(dw, ref_w) < 1e-5


@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("conv", [False, True])
@pytest.mark.parametrize("variant", [0, 2, 11, 12, 13])
def test_wgrad_fused_bias_ksum(splits, conv, variant):
    """Weight-gradient GEMM with the bias gradient (row sums of A = dY^T over k) fused."""
    Bsz, T, cin, cout, KS, pad = 3, 150, 64, 200, 5, 2
    M = Bsz * T
    g = torch.Generator().manual_seed(11 + splits + conv)
    dy = torch.randn(M, cout, generator=g).bfloat16().cuda()
    x = torch.randn(M, cin, generator=g).bfloat16().cuda()
    kin = KS * cin if conv else cin
    dw = torch.empty(cout, kin, device="cuda")
    gb = torch.full((cout,), 3.0, device="cuda")
    ops.gemm(dy, x, dw, cout, kin, M, cout, cin, kin, trans_a=True, trans_b=True, splits=splits,
             b_conv=(T, cin, pad) if conv else None, a_ksum=gb, a_ksum_beta=0.5, variant=variant)
    ref_b = 1.5 + dy.double().sum(0)
    assert rel(gb, ref_b) < 1e-6
    if not conv:
        assert rel(dw, dy.double().t() @ x.double()) < 1e-5


@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_grouped_matches_single(splits):
    """tt2_gemm_grouped over weight-gradient problems of different shapes (with fused
    bias sums, one conv-B problem, a K tail) equals the float64 reference."""
    g = torch.Generator().manual_seed(5 + splits)
    T, cin, pad = 100, 64, 2
    M = 3 * T
    probs, refs = [], []
    for n_out, n_in, conv in [(512, 512, False), (200, 64, False), (136, 5 * cin, True), (1536, 128, False)]:
        dy = torch.randn(M, n_out, generator=g).bfloat16().cuda()
        x = torch.randn(M, cin if conv else n_in, generator=g).bfloat16().cuda()
        dw = torch.empty(n_out, n_in, device="cuda")
        gb = torch.full((n_out,), 2.0, device="cuda")
        probs.append(dict(a=dy, b=x, c=dw, m=n_out, n=n_in, k=M, lda=n_out, ldb=x.shape[1], ldc=n_in, trans_a=True,
                          trans_b=True, splits=splits, b_conv=(T, cin, pad) if conv else None, a_ksum=gb,
                          a_ksum_beta=0.5))
        if conv:
            xp = torch.nn.functional.pad(x.double().view(3, T, cin), (0, 0, pad, pad))
            cols = torch.cat([xp[:, t:t + T] for t in range(5)], dim=2).reshape(M, 5 * cin)
            ref = dy.double().t() @ cols
        else:
            ref = dy.double().t() @ x.double()
        refs.append((dw, ref, gb, 1.0 + dy.double().sum(0)))
    ops.gemm_grouped(probs)
    for dw, ref, gb, ref_b in refs:
        assert rel(dw, ref) < 1e-5
        assert rel(gb, ref_b) < 1e-6
