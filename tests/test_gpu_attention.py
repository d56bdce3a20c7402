"""Fused attention kernels vs a float64 torch reference (GPU)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def ref_attn(q, k, v, key_len, causal, scale):
    """q [B,H,Tq,64] ... float64; masked probs exactly 0; empty rows -> 0."""
    B, H, Tq, _ = q.shape
    Tk = k.shape[2]
    s = (q @ k.transpose(-1, -2)) * scale
    allowed = torch.ones(B, 1, Tq, Tk, dtype=torch.bool)
    if key_len is not None:
        allowed &= torch.arange(Tk)[None, None, None, :] < key_len.view(B, 1, 1, 1).cpu()
    if causal:
        allowed &= torch.ones(Tq, Tk, dtype=torch.bool).tril()[None, None]
    s = s.masked_fill(~allowed, float("-inf"))
    mx = s.amax(-1, keepdim=True)
    mx = torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))
    e = torch.exp(s - mx) * allowed
    den = e.sum(-1, keepdim=True)
    p = e / torch.where(den > 0, den, torch.ones_like(den))
    return p @ v


CASES = [
    # B, H, Tq, Tk, causal, self(packed qkv), key_len
    (2, 3, 70, 70, True, True, [70, 41]),
    (2, 2, 130, 130, False, True, [130, 5]),
    (3, 2, 100, 37, False, False, [37, 20, 0]),
    (1, 8, 64, 128, False, False, None),
    (2, 2, 200, 200, True, True, None),
    (2, 2, 300, 300, True, True, [300, 257]),
    (2, 1, 131, 333, False, False, [333, 129]),
]


@pytest.fixture(params=[0, 1, 2, 3], ids=["auto", "v1", "v3w2", "v3w4"])
def attn_variant(request):
    old = ops.ATTN_VARIANT
    ops.ATTN_VARIANT = request.param
    yield request.param
    ops.ATTN_VARIANT = old


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
def test_attention_fwd_bwd(dtype, case, attn_variant):
    B, H, Tq, Tk, causal, packed, kl = case
    D = 64
    scale = 1.0 / math.sqrt(D)
    g = torch.Generator().manual_seed(B * 100 + Tq + Tk + causal)
    HD = H * D
    if packed:
        qkv = torch.randn(B * Tq, 3 * HD, generator=g)
        qkv_d = qkv.to(dtype).cuda()
        q_t, k_t, v_t = qkv_d[:, :HD], qkv_d[:, HD:2 * HD], qkv_d[:, 2 * HD:]
        ld_q = ld_k = ld_v = 3 * HD
        qh = qkv[:, :HD].to(dtype).double()
        kh = qkv[:, HD:2 * HD].to(dtype).double()
        vh = qkv[:, 2 * HD:].to(dtype).double()
    else:
        q = torch.randn(B * Tq, HD, generator=g)
        kv = torch.randn(B * Tk, 2 * HD, generator=g)
        q_t = q.to(dtype).cuda()
        kv_d = kv.to(dtype).cuda()
        k_t, v_t = kv_d[:, :HD], kv_d[:, HD:]
        ld_q, ld_k, ld_v = HD, 2 * HD, 2 * HD
        qh, kh, vh = q.to(dtype).double(), kv[:, :HD].to(dtype).double(), kv[:, HD:].to(dtype).double()
    key_len = None if kl is None else torch.tensor(kl, dtype=torch.int32)
    klen_d = None if key_len is None else key_len.cuda()

    def heads(x, T):
        return x.view(B, T, H, D).transpose(1, 2)

    qr = heads(qh, Tq).clone().requires_grad_(True)
    kr = heads(kh, Tk).clone().requires_grad_(True)
    vr = heads(vh, Tk).clone().requires_grad_(True)
    o_ref = ref_attn(qr, kr, vr, key_len, causal, scale)

    out = torch.empty(B * Tq, HD, dtype=dtype, device="cuda")
    lse = torch.empty(B * H, Tq, dtype=torch.float32, device="cuda")
    ops.attn_fwd(q_t, k_t, v_t, out, lse, ld_q, ld_k, ld_v, HD, B, H, Tq, Tk, klen_d, causal, scale)
    o_ref_flat = o_ref.transpose(1, 2).reshape(B * Tq, HD)
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert rel(out, o_ref_flat) < tol

    dout = torch.randn(B * Tq, HD, generator=g)
    dout_d = dout.to(dtype).cuda()
    (o_ref * heads(dout.to(dtype).double(), Tq)).sum().backward()
    dq = torch.zeros(B * Tq, HD, dtype=dtype, device="cuda")
    dkv = torch.zeros(B * Tk, 2 * HD, dtype=dtype, device="cuda")
    delta = torch.empty(B * H, Tq, dtype=torch.float32, device="cuda")
    ops.attn_bwd(q_t, k_t, v_t, out, dout_d, lse, delta, dq, dkv[:, :HD], dkv[:, HD:], ld_q, ld_k, ld_v, HD, HD,
                 HD, 2 * HD, 2 * HD, B, H, Tq, Tk, klen_d, causal, scale)
    flat = lambda x, T: x.transpose(1, 2).reshape(B * T, HD)  # noqa: E731
    tol_b = 5e-6 if dtype == torch.float32 else 2e-2
    assert rel(dq, flat(qr.grad, Tq)) < tol_b
    assert rel(dkv[:, :HD], flat(kr.grad, Tk)) < tol_b
    assert rel(dkv[:, HD:], flat(vr.grad, Tk)) < tol_b
    if key_len is not None:
        # keys past the length get exactly zero gradient
        for b, L in enumerate(kl):
            assert dkv.view(B, Tk, 2 * HD)[b, L:].abs().max().item() == 0 if L < Tk else True
