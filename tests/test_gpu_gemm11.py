"""v11 GEMM (v7's 256 x 128 tile with 4 MFMA waves of 128 x 64 and 8 loader waves; tt2_gemm
variant 17, the auto choice for the NT forward products with K <= 1024): bit for bit the same
as v7 through its LDS-image epilogue (variant 14) -- the same K order per output and the same
epilogue -- for M tails, one and many K steps, the forward epilogue codes (bias / ReLU /
dropout, alpha) and the activation-gradient form (N-contiguous B) with a residual or a ReLU
gate; and against float64 torch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402


def _run(A, B, m, n, k, tb, kw, v):
    C = torch.full((m, n), float("nan"), device="cuda", dtype=torch.bfloat16)
    ops.gemm(A, B, C, m, n, k, k, B.shape[1], n, trans_b=tb, variant=v, **kw)
    return C


@pytest.mark.parametrize("mnk", [(256, 128, 64), (300, 256, 128), (12800, 512, 512), (2048, 1536, 1024),
                                 (520, 384, 192)])
@pytest.mark.parametrize("epi", ["", "b", "br", "brd", "d"])
def test_gemm11_forward_matches_v7(mnk, epi):
    m, n, k = mnk
    g = torch.Generator(device="cuda").manual_seed(m + n + k + len(epi))
    A = torch.randn(m, k, device="cuda", generator=g).bfloat16()
    B = (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).bfloat16()
    seed = torch.tensor([4321], dtype=torch.int32, device="cuda")
    kw = {"alpha": 0.75}
    if "b" in epi:
        kw["bias"] = torch.randn(n, device="cuda", generator=g)
    if "r" in epi:
        kw["act"] = ACT_RELU
    if "d" in epi:
        kw["drop"] = ops.Drop(seed, 11, 0.2)
    c7, c11 = _run(A, B, m, n, k, False, kw, 14), _run(A, B, m, n, k, False, kw, 17)
    torch.cuda.synchronize()
    assert not torch.isnan(c11).any()
    assert torch.equal(c7, c11)
    if not epi:
        ref = 0.75 * (A.double() @ B.double().t())
        assert ((c11.double() - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("mnk", [(300, 256, 128), (12800, 512, 512), (2048, 512, 1024)])
@pytest.mark.parametrize("epi", ["", "res", "gate"])
def test_gemm11_dgrad_matches_v7(mnk, epi):
    """The activation-gradient form (B N-contiguous, forced: auto keeps v7 there)."""
    m, n, k = mnk
    g = torch.Generator(device="cuda").manual_seed(7 * m + n + k + len(epi))
    A = torch.randn(m, k, device="cuda", generator=g).bfloat16()
    B = (torch.randn(k, n, device="cuda", generator=g) / k ** 0.5).bfloat16()
    X = torch.randn(m, n, device="cuda", generator=g).bfloat16()
    kw = {}
    if epi == "res":
        kw.update(res=X, ldr=n)
    if epi == "gate":
        kw.update(gate=X.relu(), ldg=n, gate_scale=1.25)
    c7, c11 = _run(A, B, m, n, k, True, kw, 14), _run(A, B, m, n, k, True, kw, 17)
    torch.cuda.synchronize()
    assert not torch.isnan(c11).any()
    assert torch.equal(c7, c11)
    ref = A.double() @ B.double()
    if epi == "res":
        ref = ref + X.double()
    if epi == "gate":
        ref = torch.where(X.double() > 0, ref * 1.25, torch.zeros_like(ref))
    assert ((c11.double() - ref).norm() / ref.norm()).item() < 1e-2


def test_gemm11_is_the_auto_choice():
    """The forward NT product with K <= 1024 runs v11 under auto: same bits as variant 17."""
    m, n, k = 12800, 512, 512
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    bias = torch.randn(n, device="cuda")
    c0, c17 = _run(A, B, m, n, k, False, {"bias": bias}, 0), _run(A, B, m, n, k, False, {"bias": bias}, 17)
    torch.cuda.synchronize()
    assert torch.equal(c0, c17)
