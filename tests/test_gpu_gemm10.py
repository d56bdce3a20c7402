"""v10 GEMM (256 x 256 NT tile, 8 MFMA waves + 4 loader waves, 5-slot single-operand ring;
tt2_gemm variant 16): same results as v7 (variant 13) -- the accumulation order per output and
the epilogue's operation order are the same, so bit for bit -- and against float64 torch; M
tails, one and many K steps, every epilogue code (bias / ReLU / dropout), alpha, the launch
probe's span."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2 import ops  # noqa: E402
from tt2._lib import ACT_RELU  # noqa: E402


@pytest.mark.parametrize("mnk", [(256, 256, 64), (300, 512, 128), (1000, 768, 576), (4096, 2048, 512),
                                 (512, 256, 192)])
@pytest.mark.parametrize("epi", ["", "b", "br", "brd", "d"])
def test_gemm10_matches_v7(mnk, epi):
    m, n, k = mnk
    g = torch.Generator(device="cuda").manual_seed(m + n + k + len(epi))
    A = torch.randn(m, k, device="cuda", generator=g).bfloat16()
    B = (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).bfloat16()
    seed = torch.tensor([1234], dtype=torch.int32, device="cuda")
    kw = {}
    if "b" in epi:
        kw["bias"] = torch.randn(n, device="cuda", generator=g)
    if "r" in epi:
        kw["act"] = ACT_RELU
    if "d" in epi:
        kw["drop"] = ops.Drop(seed, 9, 0.2)
    out = {}
    for v in (13, 16):
        C = torch.full((m, n), float("nan"), device="cuda", dtype=torch.bfloat16)
        ops.gemm(A, B, C, m, n, k, k, k, n, alpha=0.75, variant=v, **kw)
        out[v] = C
    torch.cuda.synchronize()
    assert not torch.isnan(out[16]).any()
    assert torch.equal(out[13], out[16])
    if not epi:
        ref = 0.75 * (A.double() @ B.double().t())
        assert ((out[16].double() - ref).norm() / ref.norm()).item() < 1e-2


def test_gemm10_probe_span():
    m, n, k = 2048, 1024, 512
    A = torch.randn(m, k, device="cuda").bfloat16()
    B = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    ops.gemm(A, B, C, m, n, k, k, k, n, variant=16)
    torch.cuda.synchronize()
    ops.PROBE = probe = ops.LaunchProbe()
    try:
        ops.gemm(A, B, C, m, n, k, k, k, n, variant=16)
        sp = probe.summary(span=True)
    finally:
        ops.PROBE = None
        probe.close()
    (key, v), = sp.items()
    assert v[0] == 1 and v[2] > 0
    ref = A.float() @ B.float().t()
    assert ((C.float() - ref).norm() / ref.norm()).item() < 1e-2
