"""AR decode path vs the CPU oracle (GPU): forced length, prenet dropout off.
fp32 mode must match within 1e-3; the hipGraph replay must equal eager launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.infer import Decoder  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402
from tt2 import ops  # noqa: E402
from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def setup(dtype):
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 3).eval()
    model = TransformerTTS(TTSConfig(), dtype=dtype).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(5)
    B, Tx = 3, 17
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.tensor([17, 12, 6])
    for b in range(B):
        text[b, tl[b]:] = 0
    return oracle, model, text, tl


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 6e-2)])
def test_decode_matches_oracle(dtype, tol):
    oracle, model, text, tl = setup(dtype)
    T = 14
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    after, out_len = model.infer(text, tl, T, stop_threshold=None)
    assert after.shape == ref_after.shape
    assert rel(after, ref_after) < tol
    dec = model._decoders[(3, 17, T, False)]
    assert rel(dec.mel_seq[:, :T], ref_before) < tol
    assert rel(dec.stop_seq[:, :T], ref_stop) < tol
    assert (out_len.cpu() == T).all()


def test_graph_replay_equals_eager():
    _, model, text, tl = setup(torch.bfloat16)
    T = 10
    a1, _ = model.infer(text, tl, T, stop_threshold=None, use_graph=True)
    a2, _ = model.infer(text, tl, T, stop_threshold=None, use_graph=False)
    assert torch.equal(a1, a2)


@pytest.mark.parametrize("fuse", [0, 2, 3])
def test_decode_fusion_levels_match(fuse):
    """bf16 decode with the KV scatter (default level 1) vs no fusion / also the fused
    LayerNorm prologues: same frames within bf16 rounding of the LN output."""
    _, model, text, tl = setup(torch.bfloat16)
    T = 10
    model.eval()
    ref = Decoder(model.engine, 3, 17, T)
    ref.fuse = 1
    out = Decoder(model.engine, 3, 17, T)
    out.fuse = fuse
    a, _ = ref.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    b, _ = out.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
    assert rel(b, a) < (1e-6 if fuse == 0 else 2e-2)
    # the frame-emit epilogue advanced the device step counter once per frame
    assert out.t.item() == T


def test_stop_token_early_exit():
    _, model, text, tl = setup(torch.bfloat16)
    e = model.engine
    with torch.no_grad():   # push the stop logit up so every utterance stops immediately
        e.P("heads.b")[80] = 50.0
        e.sync_shadow()
    after, out_len = model.infer(text, tl, 64, stop_threshold=0.5)
    assert (out_len.cpu() == 1).all()
    assert after.shape[1] < 64


@pytest.mark.parametrize("m", [1, 5, 32])
def test_skinny_gemm(m):
    g = torch.Generator().manual_seed(m)
    n, k = 200, 520
    A = torch.randn(m, k, generator=g).bfloat16().cuda()
    B = torch.randn(n, k, generator=g).bfloat16().cuda()
    bias = torch.randn(n, generator=g).cuda()
    C = torch.empty(m, n, dtype=torch.float32, device="cuda")
    ops.gemm(A, B, C, m, n, k, k, k, n, bias=bias, act=1, variant=3)
    ref = (A.double() @ B.double().t() + bias.double()).relu()
    assert rel(C, ref) < 1e-5


def test_decode_wide_batch_matches_oracle():
    """A 40-utterance batch takes the 64-row skinny kernels (4 row blocks per MFMA column
    tile): bf16 frames match the fp32 CPU oracle at the bf16 tolerance."""
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 4).eval()
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).eval()
    model.load_state_dict(oracle.state_dict())
    g = torch.Generator().manual_seed(8)
    B, Tx, T = 40, 11, 6
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.randint(3, Tx + 1, (B,), generator=g)
    for b in range(B):
        text[b, tl[b]:] = 0
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    after, out_len = model.infer(text, tl, T, stop_threshold=None)
    assert rel(after, ref_after) < 6e-2
    dec = model._decoders[(B, Tx, T, False)]
    assert dec.fuse == 3 and dec.fused_io
    assert rel(dec.mel_seq[:, :T], ref_before) < 6e-2


def test_long_form_limits_early_exit():
    """cfg5 shape (B=64, T_max=2000): per-utterance frame caps end the loop at the last
    cap (polled every 32 frames), out_len = caps, frames stay finite, and the first frames
    equal a short run of the same batch."""
    torch.manual_seed(0)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).eval()
    g = torch.Generator().manual_seed(2)
    B, Tx, Tm = 64, 128, 2000
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.full((B,), Tx, dtype=torch.long, device="cuda")
    caps = torch.randint(300, 700, (B,), generator=g)
    dec = Decoder(model.engine, B, Tx, Tm)
    after, out_len = dec.run(text, tl, Tm, stop_threshold=None, limits=caps)
    n = after.shape[1]
    assert int(caps.max()) <= n < int(caps.max()) + 32
    assert torch.equal(out_len.cpu(), caps)
    assert torch.isfinite(dec.mel_seq[:, :n]).all()
    short = Decoder(model.engine, B, Tx, 8)
    short.run(text, tl, 8, stop_threshold=None)
    assert rel(short.mel_seq[:, :8], dec.mel_seq[:, :8]) < 1e-6


def test_decode_fp16_matches_oracle():
    """cfg5's fp16 decode step (f16 weights copy, f16 KV cache, f16 cross K/V) on a bf16
    engine: frames match the fp32 oracle within the fp16 tolerance, and the fp16 frames sit
    at least as close to the oracle as the bf16 ones (more mantissa bits)."""
    oracle, model, text, tl = setup(torch.bfloat16)
    T = 12
    ref_after, _, ref_before, ref_stop = oracle.infer(text, tl, T, force_len=True)
    errs = {}
    for dt in (torch.float16, torch.bfloat16):
        dec = Decoder(model.engine, 3, 17, T, dtype=dt)
        after, out_len = dec.run(text.cuda(), tl.cuda(), T, stop_threshold=None)
        errs[dt] = rel(dec.mel_seq[:, :T], ref_before)
        assert rel(after, ref_after) < 6e-2
        assert (out_len.cpu() == T).all()
    assert errs[torch.float16] < 3e-2
    assert errs[torch.float16] <= errs[torch.bfloat16] * 1.5
