"""End-to-end parity: the MI355X engine vs the CPU oracle (GPU).

fp32 mode runs the same kernels with exact-f32 MFMA and must match the oracle
within the north_star bar (1e-3 relative L2 on the mels; gradients too).
bf16 mode is checked at a looser, stated tolerance."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402
from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def make_batch(B=2, Tx=17, Ty=23, text_len=(17, 11), mel_len=(23, 15), seed=0):
    g = torch.Generator().manual_seed(seed)
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl = torch.tensor(text_len)
    ml = torch.tensor(mel_len)
    for b in range(B):
        text[b, tl[b]:] = 0
    mel = torch.randn(B, Ty, 80, generator=g)
    for b in range(B):
        mel[b, ml[b]:] = 0
    return text, tl, mel, ml


def build(dtype, seed=0):
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), seed)
    model = TransformerTTS(TTSConfig(), dtype=dtype)
    model.load_state_dict(oracle.state_dict())
    return oracle, model


@pytest.fixture(scope="module")
def pair32():
    return build(torch.float32)


def test_state_dict_roundtrip(pair32):
    oracle, model = pair32
    sd_o, sd_m = oracle.state_dict(), model.state_dict()
    assert list(sd_o.keys()) == list(sd_m.keys())
    for k in sd_o:
        assert torch.equal(sd_o[k].float(), sd_m[k].float()), k


# Dropout seed: with seed 1234 one kept encoder-layer-3 FFN pre-activation is +1.3e-6 (f64)
# and the engine's f32 sum lands on the other side of the ReLU kink (the CPU f32 oracle does
# not), which moves every gradient below that layer by ~1.4e-3; seeds 1-5 give <= 6e-6 on
# every gradient against a float64 oracle (tools/fp32_grad_err.py; round 1's tools/kink_check.py is in git history).
@pytest.mark.parametrize("train,drop_seed", [(False, None), (True, None), (True, 1)])
def test_forward_backward_fp32(train, drop_seed):
    oracle, model = build(torch.float32)
    text, tl, mel, ml = make_batch()
    oracle.train(train)
    model.train(train)
    model.engine.dropout_enabled = drop_seed is not None
    oracle.set_seed(drop_seed)
    if drop_seed is not None:
        model.set_seed(drop_seed)
    ob, oa, os_, _ = oracle(text, tl, mel, ml)
    mb, ma, ms, _ = model(text, tl.int(), mel, ml.int())
    assert rel(mb, ob) < 1e-4
    assert rel(ma, oa) < 1e-4
    assert rel(ms, os_) < 1e-4
    if not train:
        return
    lo, parts_o = oracle.loss((ob, oa, os_), mel, ml)
    lm, parts_m = model.loss()
    assert abs(lm.item() - lo.item()) / abs(lo.item()) < 1e-4
    for k in parts_o:
        assert abs(parts_m[k].item() - parts_o[k].item()) <= 1e-4 * abs(parts_o[k].item()) + 1e-7, k
    lo.backward()
    model.backward()
    gm = model.grads_state_dict()
    bad = []
    gnorm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in oracle.parameters() if p.grad is not None))
    for k, p in oracle.named_parameters():
        ref = p.grad if p.grad is not None else torch.zeros_like(p)
        if ref.double().norm() < 1e-6 * gnorm:
            # e.g. conv biases in front of training-mode BatchNorm: analytically zero
            if gm[k].double().norm() >= 1e-5 * gnorm:
                bad.append((k, "nonzero", gm[k].abs().max().item()))
            continue
        r = rel(gm[k], ref)
        if r >= 1e-3:
            bad.append((k, r))
    if bad:
        pytest.fail("\n".join(map(str, bad)))
    # running statistics after one training forward
    sd_o, sd_m = oracle.state_dict(), model.state_dict()
    for k in sd_o:
        if "running_" in k:
            assert rel(sd_m[k], sd_o[k]) < 1e-4, k


def test_forward_bf16():
    oracle, model = build(torch.bfloat16)
    text, tl, mel, ml = make_batch()
    oracle.eval()
    model.eval()
    ob, oa, os_, _ = oracle(text, tl, mel, ml)
    mb, ma, ms, _ = model(text, tl.int(), mel, ml.int())
    assert rel(mb, ob) < 5e-2
    assert rel(ma, oa) < 5e-2


def test_train_step_and_graph():
    """Eager steps then a captured step: loss finite, replay == eager on the same state."""
    torch.manual_seed(0)
    _, model = build(torch.bfloat16)
    text, tl, mel, ml = make_batch(B=4, Tx=32, Ty=64, text_len=(32, 30, 20, 9), mel_len=(64, 50, 33, 10))
    model.train()
    model.configure_optimizer(lr=1.0, warmup=100.0)
    l0 = model.train_step(text.cuda(), tl.cuda(), mel.cuda(), ml.cuda())[0].item()
    for _ in range(3):
        l = model.train_step(text.cuda(), tl.cuda(), mel.cuda(), ml.cuda())[0].item()
    assert l == l and l < l0 * 1.5
    run = model.capture_train_step(4, 32, 64)
    for _ in range(3):
        lg = run(text.cuda(), tl.cuda(), mel.cuda(), ml.cuda())[0].item()
    assert lg == lg


def test_backward_bf16_grads_close_to_oracle():
    """bf16 training backward (the path the bench runs, incl. the 88-row padded heads
    GEMMs) vs the fp32 oracle's gradients, at a bf16 tolerance."""
    oracle, model = build(torch.bfloat16, seed=3)
    text, tl, mel, ml = make_batch(B=2, Tx=17, Ty=40, mel_len=(40, 27))
    oracle.train()
    model.train()
    model.engine.dropout_enabled = False
    oracle.set_seed(None)
    ob, oa, os_, _ = oracle(text, tl, mel, ml)
    lo, _ = oracle.loss((ob, oa, os_), mel, ml)
    lo.backward()
    grads = []
    for pad in (True, False):   # the padded heads GEMMs vs the unpadded register-staged ones
        model.engine.pad_heads = pad
        model(text, tl.int(), mel, ml.int())
        model.loss()
        model.backward()
        grads.append({k: v.clone() for k, v in model.grads_state_dict().items()})
    gm = grads[0]
    og = dict(oracle.named_parameters())
    for k in ("mel_linear.weight", "mel_linear.bias", "stop_linear.weight", "stop_linear.bias",
              "decoder.layers.5.ffn.w2.weight", "postnet.convs.0.conv.weight", "encoder.embed.weight"):
        # the padded heads dgrad (K = 88) runs the 64 x 64 v8 kernel, the unpadded one (K = 81) the
        # register-staged kernel: they sum k in different orders, so they agree to bf16 rounding,
        # which the BN-normalised encoder convs amplify on the way to the embedding
        tol = 2e-2 if k == "encoder.embed.weight" else 2e-3
        assert rel(gm[k], grads[1][k]) < tol, (k, rel(gm[k], grads[1][k]))
        # vs the fp32 oracle only near the output: the gradients that pass through the
        # BN-normalised convs (post-net, encoder pre-net) amplify bf16 rounding to ~25 %
        if k.startswith(("mel_", "stop_", "decoder.layers.5")):
            assert rel(gm[k], og[k].grad) < 0.12, (k, rel(gm[k], og[k].grad))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 5e-2)])
def test_alignments_match_oracle(dtype, tol):
    """model.alignments(l): the encoder-decoder attention probabilities recomputed from the
    saved LSE equal the oracle's nn.MultiheadAttention-style weights (masked keys exactly 0)."""
    oracle, model = build(dtype, seed=5)
    text, tl, mel, ml = make_batch()
    oracle.eval()
    model.eval()
    _, _, _, attn = oracle(text, tl, mel, ml, return_attn=True)
    model(text, tl.int(), mel, ml.int())
    for l in (0, 5):
        ref = attn["dec_cross"][l]
        got = model.alignments(l).cpu()
        assert got.shape == ref.shape
        assert rel(got, ref) < tol
        assert got[1, :, :, int(tl[1]):].abs().max().item() == 0.0
    f = TransformerTTS.diagonal_focus(model.alignments(-1), tl, ml)
    assert f.shape == (2,) and ((f > 0) & (f <= 1.0001)).all()
