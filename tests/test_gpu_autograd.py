"""The drop-in training surface: TransformerTTS is a torch.nn.Module whose
parameters() alias the engine's flat master buffer and whose forward / loss are autograd
Functions over libtt2, so a reference-shaped loop

    opt.zero_grad(); out = model(...); total, _ = model.loss(out, mel, mel_len)
    total.backward(); opt.step()

runs on the GPU engine with a stock torch optimizer.  Checked against the same loop on the
CPU oracle (f32 mode, dropout on, hash-identical masks)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402
from tt2_oracle import OracleConfig, TransformerTTSOracle, init_deterministic, tts_loss  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def batch(seed=0, B=2, Tx=13, Ty=19):
    g = torch.Generator().manual_seed(seed)
    text = torch.randint(1, 80, (B, Tx), generator=g)
    tl, ml = torch.tensor([Tx, Tx - 4]), torch.tensor([Ty, Ty - 7])
    text[1, Tx - 4:] = 0
    mel = torch.randn(B, Ty, 80, generator=g)
    return text, tl, mel, ml


def test_sgd_loop_matches_oracle():
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 0).train()
    model = TransformerTTS(TTSConfig(), dtype=torch.float32).train()
    model.load_state_dict(oracle.state_dict())
    p0 = {k: v.clone() for k, v in oracle.state_dict().items()}
    opt_o = torch.optim.SGD(oracle.parameters(), lr=0.05)
    opt_m = torch.optim.SGD(model.parameters(), lr=0.05)
    assert sum(p.numel() for p in model.parameters()) == model.n_params()
    for step in range(3):
        text, tl, mel, ml = batch(step)
        oracle.set_seed(100 + step)
        model.set_seed(100 + step)
        opt_o.zero_grad()
        out = oracle(text, tl, mel, ml)
        lo, _ = oracle.loss(out[:3], mel, ml)
        lo.backward()
        opt_o.step()
        opt_m.zero_grad()
        out_m = model(text.cuda(), tl.cuda(), mel.cuda(), ml.cuda())
        assert out_m[0].requires_grad and out_m[0].grad_fn is not None
        lm, parts = model.loss(out_m, mel.cuda(), ml.cuda())
        lm.backward()
        opt_m.step()
        assert abs(lm.item() - lo.item()) < 1e-4 * abs(lo.item())
    sd_o, sd_m = oracle.state_dict(), model.state_dict()
    for k, v in sd_o.items():
        if "num_batches" in k:
            assert int(sd_m[k]) == int(v), k
            continue
        assert rel(sd_m[k], v) < 1e-4, k
        # (conv biases in front of training-mode BatchNorm have an analytically zero gradient:
        # both sides update them by rounding noise only)
        if "running" not in k and "conv.bias" not in k and not torch.equal(v, p0[k]):
            assert rel(sd_m[k].cpu() - p0[k], v - p0[k]) < 2e-3, k   # the SGD updates themselves


def test_loss_honours_arguments():
    model = TransformerTTS(TTSConfig(), dtype=torch.float32).eval()
    text, tl, mel, ml = batch(5)
    with torch.no_grad():
        out = model(text.cuda(), tl.cuda(), mel.cuda(), ml.cuda())
    g = torch.Generator().manual_seed(9)
    mel2 = torch.randn(mel.shape, generator=g)
    ml2 = torch.tensor([15, 9])
    leaves = [(out[0] * 1.5 + 0.1).detach().requires_grad_(), (out[1] - 0.2).detach().requires_grad_(),
              (out[2] + 1.0).detach().requires_grad_()]
    total, parts = model.loss(leaves, mel2.cuda(), ml2.cuda())
    total.backward()
    cpu = [x.detach().cpu().requires_grad_() for x in leaves]
    ref, ref_parts = tts_loss(cpu[0], cpu[1], cpu[2], mel2, ml2)
    ref.backward()
    assert abs(total.item() - ref.item()) < 1e-5 * ref.item()
    for k in ("mel_before", "mel_after", "stop"):
        assert abs(parts[k].item() - ref_parts[k].item()) < 1e-5 * abs(ref_parts[k].item()) + 1e-7
    for a, b in zip(leaves, cpu):
        assert rel(a.grad, b.grad) < 1e-5


def test_adam_loop_bf16_reduces_loss():
    """bf16 model + stock torch.optim.Adam: the external optimizer updates the f32 master
    weights in place and the next forward refreshes the bf16 shadow the kernels read."""
    torch.manual_seed(0)
    oracle = init_deterministic(TransformerTTSOracle(OracleConfig()), 1)
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
    model.load_state_dict(oracle.state_dict())
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    text, tl, mel, ml = [t.cuda() for t in batch(3)]
    losses = []
    for step in range(8):
        model.set_seed(step)
        opt.zero_grad()
        out = model(text, tl, mel, ml)
        total, _ = model.loss(out, mel, ml)
        total.backward()
        opt.step()
        losses.append(total.item())
    out = model(text, tl, mel, ml)     # the forward refreshed the shadow from the updated master
    e = model.engine
    assert torch.equal(e.shadow, e.params.bfloat16())
    assert losses[-1] < 0.8 * losses[0], losses


def test_backward_after_overwriting_forward_raises():
    model = TransformerTTS(TTSConfig(), dtype=torch.float32).train()
    text, tl, mel, ml = [t.cuda() for t in batch(1)]
    out1 = model(text, tl, mel, ml)
    l1, _ = model.loss(out1, mel, ml)
    model(text, tl, mel, ml)            # same shape: reuses (overwrites) the activation arena
    with pytest.raises(RuntimeError, match="overwrote"):
        l1.backward()
