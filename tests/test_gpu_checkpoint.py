"""Checkpoint save/resume (GPU): 2 steps + save + load into a fresh
model + 2 steps equals 4 uninterrupted steps bit for bit (parameters, Adam moments,
optimizer step, BN running statistics and the dropout-seed stream all restored)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def _model():
    torch.manual_seed(0)
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16, seed=11)
    with torch.no_grad():
        for name, (off, shape, n) in m.engine.lay.slots.items():
            if len(shape) >= 2:
                m.engine.P(name).normal_(0, 0.02)
        m.engine.sync_shadow()
    m.configure_optimizer(lr=1e-3, warmup=10.0)
    return m.train()


def test_resume_is_bitwise(tmp_path):
    g = torch.Generator().manual_seed(4)
    B, Tx, Ty = 2, 20, 40
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([20, 13]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([40, 25]).cuda()
    a = _model()
    losses = [a.train_step(text, tl, mel, ml).clone() for _ in range(4)]
    b = _model()
    for _ in range(2):
        b.train_step(text, tl, mel, ml)
    path = str(tmp_path / "ck.pt")
    b.save_checkpoint(path)
    c = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
    c.load_checkpoint(path)
    resumed = [c.train_step(text, tl, mel, ml).clone() for _ in range(2)]
    torch.cuda.synchronize()
    assert torch.equal(resumed[0], losses[2]) and torch.equal(resumed[1], losses[3])
    assert torch.equal(c.engine.params, a.engine.params)
    assert torch.equal(c.engine.exp_avg_sq, a.engine.exp_avg_sq)
    assert torch.equal(c.engine.stats, a.engine.stats)
    assert c.engine.seed.item() == a.engine.seed.item() and c.engine.step_t.item() == 4
