"""Per-step JSONL metrics on the GPU (tt2/metrics.py): eager and captured steps each write
one line, lagged by one step (flushed at close), whose loss terms equal the step's device
loss vector and whose timing fields are positive."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu

from tt2.config import TTSConfig  # noqa: E402
from tt2.model import TransformerTTS  # noqa: E402


def test_metrics_jsonl(tmp_path):
    g = torch.Generator().manual_seed(3)
    B, Tx, Ty = 2, 24, 48
    text = torch.randint(1, 80, (B, Tx), generator=g).cuda()
    tl = torch.tensor([24, 17]).cuda()
    mel = torch.randn(B, Ty, 80, generator=g).cuda()
    ml = torch.tensor([48, 30]).cuda()
    m = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
    m.configure_optimizer(lr=1e-3, warmup=10.0)
    path = tmp_path / "m.jsonl"
    m.train_step(text, tl, mel, ml)            # sizes the workspaces (before metrics: no line)
    m.enable_metrics(str(path))
    losses = [m.train_step(text, tl, mel, ml).clone() for _ in range(2)]
    run = m.capture_train_step(B, Tx, Ty)
    losses += [run(text, tl, mel, ml).clone() for _ in range(2)]
    assert len(path.read_text().splitlines()) == 3          # the last step is still pending
    m.enable_metrics(None)                                   # close() flushes it
    lines = [json.loads(x) for x in path.read_text().splitlines()]
    assert [r["step"] for r in lines] == [0, 1, 2, 3]
    for r, lv in zip(lines, losses):
        assert r["ms"] > 0 and r["frames_per_s"] > 0 and r["tflops"] > 0
        assert r["allreduce_ms"] is None and r["batch"] == B and r["frames"] == Ty and r["world"] == 1
        # frames_per_s counts padded frames (B x Ty), valid_frames_per_s the mel_len frames
        assert r["valid_frames_per_s"] / r["frames_per_s"] == pytest.approx((48 + 30) / (B * Ty), rel=1e-3)
        got = [r["loss"][k] for k in ("total", "mse_before", "mse_after", "bce_stop")]
        assert got == pytest.approx(lv.float().cpu().tolist(), rel=1e-6)
