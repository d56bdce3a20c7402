"""Per-step JSONL metrics (tt2/metrics.py): the useful-FLOP count the lines
report, checked against SURVEY §8(a)'s per-block figures for cfg2 (CPU only)."""
from tt2.config import TTSConfig
from tt2.metrics import step_flops


def test_step_flops_cfg2_matches_survey():
    f = step_flops(TTSConfig(), 16, 128, 800)
    assert abs(f / 2.63e12 - 1) < 0.005, f          # 2.63e12 useful FLOPs per step
    assert abs(f / (16 * 800) / 2.05e8 - 1) < 0.005  # 2.05e8 FLOPs per mel frame


def test_step_flops_scales():
    c = TTSConfig()
    # linear in batch; the causal term makes it superlinear in frames
    assert abs(step_flops(c, 32, 128, 800) / step_flops(c, 16, 128, 800) - 2) < 1e-12
    assert step_flops(c, 16, 128, 1600) > 2 * step_flops(c, 16, 128, 800)
