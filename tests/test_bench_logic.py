"""bench.py host logic that must hold at N > 1 (CPU, no GPU calls).

The roofline leg runs one instrumented eager step on rank 0 only; the DP gradient hook
must be detached for it (its bucket all-reduces would have no peers on the other ranks)
and restored afterwards."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tt2 import ops  # noqa: E402


class _Probe:
    def summary(self):
        # key -> (launches, flops, seconds, algorithmic bytes)
        return {("gemm", 13, 0, 0): (2, 4.0e12, 2e-3, 2 << 20)}

    def replay_time(self, key):
        return 2e-3


class _Engine:
    grad_ready_hook = "dp-hook"


class _Model:
    def __init__(self):
        self.engine = _Engine()
        self.hook_seen = "unset"

    def train_step(self, *batch):
        self.hook_seen = self.engine.grad_ready_hook


def test_roofline_detaches_dp_hook(monkeypatch):
    monkeypatch.setattr(ops, "LaunchProbe", _Probe)
    m = _Model()
    r = bench.roofline(m, None, None, None, None)
    assert m.hook_seen is None                      # no all-reduce from the rank-0-only step
    assert m.engine.grad_ready_hook == "dp-hook"    # restored for later steps
    assert ops.PROBE is None
    assert r["kernel"] == "gemm7_kernel<true, true>" and r["launches_per_step"] == 2
    assert abs(r["achieved"] - 2000.0) < 1e-6 and r["bound"] == "mfma"


def test_longform_algo_bytes_counts_running_utterances_only():
    """cfg5's roofline bytes: weights once per step, each utterance's cross K/V and t + 1 self
    K/V rows only while it runs (its attention exits after its stop)."""
    import torch
    lens = torch.tensor([1, 3])
    got = bench.longform_algo_bytes(lens, 3)
    want = 3 * bench.LF_W_BYTES + 4 * bench.LF_CROSS_BYTES + bench.LF_KEY_BYTES * (1 + (1 + 2 + 3))
    assert abs(got - want) < 1e-6 * want
