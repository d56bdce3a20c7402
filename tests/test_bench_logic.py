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
    def summary(self, span=False):
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
    assert r["kernel"] == "gemm7_kernel<true, true, 0>" and r["launches_per_step"] == 2
    assert abs(r["achieved"] - 2000.0) < 1e-6 and r["bound"] == "mfma"


def test_longform_algo_bytes_counts_running_utterances_only():
    """cfg5's roofline bytes: weights once per step, each utterance's cross K/V and t + 1 self
    K/V rows only while it runs (its attention exits after its stop)."""
    import torch
    lens = torch.tensor([1, 3])
    got = bench.longform_algo_bytes(lens, 3)
    want = 3 * bench.LF_W_BYTES + 4 * bench.LF_CROSS_BYTES + bench.LF_KEY_BYTES * (1 + (1 + 2 + 3))
    assert abs(got - want) < 1e-6 * want


def test_multi_gpu_request_without_torchrun_spawns_ranks_and_fails_loudly():
    """`bench.py --gpus 2` with no WORLD_SIZE starts 2 rank processes itself.  Here (no GPU)
    the ranks rendezvous over gloo and then fail at their first device call: the launcher
    must exit non-zero and print no JSON line (never a dp1 line for a dp2 request)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["TT2_DIST_TIMEOUT_S"] = "60"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "launched 2 ranks" in r.stderr


def test_world_size_mismatch_is_refused():
    """Under torchrun with WORLD_SIZE != --gpus the rank refuses to report."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "refusing" in r.stderr
