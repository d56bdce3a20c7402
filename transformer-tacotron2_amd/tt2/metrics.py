"""Per-step JSONL metrics (SURVEY.md §5 "metrics/logging"; off by default).

    model.enable_metrics("run/metrics.jsonl")      # or TT2_METRICS=<path> in the environment
    for batch in loader:
        model.train_step(*batch, sync_grads=sync.finish)   # or a captured run(...)

One JSON object per training step: wall time of the step on the device (HIP events on
the compute stream around it), mel frames/s (padded frames, B x Ty per rank, times the world size; valid_frames_per_s counts
the mel_len frames of this rank's batch times the world size), the loss terms, the span of the gradient
all-reduce on the comm stream (RcclGradSync; null without data parallelism) and the
achieved useful TFLOP/s against the dense bf16 MFMA peak.  Nothing blocks the step: a
step's events and loss are read back once the NEXT step has been issued (and at close()),
so the host never waits on the step it just launched.
"""
from __future__ import annotations

import json
import os
import time

import torch

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)


def step_flops(cfg, B: int, Tx: int, Ty: int) -> float:
    """Useful FLOPs of one training step (forward counted per block,
    causal self-attention at half, backward = 2x forward).  cfg2 (16, 128, 800): 2.63e12."""
    d, f, h_dim = cfg.d_model, cfg.d_ffn, cfg.d_model
    Me, Md = B * Tx, B * Ty
    k, ck = cfg.enc_conv_kernel, cfg.postnet_kernel
    enc = (2 * Me * d * d * k * cfg.enc_conv_layers + 2 * Me * d * d
           + cfg.n_enc * (2 * Me * 4 * d * d + 4 * B * Tx * Tx * h_dim + 2 * Me * 2 * d * f))
    p = cfg.dec_prenet
    dec = 2 * Md * (cfg.n_mels * p + p * p + p * d)
    dec += cfg.n_dec * (2 * Md * 4 * d * d + 4 * B * Ty * Ty * h_dim / 2
                        + 2 * Md * 2 * d * d + 2 * Me * 2 * d * d + 4 * B * Ty * Tx * h_dim
                        + 2 * Md * 2 * d * f)
    heads = 2 * Md * d * (cfg.n_mels + 1)
    c = cfg.postnet_channels
    chans = [cfg.n_mels] + [c] * (cfg.postnet_layers - 1) + [cfg.n_mels]
    post = sum(2 * Md * ck * chans[i] * chans[i + 1] for i in range(cfg.postnet_layers))
    return 3.0 * (enc + dec + heads + post)


class StepMetrics:
    """Appends one JSON line per step to `path` (see the module docstring)."""

    LOSS_KEYS = ("total", "mse_before", "mse_after", "bce_stop")

    def __init__(self, path: str, cfg, world: int | None = None):
        """world: ranks whose frames count in frames/s; None: torch.distributed's world size,
        looked up when the first line is written (after init_process_group, wherever the
        model was built)."""
        self.path, self.cfg, self.world = path, cfg, world
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", buffering=1)
        self._pending = None
        self._open = None
        self.step = 0

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._open = ev

    def _world(self) -> int:
        if self.world is None:
            import torch.distributed as dist
            self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        return self.world

    def end(self, loss: torch.Tensor, B: int, Tx: int, Ty: int, sync=None, mel_len: torch.Tensor | None = None):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        ar = sync.pop_span() if sync is not None and hasattr(sync, "pop_span") else None
        valid = mel_len.detach().to(torch.int64).sum() if mel_len is not None else None   # device scalar, no sync
        cur = (self._open, ev, loss.detach().clone(), (B, Tx, Ty), ar, time.time(), valid)
        self._open = None
        self.flush()
        self._pending = cur

    def flush(self):
        if self._pending is None:
            return
        t0, t1, loss, (B, Tx, Ty), ar, wall, valid = self._pending
        self._pending = None
        t1.synchronize()
        ms = t0.elapsed_time(t1)
        vals = loss.float().cpu().tolist()
        fl = step_flops(self.cfg, B, Tx, Ty)
        world = self._world()
        rec = {"step": self.step, "time": round(wall, 3), "ms": round(ms, 4),
               "frames_per_s": round(world * B * Ty / (ms / 1e3), 1),
               "valid_frames_per_s": round(world * int(valid.item()) / (ms / 1e3), 1) if valid is not None else None,
               "loss": {k: v for k, v in zip(self.LOSS_KEYS, vals)},
               "allreduce_ms": round(ar[0].elapsed_time(ar[1]), 4) if ar is not None else None,
               "tflops": round(fl / (ms / 1e3) / 1e12, 2),
               "frac_of_peak": round(fl / (ms / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4),
               "batch": B, "text_len": Tx, "frames": Ty, "world": world}
        self._f.write(json.dumps(rec) + "\n")
        self.step += 1

    def close(self):
        self.flush()
        self._f.close()
