"""Audio data path either side of the mel engine.

* ``MelExtractor``: waveform batch -> log-mel targets [B, T, 80] in the model's
  channels-last layout, Tacotron2 convention (22.05 kHz, n_fft 1024, hop 256,
  periodic Hann, centre reflect padding, magnitude, 80 Slaney mel bands over
  0..8000 Hz, log(max(x, 1e-5))).
* ``GriffinLim``: synthesised log-mels -> waveform (mel -> linear magnitude by the
  filterbank's pseudo-inverse, then Griffin-Lim with the least-squares iSTFT): the
  vocoder hand-off for listening tests.

Every transform runs on the GPU through libtt2: the window-folded DFT basis, its
inverse and the mel filterbank are f32 ``tt2_gemm`` operands (constant tables built
once at construction), and csrc/audio.hip does the padding, magnitude, phase
projection, overlap-add and log/exp row moves.  The frames of the whole batch are
one strided GEMM operand (ld = hop) over a padded buffer whose per-utterance length
is a multiple of the hop (see include/tt2_capi.h).
"""
from __future__ import annotations

import math

import torch

from . import ops
from ._lib import ACT_RELU, check, lib, ptr, stream_ptr

SR, N_FFT, HOP, N_MELS, FMIN, FMAX, LOG_CLAMP = 22050, 1024, 256, 80, 0.0, 8000.0, 1e-5
NB = N_FFT // 2 + 1          # 513 frequency bins
LD_SPEC = 1032               # [re 513 | im 513 | pad] columns of a spectrum row (16-B rows)
LD_MAG = 516                 # 513 magnitudes + pad


def _hz_to_mel(f: torch.Tensor) -> torch.Tensor:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return torch.where(f >= min_log_hz, min_log_mel + torch.log(f.clamp_min(1e-12) / min_log_hz) / logstep, f / f_sp)


def _mel_to_hz(m: torch.Tensor) -> torch.Tensor:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr=SR, n_fft=N_FFT, n_mels=N_MELS, fmin=FMIN, fmax=FMAX) -> torch.Tensor:
    """[n_mels, n_fft/2 + 1] Slaney-normalised triangular filters (the algorithm of
    librosa.filters.mel, htk=False, norm='slaney'), float64 on the host."""
    d = torch.float64
    fft_f = torch.linspace(0, sr / 2, n_fft // 2 + 1, dtype=d)
    edges = _mel_to_hz(torch.linspace(float(_hz_to_mel(torch.tensor(fmin, dtype=d))),
                                      float(_hz_to_mel(torch.tensor(fmax, dtype=d))), n_mels + 2, dtype=d))
    fdiff = edges[1:] - edges[:-1]
    ramps = edges[:, None] - fft_f[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = torch.clamp(torch.minimum(lower, upper), min=0.0)
    return w * (2.0 / (edges[2:] - edges[:-2]))[:, None]


def _window(n=N_FFT) -> torch.Tensor:
    return 0.5 - 0.5 * torch.cos(2 * math.pi * torch.arange(n, dtype=torch.float64) / n)


def n_frames(n_samples: int) -> int:
    return 1 + n_samples // HOP


class _Plan:
    """Buffers of one (batch, samples) shape."""

    def __init__(self, B: int, L: int, dev):
        self.B, self.L = B, L
        self.Lp = -(-(L + N_FFT) // HOP) * HOP          # padded length per utterance, multiple of hop
        self.R = self.Lp // HOP                          # frame rows per utterance
        self.M = B * self.R - (N_FFT // HOP - 1)         # frame rows of the batch matrix (last one in bounds)
        self.T = n_frames(L)
        f32 = dict(dtype=torch.float32, device=dev)
        self.padded = torch.zeros(B * self.Lp, **f32)
        self.spec = torch.zeros(B * self.R, LD_SPEC, **f32)
        self.mag = torch.zeros(B * self.R, LD_MAG, **f32)
        self.rows = torch.zeros(B * self.R, N_MELS, **f32)


class MelExtractor:
    def __init__(self, device="cuda"):
        self.dev = torch.device(device)
        w = _window()
        n = torch.arange(N_FFT, dtype=torch.float64)
        k = torch.arange(NB, dtype=torch.float64)
        ang = 2 * math.pi * k[:, None] * n[None, :] / N_FFT
        basis = torch.zeros(LD_SPEC, N_FFT, dtype=torch.float64)
        basis[:NB] = torch.cos(ang) * w            # Re X_k = sum_n w[n] x[n] cos(2 pi k n / N)
        basis[NB:2 * NB] = -torch.sin(ang) * w     # Im X_k = -sum_n w[n] x[n] sin(2 pi k n / N)
        self.basis = basis.float().to(self.dev)
        fb = torch.zeros(N_MELS, LD_MAG, dtype=torch.float64)
        fb[:, :NB] = mel_filterbank()
        self.fb = fb.float().to(self.dev)
        self.plans: dict[tuple[int, int], _Plan] = {}

    def plan(self, B: int, L: int) -> _Plan:
        if L <= N_FFT // 2:
            raise ValueError(f"utterances need more than {N_FFT // 2} samples (reflect padding)")
        key = (B, L)
        if key not in self.plans:
            self.plans[key] = _Plan(B, L, self.dev)
        return self.plans[key]

    def stft(self, x: torch.Tensor, lens: torch.Tensor | None, P: _Plan):
        """P.spec rows [b * R + f] = [Re | Im] STFT of utterance b's frame f (f32)."""
        L = lib()
        check(L.tt2_reflect_pad(x.data_ptr(), x.stride(0), ptr(lens), P.B, P.L, P.padded.data_ptr(), P.Lp,
                                N_FFT // 2, stream_ptr()), "tt2_reflect_pad")
        ops.gemm(P.padded, self.basis, P.spec, P.M, LD_SPEC, N_FFT, HOP, N_FFT, LD_SPEC)

    def __call__(self, audio: torch.Tensor, lens: torch.Tensor | None = None):
        """audio [B, L] f32 (device), lens [B] samples (optional, each > 512).
        Returns (log-mel [B, T, 80] f32, frames [B] int32) with T = 1 + L // 256;
        frames past an utterance's own 1 + len // 256 hold log(1e-5) (silence)."""
        B, Lx = audio.shape
        audio = audio.to(self.dev, torch.float32).contiguous()
        P = self.plan(B, Lx)
        lens32 = lens.to(self.dev, torch.int32) if lens is not None else None
        self.stft(audio, lens32, P)
        L = lib()
        check(L.tt2_spec_magnitude(P.spec.data_ptr(), LD_SPEC, P.M, NB, P.mag.data_ptr(), LD_MAG, stream_ptr()),
              "tt2_spec_magnitude")
        ops.gemm(P.mag, self.fb, P.rows, P.M, N_MELS, LD_MAG, LD_MAG, LD_MAG, N_MELS)
        frames = (1 + lens32 // HOP) if lens32 is not None else torch.full((B,), P.T, dtype=torch.int32,
                                                                              device=self.dev)
        mel = torch.empty(B, P.T, N_MELS, dtype=torch.float32, device=self.dev)
        check(L.tt2_mel_rows(P.rows.data_ptr(), N_MELS, mel.data_ptr(), frames.data_ptr(), B, P.T, N_MELS, P.R,
                             LOG_CLAMP, 0, stream_ptr()), "tt2_mel_rows")
        return mel, frames


class GriffinLim:
    """log-mel [B, T, 80] -> waveform [B, (T - 1) * 256] by Griffin-Lim (zero initial phase)."""

    def __init__(self, extractor: MelExtractor | None = None, n_iter: int = 32):
        self.mx = extractor or MelExtractor()
        self.n_iter = n_iter
        dev = self.mx.dev
        w = _window()
        n = torch.arange(N_FFT, dtype=torch.float64)
        k = torch.arange(NB, dtype=torch.float64)
        ang = 2 * math.pi * n[:, None] * k[None, :] / N_FFT
        ck = torch.full((NB,), 2.0, dtype=torch.float64)
        ck[0] = ck[-1] = 1.0
        ib = torch.zeros(N_FFT, LD_SPEC, dtype=torch.float64)
        ib[:, :NB] = torch.cos(ang) * ck / N_FFT * w[:, None]        # irfft, synthesis window folded in
        ib[:, NB:2 * NB] = -torch.sin(ang) * ck / N_FFT * w[:, None]
        ib[:, NB] = 0.0
        ib[:, 2 * NB - 1] = 0.0                                     # imaginary DC / Nyquist ignored
        self.ibasis = ib.float().to(dev)
        pinv = torch.zeros(LD_MAG, N_MELS, dtype=torch.float64)
        pinv[:NB] = torch.linalg.pinv(mel_filterbank())
        self.pinv = pinv.float().to(dev)

    def __call__(self, logmel: torch.Tensor, frames: torch.Tensor | None = None):
        B, T, _ = logmel.shape
        Ls = (T - 1) * HOP
        mx = self.mx
        P = mx.plan(B, Ls)
        dev = mx.dev
        logmel = logmel.to(dev, torch.float32).contiguous()
        fr = frames.to(dev, torch.int32) if frames is not None else torch.full((B,), T, dtype=torch.int32, device=dev)
        lens = ((fr - 1) * HOP).clamp_min(N_FFT // 2 + 1).to(torch.int32)
        L = lib()
        # linear magnitude = relu(pinv(fb) exp(logmel)), in the frame-row layout
        check(L.tt2_mel_rows(P.rows.data_ptr(), N_MELS, logmel.data_ptr(), fr.data_ptr(), B, T, N_MELS, P.R,
                             LOG_CLAMP, 1, stream_ptr()), "tt2_mel_rows")
        mag = torch.zeros(B * P.R, LD_MAG, dtype=torch.float32, device=dev)
        ops.gemm(P.rows, self.pinv, mag, B * P.R, LD_MAG, N_MELS, N_MELS, N_MELS, LD_MAG, act=ACT_RELU)
        spec = torch.empty(B * P.R, LD_SPEC, dtype=torch.float32, device=dev)
        frames_td = torch.empty(B * P.R, N_FFT, dtype=torch.float32, device=dev)
        y = torch.zeros(B, Ls, dtype=torch.float32, device=dev)
        est = None
        for it in range(self.n_iter + 1):
            check(L.tt2_spec_rephase(mag.data_ptr(), LD_MAG, ptr(est), LD_SPEC, B * P.R, NB, spec.data_ptr(),
                                     LD_SPEC, stream_ptr()), "tt2_spec_rephase")
            ops.gemm(spec, self.ibasis, frames_td, B * P.R, N_FFT, LD_SPEC, LD_SPEC, LD_SPEC, N_FFT)
            check(L.tt2_overlap_add(frames_td.data_ptr(), N_FFT, lens.data_ptr(), B, Ls, P.R, N_FFT, HOP,
                                    y.data_ptr(), Ls, stream_ptr()), "tt2_overlap_add")
            if it == self.n_iter:
                break
            mx.stft(y, lens, P)
            est = P.spec
        return y, lens
