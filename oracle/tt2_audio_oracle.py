"""CPU oracle for the audio data path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this file; the shipped GPU path (``tt2/audio.py`` +
``csrc/audio.hip``) never imports or falls back to it.

What it restates (the steps either side of the hot path):

* log-mel extraction, Tacotron2 convention [P]: 22.05 kHz audio, STFT with a
  periodic Hann window of 1024, hop 256, centre reflect padding of n_fft/2,
  magnitude (power 1), an 80-band Slaney-style mel filterbank over 0..8000 Hz
  (the algorithm of librosa.filters.mel with htk=False, norm="slaney"),
  then log(max(x, 1e-5));
* Griffin-Lim inversion of a linear magnitude spectrogram: x = iSTFT(S e^{i phi}),
  phi = angle(STFT(x)), with the weighted overlap-add normalised by the summed
  squared window (the standard least-squares iSTFT).

Pinning: librosa is not installed here, so the filterbank is a restatement of its
published algorithm ("parity unpinned" against librosa itself).  The STFT is pinned
against ``scipy.signal.stft`` (same window / hop / reflect boundary) and the
filterbank against known-answer properties (triangle peaks at the band centres,
Slaney area normalisation, a pure tone lands in the band that contains it) in
``tests/test_audio_oracle.py``.  The iSTFT is pinned by perfect reconstruction.
"""
from __future__ import annotations

import numpy as np

SR, N_FFT, HOP, N_MELS, FMIN, FMAX, LOG_CLAMP = 22050, 1024, 256, 80, 0.0, 8000.0, 1e-5


def hann(n: int = N_FFT) -> np.ndarray:
    """Periodic Hann window (scipy.signal.get_window('hann', n, fftbins=True))."""
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / n)


def hz_to_mel(f):
    """Slaney mel scale: linear below 1 kHz (3 mels / 200 Hz), log above."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-12) / min_log_hz) / logstep, f / f_sp)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr=SR, n_fft=N_FFT, n_mels=N_MELS, fmin=FMIN, fmax=FMAX) -> np.ndarray:
    """[n_mels, n_fft // 2 + 1] triangles between n_mels + 2 mel-spaced edges, each
    scaled by 2 / (f_hi - f_lo) (Slaney area normalisation)."""
    fft_f = np.linspace(0, sr / 2, n_fft // 2 + 1)
    edges = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(edges)
    ramps = edges[:, None] - fft_f[None, :]
    w = np.zeros((n_mels, n_fft // 2 + 1))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (edges[2:n_mels + 2] - edges[:n_mels]))[:, None]
    return w


def n_frames(n_samples: int, hop: int = HOP) -> int:
    return 1 + n_samples // hop


def stft(x: np.ndarray, n_fft=N_FFT, hop=HOP) -> np.ndarray:
    """Complex STFT [frames, n_fft // 2 + 1] of one 1-D signal (centre reflect padding)."""
    xp = np.pad(x.astype(np.float64), n_fft // 2, mode="reflect")
    nf = n_frames(len(x), hop)
    idx = np.arange(n_fft)[None, :] + hop * np.arange(nf)[:, None]
    return np.fft.rfft(xp[idx] * hann(n_fft)[None, :], axis=1)


def log_mel(x: np.ndarray) -> np.ndarray:
    """[frames, 80] log-mel of one utterance (the model's channels-last mel layout)."""
    mag = np.abs(stft(x))
    return np.log(np.maximum(mag @ mel_filterbank().T, LOG_CLAMP))


def istft(spec: np.ndarray, length: int, n_fft=N_FFT, hop=HOP) -> np.ndarray:
    """Least-squares inverse of ``stft``: windowed overlap-add / summed squared window."""
    nf = spec.shape[0]
    frames = np.fft.irfft(spec, n=n_fft, axis=1) * hann(n_fft)[None, :]
    total = n_fft + hop * (nf - 1)
    y = np.zeros(total)
    wss = np.zeros(total)
    w2 = hann(n_fft) ** 2
    for f in range(nf):
        y[f * hop:f * hop + n_fft] += frames[f]
        wss[f * hop:f * hop + n_fft] += w2
    y = np.where(wss > 1e-8, y / np.maximum(wss, 1e-8), 0.0)
    return y[n_fft // 2:n_fft // 2 + length]


def griffin_lim(mag: np.ndarray, length: int, n_iter: int = 32) -> np.ndarray:
    """Griffin-Lim from a linear magnitude [frames, n_fft // 2 + 1], zero initial phase."""
    spec = mag.astype(np.complex128)
    for _ in range(n_iter):
        x = istft(spec, length)
        e = stft(x)
        spec = mag * np.exp(1j * np.angle(e))
    return istft(spec, length)
