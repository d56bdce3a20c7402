"""CPU: pin the audio oracle (oracle/tt2_audio_oracle.py): STFT vs scipy.signal.stft,
the Slaney mel filterbank's known-answer properties, iSTFT perfect reconstruction,
Griffin-Lim convergence."""
import numpy as np
import scipy.signal

import tt2_audio_oracle as ao


def test_stft_matches_scipy():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(5000)
    ours = ao.stft(x)
    _, _, z = scipy.signal.stft(x, fs=ao.SR, window="hann", nperseg=ao.N_FFT, noverlap=ao.N_FFT - ao.HOP,
                                nfft=ao.N_FFT, boundary="even", padded=False, detrend=False,
                                return_onesided=True)
    ref = z.T * ao.hann().sum()          # scipy scales the spectrum by 1 / sum(window)
    assert ours.shape == ref.shape == (ao.n_frames(5000), ao.N_FFT // 2 + 1)
    assert np.abs(ours - ref).max() < 1e-9 * np.abs(ref).max()


def test_mel_filterbank_known_answers():
    fb = ao.mel_filterbank()
    assert fb.shape == (80, 513) and (fb >= 0).all()
    edges = ao.mel_to_hz(np.linspace(ao.hz_to_mel(0.0), ao.hz_to_mel(8000.0), 82))
    assert abs(edges[-1] - 8000.0) < 1e-6 and edges[0] == 0.0
    fft_f = np.linspace(0, ao.SR / 2, 513)
    for i in (0, 10, 40, 79):
        # peak at the FFT bin nearest the band centre; Slaney area: sum ~ 2 / df_bins * ...
        assert abs(fft_f[fb[i].argmax()] - edges[i + 1]) <= ao.SR / ao.N_FFT
        area = np.trapezoid(fb[i], fft_f) if hasattr(np, "trapezoid") else np.trapz(fb[i], fft_f)
        assert abs(area - 1.0) < 0.15     # triangle of height 2/(hi-lo) over (hi-lo): unit area
    assert fb[:, fft_f > 8000.0 + ao.SR / ao.N_FFT].max() == 0.0
    # Slaney scale: linear below 1 kHz
    assert abs(ao.hz_to_mel(600.0) - 9.0) < 1e-9 and abs(ao.mel_to_hz(ao.hz_to_mel(3000.0)) - 3000.0) < 1e-6


def test_log_mel_tone_lands_in_its_band():
    t = np.arange(ao.SR) / ao.SR
    f0 = 1500.0
    m = ao.log_mel(np.sin(2 * np.pi * f0 * t))
    edges = ao.mel_to_hz(np.linspace(ao.hz_to_mel(0.0), ao.hz_to_mel(8000.0), 82))
    band = int(m[10:-10].mean(0).argmax())
    assert edges[band] <= f0 <= edges[band + 2]
    assert m.shape == (ao.n_frames(ao.SR), 80)


def test_istft_reconstructs():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(7000)
    y = ao.istft(ao.stft(x), len(x))
    assert np.abs(y - x).max() < 1e-9


def test_griffin_lim_reduces_spectral_error():
    t = np.arange(8192) / ao.SR
    x = np.sin(2 * np.pi * 440 * t) + 0.5 * np.sin(2 * np.pi * 1250 * t)
    mag = np.abs(ao.stft(x))

    def err(y):
        return np.linalg.norm(np.abs(ao.stft(y)) - mag) / np.linalg.norm(mag)

    e1 = err(ao.griffin_lim(mag, len(x), n_iter=1))
    e16 = err(ao.griffin_lim(mag, len(x), n_iter=16))
    assert e16 < 0.8 * e1      # Griffin-Lim never increases the spectral distance
