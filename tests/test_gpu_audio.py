"""Audio data path on the GPU vs the numpy oracle: log-mel
extraction (ragged batch, tone + noise) and Griffin-Lim inversion."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import tt2_audio_oracle as ao  # noqa: E402
from tt2.audio import GriffinLim, MelExtractor, mel_filterbank  # noqa: E402


def _signals(B, L, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(L) / ao.SR
    x = np.stack([0.3 * np.sin(2 * np.pi * (200 + 300 * b) * t) + 0.05 * rng.standard_normal(L) for b in range(B)])
    return x.astype(np.float32)


def test_filterbank_matches_oracle():
    assert np.abs(mel_filterbank().numpy() - ao.mel_filterbank()).max() < 1e-12


@pytest.mark.parametrize("L", [4000, 22050])
def test_log_mel_matches_oracle_ragged(L):
    B = 3
    x = _signals(B, L, L)
    lens = np.array([L, L - 1000, 700])
    mx = MelExtractor()
    mel, frames = mx(torch.from_numpy(x).cuda(), torch.from_numpy(lens).cuda())
    mel = mel.cpu().numpy()
    assert mel.shape == (B, ao.n_frames(L), 80)
    for b in range(B):
        ref = ao.log_mel(x[b, :lens[b]].astype(np.float64))
        nf = ref.shape[0]
        assert frames[b].item() == nf
        assert np.abs(mel[b, :nf] - ref).max() < 2e-3          # log domain, f32 vs f64
        assert np.allclose(mel[b, nf:], np.log(1e-5))           # past the utterance: silence


def test_griffin_lim_matches_oracle():
    B, L = 2, 6000
    x = _signals(B, L, 1)
    mx = MelExtractor()
    mel, frames = mx(torch.from_numpy(x).cuda())
    gl = GriffinLim(mx, n_iter=3)
    y, lens = gl(mel, frames)
    y = y.cpu().numpy()
    pinv = np.linalg.pinv(ao.mel_filterbank())
    for b in range(B):
        n = int(lens[b])
        mag = np.maximum(0.0, np.exp(mel[b].cpu().numpy().astype(np.float64)) @ pinv.T)
        ref = ao.griffin_lim(mag, n, n_iter=3)
        assert np.linalg.norm(y[b, :n] - ref) / np.linalg.norm(ref) < 1e-3


def test_griffin_lim_converges():
    B, L = 1, 8192
    x = _signals(B, L, 2)
    mx = MelExtractor()
    mel, frames = mx(torch.from_numpy(x).cuda())
    errs = []
    for it in (1, 24):
        y, _ = GriffinLim(mx, n_iter=it)(mel, frames)
        m2, _ = mx(y[:, :y.shape[1]])
        errs.append((m2[:, :-2] - mel[:, :m2.shape[1] - 2]).abs().mean().item())
    assert errs[1] < errs[0]


def test_ljspeech_collate_and_train_step(tmp_path):
    """A mini LJSpeech-format directory -> collate (GPU log-mels match the oracle per
    utterance) -> one bf16 training step on that batch."""
    from test_data import _mini_ljspeech
    from tt2.config import TTSConfig
    from tt2.data import LJSpeech, collate
    from tt2.model import TransformerTTS
    ds = LJSpeech(_mini_ljspeech(str(tmp_path / "lj")))
    mx = MelExtractor()
    text, tl, mel, ml = collate(ds, [0, 3, 4], mx)
    assert text.shape[0] == 3 and int(tl.max()) == text.shape[1]
    for row, i in enumerate([0, 3, 4]):
        ref = ao.log_mel(ds.wav(i).astype(np.float64))
        assert int(ml[row]) == ref.shape[0]
        assert np.abs(mel[row, :ref.shape[0]].cpu().numpy() - ref).max() < 2e-3
    model = TransformerTTS(TTSConfig(), dtype=torch.bfloat16).train()
    loss = model.train_step(text, tl, mel, ml)
    assert torch.isfinite(loss).all()
