"""CPU: the LJSpeech-format data path host logic: text front end,
metadata parsing, WAV loading, length-bucketed batching."""
import os

import numpy as np
from scipy.io import wavfile

from tt2.data import SYMBOLS, LJSpeech, bucket_batches, clean_text, ids_to_text, text_to_ids


def test_symbol_table_fits_the_embedding():
    assert len(SYMBOLS) <= 80 and SYMBOLS[0] == "_" and len(set(SYMBOLS)) == len(SYMBOLS)


def test_text_front_end_known_answers():
    assert clean_text("  Mr. Smith   met Dr. Jones.\n") == "mister smith met doctor jones."
    ids = text_to_ids("Hi, there!")
    assert ids[-1] == SYMBOLS.index("~") and 0 not in ids
    assert ids_to_text(ids) == "hi, there!"
    assert text_to_ids("aéb", eos=False) == [SYMBOLS.index("a"), SYMBOLS.index("b")]   # unknown dropped


def _mini_ljspeech(root, n=5, sr=22050):
    os.makedirs(os.path.join(root, "wavs"))
    rng = np.random.default_rng(0)
    lines = []
    for i in range(n):
        uid = f"LJ001-{i:04d}"
        x = (0.3 * np.sin(2 * np.pi * (200 + 50 * i) * np.arange(sr // 4 + 1000 * i) / sr)
             + 0.01 * rng.standard_normal(sr // 4 + 1000 * i))
        wavfile.write(os.path.join(root, "wavs", uid + ".wav"), sr, (x * 32767).astype(np.int16))
        lines.append(f"{uid}|Raw text {i}, Mr. X.|Normalized text number {i}, mister X.")
    with open(os.path.join(root, "metadata.csv"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return root


def test_ljspeech_parsing_and_wavs(tmp_path):
    ds = LJSpeech(_mini_ljspeech(str(tmp_path / "lj")))
    assert len(ds) == 5 and ds.items[2][0] == "LJ001-0002"
    assert ids_to_text(ds.ids(1)) == "normalized text number 1, mister x."
    w = ds.wav(3)
    assert w.dtype == np.float32 and len(w) == 22050 // 4 + 3000 and np.abs(w).max() <= 1.0
    raw = LJSpeech(str(tmp_path / "lj"), use_normalized=False)
    assert raw.items[0][1] == "Raw text 0, Mr. X."


def test_bucket_batches_cover_and_group():
    lengths = list(np.random.default_rng(3).integers(10, 1000, 203))
    bs = bucket_batches(lengths, 8, bucket_mult=4, seed=1)
    flat = sorted(i for b in bs for i in b)
    assert flat == list(range(203))
    assert all(len(b) <= 8 for b in bs)
    spread = np.mean([max(lengths[i] for i in b) - min(lengths[i] for i in b) for b in bs if len(b) > 1])
    assert spread < 0.5 * (max(lengths) - min(lengths))
    assert bucket_batches(lengths, 8, seed=1) == bucket_batches(lengths, 8, seed=1)
    assert all(len(b) == 8 for b in bucket_batches(lengths, 8, seed=2, drop_last=True))
