"""LJSpeech-format data path: the on-disk input of real training.

* ``LJSpeech(root)``: ``root/metadata.csv`` (``id|raw text|normalised text`` per line,
  pipe-separated, no header, as LJSpeech-1.1 ships it) and ``root/wavs/<id>.wav``
  (22.05 kHz mono PCM);
* ``text_to_ids``: a character front end -- lower-casing, the English abbreviation
  expansions of the Tacotron2 ``english_cleaners``, whitespace collapse, unknown
  characters dropped, an end-of-sentence id appended -- onto a 50-symbol table that
  fits the model's 80-id embedding (id 0 = pad).  Grapheme-to-phoneme conversion is
  out of scope; characters are what Tacotron2 trains on by default;
* ``bucket_batches``: length-bucketed, shuffled batches (similar lengths together, so
  padding -- and the masked compute it costs -- stays small);
* ``collate``: padded id / length tensors and log-mel targets [B, T, 80] computed on the
  GPU by ``tt2.audio.MelExtractor`` (one batched STFT per batch).
"""
from __future__ import annotations

import csv
import os
import random
import re

import numpy as np
import torch

PAD, EOS = "_", "~"
_PUNCT = "!'(),.:;?-\""
SYMBOLS = [PAD, EOS, " "] + list(_PUNCT) + [chr(c) for c in range(ord("a"), ord("z") + 1)] + \
          [str(d) for d in range(10)]
SYMBOL_ID = {s: i for i, s in enumerate(SYMBOLS)}

_ABBREV = [(re.compile(r"\b%s\." % k, re.IGNORECASE), v) for k, v in [
    ("mrs", "misess"), ("mr", "mister"), ("dr", "doctor"), ("st", "saint"), ("co", "company"), ("jr", "junior"),
    ("maj", "major"), ("gen", "general"), ("drs", "doctors"), ("rev", "reverend"), ("lt", "lieutenant"),
    ("hon", "honorable"), ("sgt", "sergeant"), ("capt", "captain"), ("esq", "esquire"), ("ltd", "limited"),
    ("col", "colonel"), ("ft", "fort")]]
_WS = re.compile(r"\s+")


def clean_text(text: str) -> str:
    text = text.lower()
    for pat, rep in _ABBREV:
        text = pat.sub(rep, text)
    return _WS.sub(" ", text).strip()


def text_to_ids(text: str, eos: bool = True) -> list[int]:
    ids = [SYMBOL_ID[c] for c in clean_text(text) if c in SYMBOL_ID and c not in (PAD, EOS)]
    return ids + [SYMBOL_ID[EOS]] if eos else ids


def ids_to_text(ids) -> str:
    return "".join(SYMBOLS[i] for i in ids if 0 < i < len(SYMBOLS) and SYMBOLS[i] != EOS)


def load_wav(path: str, sr: int = 22050) -> np.ndarray:
    """Mono float32 in [-1, 1] (PCM16 / PCM32 / float WAV); no resampling."""
    from scipy.io import wavfile
    rate, x = wavfile.read(path)
    if rate != sr:
        raise ValueError(f"{path}: {rate} Hz, expected {sr} (resample offline)")
    if x.ndim > 1:
        x = x.mean(axis=1)
    if x.dtype == np.int16:
        return (x / 32768.0).astype(np.float32)
    if x.dtype == np.int32:
        return (x / 2147483648.0).astype(np.float32)
    return x.astype(np.float32)


class LJSpeech:
    def __init__(self, root: str, use_normalized: bool = True):
        self.root = root
        self.items = []   # (id, text)
        with open(os.path.join(root, "metadata.csv"), encoding="utf-8", newline="") as f:
            for row in csv.reader(f, delimiter="|", quoting=csv.QUOTE_NONE):
                if not row:
                    continue
                uid, raw = row[0], row[1]
                norm = row[2] if len(row) > 2 and row[2] else raw
                self.items.append((uid, norm if use_normalized else raw))

    def __len__(self):
        return len(self.items)

    def wav(self, i: int) -> np.ndarray:
        return load_wav(os.path.join(self.root, "wavs", self.items[i][0] + ".wav"))

    def ids(self, i: int) -> list[int]:
        return text_to_ids(self.items[i][1])


def bucket_batches(lengths, batch_size: int, bucket_mult: int = 8, seed: int = 0, drop_last: bool = False):
    """Shuffle, cut into chunks of batch_size * bucket_mult, sort each chunk by length,
    split into batches, shuffle the batches: every index appears exactly once."""
    rng = random.Random(seed)
    idx = list(range(len(lengths)))
    rng.shuffle(idx)
    chunk = batch_size * bucket_mult
    batches = []
    for c in range(0, len(idx), chunk):
        part = sorted(idx[c:c + chunk], key=lambda i: lengths[i])
        for b in range(0, len(part), batch_size):
            bb = part[b:b + batch_size]
            if len(bb) == batch_size or not drop_last:
                batches.append(bb)
    rng.shuffle(batches)
    return batches


def collate(ds: LJSpeech, indices, extractor, device="cuda"):
    """(text [B, Tx] i64, text_len [B], mel [B, T, 80] f32, mel_len [B]) for one batch;
    the log-mels come from one batched GPU STFT (tt2.audio.MelExtractor)."""
    ids = [ds.ids(i) for i in indices]
    wavs = [ds.wav(i) for i in indices]
    B = len(indices)
    tx = max(len(s) for s in ids)
    text = torch.zeros(B, tx, dtype=torch.long)
    for b, s in enumerate(ids):
        text[b, :len(s)] = torch.tensor(s)
    text_len = torch.tensor([len(s) for s in ids])
    L = max(len(w) for w in wavs)
    audio = torch.zeros(B, L, dtype=torch.float32)
    for b, w in enumerate(wavs):
        audio[b, :len(w)] = torch.from_numpy(w)
    lens = torch.tensor([len(w) for w in wavs], dtype=torch.int32)
    mel, frames = extractor(audio.to(device), lens.to(device))
    return text.to(device), text_len.to(device), mel, frames.to(torch.long)
