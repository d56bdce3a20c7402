"""CPU oracle for the Transformer-TTS mel path -- TEST INFRASTRUCTURE ONLY.

This file is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped GPU path (``transformer-tacotron2_amd/tt2``) never imports,
links or falls back to anything in ``oracle/``.

What it restates
----------------
The reference (keonlee9420/Transformer-tacotron2, ``/root/reference``) ships no
code: ``README.md:1-3`` names "transformer + Tacotron2" and the paper *Neural
Speech Synthesis with Transformer Network* (Li et al., AAAI 2019).  SURVEY.md
section 8(a)/(b) turns that into a concrete spec, and this module is a plain
PyTorch (fp32, CPU) statement of it:

* encoder pre-net: embedding -> 3 x [Conv1d(k5) + BatchNorm + ReLU + dropout]
  -> Linear -> scaled positional encoding (``x + alpha * PE``) -> dropout
  (PE follows transformers ``modeling_speecht5.py:400-422``)
* 6 post-LN encoder layers: fused-QKV self-attention with key-padding mask,
  position-wise FFN (ReLU) (rows a3, a4)
* decoder pre-net: 80 -> 256 -> 256 (ReLU + dropout 0.5, Tacotron2 style,
  ``modeling_speecht5.py:648-697``) -> Linear(256, 512) -> scaled PE (row a5)
* 6 post-LN decoder layers: causal + padded self-attention, cross-attention
  over the encoder memory, FFN (rows a6, a7)
* mel (80) + stop (1) linear heads (row a8, ``modeling_speecht5.py:745-756``)
* 5-layer Conv1d(k5) + BatchNorm (+tanh) post-net with residual (row a9,
  ``modeling_speecht5.py:700-737,758-762``; this spec keeps the conv bias)
* loss: masked MSE(before) + masked MSE(after) + BCE(stop, pos_weight 5)
  (row a10; stop labels as ``modeling_speecht5.py:1822-1826``)

Deterministic dropout
---------------------
Every dropout site draws its keep-mask from a counter hash of
(seed, site, flat element index) -- ``dropout_keep`` below -- which the HIP
kernels evaluate bit-identically.  That lets GPU-vs-oracle parity run with
dropout ON.

Parity status: the reference has no code, fixtures or known-answer tests, so
parity against keonlee9420's implementation is UNPINNED.  The sub-blocks are
pinned against torch stock modules and transformers SpeechT5 blocks in
``tests/test_oracle.py`` and ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------
# configuration (SURVEY 8 defaults)
# ----------------------------------------------------------------------------
@dataclass
class OracleConfig:
    vocab: int = 80
    d_model: int = 512
    n_heads: int = 8
    d_ffn: int = 2048
    n_enc: int = 6
    n_dec: int = 6
    n_mels: int = 80
    enc_conv_layers: int = 3
    enc_conv_kernel: int = 5
    dec_prenet: int = 256
    postnet_channels: int = 512
    postnet_layers: int = 5
    postnet_kernel: int = 5
    dropout: float = 0.1          # residual / FFN / PE dropout
    prenet_dropout: float = 0.5   # encoder conv + decoder prenet dropout
    postnet_dropout: float = 0.5
    stop_pos_weight: float = 5.0
    max_len: int = 4096
    bn_momentum: float = 0.1
    bn_eps: float = 1e-5
    ln_eps: float = 1e-5


# ----------------------------------------------------------------------------
# dropout sites & hash (shared spec with csrc/tt2_common.h::drop_keep)
# ----------------------------------------------------------------------------
SITE_ENC_CONV = 1        # + i, i < 3
SITE_ENC_PE = 4
SITE_ENC_LAYER = 16      # + 4*l + {0: attn residual, 1: ffn hidden, 2: ffn out}
SITE_DEC_FC1 = 64
SITE_DEC_FC2 = 65
SITE_DEC_PE = 66
SITE_DEC_LAYER = 80      # + 4*l + {0: self residual, 1: cross residual, 2: ffn hidden, 3: ffn out}
SITE_POSTNET = 112       # + i, i < 5
SITE_INFER_FC1 = 128
SITE_INFER_FC2 = 129

_M32 = np.uint64(0xFFFFFFFF)


def drop_threshold(p: float) -> int:
    return int(p * 4294967296.0) if p > 0 else 0


def dropout_keep(seed: int, site: int, n: int, p: float, offset: int = 0) -> np.ndarray:
    """Keep-mask (bool[n]) for flat indices offset..offset+n-1.

    uint32 hash of the element pair j = idx >> 1: x = j*0x9E3779B1 + seed*0x85EBCA77 +
    site*0xC2B2AE3D, then the murmur3-style finaliser; element idx takes the low 16 bits
    (even idx) or the high 16 bits (odd idx) and is kept iff they are >= floor(p * 2^16)
    (= floor(p * 2^32) >> 16).  Restates csrc/tt2_common.h drop_keep / drop_bits8.
    """
    with np.errstate(over="ignore"):
        idx = np.arange(offset, offset + n, dtype=np.uint64)
        x = ((idx >> np.uint64(1)) * np.uint64(0x9E3779B1) + np.uint64((seed * 0x85EBCA77) & 0xFFFFFFFF)
             + np.uint64((site * 0xC2B2AE3D) & 0xFFFFFFFF)) & _M32
        x ^= x >> np.uint64(16)
        x = (x * np.uint64(0x7FEB352D)) & _M32
        x ^= x >> np.uint64(15)
        x = (x * np.uint64(0x846CA68B)) & _M32
        x ^= x >> np.uint64(16)
        half = np.where((idx & np.uint64(1)) == 1, x >> np.uint64(16), x & np.uint64(0xFFFF))
    return half >= np.uint64(drop_threshold(p) >> 16)


class HashDropout(nn.Module):
    """Dropout whose mask is dropout_keep(seed, site, numel); active when
    ``self.training`` (or ``always``) and the owning model has a seed set."""

    def __init__(self, p: float, site: int, always: bool = False):
        super().__init__()
        self.p, self.site, self.always = p, site, always
        self.seed: int | None = None

    def forward(self, x):
        if self.p <= 0 or self.seed is None or not (self.training or self.always):
            return x
        keep = dropout_keep(self.seed, self.site, x.numel(), self.p)
        keep = torch.from_numpy(keep).reshape(x.shape).to(x.dtype)
        return x * keep * (1.0 / (1.0 - self.p))


# ----------------------------------------------------------------------------
# blocks
# ----------------------------------------------------------------------------
def sinusoid_table(max_len: int, dim: int) -> torch.Tensor:
    """PE table exactly as transformers modeling_speecht5.py:404-409."""
    pe = torch.zeros(max_len, dim)
    position = torch.arange(0, max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, dim, 2, dtype=torch.int64).float() * -(math.log(10000.0) / dim))
    pe[:, 0::2] = torch.sin(position.float() * div_term)
    pe[:, 1::2] = torch.cos(position.float() * div_term)
    return pe


class ScaledPositionalEncoding(nn.Module):
    """x + alpha * PE[:T], alpha init 1.0 (modeling_speecht5.py:399-422)."""

    def __init__(self, dim: int, max_len: int):
        super().__init__()
        self.register_buffer("pe", sinusoid_table(max_len, dim), persistent=False)
        self.alpha = nn.Parameter(torch.tensor(1.0))

    def forward(self, x):
        return x + self.alpha * self.pe[: x.size(1)]


class MHA(nn.Module):
    """Multi-head attention with nn.MultiheadAttention's parameter names
    (in_proj_weight [3d, d], in_proj_bias, out_proj).  Masked logits get
    probability exactly 0; a fully masked row outputs 0."""

    def __init__(self, d: int, h: int):
        super().__init__()
        self.d, self.h = d, h
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, q_in, kv_in, key_len=None, causal=False):
        B, Tq, d = q_in.shape
        Tk = kv_in.size(1)
        h, dh = self.h, d // self.h
        W, b = self.in_proj_weight, self.in_proj_bias
        q = F.linear(q_in, W[:d], b[:d])
        k = F.linear(kv_in, W[d:2 * d], b[d:2 * d])
        v = F.linear(kv_in, W[2 * d:], b[2 * d:])
        q = q.view(B, Tq, h, dh).transpose(1, 2)
        k = k.view(B, Tk, h, dh).transpose(1, 2)
        v = v.view(B, Tk, h, dh).transpose(1, 2)
        # scores and softmax in f32 (a no-op for the f32 oracle; under torch.autocast it mirrors
        # AMP's f32 softmax, so the autocast oracle is a standard bf16 mixed-precision reference)
        s = (q @ k.transpose(-1, -2)).to(torch.promote_types(q.dtype, torch.float32)) / math.sqrt(dh)
        allowed = torch.ones(B, 1, Tq, Tk, dtype=torch.bool)
        if key_len is not None:
            allowed = allowed & (torch.arange(Tk)[None, None, None, :] < key_len.view(B, 1, 1, 1))
        if causal:
            allowed = allowed & torch.ones(Tq, Tk, dtype=torch.bool).tril()[None, None]
        s = s.masked_fill(~allowed, float("-inf"))
        mx = s.amax(-1, keepdim=True)
        mx = torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))
        e = torch.exp(s - mx) * allowed
        den = e.sum(-1, keepdim=True)
        p = e / torch.where(den > 0, den, torch.ones_like(den))
        o = (p @ v).transpose(1, 2).reshape(B, Tq, d)
        return self.out_proj(o), p


class FFN(nn.Module):
    def __init__(self, d: int, f: int, p: float, site: int):
        super().__init__()
        self.w1 = nn.Linear(d, f)
        self.w2 = nn.Linear(f, d)
        self.drop = HashDropout(p, site)

    def forward(self, x):
        return self.w2(self.drop(F.relu(self.w1(x))))


class ConvBN(nn.Module):
    """Conv1d(k, pad (k-1)/2, bias) + BatchNorm1d on channels-last input.

    ``ConvBN.stats_f64`` (class-wide, off by default) is a conditioning probe for the tests,
    not a model option: the training-mode normalisation is then evaluated in float64 from
    the f32 conv output and rounded back, i.e. the same model with the BatchNorm's
    reductions rounded differently.  How far a gradient moves under it measures that
    gradient's own sensitivity to BatchNorm rounding (tests/test_gpu_fullsize.py)."""
    stats_f64 = False

    def __init__(self, cin: int, cout: int, k: int, momentum: float, eps: float):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, padding=(k - 1) // 2)
        self.bn = nn.BatchNorm1d(cout, momentum=momentum, eps=eps)

    def forward(self, x):  # x [B, T, C]
        y = self.conv(x.transpose(1, 2))
        if self.stats_f64 and self.training and y.dtype == torch.float32:
            bn = self.bn
            with torch.no_grad():
                bn(y)                       # running statistics exactly as the plain path
            z = F.batch_norm(y.double(), None, None, bn.weight.double(), bn.bias.double(), True, 0.0, bn.eps)
            return z.float().transpose(1, 2)
        return self.bn(y).transpose(1, 2)


class EncoderPrenet(nn.Module):
    def __init__(self, c: OracleConfig):
        super().__init__()
        self.convs = nn.ModuleList(
            [ConvBN(c.d_model, c.d_model, c.enc_conv_kernel, c.bn_momentum, c.bn_eps) for _ in range(c.enc_conv_layers)])
        self.drops = nn.ModuleList([HashDropout(c.prenet_dropout, SITE_ENC_CONV + i) for i in range(c.enc_conv_layers)])
        self.proj = nn.Linear(c.d_model, c.d_model)

    def forward(self, x):
        for conv, drop in zip(self.convs, self.drops):
            x = drop(F.relu(conv(x)))
        return self.proj(x)


class EncoderLayer(nn.Module):
    def __init__(self, c: OracleConfig, l: int):
        super().__init__()
        self.self_attn = MHA(c.d_model, c.n_heads)
        self.norm1 = nn.LayerNorm(c.d_model, eps=c.ln_eps)
        self.ffn = FFN(c.d_model, c.d_ffn, c.dropout, SITE_ENC_LAYER + 4 * l + 1)
        self.norm2 = nn.LayerNorm(c.d_model, eps=c.ln_eps)
        self.drop1 = HashDropout(c.dropout, SITE_ENC_LAYER + 4 * l + 0)
        self.drop2 = HashDropout(c.dropout, SITE_ENC_LAYER + 4 * l + 2)

    def forward(self, x, text_len):
        a, p = self.self_attn(x, x, key_len=text_len)
        x = self.norm1(x + self.drop1(a))
        x = self.norm2(x + self.drop2(self.ffn(x)))
        return x, p


class Encoder(nn.Module):
    def __init__(self, c: OracleConfig):
        super().__init__()
        self.embed = nn.Embedding(c.vocab, c.d_model, padding_idx=0)
        self.prenet = EncoderPrenet(c)
        self.pos = ScaledPositionalEncoding(c.d_model, c.max_len)
        self.pos_drop = HashDropout(c.dropout, SITE_ENC_PE)
        self.layers = nn.ModuleList([EncoderLayer(c, l) for l in range(c.n_enc)])

    def forward(self, text, text_len):
        x = self.pos_drop(self.pos(self.prenet(self.embed(text))))
        attn = []
        for layer in self.layers:
            x, p = layer(x, text_len)
            attn.append(p)
        return x, attn


class DecoderPrenet(nn.Module):
    def __init__(self, c: OracleConfig):
        super().__init__()
        self.fc1 = nn.Linear(c.n_mels, c.dec_prenet)
        self.fc2 = nn.Linear(c.dec_prenet, c.dec_prenet)
        self.proj = nn.Linear(c.dec_prenet, c.d_model)
        self.drop1 = HashDropout(c.prenet_dropout, SITE_DEC_FC1)
        self.drop2 = HashDropout(c.prenet_dropout, SITE_DEC_FC2)

    def forward(self, x):
        x = self.drop1(F.relu(self.fc1(x)))
        x = self.drop2(F.relu(self.fc2(x)))
        return self.proj(x)


class DecoderLayer(nn.Module):
    def __init__(self, c: OracleConfig, l: int):
        super().__init__()
        base = SITE_DEC_LAYER + 4 * l
        self.self_attn = MHA(c.d_model, c.n_heads)
        self.cross_attn = MHA(c.d_model, c.n_heads)
        self.norm1 = nn.LayerNorm(c.d_model, eps=c.ln_eps)
        self.norm2 = nn.LayerNorm(c.d_model, eps=c.ln_eps)
        self.norm3 = nn.LayerNorm(c.d_model, eps=c.ln_eps)
        self.ffn = FFN(c.d_model, c.d_ffn, c.dropout, base + 2)
        self.drop1 = HashDropout(c.dropout, base + 0)
        self.drop2 = HashDropout(c.dropout, base + 1)
        self.drop3 = HashDropout(c.dropout, base + 3)

    def forward(self, x, mem, text_len, mel_len):
        a, ps = self.self_attn(x, x, key_len=mel_len, causal=True)
        x = self.norm1(x + self.drop1(a))
        a, pc = self.cross_attn(x, mem, key_len=text_len)
        x = self.norm2(x + self.drop2(a))
        x = self.norm3(x + self.drop3(self.ffn(x)))
        return x, ps, pc


class Decoder(nn.Module):
    def __init__(self, c: OracleConfig):
        super().__init__()
        self.prenet = DecoderPrenet(c)
        self.pos = ScaledPositionalEncoding(c.d_model, c.max_len)
        self.pos_drop = HashDropout(c.dropout, SITE_DEC_PE)
        self.layers = nn.ModuleList([DecoderLayer(c, l) for l in range(c.n_dec)])

    def forward(self, dec_in, mem, text_len, mel_len, prenet_out=None):
        x = self.pos_drop(self.pos(self.prenet(dec_in) if prenet_out is None else prenet_out))
        ps, pc = [], []
        for layer in self.layers:
            x, a, b = layer(x, mem, text_len, mel_len)
            ps.append(a)
            pc.append(b)
        return x, ps, pc


class Postnet(nn.Module):
    def __init__(self, c: OracleConfig):
        super().__init__()
        n = c.postnet_layers
        chans = [c.n_mels] + [c.postnet_channels] * (n - 1) + [c.n_mels]
        self.convs = nn.ModuleList(
            [ConvBN(chans[i], chans[i + 1], c.postnet_kernel, c.bn_momentum, c.bn_eps) for i in range(n)])
        self.drops = nn.ModuleList([HashDropout(c.postnet_dropout, SITE_POSTNET + i) for i in range(n)])

    def forward(self, x):
        y = x
        n = len(self.convs)
        for i, (conv, drop) in enumerate(zip(self.convs, self.drops)):
            y = conv(y)
            if i < n - 1:
                y = torch.tanh(y)
            y = drop(y)
        return x + y


class TransformerTTSOracle(nn.Module):
    """state_dict keys == SURVEY 8(b) checkpoint layout."""

    def __init__(self, cfg: OracleConfig | None = None):
        super().__init__()
        self.cfg = c = cfg or OracleConfig()
        self.encoder = Encoder(c)
        self.decoder = Decoder(c)
        self.mel_linear = nn.Linear(c.d_model, c.n_mels)
        self.stop_linear = nn.Linear(c.d_model, 1)
        self.postnet = Postnet(c)
        self.seed: int | None = None

    def set_seed(self, seed: int | None):
        """Enable hash dropout with this per-step seed (None disables it)."""
        self.seed = seed
        for m in self.modules():
            if isinstance(m, HashDropout):
                m.seed = seed

    @staticmethod
    def shift_right(mel):
        return torch.cat([torch.zeros_like(mel[:, :1]), mel[:, :-1]], dim=1)

    def forward(self, text, text_len, mel, mel_len, return_attn=False):
        mem, ea = self.encoder(text, text_len)
        x, ps, pc = self.decoder(self.shift_right(mel), mem, text_len, mel_len)
        mel_before = self.mel_linear(x)
        stop = self.stop_linear(x).squeeze(-1)
        mel_after = self.postnet(mel_before)
        attn = {"enc": ea, "dec_self": ps, "dec_cross": pc} if return_attn else None
        return mel_before, mel_after, stop, attn

    def loss(self, outputs, mel, mel_len):
        return tts_loss(outputs[0], outputs[1], outputs[2], mel, mel_len, self.cfg.stop_pos_weight)

    def infer_prenet(self, frames, seed0: int):
        """Decoder pre-net at inference with Tacotron2's always-on dropout (sites 128 / 129):
        frame j of the prefix (the input of decode step j) draws its masks with seed
        seed0 + j over the flat [B, 256] index, as the GPU decode step does."""
        c, pn = self.cfg, self.decoder.prenet
        B, T, _ = frames.shape
        p = c.prenet_dropout
        keep = lambda site, j: torch.from_numpy(  # noqa: E731
            dropout_keep(seed0 + j, site, B * c.dec_prenet, p)).reshape(B, c.dec_prenet).float() / (1.0 - p)
        outs = []
        for j in range(T):
            h = F.relu(pn.fc1(frames[:, j])) * keep(SITE_INFER_FC1, j)
            h = F.relu(pn.fc2(h)) * keep(SITE_INFER_FC2, j)
            outs.append(pn.proj(h))
        return torch.stack(outs, 1)

    @torch.no_grad()
    def infer(self, text, text_len, max_len: int, stop_threshold: float = 0.5, force_len: bool = False,
              prenet_dropout_seed: int | None = None, stop_bias=None):
        """Greedy AR decode (loop shape of modeling_speecht5.py:2215-2267),
        recomputing the full prefix each step.  Returns (mel_after, out_len,
        mel_before, stop_logits).  prenet_dropout_seed: Tacotron2's always-on pre-net
        dropout (see infer_prenet); stop_bias [B, max_len]: added to the stop logits
        (per-utterance length injection).  An utterance's out_len is its
        first frame with sigmoid(stop) >= threshold, + 1."""
        B = text.size(0)
        c = self.cfg
        mem, _ = self.encoder(text, text_len)
        frames = torch.zeros(B, 1, c.n_mels)
        befores, stops = [], []
        out_len = torch.full((B,), max_len, dtype=torch.long)
        done = torch.zeros(B, dtype=torch.bool)
        full_len = torch.full((B,), max_len, dtype=torch.long)
        for t in range(max_len):
            pre = None if prenet_dropout_seed is None else self.infer_prenet(frames, prenet_dropout_seed)
            x, _, _ = self.decoder(frames, mem, text_len, full_len, prenet_out=pre)
            last = x[:, -1]
            f = self.mel_linear(last)
            s = self.stop_linear(last).squeeze(-1)
            if stop_bias is not None:
                s = s + stop_bias[:, t]
            befores.append(f)
            stops.append(s)
            frames = torch.cat([frames, f[:, None]], dim=1)
            if not force_len:
                hit = (torch.sigmoid(s) >= stop_threshold) & ~done
                out_len[hit] = t + 1
                done |= hit
                if bool(done.all()):
                    break
        mel_before = torch.stack(befores, 1)
        mel_after = self.postnet(mel_before)
        return mel_after, out_len, mel_before, torch.stack(stops, 1)


def tts_loss(mel_before, mel_after, stop, mel, mel_len, pos_weight=5.0):
    """Masked MSE(before) + MSE(after) + BCE(stop, pos_weight); stop label is 1
    at the last valid frame (modeling_speecht5.py:1822-1826)."""
    B, T, M = mel.shape
    valid = torch.arange(T)[None, :] < mel_len[:, None]
    n = valid.sum().clamp(min=1)
    vm = valid[..., None].to(mel.dtype)
    l_before = (((mel_before - mel) ** 2) * vm).sum() / (n * M)
    l_after = (((mel_after - mel) ** 2) * vm).sum() / (n * M)
    label = (torch.arange(T)[None, :] == (mel_len[:, None] - 1)).to(stop.dtype)
    bce = F.binary_cross_entropy_with_logits(stop, label, reduction="none",
                                             pos_weight=torch.tensor(pos_weight, dtype=stop.dtype))
    l_stop = (bce * valid).sum() / n
    total = l_before + l_after + l_stop
    return total, {"mel_before": l_before, "mel_after": l_after, "stop": l_stop}


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def init_deterministic(model: TransformerTTSOracle, seed: int = 0):
    """Seeded init used by tests/bench so oracle and GPU model share weights."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("alpha"):
                p.fill_(1.0)
            elif p.dim() == 1:
                if ".norm" in name or ".bn." in name:
                    p.copy_((1.0 if name.endswith("weight") else 0.0) + 0.05 * torch.randn(p.shape, generator=g))
                else:
                    p.copy_(0.02 * torch.randn(p.shape, generator=g))
            else:
                fan_in = p[0].numel()
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(fan_in))
        model.encoder.embed.weight[0].zero_()
    return model
