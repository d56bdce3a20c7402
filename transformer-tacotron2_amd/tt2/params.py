"""Flat parameter store and the checkpoint (state_dict) mapping.

All 52.99M parameters live in ONE flat f32 buffer (and one flat f32 gradient
buffer, Adam moments, and a bf16 shadow for the bf16 kernels), each slot
16-element aligned.  The internal slot layout is chosen for the kernels:

* conv weights are [Cout][tap][Cin] (implicit-GEMM K order), not torch's
  [Cout][Cin][k];
* the six decoder layers' cross-attention K/V projection rows are contiguous
  (``dec.kv.w`` [6*1024, 512]) so the encoder memory is projected for all
  layers by ONE GEMM;
* mel_linear and stop_linear are one [81, 512] head.

``to_state_dict`` / ``load_state_dict`` convert to and from the SURVEY 8(b)
checkpoint layout (nn.MultiheadAttention-compatible keys), so the on-disk
format never changes.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from .config import TTSConfig

ALIGN = 16


def build_slots(c: TTSConfig):
    d, F, K = c.d_model, c.d_ffn, c.enc_conv_kernel
    s = []
    s.append(("enc.embed", (c.vocab, d)))
    for i in range(c.enc_conv_layers):
        s += [(f"enc.conv{i}.w", (d, K, d)), (f"enc.conv{i}.b", (d,)),
              (f"enc.bn{i}.g", (d,)), (f"enc.bn{i}.b", (d,))]
    s += [("enc.proj.w", (d, d)), ("enc.proj.b", (d,)), ("enc.alpha", (1,))]
    for l in range(c.n_enc):
        p = f"enc{l}."
        s += [(p + "qkv.w", (3 * d, d)), (p + "qkv.b", (3 * d,)), (p + "o.w", (d, d)), (p + "o.b", (d,)),
              (p + "ln1.g", (d,)), (p + "ln1.b", (d,)), (p + "ffn1.w", (F, d)), (p + "ffn1.b", (F,)),
              (p + "ffn2.w", (d, F)), (p + "ffn2.b", (d,)), (p + "ln2.g", (d,)), (p + "ln2.b", (d,))]
    s += [("dec.fc1.w", (c.dec_prenet, c.n_mels)), ("dec.fc1.b", (c.dec_prenet,)),
          ("dec.fc2.w", (c.dec_prenet, c.dec_prenet)), ("dec.fc2.b", (c.dec_prenet,)),
          ("dec.proj.w", (d, c.dec_prenet)), ("dec.proj.b", (d,)), ("dec.alpha", (1,)),
          ("dec.kv.w", (c.n_dec * 2 * d, d)), ("dec.kv.b", (c.n_dec * 2 * d,))]
    for l in range(c.n_dec):
        p = f"dec{l}."
        s += [(p + "qkv.w", (3 * d, d)), (p + "qkv.b", (3 * d,)), (p + "o.w", (d, d)), (p + "o.b", (d,)),
              (p + "ln1.g", (d,)), (p + "ln1.b", (d,)),
              (p + "cq.w", (d, d)), (p + "cq.b", (d,)), (p + "co.w", (d, d)), (p + "co.b", (d,)),
              (p + "ln2.g", (d,)), (p + "ln2.b", (d,)), (p + "ffn1.w", (F, d)), (p + "ffn1.b", (F,)),
              (p + "ffn2.w", (d, F)), (p + "ffn2.b", (d,)), (p + "ln3.g", (d,)), (p + "ln3.b", (d,))]
    s += [("heads.w", (c.n_mels + 1, d)), ("heads.b", (c.n_mels + 1,))]
    chans = postnet_channels(c)
    for i in range(c.postnet_layers):
        s += [(f"post.conv{i}.w", (chans[i + 1], c.postnet_kernel, chans[i])), (f"post.conv{i}.b", (chans[i + 1],)),
              (f"post.bn{i}.g", (chans[i + 1],)), (f"post.bn{i}.b", (chans[i + 1],))]
    return s


def postnet_channels(c: TTSConfig):
    n = c.postnet_layers
    return [c.n_mels] + [c.postnet_channels] * (n - 1) + [c.n_mels]


def bn_layers(c: TTSConfig):
    """(name, channels) of every BatchNorm (running stats live in a side buffer)."""
    out = [(f"enc.bn{i}", c.d_model) for i in range(c.enc_conv_layers)]
    chans = postnet_channels(c)
    out += [(f"post.bn{i}", chans[i + 1]) for i in range(c.postnet_layers)]
    return out


class Layout:
    """Offsets of every slot in the flat buffer."""

    def __init__(self, slots, align=ALIGN):
        self.slots = OrderedDict()
        off = 0
        for name, shape in slots:
            n = 1
            for x in shape:
                n *= x
            self.slots[name] = (off, shape, n)
            off += (n + align - 1) // align * align
        self.numel = off

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        off, shape, n = self.slots[name]
        return flat[off:off + n].view(shape)

    def offset(self, name: str) -> int:
        return self.slots[name][0]

    def n_params(self) -> int:
        return sum(n for _, _, n in self.slots.values())


def stats_layout(c: TTSConfig) -> Layout:
    slots = []
    for name, ch in bn_layers(c):
        slots += [(name + ".rm", (ch,)), (name + ".rv", (ch,))]
    return Layout(slots)


# ------------------------------------------------------------ checkpoint map
def to_state_dict(c: TTSConfig, lay: Layout, flat: torch.Tensor, st: Layout, stats: torch.Tensor,
                  nbt: dict) -> "OrderedDict[str, torch.Tensor]":
    """Internal flat buffers -> SURVEY 8(b) state_dict (CPU f32 tensors)."""
    V = lambda n: lay.view(flat, n).detach().float().cpu()  # noqa: E731
    S = lambda n: st.view(stats, n).detach().float().cpu()  # noqa: E731
    d = c.d_model
    sd = OrderedDict()
    sd["encoder.embed.weight"] = V("enc.embed").clone()
    for i in range(c.enc_conv_layers):
        p = f"encoder.prenet.convs.{i}."
        sd[p + "conv.weight"] = V(f"enc.conv{i}.w").permute(0, 2, 1).contiguous()
        sd[p + "conv.bias"] = V(f"enc.conv{i}.b").clone()
        sd[p + "bn.weight"] = V(f"enc.bn{i}.g").clone()
        sd[p + "bn.bias"] = V(f"enc.bn{i}.b").clone()
        sd[p + "bn.running_mean"] = S(f"enc.bn{i}.rm").clone()
        sd[p + "bn.running_var"] = S(f"enc.bn{i}.rv").clone()
        sd[p + "bn.num_batches_tracked"] = torch.tensor(nbt.get(f"enc.bn{i}", 0), dtype=torch.long)
    sd["encoder.prenet.proj.weight"] = V("enc.proj.w").clone()
    sd["encoder.prenet.proj.bias"] = V("enc.proj.b").clone()
    sd["encoder.pos.alpha"] = V("enc.alpha").reshape(()).clone()
    for l in range(c.n_enc):
        p, q = f"encoder.layers.{l}.", f"enc{l}."
        sd[p + "self_attn.in_proj_weight"] = V(q + "qkv.w").clone()
        sd[p + "self_attn.in_proj_bias"] = V(q + "qkv.b").clone()
        sd[p + "self_attn.out_proj.weight"] = V(q + "o.w").clone()
        sd[p + "self_attn.out_proj.bias"] = V(q + "o.b").clone()
        sd[p + "norm1.weight"], sd[p + "norm1.bias"] = V(q + "ln1.g").clone(), V(q + "ln1.b").clone()
        sd[p + "ffn.w1.weight"], sd[p + "ffn.w1.bias"] = V(q + "ffn1.w").clone(), V(q + "ffn1.b").clone()
        sd[p + "ffn.w2.weight"], sd[p + "ffn.w2.bias"] = V(q + "ffn2.w").clone(), V(q + "ffn2.b").clone()
        sd[p + "norm2.weight"], sd[p + "norm2.bias"] = V(q + "ln2.g").clone(), V(q + "ln2.b").clone()
    for n in ("fc1", "fc2", "proj"):
        sd[f"decoder.prenet.{n}.weight"] = V(f"dec.{n}.w").clone()
        sd[f"decoder.prenet.{n}.bias"] = V(f"dec.{n}.b").clone()
    sd["decoder.pos.alpha"] = V("dec.alpha").reshape(()).clone()
    kvw, kvb = V("dec.kv.w"), V("dec.kv.b")
    for l in range(c.n_dec):
        p, q = f"decoder.layers.{l}.", f"dec{l}."
        sd[p + "self_attn.in_proj_weight"] = V(q + "qkv.w").clone()
        sd[p + "self_attn.in_proj_bias"] = V(q + "qkv.b").clone()
        sd[p + "self_attn.out_proj.weight"] = V(q + "o.w").clone()
        sd[p + "self_attn.out_proj.bias"] = V(q + "o.b").clone()
        sd[p + "cross_attn.in_proj_weight"] = torch.cat([V(q + "cq.w"), kvw[2 * d * l:2 * d * (l + 1)]], 0)
        sd[p + "cross_attn.in_proj_bias"] = torch.cat([V(q + "cq.b"), kvb[2 * d * l:2 * d * (l + 1)]], 0)
        sd[p + "cross_attn.out_proj.weight"] = V(q + "co.w").clone()
        sd[p + "cross_attn.out_proj.bias"] = V(q + "co.b").clone()
        for k in (1, 2, 3):
            sd[p + f"norm{k}.weight"] = V(q + f"ln{k}.g").clone()
            sd[p + f"norm{k}.bias"] = V(q + f"ln{k}.b").clone()
        sd[p + "ffn.w1.weight"], sd[p + "ffn.w1.bias"] = V(q + "ffn1.w").clone(), V(q + "ffn1.b").clone()
        sd[p + "ffn.w2.weight"], sd[p + "ffn.w2.bias"] = V(q + "ffn2.w").clone(), V(q + "ffn2.b").clone()
    hw, hb = V("heads.w"), V("heads.b")
    sd["mel_linear.weight"], sd["mel_linear.bias"] = hw[:c.n_mels].clone(), hb[:c.n_mels].clone()
    sd["stop_linear.weight"], sd["stop_linear.bias"] = hw[c.n_mels:].clone(), hb[c.n_mels:].clone()
    for i in range(c.postnet_layers):
        p = f"postnet.convs.{i}."
        sd[p + "conv.weight"] = V(f"post.conv{i}.w").permute(0, 2, 1).contiguous()
        sd[p + "conv.bias"] = V(f"post.conv{i}.b").clone()
        sd[p + "bn.weight"] = V(f"post.bn{i}.g").clone()
        sd[p + "bn.bias"] = V(f"post.bn{i}.b").clone()
        sd[p + "bn.running_mean"] = S(f"post.bn{i}.rm").clone()
        sd[p + "bn.running_var"] = S(f"post.bn{i}.rv").clone()
        sd[p + "bn.num_batches_tracked"] = torch.tensor(nbt.get(f"post.bn{i}", 0), dtype=torch.long)
    return sd


def from_state_dict(c: TTSConfig, sd) -> tuple[dict, dict, dict]:
    """SURVEY 8(b) state_dict -> ({slot: tensor}, {stat slot: tensor}, num_batches_tracked)."""
    d = c.d_model
    P, S, nbt = {}, {}, {}
    g = lambda k: sd[k].detach().float().cpu()  # noqa: E731
    P["enc.embed"] = g("encoder.embed.weight")
    for i in range(c.enc_conv_layers):
        p = f"encoder.prenet.convs.{i}."
        P[f"enc.conv{i}.w"] = g(p + "conv.weight").permute(0, 2, 1).contiguous()
        P[f"enc.conv{i}.b"] = g(p + "conv.bias")
        P[f"enc.bn{i}.g"], P[f"enc.bn{i}.b"] = g(p + "bn.weight"), g(p + "bn.bias")
        S[f"enc.bn{i}.rm"], S[f"enc.bn{i}.rv"] = g(p + "bn.running_mean"), g(p + "bn.running_var")
        nbt[f"enc.bn{i}"] = int(sd[p + "bn.num_batches_tracked"])
    P["enc.proj.w"], P["enc.proj.b"] = g("encoder.prenet.proj.weight"), g("encoder.prenet.proj.bias")
    P["enc.alpha"] = g("encoder.pos.alpha").reshape(1)
    for l in range(c.n_enc):
        p, q = f"encoder.layers.{l}.", f"enc{l}."
        P[q + "qkv.w"], P[q + "qkv.b"] = g(p + "self_attn.in_proj_weight"), g(p + "self_attn.in_proj_bias")
        P[q + "o.w"], P[q + "o.b"] = g(p + "self_attn.out_proj.weight"), g(p + "self_attn.out_proj.bias")
        P[q + "ln1.g"], P[q + "ln1.b"] = g(p + "norm1.weight"), g(p + "norm1.bias")
        P[q + "ffn1.w"], P[q + "ffn1.b"] = g(p + "ffn.w1.weight"), g(p + "ffn.w1.bias")
        P[q + "ffn2.w"], P[q + "ffn2.b"] = g(p + "ffn.w2.weight"), g(p + "ffn.w2.bias")
        P[q + "ln2.g"], P[q + "ln2.b"] = g(p + "norm2.weight"), g(p + "norm2.bias")
    for n in ("fc1", "fc2", "proj"):
        P[f"dec.{n}.w"], P[f"dec.{n}.b"] = g(f"decoder.prenet.{n}.weight"), g(f"decoder.prenet.{n}.bias")
    P["dec.alpha"] = g("decoder.pos.alpha").reshape(1)
    kvw, kvb = [], []
    for l in range(c.n_dec):
        p, q = f"decoder.layers.{l}.", f"dec{l}."
        P[q + "qkv.w"], P[q + "qkv.b"] = g(p + "self_attn.in_proj_weight"), g(p + "self_attn.in_proj_bias")
        P[q + "o.w"], P[q + "o.b"] = g(p + "self_attn.out_proj.weight"), g(p + "self_attn.out_proj.bias")
        cw, cb = g(p + "cross_attn.in_proj_weight"), g(p + "cross_attn.in_proj_bias")
        P[q + "cq.w"], P[q + "cq.b"] = cw[:d], cb[:d]
        kvw.append(cw[d:])
        kvb.append(cb[d:])
        P[q + "co.w"], P[q + "co.b"] = g(p + "cross_attn.out_proj.weight"), g(p + "cross_attn.out_proj.bias")
        for k in (1, 2, 3):
            P[q + f"ln{k}.g"], P[q + f"ln{k}.b"] = g(p + f"norm{k}.weight"), g(p + f"norm{k}.bias")
        P[q + "ffn1.w"], P[q + "ffn1.b"] = g(p + "ffn.w1.weight"), g(p + "ffn.w1.bias")
        P[q + "ffn2.w"], P[q + "ffn2.b"] = g(p + "ffn.w2.weight"), g(p + "ffn.w2.bias")
    P["dec.kv.w"], P["dec.kv.b"] = torch.cat(kvw, 0), torch.cat(kvb, 0)
    P["heads.w"] = torch.cat([g("mel_linear.weight"), g("stop_linear.weight")], 0)
    P["heads.b"] = torch.cat([g("mel_linear.bias"), g("stop_linear.bias")], 0)
    for i in range(c.postnet_layers):
        p = f"postnet.convs.{i}."
        P[f"post.conv{i}.w"] = g(p + "conv.weight").permute(0, 2, 1).contiguous()
        P[f"post.conv{i}.b"] = g(p + "conv.bias")
        P[f"post.bn{i}.g"], P[f"post.bn{i}.b"] = g(p + "bn.weight"), g(p + "bn.bias")
        S[f"post.bn{i}.rm"], S[f"post.bn{i}.rv"] = g(p + "bn.running_mean"), g(p + "bn.running_var")
        nbt[f"post.bn{i}"] = int(sd[p + "bn.num_batches_tracked"])
    return P, S, nbt


def grads_to_state_dict_names(c: TTSConfig, lay: Layout, gflat: torch.Tensor):
    """Gradient buffer in checkpoint naming (for parity tests vs autograd)."""
    zeros = torch.zeros(stats_layout(c).numel)
    sd = to_state_dict(c, lay, gflat, stats_layout(c), zeros, {})
    return {k: v for k, v in sd.items() if "running_" not in k and "num_batches" not in k}
