"""Autoregressive inference (call stack (C)).

    dec = Decoder(model.engine, batch=32, text_len=128, t_max=800)
    mel_after, out_len = dec.run(text, text_len, max_len=800)

The encoder runs once (eval mode) and its memory is projected to K/V for all six
decoder layers by one GEMM.  The per-frame decode step -- pre-net on the previous
frame, scaled PE, 6 x [self-attention with KV-cache append, cross-attention over the
cached memory K/V, FFN, post-LN], mel/stop heads, emit -- is composed by libtt2
itself (``tt2_decode_step``; csrc/decoder.cpp) and captured ONCE as a hipGraph the
library owns (``tt2_decode_graph_create``); ``tt2_decode_graph_launch`` replays it per
frame.  The step reads the frame index from a DEVICE counter, tracks each utterance's
stop frame on the device (``stop_len``) and stops reading keys for finished utterances;
the host only polls ``stop_len`` every ``check_every`` frames.  The post-net runs once
over the whole sequence afterwards (as modeling_speecht5.py:2261-2263 does).

This module only fills the C descriptor (pointers into the engine's weights and this
decoder's buffers); every launch happens inside libtt2.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from .trace import ranged
from . import _lib, ops
from ._lib import check, dt, lib, stream_ptr
from .engine import TTSEngine

SCHEDULE_AUTO, SCHEDULE_PLAIN, SCHEDULE_SPLIT = 0, 1, 2
SCHEDULE_SPLIT_UNFUSED = 3   # split-K, the attention launches without the fused projections
SCHEDULE_SPLIT_FFN1 = 4      # split-K, each FFN sublayer in one tt2_ffn_decode launch (opt-in: slower)
STOP_FORCE = 1e4   # |injected stop logit|: dominates any logit the heads produce


def stop_logit(threshold: float | None) -> float:
    """Probability threshold -> logit (None: never stop).  sigmoid(s) >= threshold, so a
    threshold of 1 never stops (+inf) and 0 stops at the first frame (-inf)."""
    if threshold is None:
        return math.inf
    if not 0.0 <= threshold <= 1.0:
        raise ValueError(f"stop_threshold must be in [0, 1], got {threshold}")
    if threshold >= 1.0:
        return math.inf
    if threshold <= 0.0:
        return -math.inf
    return math.log(threshold / (1.0 - threshold))


class Decoder:
    def __init__(self, engine: TTSEngine, batch: int, text_len: int, t_max: int, prenet_dropout: bool = True,
                 seed: int = 0, dtype: torch.dtype | None = None, schedule: int = SCHEDULE_AUTO):
        """dtype: the decode step's storage type -- the engine's (bf16 / f32) by default, or
        torch.float16 on a bf16 engine: the step then runs on an f16 copy of
        the weights (refreshed from the f32 master at every encode()), an f16 KV cache and the
        encoder memory's K/V cast to f16; the encoder and post-net stay in the engine's dtype.
        prenet_dropout: Tacotron2's always-on pre-net dropout at inference (sites 128 / 129,
        seed `seed` + frame index); on by default, False for parity runs against a
        dropout-free reference."""
        self.e = e = engine
        c = e.cfg
        self.B, self.Tx, self.Tmax = batch, text_len, t_max
        if t_max >= c.max_len:   # a replay at the saturated counter reads PE row t_max
            raise ValueError(f"t_max {t_max} must be below the positional table's {c.max_len} rows")
        self.prenet_dropout = prenet_dropout
        self.seed0 = seed
        dev = e.dev
        cd = dtype or e.cd
        self.dd = cd
        if cd == torch.float16 and (e.cd != torch.bfloat16 or batch > 64):
            raise ValueError("f16 decode needs a bf16 engine and batch <= 64 (the skinny decode kernels)")
        # TT2_DEC_SCHEDULE (dev knob, A/B runs): overrides the default schedule
        if schedule == SCHEDULE_AUTO and os.environ.get("TT2_DEC_SCHEDULE"):
            schedule = int(os.environ["TT2_DEC_SCHEDULE"])
        self.schedule = schedule
        # steps per decode graph launch (tt2_decode_graph_create_n; TT2_DEC_GRAPH_STEPS): one
        # graph boundary per 8 frames, +0.6-1.2 % frames/s over one per frame
        self.graph_steps = int(os.environ.get("TT2_DEC_GRAPH_STEPS", "8"))
        self.A = e.arena(batch, text_len, t_max)   # encoder + post-net buffers (lazy)
        B = batch
        self.mel_seq = torch.zeros(B, t_max, c.n_mels, dtype=torch.float32, device=dev)
        self.stop_seq = torch.zeros(B, t_max, dtype=torch.float32, device=dev)
        self.stop_len = torch.full((B,), 2 ** 31 - 1, dtype=torch.int32, device=dev)
        self.stop_bias = torch.zeros(B, t_max, dtype=torch.float32, device=dev)
        self.t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = torch.zeros(1, dtype=torch.int32, device=dev)
        if cd == torch.float16:
            self.w16 = torch.zeros(e.lay.numel, dtype=torch.float16, device=dev)
            self.mkv16 = torch.zeros(B * text_len, c.n_dec * 2 * c.d_model, dtype=torch.float16, device=dev)
        self._graphs: dict[float, int] = {}
        self._desc_cache: dict[float, _lib.DecodeDesc] = {}
        self.ws = None
        self.ws = torch.empty(lib().tt2_decode_workspace_size(C.byref(self.desc(math.inf))), dtype=torch.uint8,
                              device=dev)

    # ----------------------------------------------------------------- descriptor
    def W(self, name):
        """Weight view in the decode step's dtype."""
        if self.dd == torch.float16:
            return self.e.lay.view(self.w16, name)
        return self.e.W(name)

    @property
    def mkv(self):
        """Encoder memory K/V of all decoder layers [B * Tx, 6144] in the step's dtype."""
        return self.mkv16 if self.dd == torch.float16 else self.A["mkv"]

    def desc(self, logit: float) -> _lib.DecodeDesc:
        """The tt2_decode_desc of this decoder with stop threshold `logit` (cached: the
        pointers never change after construction)."""
        d = self._desc_cache.get(logit)
        if d is not None:
            return d
        e, c = self.e, self.e.cfg
        d = _lib.DecodeDesc()
        d.batch, d.text_len, d.t_max, d.n_layers = self.B, self.Tx, self.Tmax, c.n_dec
        d.d_model, d.n_heads, d.d_ffn, d.n_mels, d.prenet_dim = c.d_model, c.n_heads, c.d_ffn, c.n_mels, c.dec_prenet
        d.dtype = dt(self.W("heads.w"))
        d.schedule = self.schedule
        d.ln_eps = c.ln_eps
        d.prenet_dropout = c.prenet_dropout if self.prenet_dropout else 0.0
        d.stop_logit = logit
        W, P = (lambda n: self.W(n).data_ptr()), (lambda n: e.P(n).data_ptr())  # noqa: E731
        d.fc1_w, d.fc1_b, d.fc2_w, d.fc2_b = W("dec.fc1.w"), P("dec.fc1.b"), W("dec.fc2.w"), P("dec.fc2.b")
        d.proj_w, d.proj_b, d.alpha, d.pe_table = W("dec.proj.w"), P("dec.proj.b"), P("dec.alpha"), e.pe.data_ptr()
        for l in range(c.n_dec):
            L, p = d.layers[l], f"dec{l}."
            for f in ("qkv", "o", "cq", "co", "ffn1", "ffn2"):
                setattr(L, f + "_w", W(p + f + ".w"))
                setattr(L, f + "_b", P(p + f + ".b"))
            for k in (1, 2, 3):
                setattr(L, f"ln{k}_g", P(p + f"ln{k}.g"))
                setattr(L, f"ln{k}_b", P(p + f"ln{k}.b"))
        d.heads_w, d.heads_b = W("heads.w"), P("heads.b")
        d.mem_kv, d.text_lens = self.mkv.data_ptr(), self.A["text_len"].data_ptr()
        d.mel_seq, d.stop_seq, d.stop_len = self.mel_seq.data_ptr(), self.stop_seq.data_ptr(), self.stop_len.data_ptr()
        d.stop_bias = self.stop_bias.data_ptr()
        d.step, d.seed = self.t.data_ptr(), self.seed.data_ptr()
        if self.ws is not None:
            d.workspace, d.ws_bytes = self.ws.data_ptr(), self.ws.numel()
            self._desc_cache[logit] = d
        return d

    def inject_stop(self, lengths: torch.Tensor | None):
        """Force each utterance's stop at frame lengths[b] - 1 by injecting stop logits
        (-STOP_FORCE before, +STOP_FORCE at the stop frame); None clears."""
        self.stop_bias.zero_()
        if lengths is None:
            return
        lengths = lengths.to(self.stop_bias.device, torch.long).clamp(1, self.Tmax)
        t = torch.arange(self.Tmax, device=self.stop_bias.device)[None, :]
        self.stop_bias.copy_(torch.where(t < lengths[:, None] - 1, -STOP_FORCE, 0.0))
        self.stop_bias.scatter_(1, (lengths - 1)[:, None], STOP_FORCE)

    # ----------------------------------------------------------------- one step
    def step(self, stop_threshold: float | None = None):
        """Launch one decode step as eager launches (libtt2 composes them)."""
        check(lib().tt2_decode_step(C.byref(self.desc(stop_logit(stop_threshold))), stream_ptr()), "tt2_decode_step")

    # ----------------------------------------------------------------- driver
    def reset(self):
        check(lib().tt2_decode_reset(C.byref(self.desc(math.inf)), self.seed0 & 0xFFFFFFFF, stream_ptr()),
              "tt2_decode_reset")

    @ranged("tt2.decode.encode")
    def encode(self, text, text_len):
        e, A = self.e, self.A
        was = e.training
        e.training = False
        A["text"].copy_(text.reshape(-1))
        A["text_len"].copy_(text_len.to(torch.int32))
        e.forward_encoder(A)
        e.training = was
        if self.dd == torch.float16:
            self.w16.copy_(e.params)
            kvld = self.mkv16.shape[1]
            ops.cast2d(A["mkv"], kvld, self.mkv16, kvld, self.mkv16.shape[0], kvld)

    def capture(self, stop_threshold: float | None = 0.5):
        """Have libtt2 capture one decode step (stop threshold baked in) as a hipGraph."""
        logit = stop_logit(stop_threshold)
        if logit not in self._graphs:
            h = C.c_void_p()
            check(lib().tt2_decode_graph_create_n(C.byref(self.desc(logit)), self.graph_steps, stream_ptr(),
                                                  C.byref(h)), "tt2_decode_graph_create_n")
            self._graphs[logit] = h.value
        return self._graphs[logit]

    def close(self):
        for h in self._graphs.values():
            lib().tt2_decode_graph_destroy(h)
        self._graphs.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown: the library may be gone
            pass

    @ranged("tt2.decode.loop")
    def decode_loop(self, n_steps: int, use_graph: bool = True, stop_threshold: float | None = None,
                    check_every: int = 32, limits: torch.Tensor | None = None) -> int:
        """Run up to n_steps frames; with stop_threshold, an utterance finishes at its first
        stop probability >= threshold (tracked on the device, its attention then reads no keys)
        or at its own frame limit (limits: [B] caps).  The loop ends once every utterance is
        done (polled every check_every frames).  Returns frames run."""
        n_steps = min(n_steps, self.Tmax)   # the cache holds t_max frames
        if limits is not None:
            limits = limits.to(device=self.stop_len.device, dtype=torch.long)
            n_steps = min(n_steps, int(limits.max()))
        graph = self.capture(stop_threshold) if use_graph else None
        L = lib()
        done = 0
        while done < n_steps:
            k = min(check_every, n_steps - done)
            if graph is not None:
                check(L.tt2_decode_graph_launch(graph, k, stream_ptr()), "tt2_decode_graph_launch")
            else:
                for _ in range(k):
                    self.step(stop_threshold)
            done += k
            if stop_threshold is not None or limits is not None:
                fin = torch.zeros(self.B, dtype=torch.bool, device=self.stop_len.device)
                if stop_threshold is not None:
                    fin |= self.stop_len <= done
                if limits is not None:
                    fin |= limits <= done
                if bool(fin.all()):
                    break
        return done

    def out_lengths(self, n_frames: int, stop_threshold: float | None, limits: torch.Tensor | None = None):
        out_len = torch.full((self.B,), n_frames, dtype=torch.long, device=self.e.dev)
        if stop_threshold is not None:
            out_len = torch.minimum(out_len, self.stop_len.long())
        if limits is not None:
            out_len = torch.minimum(out_len, limits.to(out_len.device, torch.long))
        return out_len

    @ranged("tt2.decode.postnet")
    def postnet(self, n_frames: int, stop_threshold: float | None, limits: torch.Tensor | None = None):
        e, c, A = self.e, self.e.cfg, self.A
        B, T = self.B, n_frames
        was = e.training
        e.training = False
        # the post-net sees exactly the n decoded frames (conv zero padding at n); an utterance
        # that stopped earlier has zero frames after its stop (the emit writes them), i.e. it
        # is post-processed as if zero-padded to the batch length
        Md = B * T
        before = self.mel_seq[:, :T].reshape(Md, c.n_mels).contiguous()
        ops.cast2d(before, c.n_mels, A["pin"], c.n_mels, Md, c.n_mels)
        e._postnet_fwd(A, A["pin"], before, c.n_mels, Md, T, False)
        e.training = was
        mel_after = A["mel_after"][:Md].view(B, T, c.n_mels).clone()
        return mel_after, self.out_lengths(n_frames, stop_threshold, limits)

    def run(self, text, text_len, max_len: int | None = None, stop_threshold: float | None = 0.5,
            use_graph: bool = True, limits: torch.Tensor | None = None):
        """Greedy decode; returns (mel_after [B, T, 80] f32, out_len [B]).  limits: optional
        per-utterance frame caps [B] (out_len <= limits)."""
        max_len = min(max_len or self.Tmax, self.Tmax)
        self.encode(text, text_len)
        self.reset()
        n = self.decode_loop(max_len, use_graph, stop_threshold, limits=limits)
        return self.postnet(n, stop_threshold, limits)
