"""Autoregressive inference (call stack (C)).

    dec = Decoder(model.engine, batch=32, text_len=128, t_max=800)
    mel_after, out_len = dec.run(text, text_len, max_len=800)

The encoder runs once (eval mode) and its memory is projected to K/V for all
six decoder layers by one GEMM.  The per-frame decode step -- pre-net on the
previous frame, scaled PE, 6 x [self-attention with KV-cache append, cross-
attention over the cached memory K/V, FFN, post-LN], mel/stop heads, emit --
reads the step index from a DEVICE counter, so it is captured ONCE as a
hipGraph (torch.cuda.CUDAGraph records the libtt2 launches) and replayed per
frame; the host only polls the stop flags every ``check_every`` frames.  The
post-net runs once over the whole sequence afterwards (as
modeling_speecht5.py:2261-2263 does).
"""
from __future__ import annotations

import math

import torch

from . import ops
from ._lib import ACT_RELU
from .config import SITE_INFER_FC1, SITE_INFER_FC2
from .engine import TTSEngine
from .ops import NO_DROP, Drop


class _Slab:
    """Fixed buffer for the split-K partial slabs (a Workspace stand-in that never grows,
    so the captured graph keeps its pointer)."""

    def __init__(self, t: torch.Tensor):
        self.t = t

    def get(self, nbytes: int) -> torch.Tensor:
        if nbytes > self.t.numel() * 4:
            raise ValueError(f"decode slab too small: {nbytes} bytes")
        return self.t


class Decoder:
    def __init__(self, engine: TTSEngine, batch: int, text_len: int, t_max: int, prenet_dropout: bool = False,
                 seed: int = 0, dtype: torch.dtype | None = None):
        """dtype: the decode step's storage type -- the engine's (bf16 / f32) by default, or
        torch.float16 on a bf16 engine: the step then runs on an f16 copy of
        the weights (refreshed from the f32 master at every encode()), an f16 KV cache and the
        encoder memory's K/V cast to f16; the encoder and post-net stay in the engine's dtype."""
        self.e = e = engine
        c = e.cfg
        self.B, self.Tx, self.Tmax = batch, text_len, t_max
        if t_max > c.max_len:
            raise ValueError(f"t_max {t_max} exceeds the positional table ({c.max_len})")
        self.prenet_dropout = prenet_dropout
        self.seed0 = seed
        dev = e.dev
        cd = dtype or e.cd
        self.dd = cd
        if cd == torch.float16 and (e.cd != torch.bfloat16 or batch > 64):
            raise ValueError("f16 decode needs a bf16 engine and batch <= 64 (the skinny decode kernels)")
        d, F = c.d_model, c.d_ffn
        B = batch
        self.A = e.arena(batch, text_len, t_max)   # encoder + post-net buffers (lazy)
        z = lambda *s, dt=cd: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self.prev = z(B, c.n_mels)
        self.p1, self.p2 = z(B, c.dec_prenet), z(B, c.dec_prenet)
        self.proj, self.x0 = z(B, d), z(B, d)
        self.xa, self.xb = z(B, d), z(B, d)
        self.qkv = z(B, 3 * d)
        self.att, self.o, self.h1, self.cq, self.catt, self.co, self.h2 = (z(B, d) for _ in range(7))
        self.f1, self.f2 = z(B, F), z(B, d)
        self.cache = z(c.n_dec, B, t_max, 2 * d)           # per layer [B][t_max][K | V]
        self.heads = z(B, 96, dt=torch.float32)
        self.mel_seq = z(B, t_max, c.n_mels, dt=torch.float32)
        self.stop_seq = z(B, t_max, dt=torch.float32)
        self.t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = torch.zeros(1, dtype=torch.int32, device=dev)
        self.emit_done = torch.zeros(1, dtype=torch.int32, device=dev)   # heads-GEMM arrival counter
        # bf16: the scaled PE rides in the pre-net projection's epilogue and the frame emit
        # in the heads GEMM's (skinny-path epilogues; 2 launches fewer per step)
        half = cd in (torch.bfloat16, torch.float16)
        self.fused_io = half and batch <= 64
        self.graph = None
        # bf16 decode-step schedules: 0 no fusion, 1 KV-cache scatter in the QKV epilogue,
        # 2 also the LayerNorms as GEMM prologues (every workgroup recomputes the 32-row
        # statistics), 3 (default) KV scatter + split-K o / co / ffn2 whose slabs a
        # residual + LayerNorm combine kernel folds (tools/decode_ab.py measures them).
        # The skinny-path fusions need batch <= 64 (the LN prologues <= 32); larger batches
        # run unfused.
        self.fuse = 3 if half and batch <= 64 else 0
        self.split_o, self.split_f = 4, 8
        self.slab = _Slab(torch.zeros(16 * max(B, 32) * d, dtype=torch.float32, device=dev))
        if cd == torch.float16:
            self.w16 = torch.zeros(e.lay.numel, dtype=torch.float16, device=dev)
            self.mkv16 = torch.zeros(B * text_len, c.n_dec * 2 * d, dtype=torch.float16, device=dev)

    def W(self, name):
        """Weight view in the decode step's dtype."""
        if self.dd == torch.float16:
            return self.e.lay.view(self.w16, name)
        return self.e.W(name)

    @property
    def mkv(self):
        """Encoder memory K/V of all decoder layers [B * Tx, 6144] in the step's dtype."""
        return self.mkv16 if self.dd == torch.float16 else self.A["mkv"]

    # ----------------------------------------------------------------- one step
    def step(self):
        """Launch one decode step (graph-capturable: no host sync, no allocation)."""
        e, c = self.e, self.e.cfg
        A, B = self.A, self.B
        d, F, H = c.d_model, c.d_ffn, c.n_heads
        scale = 1.0 / math.sqrt(c.head_dim)
        pd = c.prenet_dropout if self.prenet_dropout else 0.0
        d1 = Drop(self.seed, SITE_INFER_FC1, pd) if pd > 0 else NO_DROP
        d2 = Drop(self.seed, SITE_INFER_FC2, pd) if pd > 0 else NO_DROP
        lin = e._lin
        lin(self.prev, self.W("dec.fc1.w"), self.p1, B, c.dec_prenet, c.n_mels, bias=e.P("dec.fc1.b"), act=ACT_RELU,
            drop=d1)
        lin(self.p1, self.W("dec.fc2.w"), self.p2, B, c.dec_prenet, c.dec_prenet, bias=e.P("dec.fc2.b"), act=ACT_RELU,
            drop=d2)
        if self.fused_io:
            # x0 = proj(p2) + alpha * pe[t], the scaled PE in the projection's epilogue
            lin(self.p2, self.W("dec.proj.w"), self.x0, B, d, c.dec_prenet, bias=e.P("dec.proj.b"),
                pe=(e.pe, e.P("dec.alpha"), self.t))
        else:
            lin(self.p2, self.W("dec.proj.w"), self.proj, B, d, c.dec_prenet, bias=e.P("dec.proj.b"))
            ops.posenc_fwd(self.proj, e.P("dec.alpha"), e.pe, self.x0, B, 1, t_ptr=self.t)
        mkv = self.mkv
        kvld = c.n_dec * 2 * d
        eps = c.ln_eps
        # Each post-LN is fused into the GEMM that consumes it (the skinny kernel
        # normalises its A rows and publishes the LN output for the residual path), and
        # the K/V columns of the QKV projection go straight into the KV cache: 8 kernels
        # per layer instead of 12.
        if self.dd == torch.float16 or (e.cd == torch.bfloat16 and self.fuse == 3):
            return self._step_layers_split(B, d, F, H, scale)
        if e.cd != torch.bfloat16 or self.fuse < 2:
            return self._step_layers_unfused(lin, B, d, F, H, scale, kv_fused=e.cd == torch.bfloat16 and self.fuse == 1)
        x, ln_prev = self.x0, None          # ln_prev: (branch, gamma, beta, out) pending on x
        xs = (self.xa, self.xb)
        for l in range(c.n_dec):
            p = f"dec{l}."
            cache = self.cache[l]
            kv = (cache, self.t, d, self.Tmax * 2 * d, 2 * d)
            if ln_prev is None:
                lin(x, self.W(p + "qkv.w"), self.qkv, B, 3 * d, d, bias=e.P(p + "qkv.b"), kv=kv)
            else:
                lin(x, self.W(p + "qkv.w"), self.qkv, B, 3 * d, d, bias=e.P(p + "qkv.b"), kv=kv, a_ln=ln_prev + (eps,))
                x = ln_prev[3]
            ops.attn_decode(self.qkv, cache, cache[:, :, d:], self.att, 3 * d, self.Tmax * 2 * d, 2 * d,
                            self.Tmax * 2 * d, 2 * d, d, B, H, self.Tmax, t_ptr=self.t, scale=scale)
            lin(self.att, self.W(p + "o.w"), self.o, B, d, d, bias=e.P(p + "o.b"))
            # h1 = LN1(x + o), fused into the cross-attention query projection
            lin(x, self.W(p + "cq.w"), self.cq, B, d, d, bias=e.P(p + "cq.b"),
                a_ln=(self.o, e.P(p + "ln1.g"), e.P(p + "ln1.b"), self.h1, eps))
            ko = 2 * d * l
            ops.attn_decode(self.cq, mkv[:, ko:], mkv[:, ko + d:], self.catt, d, self.Tx * kvld, kvld,
                            self.Tx * kvld, kvld, d, B, H, self.Tx, key_len=A["text_len"], scale=scale)
            lin(self.catt, self.W(p + "co.w"), self.co, B, d, d, bias=e.P(p + "co.b"))
            # h2 = LN2(h1 + co), fused into FFN1
            lin(self.h1, self.W(p + "ffn1.w"), self.f1, B, F, d, bias=e.P(p + "ffn1.b"), act=ACT_RELU,
                a_ln=(self.co, e.P(p + "ln2.g"), e.P(p + "ln2.b"), self.h2, eps))
            lin(self.f1, self.W(p + "ffn2.w"), self.f2, B, d, F, bias=e.P(p + "ffn2.b"))
            # LN3(h2 + f2) is fused into the next consumer (next layer's QKV, or the heads)
            x, ln_prev = self.h2, (self.f2, e.P(p + "ln3.g"), e.P(p + "ln3.b"), xs[l % 2])
        lin(x, self.W("heads.w"), self.heads, B, c.n_mels + 1, d, bias=e.P("heads.b"), ldo=96,
            a_ln=ln_prev + (eps,), emit=self._emit_args())

    def _step_layers_split(self, B, d, F, H, scale):
        """Decoder layers with split-K output projections: o, co and ffn2 (the K = 512 /
        2048 GEMMs whose 32 column tiles would leave most CUs idle) write raw partial slabs
        from splits x more workgroups, and tt2_ln_combine folds the slabs + bias + residual
        into the sublayer's LayerNorm.  11 launches per layer, as the unfused path, but the
        weight stream of those three is spread over 4-8x the CUs."""
        e, c, A = self.e, self.e.cfg, self.A
        lin = e._lin
        x = self.x0
        mkv = self.mkv
        kvld = c.n_dec * 2 * d
        eps = c.ln_eps
        slab = self.slab

        def split(xin, w, n, k, sp):
            ops.gemm(xin, w, self.o, B, n, k, k, k, n, splits=sp, main_only=True, ws=slab)

        for l in range(c.n_dec):
            p = f"dec{l}."
            cache = self.cache[l]
            lin(x, self.W(p + "qkv.w"), self.qkv, B, 3 * d, d, bias=e.P(p + "qkv.b"),
                kv=(cache, self.t, d, self.Tmax * 2 * d, 2 * d))
            ops.attn_decode(self.qkv, cache, cache[:, :, d:], self.att, 3 * d, self.Tmax * 2 * d, 2 * d,
                            self.Tmax * 2 * d, 2 * d, d, B, H, self.Tmax, t_ptr=self.t, scale=scale)
            split(self.att, self.W(p + "o.w"), d, d, self.split_o)
            ops.ln_combine(x, slab.t, self.split_o, e.P(p + "o.b"), e.P(p + "ln1.g"), e.P(p + "ln1.b"), self.h1, B,
                           eps)
            lin(self.h1, self.W(p + "cq.w"), self.cq, B, d, d, bias=e.P(p + "cq.b"))
            ko = 2 * d * l
            ops.attn_decode(self.cq, mkv[:, ko:], mkv[:, ko + d:], self.catt, d, self.Tx * kvld, kvld,
                            self.Tx * kvld, kvld, d, B, H, self.Tx, key_len=A["text_len"], scale=scale)
            split(self.catt, self.W(p + "co.w"), d, d, self.split_o)
            ops.ln_combine(self.h1, slab.t, self.split_o, e.P(p + "co.b"), e.P(p + "ln2.g"), e.P(p + "ln2.b"),
                           self.h2, B, eps)
            lin(self.h2, self.W(p + "ffn1.w"), self.f1, B, F, d, bias=e.P(p + "ffn1.b"), act=ACT_RELU)
            split(self.f1, self.W(p + "ffn2.w"), d, F, self.split_f)
            xn = self.xa if x is not self.xa else self.xb
            ops.ln_combine(self.h2, slab.t, self.split_f, e.P(p + "ffn2.b"), e.P(p + "ln3.g"), e.P(p + "ln3.b"),
                           xn, B, eps)
            x = xn
        self._heads(x)

    def _emit_args(self):
        """Frame emit fused into the heads GEMM (bf16 skinny path): mel/stop/prev stores,
        then the last workgroup advances the step counter and the dropout seed."""
        return (self.mel_seq, self.stop_seq, self.prev, self.t, self.seed, self.emit_done, self.e.cfg.n_mels,
                self.Tmax)

    def _heads(self, x):
        c, e = self.e.cfg, self.e
        if self.fused_io:
            e._lin(x, self.W("heads.w"), self.heads, self.B, c.n_mels + 1, c.d_model, bias=e.P("heads.b"), ldo=96,
                   emit=self._emit_args())
        else:
            e._lin(x, self.W("heads.w"), self.heads, self.B, c.n_mels + 1, c.d_model, bias=e.P("heads.b"), ldo=96)
            self._emit()

    def _emit(self):
        c = self.e.cfg
        ops.decode_emit(self.heads, 96, self.B, c.n_mels, self.Tmax, self.mel_seq, self.stop_seq, self.prev, self.t,
                        self.seed)

    def _step_layers_unfused(self, lin, B, d, F, H, scale, kv_fused=False):
        """Decoder layers + heads with separate LayerNorm kernels; the K/V append is a
        separate kernel too unless kv_fused (bf16 skinny-GEMM epilogue scatter)."""
        e, c, A = self.e, self.e.cfg, self.A
        x, xn = self.x0, self.xa
        mkv = self.mkv
        kvld = c.n_dec * 2 * d
        for l in range(c.n_dec):
            p = f"dec{l}."
            cache = self.cache[l]
            if kv_fused:
                lin(x, self.W(p + "qkv.w"), self.qkv, B, 3 * d, d, bias=e.P(p + "qkv.b"),
                    kv=(cache, self.t, d, self.Tmax * 2 * d, 2 * d))
            else:
                lin(x, self.W(p + "qkv.w"), self.qkv, B, 3 * d, d, bias=e.P(p + "qkv.b"))
                ops.kv_append(self.qkv[:, d:], 3 * d, cache, self.Tmax * 2 * d, 2 * d, 2 * d, B, self.t)
            ops.attn_decode(self.qkv, cache, cache[:, :, d:], self.att, 3 * d, self.Tmax * 2 * d, 2 * d,
                            self.Tmax * 2 * d, 2 * d, d, B, H, self.Tmax, t_ptr=self.t, scale=scale)
            lin(self.att, self.W(p + "o.w"), self.o, B, d, d, bias=e.P(p + "o.b"))
            ops.layernorm_fwd(x, self.o, e.P(p + "ln1.g"), e.P(p + "ln1.b"), self.h1, None, None, B, c.ln_eps)
            lin(self.h1, self.W(p + "cq.w"), self.cq, B, d, d, bias=e.P(p + "cq.b"))
            ko = 2 * d * l
            ops.attn_decode(self.cq, mkv[:, ko:], mkv[:, ko + d:], self.catt, d, self.Tx * kvld, kvld,
                            self.Tx * kvld, kvld, d, B, H, self.Tx, key_len=A["text_len"], scale=scale)
            lin(self.catt, self.W(p + "co.w"), self.co, B, d, d, bias=e.P(p + "co.b"))
            ops.layernorm_fwd(self.h1, self.co, e.P(p + "ln2.g"), e.P(p + "ln2.b"), self.h2, None, None, B, c.ln_eps)
            lin(self.h2, self.W(p + "ffn1.w"), self.f1, B, F, d, bias=e.P(p + "ffn1.b"), act=ACT_RELU)
            lin(self.f1, self.W(p + "ffn2.w"), self.f2, B, d, F, bias=e.P(p + "ffn2.b"))
            ops.layernorm_fwd(self.h2, self.f2, e.P(p + "ln3.g"), e.P(p + "ln3.b"), xn, None, None, B, c.ln_eps)
            x, xn = xn, (self.xb if xn is self.xa else self.xa)
        self._heads(x)

    # ----------------------------------------------------------------- driver
    def reset(self):
        self.t.zero_()
        self.seed.fill_(self.seed0)
        self.prev.zero_()

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

    def capture(self):
        """Record one decode step as a hipGraph (run after encode(); the warm-up
        step it takes first is undone by reset())."""
        self.reset()
        self.step()                  # warm-up: sizes everything, touches buffers
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(self.graph, stream=s, capture_error_mode=ops.CAPTURE_MODE):
                self.step()
        torch.cuda.current_stream().wait_stream(s)
        self.reset()

    def decode_loop(self, n_steps: int, use_graph: bool = True, stop_threshold: float | None = None,
                    check_every: int = 32, limits: torch.Tensor | None = None) -> int:
        """Run up to n_steps frames; with stop_threshold, stop once every utterance has
        emitted a stop probability >= threshold or reached its own frame limit
        (limits: [B] per-utterance caps, e.g. from a length model).  The batch keeps
        stepping until the last utterance is done (polled every check_every frames).
        Returns frames run."""
        logit_thr = None if stop_threshold is None else math.log(stop_threshold / (1.0 - stop_threshold))
        if limits is not None:
            limits = limits.to(device=self.stop_seq.device, dtype=torch.long)
            n_steps = min(n_steps, int(limits.max()))
        done = 0
        while done < n_steps:
            k = min(check_every, n_steps - done)
            for _ in range(k):
                if use_graph:
                    self.graph.replay()
                else:
                    self.step()
            done += k
            if logit_thr is not None or limits is not None:
                fin = torch.zeros(self.B, dtype=torch.bool, device=self.stop_seq.device)
                if logit_thr is not None:
                    fin |= (self.stop_seq[:, :done] >= logit_thr).any(dim=1)
                if limits is not None:
                    fin |= limits <= done
                if bool(fin.all()):
                    break
        return done

    def postnet(self, n_frames: int, stop_threshold: float | None, limits: torch.Tensor | None = None):
        e, c, A = self.e, self.e.cfg, self.A
        B, T = self.B, n_frames
        was = e.training
        e.training = False
        # the post-net sees exactly the n decoded frames (conv zero padding at n)
        Md = B * T
        before = self.mel_seq[:, :T].reshape(Md, c.n_mels).contiguous()
        ops.cast2d(before, c.n_mels, A["pin"], c.n_mels, Md, c.n_mels)
        e._postnet_fwd(A, A["pin"], before, c.n_mels, Md, T, False)
        e.training = was
        mel_after = A["mel_after"][:Md].view(B, T, c.n_mels).clone()
        out_len = torch.full((B,), n_frames, dtype=torch.long, device=e.dev)
        if stop_threshold is not None:
            logit_thr = math.log(stop_threshold / (1.0 - stop_threshold))
            hit = self.stop_seq[:, :n_frames] >= logit_thr
            first = torch.where(hit.any(1), hit.float().argmax(1) + 1, torch.full_like(out_len, n_frames))
            out_len = first.long()
        if limits is not None:
            out_len = torch.minimum(out_len, limits.to(out_len.device, torch.long))
        return mel_after, out_len

    def run(self, text, text_len, max_len: int | None = None, stop_threshold: float | None = 0.5,
            use_graph: bool = True, limits: torch.Tensor | None = None):
        """Greedy decode; returns (mel_after [B, T, 80] f32, out_len [B]).  limits: optional
        per-utterance frame caps [B] (out_len <= limits)."""
        max_len = max_len or self.Tmax
        self.encode(text, text_len)
        if use_graph and self.graph is None:
            self.capture()
        self.reset()
        n = self.decode_loop(max_len, use_graph, stop_threshold, limits=limits)
        return self.postnet(n, stop_threshold, limits)
