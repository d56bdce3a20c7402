"""TTSEngine -- the training/inference step as an explicit kernel schedule.

No autograd: the forward writes every activation the backward needs into a
preallocated per-shape arena; the backward walks the network in reverse with
hand-written gradient kernels (libtt2), writing parameter gradients straight
into one flat f32 buffer.  Everything runs on the current torch stream with
no host synchronisation and no allocation after warm-up, so a whole step
(forward + loss + backward + Adam) is capturable in one hipGraph.

Layout: activations are channels-last [batch*time, channels];
Me = B*Tx encoder rows, Md = B*Ty decoder rows.  Compute dtype ``cd`` is bf16
(f32 accumulation, f32 master weights/grads/statistics) or f32 (parity mode,
exact-f32 MFMA).
"""
from __future__ import annotations

import math
import os

import torch

from . import ops
from ._lib import ACT_NONE, ACT_RELU, ACT_TANH
from .trace import ranged
from .config import (SITE_DEC_FC1, SITE_DEC_FC2, SITE_DEC_LAYER, SITE_DEC_PE, SITE_ENC_CONV, SITE_ENC_LAYER,
                     SITE_ENC_PE, SITE_POSTNET, TTSConfig)
from .ops import NO_DROP, Drop
from .params import Layout, bn_layers, build_slots, postnet_channels, stats_layout


def sinusoid_table(max_len: int, dim: int) -> torch.Tensor:
    """Scaled-PE table (same formula as transformers modeling_speecht5.py:404-409)."""
    pe = torch.zeros(max_len, dim)
    position = torch.arange(0, max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, dim, 2, dtype=torch.int64).float() * -(math.log(10000.0) / dim))
    pe[:, 0::2] = torch.sin(position.float() * div_term)
    pe[:, 1::2] = torch.cos(position.float() * div_term)
    return pe


def _wide(dtype, conv, m: int, *inner: int) -> bool:
    """True when tt2_gemm's auto plan takes the 256 x 128 kernel (v7) for a GEMM with
    m output rows: bf16, 8-aligned inner dims, conv operands (T, C, pad) with T, C >= 64,
    not the skinny decode path (see gemm.hip gemm_plan)."""
    conv_ok = conv is None or (conv[0] >= 64 and conv[1] >= 64)
    return dtype == torch.bfloat16 and conv_ok and m > 32 and all(d % 8 == 0 for d in inner)


def auto_splits(n_out: int, n_in: int, k: int, wide: bool = False, items: int = 256) -> int:
    """Split-K factor for a weight-gradient GEMM (long K = tokens, few output tiles).
    v7 (256 x 128 tiles): ~`items` workgroups, >= 512 k each, at most 16 slabs (measured alone:
    512x512x12800 sp16 < sp32 < sp8; 2048x512x12800 sp8 best)."""
    if wide:
        tiles = ((n_out + 255) // 256) * ((n_in + 127) // 128)
        return max(1, min(16, items // tiles, k // 512))
    tiles = ((n_out + 127) // 128) * ((n_in + 127) // 128)
    if tiles >= 256:
        return 1
    return max(1, min(32, 512 // tiles, k // 256))


def act_splits(m: int, n: int, k: int, wide: bool = False) -> int:
    """Split-K factor for an activation GEMM: only when its tiles cannot fill the 256
    CUs (the encoder's 2048-token GEMMs); the epilogue then runs in the split-K reduce."""
    if wide:
        tiles = ((m + 255) // 256) * ((n + 127) // 128)
        if tiles >= 128 or k < 1024 or m <= 32:
            return 1
        return max(1, min(8, 256 // tiles, k // 512))
    tiles = ((m + 127) // 128) * ((n + 127) // 128)
    if tiles >= 192 or k < 1024 or m <= 32:   # m <= 32: the decode step's skinny weight-streaming GEMM
        return 1
    return max(1, min(8, 512 // tiles, k // 512))


class Arena:
    """All activations / gradient scratch for one (B, Tx, Ty) shape."""

    def __init__(self, c: TTSConfig, B: int, Tx: int, Ty: int, cd: torch.dtype, dev):
        self.B, self.Tx, self.Ty = B, Tx, Ty
        self.gen = 0   # forward count (the autograd boundary checks its saved arena is intact)
        d, F, H = c.d_model, c.d_ffn, c.n_heads
        Me, Md = B * Tx, B * Ty
        self.Me, self.Md = Me, Md
        self.t = {}
        self.spec = {}
        self.dev = dev
        f32 = torch.float32

        def mk(name, shape, dtype=cd, zero=False):
            self.spec[name] = (shape, dtype, zero)

        mk("text", (Me,), torch.int64)
        mk("text_len", (B,), torch.int32)
        mk("mel_len", (B,), torch.int32)
        mk("mel", (B, Ty, c.n_mels), f32)
        mk("emb", (Me, d))
        for i in range(c.enc_conv_layers):
            mk(f"ecv_y{i}", (Me, d))
            mk(f"ecv_part{i}", (2 * ((Me + 63) // 64) * d,), f32)   # fused BatchNorm statistics (see pcv_part)
            mk(f"ecv_o{i}", (Me, d))
            mk(f"ecv_mean{i}", (d,), f32)
            mk(f"ecv_rstd{i}", (d,), f32)
        mk("eproj", (Me, d))
        mk("ex0", (Me, d))
        for l in range(c.n_enc):
            mk(f"eqkv{l}", (Me, 3 * d))
            mk(f"eatt{l}", (Me, d))
            mk(f"else{l}", (B * H, Tx), f32)
            mk(f"eo{l}", (Me, d))
            mk(f"eh1{l}", (Me, d))
            mk(f"eln1m{l}", (Me,), f32)
            mk(f"eln1r{l}", (Me,), f32)
            mk(f"ef1{l}", (Me, F))
            mk(f"ef2{l}", (Me, d))
            mk(f"ex{l + 1}", (Me, d))
            mk(f"eln2m{l}", (Me,), f32)
            mk(f"eln2r{l}", (Me,), f32)
        mk("mkv", (Me, c.n_dec * 2 * d))
        mk("din", (Md, c.n_mels))
        mk("dp1", (Md, c.dec_prenet))
        mk("dp2", (Md, c.dec_prenet))
        mk("dproj", (Md, d))
        mk("dx0", (Md, d))
        for l in range(c.n_dec):
            mk(f"dqkv{l}", (Md, 3 * d))
            mk(f"datt{l}", (Md, d))
            mk(f"dlse{l}", (B * H, Ty), f32)
            mk(f"do{l}", (Md, d))
            mk(f"dh1{l}", (Md, d))
            mk(f"dcq{l}", (Md, d))
            mk(f"dcatt{l}", (Md, d))
            mk(f"dclse{l}", (B * H, Ty), f32)
            mk(f"dco{l}", (Md, d))
            mk(f"dh2{l}", (Md, d))
            mk(f"df1{l}", (Md, F))
            mk(f"df2{l}", (Md, d))
            mk(f"dx{l + 1}", (Md, d))
            for k in (1, 2, 3):
                mk(f"dln{k}m{l}", (Md,), f32)
                mk(f"dln{k}r{l}", (Md,), f32)
        self.heads_ld = 96
        mk("heads", (Md, self.heads_ld), f32, zero=True)
        mk("pin", (Md, c.n_mels))
        chans = postnet_channels(c)
        for i in range(c.postnet_layers):
            mk(f"pcv_y{i}", (Md, chans[i + 1]))
            if i < c.postnet_layers - 1:
                mk(f"pcv_o{i}", (Md, chans[i + 1]))
            mk(f"pcv_mean{i}", (chans[i + 1],), f32)
            mk(f"pcv_rstd{i}", (chans[i + 1],), f32)
            # the conv GEMM's fused BatchNorm statistics (chunk moments / sums, bf16 training; sized
            # for the smallest chunk, the 64 x 64 kernel's)
            mk(f"pcv_part{i}", (2 * ((Md + 63) // 64) * chans[i + 1],), f32)
        mk("mel_after", (Md, c.n_mels), f32)
        mk("loss", (4,), f32)
        # ---- gradient scratch
        mk("g_heads", (Md, self.heads_ld), f32)
        mk("gh_cd", (Md, self.heads_ld), cd, zero=True)
        mk("g_after", (Md, c.n_mels))
        mk("g_pa", (Md, c.postnet_channels))
        mk("g_pb", (Md, c.postnet_channels))
        mk("g_xa", (Md, d))
        mk("g_xb", (Md, d))
        mk("g_res", (Md, d))
        mk("g_br", (Md, d))
        mk("g_br2", (Md, d))    # per-branch dY buffers: a layer's weight gradients run as one
        mk("g_br3", (Md, d))    # grouped GEMM at the end of its backward (Engine._flush_wgrads)
        mk("g_cq", (Md, d))
        mk("g_f1", (Md, F))
        mk("g_qkv", (Md, 3 * d))
        mk("g_att", (Md, d))
        mk("g_p1", (Md, c.dec_prenet))
        mk("g_p2", (Md, c.dec_prenet))
        mk("g_mkv", (Me, c.n_dec * 2 * d))
        mk("delta", (B * H, max(Tx, Ty)), f32)

    def __getitem__(self, k):
        t = self.t.get(k)
        if t is None:
            # allocated on first use (inference touches a subset); never inside a capture
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"arena buffer {k} first touched during graph capture")
            shape, dtype, zero = self.spec[k]
            t = (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=self.dev)
            self.t[k] = t
        return t

    def materialize(self):
        for k in self.spec:
            self[k]
        return self

    def layer_buf(self, name: str, key, shape=None) -> torch.Tensor:
        """A per-layer copy `name@key` of gradient scratch buffer `name` (optionally of another
        shape): the overlapped backward (TTSEngine.wgrad_overlap) keeps each layer's weight-
        gradient dY alive until the side stream has used it."""
        full = f"{name}@{key}"
        if full not in self.spec:
            shp, dt, zero = self.spec[name]
            self.spec[full] = (tuple(shape) if shape is not None else shp, dt, zero)
        return self[full]


class TTSEngine:
    # overlapped backward's clip-norm partials: at most NORM_RANGES gradient ranges, each summed by
    # one work group per NORM_CHUNK gradients (NORM_PARTS_MAX at most; bandwidth-bound either way)
    NORM_RANGES, NORM_CHUNK, NORM_PARTS_MAX = 64, 1 << 13, 1024

    def __init__(self, cfg: TTSConfig | None = None, dtype: torch.dtype = torch.bfloat16, device="cuda",
                 seed: int = 0):
        self.cfg = c = cfg or TTSConfig()
        assert c.d_model == 512 and c.head_dim == 64, "kernels are built for d_model 512, head_dim 64"
        self._heads_pad = None   # bf16: heads GEMMs padded to 88 rows (_pad_heads_weights)
        self._heads_pad_fresh = False
        self.pad_heads = True
        # backward: a LayerNorm's column-sum finalize rides in the next LayerNorm's launch
        # (two dedicated partials buffers alternate; see _ln_defer)
        self.ln_chain = os.environ.get("TT2_LN_CHAIN", "1") != "0"
        self._ln_parts = None
        # ... and each layer's last one in the layer's grouped weight-gradient reduce launch
        self.ln_fin_in_reduce = os.environ.get("TT2_LN_FIN_REDUCE", "1") != "0"
        self._wq = None   # weight-gradient requests queued for one grouped launch (see _defer_wgrads)
        self._in_scope = False   # between _defer_wgrads and _flush_wgrads (a layer's group)
        self.wflip_batch = os.environ.get("TT2_WFLIP_BATCH", "1") != "0"
        # bf16 backward: every weight-gradient GEMM (and the DP hook of its bucket) runs on a side
        # stream that starts with the encoder backward, whose small latency-bound launches leave
        # most of the chip idle; the decoder / post-net dgrad chain no longer waits for them
        # (see backward).  Off: each layer's weight gradients run in place, as before.
        self.wgrad_overlap = os.environ.get("TT2_WGRAD_OVERLAP", "1") != "0"
        self._jobs = None    # overlapped backward: queued weight-gradient jobs (see _push_job)
        self._side = None
        self._side_ws = None
        self._side_live = False
        self._ln_parts_l = {}   # per-layer partials of the deferred last LayerNorm of a layer
        # side-stream weight-gradient launches: split-K factor multiplier (shorter work items)
        # and work-group cap (0: none), dev knobs for the overlap's A/B
        self._norm_buf = None
        self._norm_pending = None   # (ranges, computed on the side stream) of the last overlapped backward
        self.side_split = int(os.environ.get("TT2_SIDE_SPLIT", "1"))
        # work items a grouped weight-gradient launch aims at (its split-K factor: items / tiles)
        self.wgrad_items = int(os.environ.get("TT2_WGRAD_ITEMS", "128"))
        self.wgrad_items_direct = int(os.environ.get("TT2_WGRAD_DIRECT", "128"))   # the ungrouped ones
        self.side_groups = int(os.environ.get("TT2_SIDE_WG", "0"))
        # ... for the jobs issued while the decoder backward runs (side_start >= 0): the 200-tile
        # N = 512 dgrads there leave 56 CUs idle, which a capped side grid can fill
        self.side_groups_dec = int(os.environ.get("TT2_SIDE_WG_DEC", "128"))
        self._side_cap = 0
        # the decoder layer whose backward starts the side stream (-1: the encoder backward).  Default:
        # the first one (5), with the side grid capped at 128 work groups while the decoder backward
        # runs (side_groups_dec): -0.8 % step time, same box, interleaved (gpurun_out/r05j, r05m)
        self.side_start = int(os.environ.get("TT2_SIDE_START", "5"))
        self.enc_overlap = int(os.environ.get("TT2_ENC_OVERLAP", "1"))   # see forward()
        # ... also with SyncBatchNorm (the encoder pre-net's exchanges then fork the comm stream
        # from the side stream); TT2_ENC_OVERLAP_SYNCBN=0 keeps the encoder on the main stream there
        self.enc_overlap_syncbn = os.environ.get("TT2_ENC_OVERLAP_SYNCBN", "1") != "0"
        # SyncBatchNorm under the encoder overlap: the pre-net (its BatchNorm exchanges) on the
        # main stream, the capture's origin (forward()).  False is for the capture guard's test
        # only: the exchanges then come from the side stream and the capture refuses them.
        self.syncbn_prenet_on_main = True
        # the post-net BatchNorms' statistics from their conv GEMMs' epilogues (_postnet_fwd)
        self.bn_gemm_stats = os.environ.get("TT2_BN_GEMM_STATS", "1") != "0"
        # pipelined optimizer (opt-in: TransformerTTS.pipeline_optimizer): a step's Adam is
        # deferred to the start of the next forward, where the encoder's share runs on the side
        # stream ahead of the encoder and the rest on the main stream ahead of the decoder,
        # beside the encoder's forward (the same updates in the same order: identical results).
        # Whether an update is pending lives on the device (adam_gate: armed by optimizer_step,
        # consumed by the deferred Adam or by flush_optimizer), so a captured step never applies
        # an update twice after an eager flush, nor a stale one after load_state_dict
        self.pipeline_opt = False
        self._adam_parts = None   # the clip-norm partials the deferred Adam reads (a fixed buffer)
        self.cd = dtype
        self.dev = torch.device(device)
        self.lay = Layout(build_slots(c))
        self.slay = stats_layout(c)
        n = self.lay.numel
        self.params = torch.zeros(n, dtype=torch.float32, device=self.dev)
        self.grads = torch.zeros(n, dtype=torch.float32, device=self.dev)
        self.shadow = torch.zeros(n, dtype=torch.bfloat16, device=self.dev) if dtype == torch.bfloat16 else None
        self.stats = torch.zeros(self.slay.numel, dtype=torch.float32, device=self.dev)
        self.nbt = {name: 0 for name, _ in bn_layers(c)}
        self.exp_avg = None
        self.exp_avg_sq = None
        self.pe = sinusoid_table(c.max_len, c.d_model).to(self.dev)
        self.seed = torch.tensor([seed], dtype=torch.int32, device=self.dev)   # per-step dropout seed (uint32)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.adam_gate = torch.zeros(1, dtype=torch.int32, device=self.dev)   # pipelined Adam pending
        self.ws = ops.Workspace()
        self.arenas: dict[tuple, Arena] = {}
        self.training = True
        self.dropout_enabled = True
        self.grad_scale = 1.0
        self.grad_ready_hook = None   # called as hook(flat_offset) during backward (DP bucketing)
        self._ready_set = set(self.ready_names())
        # overlapped backward with DP: hand each bucket to the comm stream after the next side job
        # is issued, ordered by an event (_fire_deferred); TT2_DEFER_FORK=0: right after its job
        self.defer_bucket_fork = os.environ.get("TT2_DEFER_FORK", "1") != "0"
        self._deferred = []
        self.bn_sync = None   # SyncBatchNorm exchange (tt2/dist.py BnSync), None: per-replica statistics
        self.opt = dict(lr=1.0, beta1=0.9, beta2=0.98, eps=1e-9, weight_decay=0.0, clip_norm=1.0, warmup=4000.0,
                        noam=True)
        self._init_defaults()

    # ------------------------------------------------------------ parameters
    def _init_defaults(self):
        for name, _ in bn_layers(self.cfg):
            self.slay.view(self.stats, name + ".rv").fill_(1.0)
        for name, (off, shape, n) in self.lay.slots.items():
            if name.endswith(".g") or name.endswith("alpha"):
                self.P(name).fill_(1.0)
        self.sync_shadow()

    def P(self, name):
        return self.lay.view(self.params, name)

    def G(self, name):
        return self.lay.view(self.grads, name)

    def W(self, name):
        return self.lay.view(self.shadow if self.shadow is not None else self.params, name)

    def S(self, name):
        return self.slay.view(self.stats, name)

    def sync_shadow(self):
        self._heads_pad_fresh = False
        if self.shadow is not None:
            self.shadow.copy_(self.params)

    def load_slots(self, P: dict, S: dict | None = None, nbt: dict | None = None):
        with torch.no_grad():
            for k, v in P.items():
                self.P(k).copy_(v.reshape(self.P(k).shape))
            for k, v in (S or {}).items():
                self.S(k).copy_(v)
        if nbt:
            self.nbt.update(nbt)
        self.sync_shadow()

    def drop(self, site: int, p: float) -> Drop:
        if self.training and self.dropout_enabled and p > 0:
            return Drop(self.seed, site, p)
        return NO_DROP

    def arena(self, B, Tx, Ty) -> Arena:
        key = (B, Tx, Ty)
        if key not in self.arenas:
            self.arenas[key] = Arena(self.cfg, B, Tx, Ty, self.cd, self.dev)
        return self.arenas[key]

    # ------------------------------------------------------------ GEMM helpers
    def _lin(self, x, w, out, m, n, k, bias=None, act=ACT_NONE, drop=NO_DROP, res=None, ldx=None, ldo=None,
             a_conv=None, beta=0.0, **fuse):
        # fused column statistics need the whole K in one tile (no split-K)
        sp = 1 if "col_stats" in fuse else act_splits(m, n, k, _wide(x.dtype, a_conv, m, k) and not fuse)
        ops.gemm(x, w, out, m, n, k, ldx or k, k, ldo or n, bias=bias, res=res, ldr=ldo or n, act=act, drop=drop,
                 a_conv=a_conv, beta=beta, ws=self.ws, splits=sp, **fuse)

    def _dgrad(self, dy, w, out, m, n_in, n_out, res=None, gate=None, gate_scale=1.0, ldy=None, ldo=None,
               a_conv=None, beta=0.0, bn_bwd=None):
        """out[m, n_in] = dy[m, n_out] @ W[n_out, n_in] (+res) (*gate); bn_bwd: see _conv_dgrad"""
        sp = 1 if bn_bwd is not None else act_splits(m, n_in, n_out, _wide(dy.dtype, a_conv, m, n_out, n_in))
        ops.gemm(dy, w, out, m, n_in, n_out, ldy or n_out, n_in, ldo or n_in, trans_b=True, res=res,
                 ldr=ldo or n_in, gate=gate, ldg=ldo or n_in, gate_scale=gate_scale, a_conv=a_conv, beta=beta,
                 ws=self.ws, splits=sp, bn_bwd=bn_bwd)

    def _conv_dgrad(self, dy, wflip, out, m, cin, cout, K, T, ldo=None, beta=0.0, bn_bwd=None):
        """out[m, cin] = conv1d(dy, flipped W): implicit im2col of dy x wflip[cin][tap][cout].
        bn_bwd: out is that BatchNorm backward's dout; the GEMM also leaves its column sums (one
        tile per output, no split-K)"""
        ops.gemm(dy, wflip, out, m, cin, K * cout, cout, K * cout, ldo or cin, a_conv=(T, cout, (K - 1) // 2),
                 beta=beta, ws=self.ws, splits=1 if bn_bwd is not None else act_splits(m, cin, K * cout),
                 bn_bwd=bn_bwd)

    def _wgrad(self, dy, x, gw, n_out, n_in, m, ldy=None, ldx=None, b_conv=None, gb=None, now=False):
        """gw[n_out, n_in] (f32) = dy[m, n_out]^T @ x[m, n_in]; gb (optional) = the
        bias gradient sum_m dy[m, :], fused into the GEMM's A-tile pass for bf16.
        Inside a _defer_wgrads() scope, v7-eligible requests are queued and launched
        together by _flush_wgrads (their inputs must stay live until then); in an overlapped
        backward every v7-eligible request is queued for the side stream (now=True: not)."""
        if (self._wq is not None or (self._jobs is not None and not now)) and _wide(dy.dtype, b_conv, n_out, n_out,
                                                                                     n_in):
            if not self._in_scope:
                # a request the in-place schedule launches on its own (outside a layer's group):
                # queued as that same launch (same plan, same split-K factor), so the overlapped
                # schedule sums every weight gradient in the same order (bit-identical)
                req = {"direct": dict(a=dy, b=x, c=gw, m=n_out, n=n_in, k=m, lda=ldy or n_out, ldb=ldx or n_in,
                                      ldc=n_in, trans_a=True, trans_b=True, b_conv=b_conv, a_ksum=gb,
                                      splits=auto_splits(n_out, n_in, m, True, self.wgrad_items_direct))}
                if self._wq is None:
                    self._wq = []
            else:
                req = dict(a=dy, b=x, c=gw, m=n_out, n=n_in, k=m, lda=ldy or n_out, ldb=ldx or n_in, ldc=n_in,
                           trans_a=True, trans_b=True, b_conv=b_conv, a_ksum=gb)
            self._wq.append(req)
            return
        # the fused path rides on the LDS-DMA kernel: bf16 with 8-aligned M and N
        fused = gb is not None and dy.dtype == torch.bfloat16 and n_out % 8 == 0 and n_in % 8 == 0
        ops.gemm(dy, x, gw, n_out, n_in, m, ldy or n_out, ldx or n_in, n_in, trans_a=True, trans_b=True,
                 splits=auto_splits(n_out, n_in, m, _wide(dy.dtype, b_conv, n_out, n_out, n_in), self.wgrad_items_direct),
                 b_conv=b_conv, ws=self.ws,
                 a_ksum=gb if fused else None)
        if gb is not None and not fused:
            self._bias(dy, ldy or n_out, m, n_out, gb)

    def _ln_defer(self, slot: int, m: int, prev=None) -> dict:
        """Keyword arguments that defer a LayerNorm backward's finalize into partials buffer
        `slot` (0/1, alternating along a chain) and complete `prev`'s in the same launch.
        Chains stop at each layer's last LayerNorm (not deferred), so every layer's
        gradients are final when its DP bucket may be launched."""
        if not self.ln_chain:
            return {}
        if self._ln_parts is None:
            nbytes = ops.layernorm_bwd_workspace_size(1 << 30, self.cfg.d_model)
            self._ln_parts = [torch.empty(nbytes, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        return {"part": self._ln_parts[slot], "defer": True, "prev": prev}

    def _ln_last(self, *args, prev=None, slot=0, **kw):
        """A layer's last LayerNorm backward: with the chain on, deferred into partials slot
        `slot` (free: its previous user was completed by `prev`'s launch) and returned for
        _flush_wgrads to finalize inside the layer's grouped weight-gradient launch, which
        precedes the layer's DP bucket (_ready) and the next use of the slot."""
        if self._jobs is not None:
            # overlapped: finalized later by the layer's weight-gradient job on the side stream,
            # so the partials get a buffer of their own (the chain slots are reused meanwhile)
            key = kw.pop("key")
            buf = self._ln_parts_l.get(key)
            if buf is None:
                buf = torch.empty(ops.layernorm_bwd_workspace_size(1 << 30, self.cfg.d_model), dtype=torch.uint8,
                                  device=self.dev)
                self._ln_parts_l[key] = buf
            extra = {"part": buf, "defer": True, "prev": prev}
        else:
            kw.pop("key", None)
            extra = self._ln_defer(slot, 0, prev) if self.ln_chain and self.ln_fin_in_reduce else {"prev": prev}
        a = ops.layernorm_bwd(*args, ws=self.ws, **kw, **extra)
        return a if extra.get("defer") else None

    def _defer_wgrads(self):
        if self._wq and self._jobs is not None:   # overlapped: earlier queued requests keep their order
            self._push_job(self._wq)
        self._wq = []
        self._in_scope = True

    def _flush_wgrads(self, fin=None):
        """Launch the queued weight gradients as grouped v7 GEMMs (<= 8 per launch), one
        split-K factor per group: about 256 work items, >= 512 tokens per split.  fin: the
        layer's last (deferred) LayerNorm backward, finalized in the first group's reduce
        launch instead of a launch of its own."""
        q, self._wq = self._wq or [], None
        self._in_scope = False
        if self._jobs is not None:
            self._push_job(q, fin)
            return
        self._launch_wgrads(q, fin, self.ws)

    def _launch_wgrads(self, q, fin, ws, side=False):
        if not q and fin is not None:
            ops.layernorm_bwd_finalize(fin)
        # requests the in-place schedule launches one by one (v7, each with its own split-K factor):
        # grouped launches with per-problem splits, which compute every problem's tiles and its
        # split-K reduce the same way (bit-identical to the single launches), in fewer launches
        direct = [p["direct"] for p in q if "direct" in p]
        for i in range(0, len(direct), 8):
            ops.gemm_grouped(direct[i:i + 8], ws=ws, max_groups=self._side_cap if side else 0)
        q = [p for p in q if "direct" not in p]
        for i in range(0, len(q), 8):
            grp = q[i:i + 8]
            tiles = sum(((p["m"] + 255) // 256) * ((p["n"] + 127) // 128) for p in grp)
            kmin = min(p["k"] for p in grp)
            sp = max(1, min(16, self.wgrad_items // tiles, kmin // 512))
            if side:   # beside the encoder backward: shorter items, a capped grid
                sp = max(1, min(16 * self.side_split, sp * self.side_split, kmin // 256))
            ops.gemm_grouped([dict(p, splits=sp) for p in grp], ws=ws, fin=fin if i == 0 else None,
                             max_groups=self._side_cap if side else 0)

    # ------------------------------------------------------------ overlapped weight gradients
    # A job = queued weight-gradient requests (+ a deferred LayerNorm finalize, + the DP hooks
    # of the buckets they complete), ordered after the main-stream work that produced its
    # inputs by an event.  Jobs run in order on the side stream, which first waits for the
    # start of the encoder backward (_start_side); the main stream joins it at the end of the
    # backward.  Every DP hook therefore fires from the side stream, in bucket order.
    def _ov_begin(self):
        if self._side is None:
            self._side = torch.cuda.Stream()
            self._side_ws = ops.Workspace()
        self._side.wait_stream(torch.cuda.current_stream())
        self._jobs = []
        self._deferred = []
        self._side_live = False

    def _push_job(self, q, fin=None, ready=()):
        ev = torch.cuda.Event()
        ev.record()
        job = {"q": q, "fin": fin, "ready": list(ready), "ev": ev, "done": False}
        self._jobs.append(job)
        return job

    def _run_job(self, job):
        self._side.wait_event(job["ev"])
        with torch.cuda.stream(self._side):
            self._launch_wgrads(job["q"], job["fin"], self._side_ws, side=True)
            self._fire_deferred()
            ev = None
            if job["ready"] and self.grad_ready_hook is not None and self.defer_bucket_fork:
                ev = torch.cuda.Event()
                ev.record()
            for name in job["ready"]:
                off = self.lay.offset(name)
                if self.grad_ready_hook is not None:
                    if ev is not None:
                        self._deferred.append((off, ev))
                    else:
                        self.grad_ready_hook(off)
                self._norm_range(off)
        job["done"] = True

    def _fire_deferred(self):
        """The bucket hand-offs of the previous side job, issued only now that this job's weight
        gradients are on the side stream, each ordered after an event recorded at the end of its
        own job (defer_bucket_fork).  Issued right after their job, the comm stream's exchange
        kernels were created ahead of the side stream's next job in the captured graph, and the
        graph's executor ran the two branches one after the other (every side job then waited for
        the previous bucket's exchange)."""
        h = self.grad_ready_hook
        after_ok = getattr(getattr(h, "__self__", None), "accepts_after", False)
        for off, ev in self._deferred:
            if after_ok:
                h(off, after=ev)
            else:   # a hook without the event form: ordered after everything issued on the side stream
                h(off)
        self._deferred = []

    def _norm_begin(self, side: bool):
        """The clip norm's squared sum is taken over fixed ranges of the flat gradients, one per
        DP bucket boundary (_ready), in every schedule, so every schedule clips identically:
        `side` (overlapped backward without DP): each range on the side stream once its job has
        run; otherwise all ranges by optimizer_step (with DP: after the exchange)."""
        if self._norm_buf is None:
            self._norm_buf = torch.empty(self.NORM_RANGES * self.NORM_PARTS_MAX, dtype=torch.float32, device=self.dev)
        self._norm_ranges, self._norm_hi, self._norm_side = [], self.lay.numel, side
        self._norm_used = 0

    def _norm_range(self, lo):
        """Gradients [lo, hi) are final (hi: the previous boundary): their squared-norm partials."""
        hi = self._norm_hi
        if lo >= hi:
            return
        if len(self._norm_ranges) >= self.NORM_RANGES:
            raise RuntimeError("overlapped backward: more gradient ranges than NORM_RANGES")
        nb = max(1, min(self.NORM_PARTS_MAX, (hi - lo + self.NORM_CHUNK - 1) // self.NORM_CHUNK))
        self._norm_ranges.append((lo, hi, self._norm_used, nb))
        self._norm_used += nb
        self._norm_hi = lo
        if self._norm_side:
            ops.sumsq_parts(self.grads[lo:hi], self._norm_buf[self._norm_ranges[-1][2]:], nb)

    def _start_side(self):
        gate = torch.cuda.Event()
        gate.record()
        self._side.wait_event(gate)
        self._side_live = True

    def _pump(self, k: int = 1):
        """Issue the next k queued jobs on the (started) side stream.  The encoder backward
        calls this between its own launches, so in the captured graph the side work is created
        interleaved with the encoder chain rather than ahead of it (issued ahead, the graph's
        executor held the encoder's first launch behind ~0.5 ms of side kernels)."""
        if not self._side_live:
            return
        for job in self._jobs:
            if k <= 0:
                break
            if not job["done"]:
                self._run_job(job)
                k -= 1

    def _ov_end(self):
        if self._wq:
            self._push_job(self._wq)
            self._wq = None
        if not self._side_live:
            self._start_side()
        self._pump(len(self._jobs))
        with torch.cuda.stream(self._side):
            self._fire_deferred()
            self._norm_range(0)
        torch.cuda.current_stream().wait_stream(self._side)
        self._jobs = None
        self._side_live = False

    def _bias(self, dy, ld, m, n, gb):
        ops.colsum(dy, ld, m, n, gb, ws=self.ws)

    # ------------------------------------------------------------ forward
    def stage_inputs(self, A: Arena, text, text_len, mel, mel_len):
        A["text"].copy_(text.reshape(-1), non_blocking=True)
        A["text_len"].copy_(text_len, non_blocking=True)
        A["mel_len"].copy_(mel_len, non_blocking=True)
        A["mel"].copy_(mel, non_blocking=True)

    def forward(self, A: Arena):
        """Teacher-forced forward: encoder -> decoder -> heads -> post-net.  enc_overlap (bf16;
        TT2_ENC_OVERLAP, default 1): the encoder runs on the side stream beside the decoder's
        pre-net and layer 0's self-attention block, which do not need the memory (the step
        6.94 vs 7.03 ms measured; 1 issues the encoder first, 2 the decoder's part first: the
        same; 0 off)."""
        self._heads_pad_fresh = False   # the padded head weights are copied again (_pad_heads_weights)
        parts = self._adam_parts if self.pipeline_opt else None   # pipelined: last step's Adam (gated)
        if self.enc_overlap and self.cd == torch.bfloat16 and (self.bn_sync is None or self.enc_overlap_syncbn):
            if self._side is None:
                self._side = torch.cuda.Stream()
                self._side_ws = ops.Workspace()
            side = self._side
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            dec = self._decoder_steps(A)
            c_ndec = self.cfg.n_dec
            enc_r = self._enc_param_ranges() if parts is not None else []

            # SyncBatchNorm: the pre-net's exchanges stay on the main stream (the capture's
            # origin).  Forked from the side stream, the comm stream would have to be joined
            # back into the side stream, and hipStreamEndCapture (ROCm 7.0 runtime in torch)
            # segfaults on any stream joined into a stream other than the origin
            # (tools/capture_topo.py nested2s).  The decoder's first block
            # then overlaps the encoder layers instead of the pre-net: the chain is the same.
            pre_main = self.bn_sync is not None and self.syncbn_prenet_on_main
            enc_r_side = [] if pre_main else enc_r   # with the pre-net on main, its update goes there
            enc_adam_done = torch.cuda.Event() if enc_r_side else None

            def encoder():
                ws, self.ws = self.ws, self._side_ws
                try:
                    with torch.cuda.stream(side):
                        for lo, hi in enc_r_side:   # the encoder's parameters first
                            self._adam(lo, hi, parts, gated=True)
                        if enc_r_side:
                            # the main stream's conv weight flip below reads these weights
                            enc_adam_done.record()
                        if not pre_main:
                            self.forward_encoder_prenet(A)
                        self.forward_encoder_layers(A, rest_kv_later=True)
                finally:
                    self.ws = ws

            def rest_adam():   # everything else, ahead of the decoder
                if parts is None:
                    return
                lo = 0
                for a, b in enc_r + [(self.lay.numel, self.lay.numel)]:
                    if a > lo:
                        self._adam(lo, a, parts, gated=True)
                    lo = b
            if pre_main:
                for lo, hi in enc_r:   # the encoder's deferred update before the pre-net reads it
                    self._adam(lo, hi, parts, gated=True)
                self.forward_encoder_prenet(A)
                side.wait_stream(main)
            if self.enc_overlap == 1:
                encoder()
                rest_adam()
                next(dec)
            else:
                rest_adam()
                next(dec)
                encoder()
            if self.training and self.wflip_batch:
                # the dgrad conv weights (tap-flipped) for the backward, on the main stream while it
                # waits for the encoder (they depend on the weights only; with the pipelined
                # optimizer, on the encoder convs' deferred update issued on the side stream)
                if enc_adam_done is not None:
                    main.wait_event(enc_adam_done)
                self._flip_conv_weights()
                self._wflip_ready = True
            self._pad_heads_weights()   # (also while the main stream waits for the encoder)
            main.wait_stream(side)   # layer 0's memory K/V, before layer 0's cross-attention
            if parts is not None:
                ops.adam_gate(self.adam_gate, self.step_t)   # both halves of the deferred Adam have read it
            if c_ndec > 1:
                ws, self.ws = self.ws, self._side_ws
                try:
                    with torch.cuda.stream(side):   # layers 1..'s memory K/V beside decoder layer 0
                        self.forward_memory_kv(A, 1)
                finally:
                    self.ws = ws
            next(dec, None)          # decoder layer 0 and layer 1's self-attention block (or all of
            main.wait_stream(side)   # a one-layer decoder)
            for _ in dec:
                pass
        else:
            if parts is not None:
                self._adam(0, self.lay.numel, parts, gated=True)
                ops.adam_gate(self.adam_gate, self.step_t)
            self.forward_encoder(A)
            for _ in self._decoder_steps(A):
                pass
        self._count_batches()

    def _count_batches(self):
        if self.training:
            for k in self.nbt:
                self.nbt[k] += 1

    @ranged("tt2.encoder")
    def forward_encoder(self, A: Arena):
        """Encoder pre-net + layers, then the K/V projection of the memory for
        all decoder layers (A["mkv"])."""
        self.forward_encoder_prenet(A)
        self.forward_encoder_layers(A)

    def forward_encoder_prenet(self, A: Arena):
        """Embedding, 3 x (conv + BatchNorm + ReLU + dropout), projection, scaled PE -> A["ex0"]."""
        c = self.cfg
        B, Tx, Me = A.B, A.Tx, A.Me
        d, F, H, K = c.d_model, c.d_ffn, c.n_heads, c.enc_conv_kernel
        pad = (K - 1) // 2
        tr = self.training
        scale = 1.0 / math.sqrt(c.head_dim)
        # ---------------- encoder pre-net
        ops.embedding_fwd(A["text"], self.W("enc.embed"), A["emb"], Me, c.vocab)
        x = A["emb"]
        for i in range(c.enc_conv_layers):
            y = A[f"ecv_y{i}"]
            conv = dict(bias=self.P(f"enc.conv{i}.b"), ldx=d, a_conv=(Tx, d, pad))
            st = self._fused_stats(tr, A[f"ecv_part{i}"], x, self.W(f"enc.conv{i}.w"), y, Me, d, K * d, **conv)
            self._lin(x, self.W(f"enc.conv{i}.w"), y, Me, d, K * d, **conv,
                      **({"col_stats": st[0]} if st is not None else {}))
            ops.batchnorm_fwd(y, self.P(f"enc.bn{i}.g"), self.P(f"enc.bn{i}.b"), A[f"ecv_mean{i}"],
                              A[f"ecv_rstd{i}"], self.S(f"enc.bn{i}.rm"), self.S(f"enc.bn{i}.rv"), A[f"ecv_o{i}"],
                              Me, d, ACT_RELU, tr, drop=self.drop(SITE_ENC_CONV + i, c.prenet_dropout),
                              eps=c.bn_eps, momentum=c.bn_momentum, ws=self.ws, sync=self.bn_sync, stats=st)
            x = A[f"ecv_o{i}"]
        self._lin(x, self.W("enc.proj.w"), A["eproj"], Me, d, d, bias=self.P("enc.proj.b"))
        ops.posenc_fwd(A["eproj"], self.P("enc.alpha"), self.pe, A["ex0"], Me, Tx,
                       drop=self.drop(SITE_ENC_PE, c.dropout))

    def forward_encoder_layers(self, A: Arena, rest_kv_later: bool = False):
        """The encoder layers on A["ex0"], then the memory's K/V projection (A["mkv"]); with
        rest_kv_later only layer 0's part (the caller issues forward_memory_kv(A, 1))."""
        c = self.cfg
        B, Tx, Me = A.B, A.Tx, A.Me
        d, F, H = c.d_model, c.d_ffn, c.n_heads
        scale = 1.0 / math.sqrt(c.head_dim)
        x = A["ex0"]
        # ---------------- encoder layers
        for l in range(c.n_enc):
            p, base = f"enc{l}.", SITE_ENC_LAYER + 4 * l
            qkv = A[f"eqkv{l}"]
            self._lin(x, self.W(p + "qkv.w"), qkv, Me, 3 * d, d, bias=self.P(p + "qkv.b"))
            ops.attn_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], A[f"eatt{l}"], A[f"else{l}"], 3 * d, 3 * d, 3 * d, d,
                         B, H, Tx, Tx, A["text_len"], False, scale)
            self._lin(A[f"eatt{l}"], self.W(p + "o.w"), A[f"eo{l}"], Me, d, d, bias=self.P(p + "o.b"))
            ops.layernorm_fwd(x, A[f"eo{l}"], self.P(p + "ln1.g"), self.P(p + "ln1.b"), A[f"eh1{l}"],
                              A[f"eln1m{l}"], A[f"eln1r{l}"], Me, c.ln_eps, drop=self.drop(base, c.dropout))
            h1 = A[f"eh1{l}"]
            self._lin(h1, self.W(p + "ffn1.w"), A[f"ef1{l}"], Me, F, d, bias=self.P(p + "ffn1.b"), act=ACT_RELU,
                      drop=self.drop(base + 1, c.dropout))
            self._lin(A[f"ef1{l}"], self.W(p + "ffn2.w"), A[f"ef2{l}"], Me, d, F, bias=self.P(p + "ffn2.b"))
            ops.layernorm_fwd(h1, A[f"ef2{l}"], self.P(p + "ln2.g"), self.P(p + "ln2.b"), A[f"ex{l + 1}"],
                              A[f"eln2m{l}"], A[f"eln2r{l}"], Me, c.ln_eps, drop=self.drop(base + 2, c.dropout))
            x = A[f"ex{l + 1}"]
        self.forward_memory_kv(A, 0)
        if not rest_kv_later:
            self.forward_memory_kv(A, 1)

    def forward_memory_kv(self, A: Arena, part: int):
        """The memory's K/V projection for the decoder layers' cross-attention, as two GEMMs into
        A["mkv"] [Me, n_dec * 1024]: part 0 = layer 0's K/V, which decoder layer 0 waits for;
        part 1 = layers 1.., which the overlapped forward issues after layer 0 can start (it runs
        beside the decoder's layer 0).  Every schedule uses the same two GEMMs (identical bits)."""
        c = self.cfg
        d, Me = c.d_model, A.Me
        kvld, w, b = c.n_dec * 2 * d, self.W("dec.kv.w"), self.P("dec.kv.b")
        lo, hi = (0, 2 * d) if part == 0 else (2 * d, kvld)
        if hi <= lo:   # a one-layer decoder has no part 1
            return
        self._lin(A[f"ex{c.n_enc}"], w[lo:hi], A["mkv"][:, lo:], Me, hi - lo, d, bias=b[lo:hi], ldo=kvld)

    @ranged("tt2.decoder")
    def forward_decoder(self, A: Arena):
        for _ in self._decoder_steps(A):
            pass

    def _decoder_steps(self, A: Arena):
        """The decoder forward as a generator: it yields once, right before the first use of
        the encoder memory (layer 0's cross-attention), so forward() can overlap what comes
        before it with the encoder."""
        c = self.cfg
        B, Tx, Ty, Md = A.B, A.Tx, A.Ty, A.Md
        d, F, H = c.d_model, c.d_ffn, c.n_heads
        tr = self.training
        scale = 1.0 / math.sqrt(c.head_dim)
        # ---------------- decoder pre-net
        ops.shift_right(A["mel"], A["din"], B, Ty, c.n_mels)
        self._lin(A["din"], self.W("dec.fc1.w"), A["dp1"], Md, c.dec_prenet, c.n_mels, bias=self.P("dec.fc1.b"),
                  act=ACT_RELU, drop=self.drop(SITE_DEC_FC1, c.prenet_dropout))
        self._lin(A["dp1"], self.W("dec.fc2.w"), A["dp2"], Md, c.dec_prenet, c.dec_prenet,
                  bias=self.P("dec.fc2.b"), act=ACT_RELU, drop=self.drop(SITE_DEC_FC2, c.prenet_dropout))
        self._lin(A["dp2"], self.W("dec.proj.w"), A["dproj"], Md, d, c.dec_prenet, bias=self.P("dec.proj.b"))
        ops.posenc_fwd(A["dproj"], self.P("dec.alpha"), self.pe, A["dx0"], Md, Ty,
                       drop=self.drop(SITE_DEC_PE, c.dropout))
        x = A["dx0"]
        mkv = A["mkv"]
        kvld = c.n_dec * 2 * d
        # ---------------- decoder layers
        for l in range(c.n_dec):
            p, base = f"dec{l}.", SITE_DEC_LAYER + 4 * l
            qkv = A[f"dqkv{l}"]
            self._lin(x, self.W(p + "qkv.w"), qkv, Md, 3 * d, d, bias=self.P(p + "qkv.b"))
            ops.attn_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], A[f"datt{l}"], A[f"dlse{l}"], 3 * d, 3 * d, 3 * d, d,
                         B, H, Ty, Ty, A["mel_len"], True, scale)
            self._lin(A[f"datt{l}"], self.W(p + "o.w"), A[f"do{l}"], Md, d, d, bias=self.P(p + "o.b"))
            ops.layernorm_fwd(x, A[f"do{l}"], self.P(p + "ln1.g"), self.P(p + "ln1.b"), A[f"dh1{l}"],
                              A[f"dln1m{l}"], A[f"dln1r{l}"], Md, c.ln_eps, drop=self.drop(base, c.dropout))
            h1 = A[f"dh1{l}"]
            self._lin(h1, self.W(p + "cq.w"), A[f"dcq{l}"], Md, d, d, bias=self.P(p + "cq.b"))
            ko = 2 * d * l
            if l <= 1:
                yield
            ops.attn_fwd(A[f"dcq{l}"], mkv[:, ko:], mkv[:, ko + d:], A[f"dcatt{l}"], A[f"dclse{l}"], d, kvld, kvld,
                         d, B, H, Ty, Tx, A["text_len"], False, scale)
            self._lin(A[f"dcatt{l}"], self.W(p + "co.w"), A[f"dco{l}"], Md, d, d, bias=self.P(p + "co.b"))
            ops.layernorm_fwd(h1, A[f"dco{l}"], self.P(p + "ln2.g"), self.P(p + "ln2.b"), A[f"dh2{l}"],
                              A[f"dln2m{l}"], A[f"dln2r{l}"], Md, c.ln_eps, drop=self.drop(base + 1, c.dropout))
            h2 = A[f"dh2{l}"]
            self._lin(h2, self.W(p + "ffn1.w"), A[f"df1{l}"], Md, F, d, bias=self.P(p + "ffn1.b"), act=ACT_RELU,
                      drop=self.drop(base + 2, c.dropout))
            self._lin(A[f"df1{l}"], self.W(p + "ffn2.w"), A[f"df2{l}"], Md, d, F, bias=self.P(p + "ffn2.b"))
            ops.layernorm_fwd(h2, A[f"df2{l}"], self.P(p + "ln3.g"), self.P(p + "ln3.b"), A[f"dx{l + 1}"],
                              A[f"dln3m{l}"], A[f"dln3r{l}"], Md, c.ln_eps, drop=self.drop(base + 3, c.dropout))
            x = A[f"dx{l + 1}"]
        # ---------------- heads (mel 80 + stop 1 in one GEMM, f32 out)
        nh = c.n_mels + 1
        if self._heads_padded():
            # the head rows padded to 88 (zero rows and bias): 8-column chunks only, 14.0 vs 16.4 us
            # (tools/heads_ab.py); output columns 81..87 are zero, the buffer's padding anyway
            _, _, w_p, b_p = self._pad_heads_weights()
            self._lin(x, w_p, A["heads"], Md, w_p.shape[0], d, bias=b_p, ldo=A.heads_ld)
        else:
            self._lin(x, self.W("heads.w"), A["heads"], Md, nh, d, bias=self.P("heads.b"), ldo=A.heads_ld)
        # ---------------- post-net
        ops.cast2d(A["heads"], A.heads_ld, A["pin"], c.n_mels, Md, c.n_mels)
        self._postnet_fwd(A, A["pin"], A["heads"], A.heads_ld, Md, Ty, tr)

    @ranged("tt2.postnet")
    def _postnet_fwd(self, A, x_in, res, res_ld, Md, Ty, tr):
        c = self.cfg
        chans = postnet_channels(c)
        K = c.postnet_kernel
        pad = (K - 1) // 2
        x = x_in
        nl = c.postnet_layers
        for i in range(nl):
            cin, cout = chans[i], chans[i + 1]
            y = A[f"pcv_y{i}"]
            # training in bf16: the conv GEMM leaves the BatchNorm's column moments from its output
            # tiles, so the statistics pass over y is skipped (_fused_stats)
            conv = dict(bias=self.P(f"post.conv{i}.b"), ldx=cin, a_conv=(Ty, cin, pad))
            st = self._fused_stats(tr, A[f"pcv_part{i}"], x, self.W(f"post.conv{i}.w"), y, Md, cout, K * cin, **conv)
            self._lin(x, self.W(f"post.conv{i}.w"), y, Md, cout, K * cin, **conv,
                      **({"col_stats": st[0]} if st is not None else {}))
            last = i == nl - 1
            out = A["mel_after"] if last else A[f"pcv_o{i}"]
            ops.batchnorm_fwd(y, self.P(f"post.bn{i}.g"), self.P(f"post.bn{i}.b"), A[f"pcv_mean{i}"],
                              A[f"pcv_rstd{i}"], self.S(f"post.bn{i}.rm"), self.S(f"post.bn{i}.rv"), out, Md, cout,
                              ACT_NONE if last else ACT_TANH, tr,
                              drop=self.drop(SITE_POSTNET + i, c.postnet_dropout),
                              res=res if last else None, res_ld=res_ld, eps=c.bn_eps, momentum=c.bn_momentum,
                              ws=self.ws, sync=self.bn_sync, stats=st)
            x = out

    # ------------------------------------------------------------ loss
    @ranged("tt2.loss")
    def loss(self, A: Arena):
        c = self.cfg
        ops.tts_loss(A["heads"], A.heads_ld, A["mel_after"], A["mel"], A["mel_len"], A["loss"], A["g_heads"],
                     A["g_after"], A.B, A.Ty, c.n_mels, c.stop_pos_weight, self.grad_scale, ws=self.ws)

    # ------------------------------------------------------------ backward
    def ready_names(self) -> list[str]:
        """The parameters whose flat offsets the backward reports as final (_ready), in the order
        it reports them: everything at or above each offset is final then.  DP buckets cut at
        these offsets (dist.attach, layer-aligned buckets) become complete as soon as their layer
        is done."""
        c = self.cfg
        return (["post.conv0.w", "heads.w"] + [f"dec{l}.qkv.w" for l in reversed(range(c.n_dec))] + ["dec.fc1.w"] +
                [f"enc{l}.qkv.w" for l in reversed(range(c.n_enc))] + ["enc.embed"])

    def ready_offsets(self) -> list[int]:
        return [self.lay.offset(n) for n in self.ready_names()]

    def _ready(self, name):
        if name not in self._ready_set:
            raise RuntimeError(f"engine._ready({name!r}): not in ready_names() (DP bucket cuts would miss it)")
        if self._jobs is not None:
            # the bucket is final once the queued weight gradients have run: its hook goes
            # with them, in a job ordered after everything the main stream has issued so far
            q, self._wq = self._wq or [], None
            self._push_job(q, ready=[name])
            return
        off = self.lay.offset(name)
        if self.grad_ready_hook is not None:
            self.grad_ready_hook(off)
        self._norm_range(off)

    @ranged("tt2.backward")
    def backward(self, A: Arena):
        c, cd = self.cfg, self.cd
        B, Tx, Ty, Me, Md = A.B, A.Tx, A.Ty, A.Me, A.Md
        d, F, H, K = c.d_model, c.d_ffn, c.n_heads, c.enc_conv_kernel
        pad = (K - 1) // 2
        scale = 1.0 / math.sqrt(c.head_dim)
        gs = lambda p: 1.0 / (1.0 - p) if (self.training and self.dropout_enabled and p > 0) else 1.0  # noqa: E731
        ov = self.wgrad_overlap and cd == torch.bfloat16
        self._norm_pending = None
        self._jobs = self._wq = None   # (a backward that raised leaves no queue behind)
        self._in_scope = False
        self._norm_begin(side=ov and self.grad_ready_hook is None)
        if ov:
            self._ov_begin()
        # a weight-gradient dY buffer: per layer (`key`) when the side stream reads it later
        gbuf = (lambda name, key, shape=None: A.layer_buf(name, key, shape)) if ov else \
            (lambda name, key, shape=None: A[name] if shape is None else A[name].view(-1)[:math.prod(shape)].view(shape))
        if not getattr(self, "_wflip_ready", False):   # (the overlapped forward flipped them)
            self._flip_conv_weights()
        self._wflip_ready = False
        # ---------------- post-net
        chans = postnet_channels(c)
        nl = c.postnet_layers
        g = A["g_after"]
        scratch = [A["g_pa"], A["g_pb"]]
        # the BatchNorm backward statistics of layer i - 1 from the conv dgrad of layer i that
        # produces their dout (_fused_stats; TT2_BN_GEMM_STATS=0: the BN's own pass)
        bstats = None   # (buf, rows) of this layer's sums, when the previous dgrad left them
        for i in reversed(range(nl)):
            cin, cout = chans[i], chans[i + 1]
            last = i == nl - 1
            act = ACT_NONE if last else ACT_TANH
            # BN backward may run in place (g is dead afterwards)
            dyv = gbuf("g_pa", f"p{i}", (Md, cout)) if ov else scratch[i % 2].view(-1)[:Md * cout].view(Md, cout)
            ops.batchnorm_bwd(A[f"pcv_y{i}"], g, self.P(f"post.bn{i}.g"), self.P(f"post.bn{i}.b"),
                              A[f"pcv_mean{i}"], A[f"pcv_rstd{i}"], dyv, self.G(f"post.bn{i}.g"),
                              self.G(f"post.bn{i}.b"), Md, cout, act,
                              drop=self.drop(SITE_POSTNET + i, c.postnet_dropout), ws=self.ws, sync=self.bn_sync,
                              stats=bstats)
            bstats = None
            x_in = A[f"pcv_o{i - 1}"] if i > 0 else A["pin"]
            self._wgrad(dyv, x_in, self.G(f"post.conv{i}.w").view(cout, K * cin), cout, K * cin, Md, ldx=cin,
                        b_conv=(Ty, cin, pad), gb=self.G(f"post.conv{i}.b"))
            wflip = self._wflip(f"post.conv{i}.w", cout, cin, K)
            if i > 0:
                gn = scratch[(i + 1) % 2].view(-1)[:Md * cin].view(Md, cin)
                j, bnb = i - 1, None
                bstats = self._fused_stats(True, A[f"pcv_part{j}"], dyv, wflip, gn, Md, cin, K * cout, ldx=cout,
                                           a_conv=(Ty, cout, pad))   # (the forward's moments are consumed)
                if bstats is not None:
                    bnb = ops.bn_bwd_args(A[f"pcv_y{j}"], self.P(f"post.bn{j}.g"), self.P(f"post.bn{j}.b"),
                                          A[f"pcv_mean{j}"], A[f"pcv_rstd{j}"], Md, cin, ACT_TANH,
                                          self.drop(SITE_POSTNET + j, c.postnet_dropout), bstats)
                self._conv_dgrad(dyv, wflip, gn, Md, cin, cout, K, Ty, bn_bwd=bnb)
                g = gn
            else:
                # d(mel_before) += postnet input gradient (g_heads already holds direct + residual terms)
                self._conv_dgrad(dyv, wflip, A["g_heads"], Md, cin, cout, K, Ty, ldo=A.heads_ld, beta=1.0)
        self._ready("post.conv0.w")
        # ---------------- heads
        nh = c.n_mels + 1
        ops.cast2d(A["g_heads"], A.heads_ld, A["gh_cd"], A.heads_ld, Md, nh)
        x_top = A[f"dx{c.n_dec}"]
        gx, gx2 = A["g_xa"], A["g_xb"]
        if cd == torch.bfloat16 and self.pad_heads:
            # the 81 head rows padded to 88 (gh_cd columns 81.. are zero) so both products take
            # the LDS-DMA kernels instead of the register-staged one (odd inner dimension)
            gw_p, gb_p, w_p, _ = self._pad_heads_weights()   # (this step's forward padded w_p)
            nhp = w_p.shape[0]
            self._wgrad(A["gh_cd"], x_top, gw_p, nhp, d, Md, ldy=A.heads_ld, gb=gb_p, now=True)
            ops.cast2d(gw_p, d, self.G("heads.w"), d, nh, d)
            ops.cast2d(gb_p, nhp, self.G("heads.b"), nh, 1, nh)
            self._dgrad(A["gh_cd"], w_p, gx, Md, d, nhp, ldy=A.heads_ld)
        else:
            self._wgrad(A["gh_cd"], x_top, self.G("heads.w"), nh, d, Md, ldy=A.heads_ld, gb=self.G("heads.b"))
            self._dgrad(A["gh_cd"], self.W("heads.w"), gx, Md, d, nh, ldy=A.heads_ld)
        self._ready("heads.w")
        # ---------------- decoder layers
        mkv = A["mkv"]
        kvld = c.n_dec * 2 * d
        g_mkv = A["g_mkv"]
        self._side_cap = self.side_groups_dec or self.side_groups   # jobs pumped beside the decoder backward
        for l in reversed(range(c.n_dec)):
            p, base = f"dec{l}.", SITE_DEC_LAYER + 4 * l
            if ov and l == self.side_start and not self._side_live:
                self._start_side()   # (dev knob) the side stream starts inside the decoder backward
            x_in = A[f"dx{l}"]
            h1, h2 = A[f"dh1{l}"], A[f"dh2{l}"]
            self._defer_wgrads()
            # LN3 + FFN
            g_br3, g_f1 = gbuf("g_br3", l), gbuf("g_f1", l)
            ln3 = ops.layernorm_bwd(gx, h2, A[f"df2{l}"], self.P(p + "ln3.g"), A[f"dln3m{l}"], A[f"dln3r{l}"],
                                    A["g_res"], g_br3, self.G(p + "ln3.g"), self.G(p + "ln3.b"), Md,
                                    drop=self.drop(base + 3, c.dropout), ws=self.ws, dbias=self.G(p + "ffn2.b"),
                                    **self._ln_defer(0, Md))
            self._wgrad(g_br3, A[f"df1{l}"], self.G(p + "ffn2.w"), d, F, Md)
            if ov:
                self._pump(1)
            self._dgrad(g_br3, self.W(p + "ffn2.w"), g_f1, Md, F, d, gate=A[f"df1{l}"],
                        gate_scale=gs(c.dropout))
            self._wgrad(g_f1, h2, self.G(p + "ffn1.w"), F, d, Md, gb=self.G(p + "ffn1.b"))
            self._dgrad(g_f1, self.W(p + "ffn1.w"), gx2, Md, d, F, res=A["g_res"])
            gx, gx2 = gx2, gx
            # LN2 + cross attention
            g_br2 = gbuf("g_br2", l)
            ln2 = ops.layernorm_bwd(gx, h1, A[f"dco{l}"], self.P(p + "ln2.g"), A[f"dln2m{l}"], A[f"dln2r{l}"],
                                    A["g_res"], g_br2, self.G(p + "ln2.g"), self.G(p + "ln2.b"), Md,
                                    drop=self.drop(base + 1, c.dropout), ws=self.ws, dbias=self.G(p + "co.b"),
                                    **self._ln_defer(1, Md, ln3))
            self._wgrad(g_br2, A[f"dcatt{l}"], self.G(p + "co.w"), d, d, Md)
            if ov:
                self._pump(1)
            self._dgrad(g_br2, self.W(p + "co.w"), A["g_att"], Md, d, d)
            ko = 2 * d * l
            g_cq = gbuf("g_cq", l)
            xargs = (A[f"dcq{l}"], mkv[:, ko:], mkv[:, ko + d:], A[f"dcatt{l}"], A["g_att"], A[f"dclse{l}"],
                     A["delta"], g_cq, g_mkv[:, ko:], g_mkv[:, ko + d:], d, kvld, kvld, d, d, d, kvld, kvld,
                     B, H, Ty, Tx, A["text_len"], False, scale)
            ops.attn_bwd(*xargs)
            self._wgrad(g_cq, h1, self.G(p + "cq.w"), d, d, Md, gb=self.G(p + "cq.b"))
            self._dgrad(g_cq, self.W(p + "cq.w"), gx2, Md, d, d, res=A["g_res"])
            gx, gx2 = gx2, gx
            # LN1 + self attention
            g_br = gbuf("g_br", l)
            ln1 = self._ln_last(gx, x_in, A[f"do{l}"], self.P(p + "ln1.g"), A[f"dln1m{l}"], A[f"dln1r{l}"],
                                A["g_res"], g_br, self.G(p + "ln1.g"), self.G(p + "ln1.b"), Md,
                                drop=self.drop(base, c.dropout), dbias=self.G(p + "o.b"), prev=ln2, slot=0,
                                key=("dec", l))
            self._wgrad(g_br, A[f"datt{l}"], self.G(p + "o.w"), d, d, Md)
            if ov:
                self._pump(1)
            self._dgrad(g_br, self.W(p + "o.w"), A["g_att"], Md, d, d)
            qkv, gq = A[f"dqkv{l}"], gbuf("g_qkv", l)
            ops.attn_bwd(qkv, qkv[:, d:], qkv[:, 2 * d:], A[f"datt{l}"], A["g_att"], A[f"dlse{l}"], A["delta"],
                         gq, gq[:, d:], gq[:, 2 * d:], 3 * d, 3 * d, 3 * d, d, d, 3 * d, 3 * d, 3 * d,
                         B, H, Ty, Ty, A["mel_len"], True, scale)
            self._wgrad(gq, x_in, self.G(p + "qkv.w"), 3 * d, d, Md, gb=self.G(p + "qkv.b"))
            self._dgrad(gq, self.W(p + "qkv.w"), gx2, Md, d, 3 * d, res=A["g_res"])
            gx, gx2 = gx2, gx
            self._flush_wgrads(fin=ln1)
            self._ready(p + "qkv.w")
        # ---------------- decoder pre-net
        g_proj = gbuf("g_br", "pre")
        ops.posenc_bwd(gx, self.pe, g_proj, self.G("dec.alpha"), Md, Ty, drop=self.drop(SITE_DEC_PE, c.dropout),
                       ws=self.ws)
        self._wgrad(g_proj, A["dp2"], self.G("dec.proj.w"), d, c.dec_prenet, Md, gb=self.G("dec.proj.b"))
        self._dgrad(g_proj, self.W("dec.proj.w"), A["g_p2"], Md, c.dec_prenet, d, gate=A["dp2"],
                    gate_scale=gs(c.prenet_dropout))
        self._wgrad(A["g_p2"], A["dp1"], self.G("dec.fc2.w"), c.dec_prenet, c.dec_prenet, Md,
                    gb=self.G("dec.fc2.b"))
        self._dgrad(A["g_p2"], self.W("dec.fc2.w"), A["g_p1"], Md, c.dec_prenet, c.dec_prenet, gate=A["dp1"],
                    gate_scale=gs(c.prenet_dropout))
        self._wgrad(A["g_p1"], A["din"], self.G("dec.fc1.w"), c.dec_prenet, c.n_mels, Md,
                    gb=self.G("dec.fc1.b"))
        # ---------------- memory (all layers' cross K/V)
        mem = A[f"ex{c.n_enc}"]
        self._wgrad(g_mkv, mem, self.G("dec.kv.w"), kvld, d, Me, gb=self.G("dec.kv.b"))
        self._ready("dec.fc1.w")
        gxe = A["g_xa"].view(-1)[:Me * d].view(Me, d)
        gxe2 = A["g_xb"].view(-1)[:Me * d].view(Me, d)
        gres = A["g_res"].view(-1)[:Me * d].view(Me, d)
        gbr = A["g_br"].view(-1)[:Me * d].view(Me, d)
        gbr2 = A["g_br2"].view(-1)[:Me * d].view(Me, d)
        gf1 = A["g_f1"].view(-1)[:Me * F].view(Me, F)
        gatt = A["g_att"].view(-1)[:Me * d].view(Me, d)
        gq = A["g_qkv"].view(-1)[:Me * 3 * d].view(Me, 3 * d)
        self._dgrad(g_mkv, self.W("dec.kv.w"), gxe, Me, d, kvld)
        if ov and not self._side_live:   # the weight gradients queued so far run beside the encoder backward
            self._start_side()
        self._side_cap = self.side_groups
        # ---------------- encoder layers
        for l in reversed(range(c.n_enc)):
            p, base = f"enc{l}.", SITE_ENC_LAYER + 4 * l
            x_in, h1 = A[f"ex{l}"], A[f"eh1{l}"]
            self._defer_wgrads()
            if ov:
                gbr, gbr2 = gbuf("g_br", f"e{l}", (Me, d)), gbuf("g_br2", f"e{l}", (Me, d))
                gf1, gq = gbuf("g_f1", f"e{l}", (Me, F)), gbuf("g_qkv", f"e{l}", (Me, 3 * d))
            ln2 = ops.layernorm_bwd(gxe, h1, A[f"ef2{l}"], self.P(p + "ln2.g"), A[f"eln2m{l}"], A[f"eln2r{l}"],
                                    gres, gbr2, self.G(p + "ln2.g"), self.G(p + "ln2.b"), Me,
                                    drop=self.drop(base + 2, c.dropout), ws=self.ws, dbias=self.G(p + "ffn2.b"),
                                    **self._ln_defer(0, Me))
            self._wgrad(gbr2, A[f"ef1{l}"], self.G(p + "ffn2.w"), d, F, Me)
            if ov:
                self._pump(1)
            self._dgrad(gbr2, self.W(p + "ffn2.w"), gf1, Me, F, d, gate=A[f"ef1{l}"], gate_scale=gs(c.dropout))
            self._wgrad(gf1, h1, self.G(p + "ffn1.w"), F, d, Me, gb=self.G(p + "ffn1.b"))
            self._dgrad(gf1, self.W(p + "ffn1.w"), gxe2, Me, d, F, res=gres)
            if ov:
                self._pump(1)
            gxe, gxe2 = gxe2, gxe
            ln1 = self._ln_last(gxe, x_in, A[f"eo{l}"], self.P(p + "ln1.g"), A[f"eln1m{l}"], A[f"eln1r{l}"], gres,
                                gbr, self.G(p + "ln1.g"), self.G(p + "ln1.b"), Me, drop=self.drop(base, c.dropout),
                                dbias=self.G(p + "o.b"), prev=ln2, slot=1, key=("enc", l))
            self._wgrad(gbr, A[f"eatt{l}"], self.G(p + "o.w"), d, d, Me)
            if ov:
                self._pump(1)
            self._dgrad(gbr, self.W(p + "o.w"), gatt, Me, d, d)
            qkv = A[f"eqkv{l}"]
            ops.attn_bwd(qkv, qkv[:, d:], qkv[:, 2 * d:], A[f"eatt{l}"], gatt, A[f"else{l}"], A["delta"],
                         gq, gq[:, d:], gq[:, 2 * d:], 3 * d, 3 * d, 3 * d, d, d, 3 * d, 3 * d, 3 * d,
                         B, H, Tx, Tx, A["text_len"], False, scale)
            self._wgrad(gq, x_in, self.G(p + "qkv.w"), 3 * d, d, Me, gb=self.G(p + "qkv.b"))
            if ov:
                self._pump(1)
            self._dgrad(gq, self.W(p + "qkv.w"), gxe2, Me, d, 3 * d, res=gres)
            gxe, gxe2 = gxe2, gxe
            self._flush_wgrads(fin=ln1)
            self._ready(p + "qkv.w")
        # ---------------- encoder pre-net
        if ov:
            gbr = gbuf("g_br", "eproj", (Me, d))
        ops.posenc_bwd(gxe, self.pe, gbr, self.G("enc.alpha"), Me, Tx, drop=self.drop(SITE_ENC_PE, c.dropout),
                       ws=self.ws)
        self._wgrad(gbr, A[f"ecv_o{c.enc_conv_layers - 1}"], self.G("enc.proj.w"), d, d, Me,
                    gb=self.G("enc.proj.b"))
        gc = gxe2
        nl_e = c.enc_conv_layers

        def enc_bnb(j, st):   # the BatchNorm backward of pre-net layer j, for the GEMM producing its dout
            if st is None:
                return None
            return ops.bn_bwd_args(A[f"ecv_y{j}"], self.P(f"enc.bn{j}.g"), self.P(f"enc.bn{j}.b"),
                                   A[f"ecv_mean{j}"], A[f"ecv_rstd{j}"], Me, d, ACT_RELU,
                                   self.drop(SITE_ENC_CONV + j, c.prenet_dropout), st)
        bstats = self._fused_stats(True, A[f"ecv_part{nl_e - 1}"], gbr, self.W("enc.proj.w"), gc, Me, d, d,
                                   trans_b=True)
        self._dgrad(gbr, self.W("enc.proj.w"), gc, Me, d, d, bn_bwd=enc_bnb(nl_e - 1, bstats))
        gdy = gres
        for i in reversed(range(nl_e)):
            if ov:
                gdy = gbuf("g_res", f"c{i}", (Me, d))
            ops.batchnorm_bwd(A[f"ecv_y{i}"], gc, self.P(f"enc.bn{i}.g"), self.P(f"enc.bn{i}.b"), A[f"ecv_mean{i}"],
                              A[f"ecv_rstd{i}"], gdy, self.G(f"enc.bn{i}.g"), self.G(f"enc.bn{i}.b"), Me, d,
                              ACT_RELU, drop=self.drop(SITE_ENC_CONV + i, c.prenet_dropout), ws=self.ws,
                              sync=self.bn_sync, stats=bstats)
            bstats = None
            x_in = A[f"ecv_o{i - 1}"] if i > 0 else A["emb"]
            if ov:
                self._pump(1)
            self._wgrad(gdy, x_in, self.G(f"enc.conv{i}.w").view(d, K * d), d, K * d, Me, ldx=d,
                        b_conv=(Tx, d, pad), gb=self.G(f"enc.conv{i}.b"))
            wflip = self._wflip(f"enc.conv{i}.w", d, d, K)
            if i > 0:
                bstats = self._fused_stats(True, A[f"ecv_part{i - 1}"], gdy, wflip, gc, Me, d, K * d, ldx=d,
                                           a_conv=(Tx, d, pad))
            self._conv_dgrad(gdy, wflip, gc, Me, d, d, K, Tx, bn_bwd=enc_bnb(i - 1, bstats) if i > 0 else None)
        ops.embedding_bwd(A["text"], gc, self.G("enc.embed"), Me, c.vocab, pad_idx=0)
        self._ready("enc.embed")
        if ov:
            self._ov_end()
        else:
            self._norm_range(0)
        self._norm_pending = (list(self._norm_ranges), self._norm_side, self._norm_used)

    def _wflip_buf(self, name, cout, cin, K):
        key = ("wflip", name)
        buf = self.__dict__.setdefault("_wflip_bufs", {}).get(key)
        if buf is None:
            buf = torch.empty(cin, K * cout, dtype=self.cd, device=self.dev)
            self._wflip_bufs[key] = buf
        return buf

    def _flip_conv_weights(self):
        """Every conv layer's dgrad weight (tap-flipped, transposed) in one launch at the start
        of the backward; _wflip then hands out the flipped copies (TT2_WFLIP_BATCH=0: one
        launch per layer where it is used, the measurement baseline)."""
        if not self.wflip_batch:
            return
        c = self.cfg
        chans = postnet_channels(c)
        convs = [(f"post.conv{i}.w", chans[i + 1], chans[i], c.postnet_kernel) for i in range(c.postnet_layers)]
        convs += [(f"enc.conv{i}.w", c.d_model, c.d_model, c.enc_conv_kernel) for i in range(c.enc_conv_layers)]
        ops.conv_weight_flip_batch([(self.W(n), self._wflip_buf(n, co, ci, k), co, ci, k) for n, co, ci, k in convs])

    def _wflip(self, name, cout, cin, K):
        buf = self._wflip_buf(name, cout, cin, K)
        if not self.wflip_batch:
            ops.conv_weight_flip(self.W(name), buf, cout, cin, K)
        return buf

    # ------------------------------------------------------------ optimizer
    def init_optimizer(self, **kw):
        self.opt.update(kw)
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.params)
            self.exp_avg_sq = torch.zeros_like(self.params)

    @ranged("tt2.optimizer")
    def optimizer_step(self):
        parts = None
        if self._norm_pending is not None:
            ranges, done, used = self._norm_pending
            self._norm_pending = None
            if not done:   # DP: the gradients are final (all-reduced) only now
                for lo, hi, at, nb in ranges:
                    ops.sumsq_parts(self.grads[lo:hi], self._norm_buf[at:], nb)
            parts = self._norm_buf[:used]
        if self.pipeline_opt:
            # pipelined: this step's Adam runs at the start of the next forward (armed on the
            # device), beside the encoder; only the dropout seed advances now
            if parts is None:
                raise RuntimeError("pipelined optimizer: no clip-norm partial sums (optimizer_step without backward)")
            if self._adam_parts is not None and self._adam_parts.data_ptr() != parts.data_ptr():
                raise RuntimeError("pipelined optimizer: the clip-norm partials moved")
            self._adam_parts = parts
            ops.adam_gate(self.adam_gate, arm=True)
            ops.step_bump(None, self.seed)
            return
        self._adam(0, self.lay.numel, parts)
        ops.step_bump(self.step_t, self.seed)

    def _adam(self, lo, hi, parts, gated: bool = False):
        self._heads_pad_fresh = False
        o = self.opt
        sl = lambda t: t[lo:hi] if t is not None else None   # noqa: E731
        ops.adam_step(sl(self.params), sl(self.grads), sl(self.exp_avg), sl(self.exp_avg_sq), sl(self.shadow),
                      self.step_t, hi - lo, o["lr"], o["beta1"], o["beta2"], o["eps"], o["weight_decay"],
                      o["clip_norm"], o["warmup"], o["noam"], self.cfg.d_model, ws=self.ws, norm_parts=parts,
                      gate=self.adam_gate if gated else None)

    def flush_optimizer(self):
        """Pipelined optimizer: run the pending Adam now (before parameters are read, saved or
        evaluated, or pipelining is switched off).  Gated on the device: with nothing pending
        (never armed, already flushed, or consumed by a replay) the launches change nothing."""
        if self._adam_parts is not None:
            self._adam(0, self.lay.numel, self._adam_parts, gated=True)
            ops.adam_gate(self.adam_gate, self.step_t)

    def drop_pending_update(self):
        """Forget a pending pipelined update (its gradients belong to replaced weights)."""
        self.adam_gate.zero_()

    def _fused_stats(self, on, buf, x, w, out, m, n, k, ldx=None, a_conv=None, trans_b=False, bias=None):
        """(buf, rows) when the GEMM out = x W^T (or its dgrad form, trans_b) can leave a BatchNorm's
        per-chunk statistics of out in buf (bf16, TT2_BN_GEMM_STATS; rows = its tile height), else
        None (the BatchNorm runs its own statistics pass)."""
        if not (on and self.bn_gemm_stats and self.cd == torch.bfloat16):
            return None
        rows = ops.gemm_stats_rows(x, w, out, m, n, k, ldx or k, n if trans_b else k, n, a_conv=a_conv,
                                   trans_b=trans_b, bias=bias)
        return (buf, rows) if rows else None

    def _heads_padded(self) -> bool:
        return self.cd == torch.bfloat16 and self.pad_heads

    def _pad_heads_weights(self):
        """bf16 with pad_heads: the mel + stop head's 81 rows as an 88-row weight / bias (rows 81..
        zero), copied from the parameters once per forward (the backward's products reuse it; the
        weights do not change in between).  Returns (grad w, grad b, w, b) padded buffers."""
        if not self._heads_padded():
            return None
        c, d = self.cfg, self.cfg.d_model
        nh, nhp = c.n_mels + 1, 88
        if self._heads_pad is None:
            z = lambda *s_, dt=torch.float32: torch.zeros(*s_, dtype=dt, device=self.dev)   # noqa: E731
            self._heads_pad = (z(nhp, d), z(nhp), z(nhp, d, dt=self.cd), z(nhp))
        if not self._heads_pad_fresh:   # cleared by forward() and by every parameter update
            _, _, w_p, b_p = self._heads_pad
            ops.cast2d(self.W("heads.w"), d, w_p, d, nh, d)
            ops.cast2d(self.P("heads.b"), nh, b_p, nhp, 1, nh)
            self._heads_pad_fresh = True
        return self._heads_pad

    def _enc_param_ranges(self):
        """Flat ranges the encoder forward reads: the encoder's slots, and the memory K/V
        projection (dec.kv) that the encoder forward applies."""
        L = self.lay
        return [(0, L.offset("dec.fc1.w")), (L.offset("dec.kv.w"), L.offset("dec0.qkv.w"))]
