"""Thin torch-tensor wrappers over the libtt2 C ABI (no compute in Python).

Every function takes preallocated output tensors and launches on the current
torch stream; nothing here allocates except ``Workspace.get`` outside capture.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib
from ._lib import GemmArgs, check, dt, lib, ptr, stream_ptr

# hipGraph capture mode of the training-step and decode-step graphs.  thread_local: RCCL's
# watchdog thread polls its work events during a capture, which a global-mode capture
# treats as a prohibited call (env TT2_CAPTURE_MODE: an A/B switch).
CAPTURE_MODE = os.environ.get("TT2_CAPTURE_MODE", "thread_local")


def drop_thr(p: float) -> int:
    """floor(p * 2^32) -- identical to the oracle's threshold."""
    return int(p * 4294967296.0) if p > 0 else 0


class Drop:
    """Dropout site descriptor: (device seed tensor uint32[1], site id, p)."""

    __slots__ = ("seed", "site", "p")

    def __init__(self, seed: torch.Tensor | None, site: int, p: float):
        self.seed, self.site, self.p = seed, site, p

    @property
    def active(self) -> bool:
        return self.seed is not None and self.p > 0

    def fields(self):
        if not self.active:
            return None, 0, 0, 1.0
        return self.seed.data_ptr(), self.site, drop_thr(self.p), 1.0 / (1.0 - self.p)


NO_DROP = Drop(None, 0, 0.0)


class Workspace:
    """Grow-only device scratch buffer (size it before graph capture)."""

    def __init__(self):
        self.buf: torch.Tensor | None = None

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.TT2Error("workspace must be sized before graph capture")
            self.buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device="cuda")
        return self.buf


_WS = Workspace()


def gemm_args(a, b, c, m, n, k, lda, ldb, ldc, trans_a=False, trans_b=False, bias=None, res=None, ldr=0,
              gate=None, ldg=0, gate_scale=1.0, alpha=1.0, beta=0.0, act=0, drop: Drop = NO_DROP, splits=1,
              a_conv=None, b_conv=None, ws: Workspace | None = None, variant: int = 0, a_ksum=None,
              a_ksum_beta=0.0, a_ln=None, kv=None, pe=None, emit=None, main_only=False,
              defer_ws: bool = False, col_stats=None, bn_bwd=None) -> GemmArgs:
    """Build the tt2_gemm_args of one request (see tt2_capi.h).  defer_ws: only size the
    split-K workspace (ws_bytes); the caller places it."""
    L = lib()
    g = GemmArgs()
    g.a, g.b, g.c = a.data_ptr(), b.data_ptr(), c.data_ptr()
    g.bias = ptr(bias)
    g.res, g.gate = ptr(res), ptr(gate)
    g.lda, g.ldb, g.ldc, g.ldr, g.ldg = lda, ldb, ldc, ldr, ldg
    g.m, g.n, g.k = m, n, k
    g.dtype_in, g.dtype_out = dt(a), dt(c)
    if b.dtype != a.dtype:
        raise _lib.TT2Error("gemm: A and B dtypes differ")
    g.res_dtype = dt(res) if res is not None else 0
    g.gate_dtype = dt(gate) if gate is not None else 0
    if bias is not None and bias.dtype != torch.float32:
        raise _lib.TT2Error("gemm: bias must be f32")
    g.trans_a, g.trans_b = int(trans_a), int(trans_b)
    g.act = act
    g.alpha, g.beta, g.gate_scale = alpha, beta, gate_scale
    g.drop_seed, g.drop_site, g.drop_thr, g.drop_scale = drop.fields()
    if a_conv is not None:
        g.a_conv_t, g.a_conv_c, g.a_conv_pad = a_conv
    if b_conv is not None:
        g.b_conv_t, g.b_conv_c, g.b_conv_pad = b_conv
    g.kernel_variant = variant
    g.col_stats = ptr(col_stats)
    if bn_bwd is not None:   # a _lib.BnArgs (bn_bwd_args); kept alive on the args for the call
        g.bn_bwd = C.addressof(bn_bwd)
        g._bn_keep = bn_bwd
    g.a_ksum, g.a_ksum_beta = ptr(a_ksum), a_ksum_beta
    if a_ln is not None:
        br, gam, bet, out, eps = a_ln
        g.a_ln_branch, g.a_ln_gamma, g.a_ln_beta, g.a_ln_out, g.a_ln_eps = ptr(br), ptr(gam), ptr(bet), ptr(out), eps
    if kv is not None:
        cache, t_ptr, col0, bstride, ld = kv
        g.kv_cache, g.kv_t, g.kv_col0, g.kv_bstride, g.kv_ld = ptr(cache), ptr(t_ptr), col0, bstride, ld
    if pe is not None:
        table, alpha, t_ptr = pe
        g.pe_table, g.pe_alpha, g.pe_t = ptr(table), ptr(alpha), ptr(t_ptr)
    if emit is not None:
        mel_seq, stop_seq, prev, t_ptr, seed, done, n_mels, t_max = emit
        g.emit_mel, g.emit_stop, g.emit_prev = ptr(mel_seq), ptr(stop_seq), ptr(prev)
        g.emit_t, g.emit_seed, g.emit_done = ptr(t_ptr), ptr(seed), ptr(done)
        g.emit_nmels, g.emit_tmax = n_mels, t_max
    g.splits = max(1, splits)
    g.main_only = int(main_only)   # dev measurement: skip the split-K reduce
    if g.splits > 1:
        need = L.tt2_gemm_workspace_size(C.byref(g))
        g.ws_bytes = need
        if not defer_ws:
            g.workspace = (ws or _WS).get(need).data_ptr()
    return g


def gemm_stats_rows(a, b, c, m, n, k, lda, ldb, ldc, **kw) -> int:
    """Rows per chunk of this request's fused BatchNorm statistics (col_stats / bn_bwd): 64 on
    the 64 x 64 kernel, 256 on the 256 x 128 one, 0 when it cannot fuse them."""
    return int(lib().tt2_gemm_stats_rows(C.byref(gemm_args(a, b, c, m, n, k, lda, ldb, ldc, defer_ws=True, **kw))))


def gemm_algo_bytes(g) -> int:
    """Algorithmic HBM bytes of one GEMM request: each operand once (an implicit-im2col
    operand as its unique sequence rows, not the tap-expanded matrix), C once, and every
    epilogue input once (residual, gate, beta * C, the BatchNorm rows of a bn_bwd epilogue,
    bias)."""
    esz = 2 if g.dtype_in == _lib.DT_BF16 else 4
    sz = lambda d: 2 if d == _lib.DT_BF16 else 4  # noqa: E731
    mn = g.m * g.n
    a_b = esz * g.m * (g.a_conv_c if g.a_conv_t > 0 else g.k)
    b_b = esz * (g.k * g.b_conv_c if g.b_conv_t > 0 else g.n * g.k)
    out = a_b + b_b + sz(g.dtype_out) * mn
    if g.res:
        out += sz(g.res_dtype) * mn
    if g.gate:
        out += sz(g.gate_dtype) * mn
    if g.beta != 0.0:
        out += sz(g.dtype_out) * mn
    if g.bn_bwd:
        out += 2 * mn
    if g.bias:
        out += 4 * g.n
    return out


def gemm(a, b, c, m, n, k, lda, ldb, ldc, **kw):
    """C[m,n] = epi(alpha * sum_k A(m,k) B(n,k)); see tt2_capi.h tt2_gemm_args.
    a_ksum (f32 [m], bf16 trans_a only): a_ksum = a_ksum_beta * a_ksum + sum_k A(m,k).
    a_ln = (branch, gamma, beta, out, eps): multiply LN(A + branch), writing it to out (skinny path).
    kv = (cache, t_ptr, col0, bstride, ld): also store columns >= col0 to the KV cache at step *t_ptr.
    pe = (table, alpha, t_ptr): add alpha * table[*t_ptr] to every output row (skinny path).
    emit = (mel_seq, stop_seq, prev, t_ptr, seed, done, n_mels, t_max): the decode frame emit
    (see tt2_capi.h), which also advances *t_ptr.
    col_stats (f32, 2 * ceil(m / rows) * n, rows = gemm_stats_rows(...)): the stored C's column
    moments per chunk (mean, M2), for batchnorm_fwd(stats=(col_stats, rows)).
    bn_bwd (bn_bwd_args(...)): C is that BatchNorm backward's dout; its per-chunk sums go to the
    args' stats buffer, for batchnorm_bwd(stats=(buf, rows))."""
    L = lib()
    g = gemm_args(a, b, c, m, n, k, lda, ldb, ldc, **kw)
    if PROBE is not None:
        key = ("gemm", L.tt2_gemm_plan(C.byref(g)), g.trans_a, g.trans_b)
        algo_bytes = gemm_algo_bytes(g)
        PROBE.begin()
        check(L.tt2_gemm(C.byref(g), stream_ptr()), "tt2_gemm")
        PROBE.end(key, 2.0 * m * n * k, algo_bytes, [g])
        return c
    check(L.tt2_gemm(C.byref(g), stream_ptr()), "tt2_gemm")
    return c


def gemm_grouped(problems, ws: Workspace | None = None, fin=None, max_groups: int = 0):
    """One tt2_gemm_grouped launch (v7) over up to 8 requests, each a dict of gemm()
    arguments (a, b, c, m, n, k, lda, ldb, ldc + keywords); their split-K slabs get
    disjoint slices of one workspace.  fin: a deferred layernorm_bwd's returned LnArgs,
    completed in the group's reduce launch (tt2_gemm_grouped_fin).  max_groups > 0: at most
    that many work groups walk the items (tt2_gemm_grouped_ex)."""
    L = lib()
    finp = C.addressof(fin) if fin is not None else None
    arr = (GemmArgs * len(problems))()
    offs, total = [], 0
    for i, p in enumerate(problems):
        arr[i] = gemm_args(defer_ws=True, **p)
        offs.append(total)
        total += (arr[i].ws_bytes + 255) // 256 * 256
    if total:
        base = (ws or _WS).get(total).data_ptr()
        for i in range(len(problems)):
            if arr[i].splits > 1:
                arr[i].workspace = base + offs[i]
    if PROBE is not None:
        key = ("gemm_grouped", 13, arr[0].trans_a, arr[0].trans_b)
        flops = sum(2.0 * g.m * g.n * g.k for g in arr)
        ab = sum(gemm_algo_bytes(g) for g in arr)
        PROBE.begin()
        check(L.tt2_gemm_grouped_ex(arr, len(problems), finp, max_groups, stream_ptr()), "tt2_gemm_grouped")
        # work groups of the call, and its kernel dispatches (a capped grid goes out as consecutive
        # launches of at most the cap, rounded down to a multiple of 8: tt2_gemm_grouped_ex)
        items = sum(((g.m + 255) // 256) * ((g.n + 127) // 128) * max(1, g.splits) for g in arr)
        grid = min(items, max(8, max_groups // 8 * 8)) if max_groups > 0 else items
        PROBE.end(key, flops, ab, list(arr), wgs=items, disp=-(-items // grid))
        return
    check(L.tt2_gemm_grouped_ex(arr, len(problems), finp, max_groups, stream_ptr()), "tt2_gemm_grouped")


class LaunchProbe:
    """Times each GEMM's main kernel inside the step with libtt2's launch probe
    (tt2_probe_arm: eager, start / stop events at the kernel's own dispatch and completion,
    as rocprofv3 measures it; eager or captured, the kernel's own wall-clock span); used by
    bench.py for the live per-kernel roofline figure."""

    def __init__(self):
        self.rec = []
        self.wgs = {}    # key -> [work groups of each recorded grouped call]
        self.disp = {}   # key -> [kernel dispatches of each recorded call] (grouped: capped grids)
        self._s = None

    def begin(self):
        self._s = lib().tt2_probe_arm()
        if self._s < 0:
            check(self._s, "tt2_probe_arm")

    def end(self, key, flops, algo_bytes=0, args=None, wgs=None, disp=1):
        if wgs is not None:
            self.wgs.setdefault(key, []).append(wgs)
        self.disp.setdefault(key, []).append(disp)
        e = None
        saved = None
        if args is not None:   # a copy of the launch's tt2_gemm_args (array for a grouped launch)
            saved = (GemmArgs * len(args))()
            for i, g in enumerate(args):
                saved[i] = g
        self.rec.append((key, flops, self._s, e, algo_bytes, saved))

    def summary(self, span: bool = False):
        """{key: [launches, flops, seconds, algorithmic bytes]}.  Seconds are the dispatch
        events' (eager launches), or with `span` the kernels' own wall-clock spans (the only
        record of a launch inside a captured graph; reading one re-arms it for the next
        replay)."""
        torch.cuda.synchronize()
        out = {}
        L = lib()
        for key, flops, slot, _, ab, _ in self.rec:
            ms = L.tt2_probe_span_ms(slot) if span else L.tt2_probe_ms(slot)
            if ms < 0:
                msg = L.tt2_last_error()
                raise _lib.TT2Error(f"launch probe {slot} ({key}) recorded no {'span' if span else 'kernel'}"
                                    f"{' (' + msg.decode() + ')' if msg else ''}")
            d = out.setdefault(key, [0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += flops
            d[2] += ms * 1e-3
            d[3] += ab
        return out

    def close(self):
        lib().tt2_probe_reset()

    def replay_time(self, key, reps: int = 10) -> float:
        """Total device time of this variant's recorded launches, each re-launched
        `reps` times back-to-back between one event pair (amortises the
        per-launch dispatch gap that single-launch brackets include)."""
        L = lib()
        total = 0.0
        for k, _, _, _, _, saved in self.rec:
            if k != key or saved is None:
                continue
            torch.cuda.synchronize()
            for g in saved:
                g.main_only = 1      # the kernel alone (a split-K reduce is a different kernel)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                if len(saved) == 1 and k[0] == "gemm":
                    check(L.tt2_gemm(C.byref(saved[0]), stream_ptr()), "tt2_gemm(replay)")
                else:
                    check(L.tt2_gemm_grouped(saved, len(saved), stream_ptr()), "tt2_gemm_grouped(replay)")
            e.record()
            torch.cuda.synchronize()
            total += s.elapsed_time(e) * 1e-3 / reps
        return total


PROBE: LaunchProbe | None = None


# 0 = auto (v2 register-resident P), 1 = v1 (P through LDS); tests A/B both,
# TT2_ATTN_VARIANT lets bench/profiling runs compare them.
ATTN_VARIANT = int(os.environ.get("TT2_ATTN_VARIANT", "0"))


def _attn_common(q, k, v, q_ld, k_ld, v_ld, batch, heads, tq, tk, key_len, causal, scale):
    a = _lib.AttnArgs()
    a.variant = ATTN_VARIANT
    a.q, a.k, a.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    a.q_ld, a.k_ld, a.v_ld = q_ld, k_ld, v_ld
    if key_len is not None and key_len.dtype != torch.int32:
        raise _lib.TT2Error("attn: key_len must be int32")
    a.key_len = ptr(key_len)
    a.batch, a.heads, a.head_dim, a.tq, a.tk, a.causal = batch, heads, 64, tq, tk, int(causal)
    a.dtype = dt(q)
    a.scale = scale
    return a


def attn_fwd(q, k, v, out, lse, q_ld, k_ld, v_ld, o_ld, batch, heads, tq, tk, key_len=None, causal=False,
             scale=0.125):
    """out[b*tq+t, 64h:64h+64] = softmax(scale q k^T + mask) v ; lse [batch*heads, tq] (log2 domain)."""
    L = lib()
    a = _attn_common(q, k, v, q_ld, k_ld, v_ld, batch, heads, tq, tk, key_len, causal, scale)
    a.o_out, a.o_ld, a.lse = out.data_ptr(), o_ld, lse.data_ptr()
    check(L.tt2_attn_fwd(C.byref(a), stream_ptr()), "tt2_attn_fwd")
    return out


def attn_probs(q, k, lse, probs, q_ld, k_ld, batch, heads, tq, tk, key_len=None, causal=False, scale=0.125):
    """Attention probabilities [B*H, Tq, Tk] f32 of a forward already run (alignment diagnostics)."""
    a = _attn_common(q, k, k, q_ld, k_ld, k_ld, batch, heads, tq, tk, key_len, causal, scale)
    a.lse = lse.data_ptr()
    check(lib().tt2_attn_probs(C.byref(a), probs.data_ptr(), stream_ptr()), "tt2_attn_probs")
    return probs


def attn_bwd(q, k, v, o, dout, lse, delta, dq, dk, dv, q_ld, k_ld, v_ld, o_ld, do_ld, dq_ld, dk_ld, dv_ld,
             batch, heads, tq, tk, key_len=None, causal=False, scale=0.125, parts=0):
    """parts: 0 dQ and dK / dV, 1 dQ only, 2 dK / dV only (non-causal bf16; see tt2_attn_args)."""
    L = lib()
    a = _attn_common(q, k, v, q_ld, k_ld, v_ld, batch, heads, tq, tk, key_len, causal, scale)
    a.parts = parts
    a.o, a.dout, a.o_ld, a.do_ld = o.data_ptr(), dout.data_ptr(), o_ld, do_ld
    a.dq, a.dk, a.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    a.dq_ld, a.dk_ld, a.dv_ld = dq_ld, dk_ld, dv_ld
    a.lse, a.delta = lse.data_ptr(), delta.data_ptr()
    check(L.tt2_attn_bwd(C.byref(a), stream_ptr()), "tt2_attn_bwd")


def _drop_into(s, drop: Drop):
    s.drop_seed, s.drop_site, s.drop_thr, s.drop_scale = drop.fields()


def colsum(x, ld, m, n, dst, beta=0.0, ws: Workspace | None = None):
    """dst[n] (f32) = beta*dst + sum over m rows of x[:, :n]  (bias gradient)."""
    L = lib()
    buf = (ws or _WS).get(L.tt2_colsum_workspace_size(m, n))
    check(L.tt2_colsum(x.data_ptr(), dt(x), ld, m, n, dst.data_ptr(), beta, buf.data_ptr(), buf.numel(),
                       stream_ptr()), "tt2_colsum")


def layernorm_fwd(x, branch, gamma, beta, y, mean, rstd, m, eps=1e-5, drop: Drop = NO_DROP):
    L = lib()
    a = _lib.LnArgs()
    a.x, a.branch, a.y = x.data_ptr(), ptr(branch), y.data_ptr()
    a.gamma, a.beta = gamma.data_ptr(), beta.data_ptr()
    a.mean, a.rstd = ptr(mean), ptr(rstd)
    a.m, a.c, a.dtype, a.eps = m, x.shape[-1], dt(x), eps
    _drop_into(a, drop)
    check(L.tt2_layernorm_fwd(C.byref(a), stream_ptr()), "tt2_layernorm_fwd")


def ln_combine(x, part, splits, bias, gamma, beta, y, m, eps=1e-5):
    """y = LN(x + bias + sum_s part[s]) (decode step; part = a skinny split-K GEMM's slabs)."""
    check(lib().tt2_ln_combine(x.data_ptr(), part.data_ptr(), splits, bias.data_ptr(), gamma.data_ptr(),
                               beta.data_ptr(), y.data_ptr(), m, x.shape[-1], eps, dt(x), stream_ptr()),
          "tt2_ln_combine")


def ffn_decode(x, w1, b1, w2, b2, gamma, beta, hidden, slab, sync, y, m, eps=1e-5, stamps=None):
    """The decode step's FFN sublayer in one launch (tt2_ffn_decode): y = LN(x + b2 + relu(x W1^T +
    b1) W2^T), hidden = relu(x W1^T + b1), slab = the 8 raw FFN2 partial slabs; sync: int32 [2048],
    zero before the first call (each call leaves it zero; sync[1088] != 0 flags a timed-out phase).
    stamps (int64 [256, 8], optional): per-work-group wall-clock stamps (tt2_ffn_decode_stamps)."""
    if sync.dtype != torch.int32 or sync.numel() < 2048:
        raise ValueError("ffn_decode: sync must be an int32 tensor of at least TT2_FFN_SYNC_INTS (2048) words")
    for t in (x, w1, w2, hidden, y, slab):
        if not t.is_contiguous():
            raise ValueError("ffn_decode: x, w1, w2, hidden, slab and y must be contiguous (packed rows)")
    a = _lib.FfnDecodeArgs()
    a.x, a.w1, a.b1, a.w2, a.b2 = x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr()
    a.gamma, a.beta, a.hidden, a.slab = gamma.data_ptr(), beta.data_ptr(), hidden.data_ptr(), slab.data_ptr()
    a.sync, a.y = sync.data_ptr(), y.data_ptr()
    a.m, a.d_model, a.d_ffn, a.dtype, a.eps = m, x.shape[-1], w1.shape[0], dt(x), eps
    if stamps is None:
        check(lib().tt2_ffn_decode(C.byref(a), stream_ptr()), "tt2_ffn_decode")
    else:
        check(lib().tt2_ffn_decode_stamps(C.byref(a), stamps.data_ptr(), stream_ptr()), "tt2_ffn_decode")


def layernorm_bwd(dy, x, branch, gamma, mean, rstd, dx, dbranch, dgamma, dbeta, m, drop: Drop = NO_DROP,
                  ws: Workspace | None = None, dbias=None, part=None, defer=False, prev=None):
    """dx = d(LN)/ds, dbranch = drop-masked dx, gamma/beta grads, and optionally
    dbias = column sums of dbranch (the producing linear layer's bias gradient).

    defer=True leaves dgamma/dbeta/dbias as column partials in `part` (a dedicated uint8
    buffer that nothing else may touch until they are finalized); a later call with
    prev=<the returned args> completes them in its own launch, or layernorm_bwd_finalize
    does.  Returns the call's LnArgs."""
    L = lib()
    a = _lib.LnArgs()
    a.dy, a.x, a.branch = dy.data_ptr(), x.data_ptr(), ptr(branch)
    a.dx, a.dbranch = dx.data_ptr(), ptr(dbranch)
    a.dbias = ptr(dbias)
    a.gamma, a.mean, a.rstd = gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    a.dgamma, a.dbeta = dgamma.data_ptr(), dbeta.data_ptr()
    a.m, a.c, a.dtype = m, x.shape[-1], dt(x)
    _drop_into(a, drop)
    need = L.tt2_layernorm_bwd_workspace_size(C.byref(a))
    if defer and part is None:
        raise ValueError("layernorm_bwd: defer needs a dedicated partials buffer")
    buf = part if part is not None else (ws or _WS).get(need)
    if buf.numel() < need:
        raise ValueError(f"layernorm_bwd: partials buffer {buf.numel()} B < {need} B")
    a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    a.defer_finalize = int(defer)
    a.finalize_prev = C.addressof(prev) if prev is not None and prev.defer_finalize else None
    check(L.tt2_layernorm_bwd(C.byref(a), stream_ptr()), "tt2_layernorm_bwd")
    return a


def layernorm_bwd_workspace_size(m: int, c: int) -> int:
    a = _lib.LnArgs()
    a.m, a.c = m, c
    return lib().tt2_layernorm_bwd_workspace_size(C.byref(a))


def layernorm_bwd_finalize(a):
    """Completes a deferred layernorm_bwd (its returned LnArgs)."""
    check(lib().tt2_layernorm_bwd_finalize(C.byref(a), stream_ptr()), "tt2_layernorm_bwd_finalize")


def _bn(y, gamma, beta, mean, rstd, m, c, act, training, drop, eps, momentum, ws):
    a = _lib.BnArgs()
    a.y, a.gamma, a.beta, a.mean, a.rstd = y.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(), \
        rstd.data_ptr()
    a.m, a.c, a.act, a.dtype, a.training, a.eps, a.momentum = m, c, act, dt(y), int(training), eps, momentum
    _drop_into(a, drop)
    return a


def _bn_sync_into(L, a, sync):
    """SyncBatchNorm exchange buffer of `sync` (tt2/dist.py BnSync: world, rank, buffer(nbytes),
    exchange(tensor)) into the args; returns the slot view that exchange() all-reduces."""
    a.sync_world, a.sync_rank = sync.world, sync.rank
    buf = sync.buffer(L.tt2_batchnorm_sync_size(C.byref(a)))
    a.sync_buf = buf.data_ptr()
    return buf[:sync.world * 3 * a.c]


def batchnorm_fwd(y, gamma, beta, mean, rstd, run_mean, run_var, out, m, c, act, training, drop: Drop = NO_DROP,
                  res=None, res_ld=0, eps=1e-5, momentum=0.1, ws: Workspace | None = None, sync=None, stats=None):
    """sync (training only): SyncBatchNorm over the data-parallel ranks -- the statistics of
    all ranks' rows (tt2_batchnorm_fwd_stats, exchange, tt2_batchnorm_fwd_apply).
    stats = (buf, rows): y's column moments are already in buf, chunks of `rows` rows (the
    producing GEMM's col_stats), so the statistics pass over y is skipped (training only)."""
    L = lib()
    a = _bn(y, gamma, beta, mean, rstd, m, c, act, training, drop, eps, momentum, ws)
    a.run_mean, a.run_var = ptr(run_mean), ptr(run_var)
    a.out, a.out_dtype = out.data_ptr(), dt(out)
    a.res, a.res_dtype, a.res_ld = ptr(res), (dt(res) if res is not None else 0), res_ld
    if stats is not None and training:
        _bn_stats_into(L, a, stats)
    else:
        buf = (ws or _WS).get(L.tt2_batchnorm_workspace_size(C.byref(a)))
        a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    if sync is None or not training:
        check(L.tt2_batchnorm_fwd(C.byref(a), stream_ptr()), "tt2_batchnorm_fwd")
        return
    slots = _bn_sync_into(L, a, sync)
    check(L.tt2_batchnorm_fwd_stats(C.byref(a), stream_ptr()), "tt2_batchnorm_fwd_stats")
    sync.exchange(slots)
    check(L.tt2_batchnorm_fwd_apply(C.byref(a), stream_ptr()), "tt2_batchnorm_fwd_apply")


def _bn_stats_into(L, a, stats):
    sbuf, a.stats_rows = stats
    need = L.tt2_batchnorm_workspace_size(C.byref(a))
    if sbuf.dtype != torch.float32 or sbuf.numel() * 4 < need:
        raise _lib.TT2Error(f"batchnorm: stats buffer needs {need} bytes of f32")
    a.workspace, a.ws_bytes = sbuf.data_ptr(), sbuf.numel() * 4


def bn_bwd_args(y, gamma, beta, mean, rstd, m, c, act, drop: Drop, stats) -> _lib.BnArgs:
    """The BatchNorm backward whose column sums a GEMM producing its dout computes
    (gemm(..., bn_bwd=...)); stats = (buf, rows) as then given to batchnorm_bwd (rows:
    gemm_stats_rows of that GEMM)."""
    L = lib()
    a = _bn(y, gamma, beta, mean, rstd, m, c, act, True, drop, 1e-5, 0.1, None)
    _bn_stats_into(L, a, stats)
    return a


def batchnorm_bwd(y, dout, gamma, beta, mean, rstd, dy, dgamma, dbeta, m, c, act, drop: Drop = NO_DROP,
                  ws: Workspace | None = None, sync=None, stats=None):
    """sync: SyncBatchNorm backward (the column sums over all ranks' rows; dgamma / dbeta
    stay this rank's sums for the gradient all-reduce).
    stats = (buf, rows): the per-chunk column sums are already in buf (the GEMM that produced
    dout, gemm(..., bn_bwd=bn_bwd_args(...))), so the statistics pass is skipped."""
    L = lib()
    a = _bn(y, gamma, beta, mean, rstd, m, c, act, True, drop, 1e-5, 0.1, ws)
    a.dout, a.dout_dtype, a.dy = dout.data_ptr(), dt(dout), dy.data_ptr()
    a.dgamma, a.dbeta = dgamma.data_ptr(), dbeta.data_ptr()
    if stats is not None:
        _bn_stats_into(L, a, stats)
    else:
        buf = (ws or _WS).get(L.tt2_batchnorm_workspace_size(C.byref(a)))
        a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    if sync is None:
        check(L.tt2_batchnorm_bwd(C.byref(a), stream_ptr()), "tt2_batchnorm_bwd")
        return
    slots = _bn_sync_into(L, a, sync)
    check(L.tt2_batchnorm_bwd_stats(C.byref(a), stream_ptr()), "tt2_batchnorm_bwd_stats")
    sync.exchange(slots)
    check(L.tt2_batchnorm_bwd_apply(C.byref(a), stream_ptr()), "tt2_batchnorm_bwd_apply")


def embedding_fwd(ids, table, out, m, vocab):
    check(lib().tt2_embedding_fwd(ids.data_ptr(), table.data_ptr(), out.data_ptr(), m, table.shape[-1], vocab,
                                  dt(table), stream_ptr()), "tt2_embedding_fwd")


def embedding_bwd(ids, dout, dtable, m, vocab, pad_idx=0):
    check(lib().tt2_embedding_bwd(ids.data_ptr(), dout.data_ptr(), dtable.data_ptr(), m, dtable.shape[-1], vocab,
                                  pad_idx, dt(dout), stream_ptr()), "tt2_embedding_bwd")


def posenc_fwd(x, alpha, pe, out, m, t, drop: Drop = NO_DROP, t_offset=0, t_ptr=None):
    a = _lib.PeArgs()
    a.x, a.out, a.alpha, a.pe = x.data_ptr(), out.data_ptr(), alpha.data_ptr(), pe.data_ptr()
    a.t_ptr = ptr(t_ptr)
    a.m, a.c, a.t, a.t_offset, a.dtype = m, x.shape[-1], t, t_offset, dt(x)
    _drop_into(a, drop)
    check(lib().tt2_posenc_fwd(C.byref(a), stream_ptr()), "tt2_posenc_fwd")


def posenc_bwd(dout, pe, dx, dalpha, m, t, drop: Drop = NO_DROP, ws: Workspace | None = None):
    L = lib()
    a = _lib.PeArgs()
    a.dout, a.dx, a.pe, a.dalpha = dout.data_ptr(), dx.data_ptr(), pe.data_ptr(), dalpha.data_ptr()
    a.m, a.c, a.t, a.dtype = m, dout.shape[-1], t, dt(dout)
    _drop_into(a, drop)
    buf = (ws or _WS).get(L.tt2_posenc_bwd_workspace_size())
    a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    check(L.tt2_posenc_bwd(C.byref(a), stream_ptr()), "tt2_posenc_bwd")


def shift_right(mel, out, batch, t, c):
    check(lib().tt2_shift_right(mel.data_ptr(), out.data_ptr(), batch, t, c, dt(out), stream_ptr()),
          "tt2_shift_right")


def cast2d(src, src_ld, dst, dst_ld, m, n):
    check(lib().tt2_cast2d(src.data_ptr(), dt(src), src_ld, dst.data_ptr(), dt(dst), dst_ld, m, n, stream_ptr()),
          "tt2_cast2d")


def tts_loss(heads, heads_ld, mel_after, target, mel_len, loss_out, g_heads, g_after, batch, t, n_mels,
             pos_weight=5.0, grad_scale=1.0, ws: Workspace | None = None, separate_grads=False):
    L = lib()
    a = _lib.LossArgs()
    a.separate_grads = int(separate_grads)
    a.heads, a.mel_after, a.target, a.mel_len = heads.data_ptr(), mel_after.data_ptr(), target.data_ptr(), \
        mel_len.data_ptr()
    a.loss_out, a.g_heads, a.g_after = loss_out.data_ptr(), g_heads.data_ptr(), g_after.data_ptr()
    a.heads_ld, a.batch, a.t, a.n_mels, a.grad_dtype = heads_ld, batch, t, n_mels, dt(g_after)
    a.pos_weight, a.grad_scale = pos_weight, grad_scale
    buf = (ws or _WS).get(L.tt2_loss_workspace_size())
    a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    check(L.tt2_tts_loss(C.byref(a), stream_ptr()), "tt2_tts_loss")


def conv_weight_flip_batch(jobs):
    """One launch flipping every (w, wd, cout, cin, k) of `jobs` (<= 16; same dtype)."""
    if not jobs:
        return
    arr = (_lib.WflipJob * len(jobs))()
    for a, (w, wd, cout, cin, k) in zip(arr, jobs):
        a.w, a.wd, a.cout, a.cin, a.k = w.data_ptr(), wd.data_ptr(), cout, cin, k
    check(lib().tt2_conv_weight_flip_batch(arr, len(jobs), dt(jobs[0][0]), stream_ptr()),
          "tt2_conv_weight_flip_batch")


def conv_weight_flip(w, wd, cout, cin, k):
    check(lib().tt2_conv_weight_flip(w.data_ptr(), wd.data_ptr(), cout, cin, k, dt(w), stream_ptr()),
          "tt2_conv_weight_flip")


def sumsq_parts(g: torch.Tensor, parts: torch.Tensor, nparts: int):
    """parts[:nparts] = partial sums of g**2 (f32, fixed split), for adam_step(norm_parts=)."""
    check(lib().tt2_sumsq_parts(g.data_ptr(), g.numel(), parts.data_ptr(), nparts, stream_ptr()), "tt2_sumsq_parts")


def adam_step(params, grads, m, v, shadow, step, n, lr, beta1=0.9, beta2=0.98, eps=1e-9, weight_decay=0.0,
              clip_norm=1.0, warmup=4000.0, noam=True, d_model=512, ws: Workspace | None = None,
              norm_parts: torch.Tensor | None = None, gate: torch.Tensor | None = None):
    """norm_parts: the squared-norm partial sums of every gradient (sumsq_parts over ranges
    covering grads), so the clip needs no pass of its own over the gradients.
    gate: int32 device flag; the update runs only while it is non-zero (adam_gate)."""
    L = lib()
    a = _lib.AdamArgs()
    if norm_parts is not None:
        a.norm_parts, a.norm_nparts = norm_parts.data_ptr(), norm_parts.numel()
    a.params, a.grads, a.exp_avg, a.exp_avg_sq = params.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr()
    a.shadow_bf16, a.step, a.n = ptr(shadow), step.data_ptr(), n
    a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = lr, beta1, beta2, eps, weight_decay
    a.clip_norm, a.warmup, a.noam, a.d_model = clip_norm, warmup, int(noam), d_model
    a.gate = ptr(gate)
    buf = (ws or _WS).get(L.tt2_adam_workspace_size())
    a.workspace, a.ws_bytes = buf.data_ptr(), buf.numel()
    check(L.tt2_adam_step(C.byref(a), stream_ptr()), "tt2_adam_step")


def step_bump(step, seed=None):
    check(lib().tt2_step_bump(ptr(step), ptr(seed), stream_ptr()), "tt2_step_bump")


def adam_gate(gate, step=None, arm: bool = False):
    """arm: gate = 1.  Otherwise (consume): if gate != 0, step += 1 and gate = 0."""
    check(lib().tt2_adam_gate(gate.data_ptr(), ptr(step), 1 if arm else 0, stream_ptr()), "tt2_adam_gate")


def attn_decode(q, k, v, out, q_ld, k_bstride, k_ld, v_bstride, v_ld, o_ld, batch, heads, tk, key_len=None,
                t_ptr=None, scale=0.125, stop_len=None, step=None, wo=None, wo_ld=0, slab=None, wq=None, wq_ld=0,
                bq=None, ln=None):
    """One query row per batch element over a key cache (see tt2_attn_decode_args).
    wo / slab: the fused output projection, slab[h, b, :] = o[b, h] @ wo[:, h*64:(h+1)*64]^T (f32).
    wq / bq: the fused query projection, q is then the projection input x and the head's
    query is x[b] @ wq[h*64:(h+1)*64]^T + bq[h*64:(h+1)*64].
    ln = (part, bias, gamma, beta, out, eps): with wq, the projection input row is first
    LN(q[b] + bias + sum of the 8 slabs part[s, b]) (as ln_combine), written to out[b]."""
    a = _lib.AttnDecodeArgs()
    a.wq, a.wq_ld, a.bq = ptr(wq), wq_ld, ptr(bq)
    if ln is not None:
        part, lb, lg, lbe, lo, eps = ln
        a.ln_part, a.ln_bias, a.ln_gamma, a.ln_beta, a.ln_out, a.ln_eps = ptr(part), ptr(lb), ptr(lg), ptr(lbe), \
            ptr(lo), eps
    a.stop_len, a.step = ptr(stop_len), ptr(step)
    a.q, a.k, a.v, a.out = q.data_ptr(), k.data_ptr(), v.data_ptr(), ptr(out)
    a.wo, a.wo_ld, a.slab = ptr(wo), wo_ld, ptr(slab)
    a.q_ld, a.k_bstride, a.k_ld, a.v_bstride, a.v_ld, a.o_ld = q_ld, k_bstride, k_ld, v_bstride, v_ld, o_ld
    a.key_len, a.t_ptr = ptr(key_len), ptr(t_ptr)
    a.batch, a.heads, a.head_dim, a.tk, a.dtype, a.scale = batch, heads, 64, tk, dt(q), scale
    check(lib().tt2_attn_decode(C.byref(a), stream_ptr()), "tt2_attn_decode")


def kv_append(src, src_ld, cache, c_bstride, c_ld, n, batch, t_ptr):
    check(lib().tt2_kv_append(src.data_ptr(), src_ld, cache.data_ptr(), c_bstride, c_ld, n, batch, t_ptr.data_ptr(),
                              dt(src), stream_ptr()), "tt2_kv_append")


def decode_emit(heads, heads_ld, batch, n_mels, t_max, mel_seq, stop_seq, prev, t_ptr, seed=None, stop_bias=None,
                stop_len=None, stop_thr=float("inf")):
    check(lib().tt2_decode_emit(heads.data_ptr(), heads_ld, batch, n_mels, t_max, mel_seq.data_ptr(),
                                stop_seq.data_ptr(), prev.data_ptr(), dt(prev), t_ptr.data_ptr(), ptr(seed),
                                ptr(stop_bias), ptr(stop_len), stop_thr, stream_ptr()), "tt2_decode_emit")
