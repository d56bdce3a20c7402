// decoder.cpp -- the autoregressive decode step composed natively (SURVEY 8(a) a13,
// 8(b) tt2_decode_graph_*): the launch schedule of one frame, its hipGraph capture
// and replay, owned by the library so any host (Python ctypes, C++, JNI / cgo) can
// drive inference through the C ABI alone.
//
// Two schedules over the same kernels:
//  * split (bf16 / f16, batch <= 64, the default): the skinny weight-streaming GEMM
//    carries the KV-cache scatter (QKV projection), the scaled PE (pre-net projection)
//    and the frame emit (heads); the attention launches carry the output projections o / co
//    (one f32 slab per head) and the cross-attention's query projection cq; ffn2 runs split-K
//    into raw f32 slabs; tt2_ln_combine folds each sublayer's slabs with bias + residual
//    into its LayerNorm, except the first post-LN of a layer, which rides in the cross-attention
//    launch's prologue (it feeds that launch's query projection).  7 launches per layer + 4.
//    Schedule 4: the same with each FFN sublayer (FFN1, FFN2 slabs, post-LN) as ONE launch
//    (tt2_ffn_decode, 5 per layer): bit-identical, but measured slower -- its two in-kernel
//    hand-offs between work groups cost more than the two launch boundaries they replace
//    (DESIGN.md section 0.5 item 4).  Schedule 3: split-K without the attention fusions.
//  * plain (f32 parity mode, or batch > 64): one launch per op (GEMM, KV append,
//    LayerNorm, PE, emit), no slabs.
// The step reads the frame index from the device counter d->step and bumps it in the
// emit, so one captured step replays for every frame with no host round trip.  The counter
// saturates at t_max: a replay past it writes no KV-cache row and emits no frame (the
// pe_table must hold t_max + 1 rows, since such a replay still reads row t_max).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstring>
#include <new>

#include "tt2_capi.h"
#include "tt2_internal.h"

namespace {

constexpr int SITE_INFER_FC1 = 128, SITE_INFER_FC2 = 129;
constexpr int HEADS_LD = 96;
#ifndef DEC_SPLIT_F
#define DEC_SPLIT_F 8
#endif
constexpr int SPLIT_O = 4, SPLIT_F = DEC_SPLIT_F;   // FFN2 (512 x 2048) split-K slabs

struct Bufs {
  char *prev, *p1, *p2, *proj, *x0, *xa, *xb, *qkv, *att, *o, *h1, *cq, *catt, *co, *h2, *f1, *f2;
  float* heads;
  float* slab;
  size_t slab_bytes;
  int32_t* emit_done;
  int32_t* ffn_sync;   // tt2_ffn_decode's counters (zeroed by tt2_decode_reset, re-armed by each launch)
  char* cache;
  size_t cache_layer;   // bytes per layer of the KV cache
  size_t total;
};

int esz_of(int dt) { return dt == TT2_DT_F32 ? 4 : 2; }

// Carves the workspace (256-B aligned regions); base == nullptr only sizes it.
Bufs carve(const tt2_decode_desc* d, char* base) {
  Bufs b{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) / 256 * 256;
    return p;
  };
  const size_t e = esz_of(d->dtype), B = d->batch, D = d->d_model;
  b.prev = take(B * d->n_mels * e);
  b.p1 = take(B * d->prenet_dim * e);
  b.p2 = take(B * d->prenet_dim * e);
  char** rows[] = {&b.proj, &b.x0, &b.xa, &b.xb, &b.att, &b.o, &b.h1, &b.cq, &b.catt, &b.co, &b.h2, &b.f2};
  for (char** r : rows) *r = take(B * D * e);
  b.qkv = take(B * 3 * D * e);
  b.f1 = take(B * d->d_ffn * e);
  b.heads = reinterpret_cast<float*>(take(B * HEADS_LD * sizeof(float)));
  b.slab_bytes = (size_t)16 * (B > 32 ? B : 32) * D * sizeof(float);
  b.slab = reinterpret_cast<float*>(take(b.slab_bytes));
  b.emit_done = reinterpret_cast<int32_t*>(take(sizeof(int32_t)));
  b.ffn_sync = reinterpret_cast<int32_t*>(take(TT2_FFN_SYNC_INTS * sizeof(int32_t)));
  b.cache_layer = B * (size_t)d->t_max * 2 * D * e;
  b.cache = take(b.cache_layer * d->n_layers);
  b.total = off;
  return b;
}

bool split_schedule(const tt2_decode_desc* d) {
  const bool half = d->dtype == TT2_DT_BF16 || d->dtype == TT2_DT_F16;
  if (d->schedule == 1) return false;
  if (d->schedule >= 2 && d->schedule <= 4) return true;
  return half && d->batch <= 64;
}

int validate(const tt2_decode_desc* d) {
  if (!d) return tt2_set_error(TT2_E_INVALID, "tt2_decode: null descriptor");
  if (d->batch <= 0 || d->text_len <= 0 || d->t_max <= 0)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: batch, text_len and t_max must be > 0");
  if (d->n_layers <= 0 || d->n_layers > TT2_MAX_DEC_LAYERS)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: 1 <= n_layers <= TT2_MAX_DEC_LAYERS");
  if (d->d_model != 512 || d->n_heads * 64 != d->d_model)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: kernels are built for d_model 512, head_dim 64");
  if (d->n_mels + 1 > HEADS_LD || d->n_mels % 8 || d->prenet_dim % 8 || d->d_ffn % 8)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: n_mels < 96 and n_mels, prenet_dim, d_ffn multiples of 8");
  if (d->dtype != TT2_DT_BF16 && d->dtype != TT2_DT_F16 && d->dtype != TT2_DT_F32)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: dtype");
  const bool split = split_schedule(d);
  if (split && (d->dtype == TT2_DT_F32 || d->batch > 64))
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: the split schedule needs bf16 / f16 and batch <= 64");
  if (!split && d->dtype == TT2_DT_F16)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: f16 runs the split schedule only (batch <= 64)");
  if (!d->mem_kv || !d->text_lens || !d->mel_seq || !d->stop_seq || !d->stop_len || !d->step || !d->seed ||
      !d->pe_table || !d->alpha)
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: null buffer in the descriptor");
  if (!(d->prenet_dropout >= 0.f && d->prenet_dropout < 1.f))
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: prenet_dropout must be in [0, 1)");
  if (!d->workspace || d->ws_bytes < tt2_decode_workspace_size(d))
    return tt2_set_error(TT2_E_INVALID, "tt2_decode: workspace smaller than tt2_decode_workspace_size()");
  return TT2_OK;
}

tt2_gemm_args lin(const void* x, const void* w, void* out, int m, int n, int k, const float* bias, int dt_in,
                  int dt_out) {
  tt2_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.a = x; g.b = w; g.c = out; g.bias = bias;
  g.lda = k; g.ldb = k; g.ldc = n;
  g.m = m; g.n = n; g.k = k;
  g.dtype_in = dt_in; g.dtype_out = dt_out;
  g.alpha = 1.f; g.gate_scale = 1.f; g.drop_scale = 1.f;
  g.splits = 1;
  return g;
}

#define TT2_TRY(x)                        \
  do {                                    \
    const int rc_ = (x);                  \
    if (rc_ != TT2_OK) return rc_;        \
  } while (0)

// One decode step: every launch on stream s (capturable: no allocation, no sync).
int step_launches(const tt2_decode_desc* d, hipStream_t s) {
  const Bufs b = carve(d, reinterpret_cast<char*>(d->workspace));
  const int B = d->batch, D = d->d_model, F = d->d_ffn, H = d->n_heads, P = d->prenet_dim, NM = d->n_mels;
  const int dt = d->dtype;
  const size_t e = esz_of(dt);
  const bool split = split_schedule(d);
  const bool fuse_o = split && d->schedule != 3;   // output projections inside the attention launches
  // schedule 4: the FFN sublayer in one launch (tt2_ffn_decode's shapes; batch <= 64 already)
  const bool fuse_ffn = fuse_o && d->schedule == 4 && D == 512 && F == 2048;
  const float scale = 1.f / std::sqrt((float)(D / H));
  const int64_t kvld = (int64_t)d->n_layers * 2 * D;

  // ---- pre-net on the previous frame (dropout always on when p > 0, as Tacotron2 decodes)
  auto prenet = [&](const void* x, const void* w, const float* bias, void* out, int n, int k, int site) {
    tt2_gemm_args g = lin(x, w, out, B, n, k, bias, dt, dt);
    g.act = 1;
    if (d->prenet_dropout > 0.f) {
      g.drop_seed = d->seed;
      g.drop_site = site;
      g.drop_thr = (uint32_t)(double(d->prenet_dropout) * 4294967296.0);
      g.drop_scale = 1.f / (1.f - d->prenet_dropout);
    }
    return tt2_gemm(&g, s);
  };
  TT2_TRY(prenet(b.prev, d->fc1_w, d->fc1_b, b.p1, P, NM, SITE_INFER_FC1));
  TT2_TRY(prenet(b.p1, d->fc2_w, d->fc2_b, b.p2, P, P, SITE_INFER_FC2));
  if (split) {
    // x0 = proj(p2) + alpha * pe[t]: the scaled PE in the projection's epilogue
    tt2_gemm_args g = lin(b.p2, d->proj_w, b.x0, B, D, P, d->proj_b, dt, dt);
    g.pe_table = d->pe_table; g.pe_alpha = d->alpha; g.pe_t = d->step;
    TT2_TRY(tt2_gemm(&g, s));
  } else {
    tt2_gemm_args g = lin(b.p2, d->proj_w, b.proj, B, D, P, d->proj_b, dt, dt);
    TT2_TRY(tt2_gemm(&g, s));
    tt2_pe_args pa;
    std::memset(&pa, 0, sizeof(pa));
    pa.x = b.proj; pa.out = b.x0; pa.alpha = d->alpha; pa.pe = d->pe_table; pa.t_ptr = d->step;
    pa.m = B; pa.c = D; pa.t = 1; pa.dtype = dt; pa.drop_scale = 1.f;
    TT2_TRY(tt2_posenc_fwd(&pa, s));
  }

  // slab: where the fused output projection writes (one f32 slab per head); ln: the fused
  // residual combine + LayerNorm of the query projection's input (tt2_attn_decode_args.ln_part)
  struct LnIn { const float* part; const float* bias; const float* gamma; const float* beta; void* out; };
  auto attn = [&](const void* q, int64_t q_ld, const void* k, const void* v, int64_t bstride, int64_t ld, int tk,
                  const int32_t* key_len, const int32_t* t_ptr, void* out, const void* wo, float* slab,
                  const void* wq = nullptr, const float* bq = nullptr, const LnIn* ln = nullptr) {
    tt2_attn_decode_args a;
    std::memset(&a, 0, sizeof(a));
    a.q = q; a.k = k; a.v = v; a.out = out;
    a.q_ld = q_ld; a.k_bstride = bstride; a.k_ld = ld; a.v_bstride = bstride; a.v_ld = ld; a.o_ld = D;
    a.key_len = key_len; a.t_ptr = t_ptr;
    a.batch = B; a.heads = H; a.head_dim = D / H; a.tk = tk; a.dtype = dt; a.scale = scale;
    a.stop_len = d->stop_len; a.step = d->step;
    if (wo) {   // split schedule: the output projection rides in the attention launch (one slab per head)
      a.out = nullptr; a.wo = wo; a.wo_ld = D; a.slab = slab;
    }
    if (wq) {   // ... and the query projection (q is then its input row)
      a.wq = wq; a.wq_ld = D; a.bq = bq;
    }
    if (ln) {   // ... whose input row is the previous sublayer's residual combine + LayerNorm
      a.ln_part = ln->part; a.ln_bias = ln->bias; a.ln_gamma = ln->gamma; a.ln_beta = ln->beta;
      a.ln_out = ln->out; a.ln_eps = d->ln_eps;
    }
    return tt2_attn_decode(&a, s);
  };
  // raw split-K partial slabs of x[B, k] W[n, k]^T (no epilogue; tt2_ln_combine folds them)
  auto slabs = [&](const void* x, const void* w, int n, int k, int sp) {
    tt2_gemm_args g = lin(x, w, b.o, B, n, k, nullptr, dt, dt);
    g.splits = sp; g.main_only = 1;
    g.workspace = b.slab; g.ws_bytes = b.slab_bytes;
    return tt2_gemm(&g, s);
  };
  auto layernorm = [&](const void* x, const void* br, const float* gamma, const float* beta, void* y) {
    tt2_ln_args a;
    std::memset(&a, 0, sizeof(a));
    a.x = x; a.branch = br; a.y = y; a.gamma = gamma; a.beta = beta;
    a.m = B; a.c = D; a.dtype = dt; a.eps = d->ln_eps; a.drop_scale = 1.f;
    return tt2_layernorm_fwd(&a, s);
  };

  const char* x = b.x0;
  const char* mkv = reinterpret_cast<const char*>(d->mem_kv);
  for (int l = 0; l < d->n_layers; ++l) {
    const tt2_dec_layer& L = d->layers[l];
    char* cache = b.cache + l * b.cache_layer;
    const int64_t cb = (int64_t)d->t_max * 2 * D;   // cache batch stride (elements)
    char* xn = (x == b.xa) ? b.xb : b.xa;
    // self-attention: QKV projection (+ K/V appended to the cache at row t), attention over 0..t
    {
      tt2_gemm_args g = lin(x, L.qkv_w, b.qkv, B, 3 * D, D, L.qkv_b, dt, dt);
      if (split) {
        g.kv_cache = cache; g.kv_t = d->step; g.kv_col0 = D; g.kv_bstride = cb; g.kv_ld = 2 * D;
      }
      TT2_TRY(tt2_gemm(&g, s));
      if (!split) TT2_TRY(tt2_kv_append(b.qkv + D * e, 3 * D, cache, cb, 2 * D, 2 * D, B, d->step, dt, s));
    }
    // fused schedule: the self-attention's slabs go to slab[0 .. H B D), the cross-attention's
    // (which reads them in its LayerNorm prologue) to slab2 = slab + H B D
    float* slab2 = b.slab + (size_t)H * B * D;
    TT2_TRY(attn(b.qkv, 3 * D, cache, cache + D * e, cb, 2 * D, d->t_max, nullptr, d->step, b.att,
                 fuse_o ? L.o_w : nullptr, b.slab));
    if (split) {
      if (!fuse_o) {
        TT2_TRY(slabs(b.att, L.o_w, D, D, SPLIT_O));
        TT2_TRY(tt2_ln_combine(x, b.slab, SPLIT_O, L.o_b, L.ln1_g, L.ln1_b, b.h1, B, D, d->ln_eps, dt, s));
      }
    } else {
      tt2_gemm_args g = lin(b.att, L.o_w, b.o, B, D, D, L.o_b, dt, dt);
      TT2_TRY(tt2_gemm(&g, s));
      TT2_TRY(layernorm(x, b.o, L.ln1_g, L.ln1_b, b.h1));
    }
    // cross-attention over the cached encoder memory K/V; in the fused schedule its query
    // projection (cq) runs inside the attention launch
    if (!fuse_o) {
      tt2_gemm_args g = lin(b.h1, L.cq_w, b.cq, B, D, D, L.cq_b, dt, dt);
      TT2_TRY(tt2_gemm(&g, s));
    }
    const char* mk = mkv + (size_t)2 * D * l * e;
    if (fuse_o) {   // h1 = LN1(x + o_b + self slabs) in the prologue; q = cq(h1); co slabs to slab2
      const LnIn ln{b.slab, L.o_b, L.ln1_g, L.ln1_b, b.h1};
      TT2_TRY(attn(x, D, mk, mk + D * e, (int64_t)d->text_len * kvld, kvld, d->text_len, d->text_lens, nullptr,
                   b.catt, L.co_w, slab2, L.cq_w, L.cq_b, &ln));
    } else {
      TT2_TRY(attn(b.cq, D, mk, mk + D * e, (int64_t)d->text_len * kvld, kvld, d->text_len, d->text_lens, nullptr,
                   b.catt, nullptr, nullptr));
    }
    if (split) {
      if (!fuse_o) TT2_TRY(slabs(b.catt, L.co_w, D, D, SPLIT_O));
      TT2_TRY(tt2_ln_combine(b.h1, fuse_o ? slab2 : b.slab, fuse_o ? H : SPLIT_O, L.co_b, L.ln2_g, L.ln2_b, b.h2, B,
                             D, d->ln_eps, dt, s));
    } else {
      tt2_gemm_args g = lin(b.catt, L.co_w, b.co, B, D, D, L.co_b, dt, dt);
      TT2_TRY(tt2_gemm(&g, s));
      TT2_TRY(layernorm(b.h1, b.co, L.ln2_g, L.ln2_b, b.h2));
    }
    // FFN
    if (fuse_ffn) {
      tt2_ffn_decode_args fa;
      std::memset(&fa, 0, sizeof(fa));
      fa.x = b.h2; fa.w1 = L.ffn1_w; fa.b1 = L.ffn1_b; fa.w2 = L.ffn2_w; fa.b2 = L.ffn2_b;
      fa.gamma = L.ln3_g; fa.beta = L.ln3_b; fa.hidden = b.f1; fa.slab = b.slab; fa.sync = b.ffn_sync; fa.y = xn;
      fa.m = B; fa.d_model = D; fa.d_ffn = F; fa.dtype = dt; fa.eps = d->ln_eps;
      TT2_TRY(tt2_ffn_decode(&fa, s));
      x = xn;
      continue;
    }
    {
      tt2_gemm_args g = lin(b.h2, L.ffn1_w, b.f1, B, F, D, L.ffn1_b, dt, dt);
      g.act = 1;
      TT2_TRY(tt2_gemm(&g, s));
    }
    if (split) {
      TT2_TRY(slabs(b.f1, L.ffn2_w, D, F, SPLIT_F));
      TT2_TRY(tt2_ln_combine(b.h2, b.slab, SPLIT_F, L.ffn2_b, L.ln3_g, L.ln3_b, xn, B, D, d->ln_eps, dt, s));
    } else {
      tt2_gemm_args g = lin(b.f1, L.ffn2_w, b.f2, B, D, F, L.ffn2_b, dt, dt);
      TT2_TRY(tt2_gemm(&g, s));
      TT2_TRY(layernorm(b.h2, b.f2, L.ln3_g, L.ln3_b, xn));
    }
    x = xn;
  }
  // mel + stop heads (f32), then the frame emit: mel_seq / stop_seq / prev, stop tracking, t += 1
  tt2_gemm_args g = lin(x, d->heads_w, b.heads, B, NM + 1, D, d->heads_b, dt, TT2_DT_F32);
  g.ldc = HEADS_LD;
  if (split) {
    g.emit_mel = d->mel_seq; g.emit_stop = d->stop_seq; g.emit_prev = b.prev; g.emit_t = d->step;
    g.emit_seed = d->seed; g.emit_done = b.emit_done; g.emit_nmels = NM; g.emit_tmax = d->t_max;
    g.emit_stop_bias = d->stop_bias; g.emit_stop_len = d->stop_len; g.emit_stop_thr = d->stop_logit;
    return tt2_gemm(&g, s);
  }
  TT2_TRY(tt2_gemm(&g, s));
  return tt2_decode_emit(b.heads, HEADS_LD, B, NM, d->t_max, d->mel_seq, d->stop_seq, b.prev, dt, d->step, d->seed,
                         d->stop_bias, d->stop_len, d->stop_logit, s);
}

}  // namespace

struct tt2_decode_graph {
  hipGraph_t graph = nullptr;     // one step
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph_n = nullptr;   // `steps` consecutive steps (steps > 1), or none
  hipGraphExec_t exec_n = nullptr;
  int steps = 1;
};

// capture `n` consecutive steps (every per-step value lives on the device: the step counter,
// the seed, the previous frame) as one graph on a private stream ordered after s
static int capture_steps(const tt2_decode_desc* d, int n, hipStream_t s, hipGraph_t* graph, hipGraphExec_t* exec) {
  // capture on a private stream (the caller's may be the legacy default stream, which
  // cannot capture), ordered after the caller's pending work.  Thread-local mode: another
  // thread's HIP calls (e.g. RCCL's watchdog) must not invalidate the capture.
  hipStream_t cs = nullptr;
  hipEvent_t ev = nullptr;
  *graph = nullptr;
  *exec = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ev, s);
  if (e == hipSuccess) e = hipStreamWaitEvent(cs, ev, 0);
  if (e == hipSuccess) e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
  int rc = tt2_check_launch(e, "tt2_decode_graph_create");
  if (rc == TT2_OK) {
    for (int i = 0; i < n && rc == TT2_OK; ++i) rc = step_launches(d, cs);
    const hipError_t ee = hipStreamEndCapture(cs, graph);   // always end a begun capture
    if (rc == TT2_OK) rc = tt2_check_launch(ee, "tt2_decode_graph_create: end capture");
  }
  if (rc == TT2_OK) rc = tt2_check_launch(hipGraphInstantiate(exec, *graph, nullptr, nullptr, 0),
                                          "tt2_decode_graph_create: instantiate");
  if (ev) hipEventDestroy(ev);
  if (cs) hipStreamDestroy(cs);
  if (rc != TT2_OK && *graph) {
    hipGraphDestroy(*graph);
    *graph = nullptr;
  }
  return rc;
}

extern "C" size_t tt2_decode_workspace_size(const tt2_decode_desc* d) {
  if (!d) return 0;
  return carve(d, nullptr).total;
}

extern "C" int tt2_decode_reset(const tt2_decode_desc* d, uint32_t seed0, hipStream_t s) {
  TT2_TRY(validate(d));
  const Bufs b = carve(d, reinterpret_cast<char*>(d->workspace));
  hipError_t e = hipMemsetAsync(d->step, 0, sizeof(int32_t), s);
  if (e == hipSuccess) e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d->seed), (int)seed0, 1, s);
  if (e == hipSuccess) e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d->stop_len), INT_MAX, d->batch, s);
  if (e == hipSuccess) e = hipMemsetAsync(b.prev, 0, (size_t)d->batch * d->n_mels * esz_of(d->dtype), s);
  if (e == hipSuccess) e = hipMemsetAsync(b.emit_done, 0, sizeof(int32_t), s);
  if (e == hipSuccess) e = hipMemsetAsync(b.ffn_sync, 0, TT2_FFN_SYNC_INTS * sizeof(int32_t), s);
  return tt2_check_launch(e, "tt2_decode_reset");
}

extern "C" int tt2_decode_step(const tt2_decode_desc* d, hipStream_t s) {
  TT2_TRY(validate(d));
  return step_launches(d, s);
}

extern "C" int tt2_decode_graph_create_n(const tt2_decode_desc* d, int32_t steps, hipStream_t s,
                                         tt2_decode_graph_t* out) {
  if (!out) return tt2_set_error(TT2_E_INVALID, "tt2_decode_graph_create: null output");
  *out = nullptr;
  if (steps < 1 || steps > 64) return tt2_set_error(TT2_E_INVALID, "tt2_decode_graph_create_n: steps in [1, 64]");
  TT2_TRY(validate(d));
  tt2_decode_graph* g = new (std::nothrow) tt2_decode_graph;
  if (!g) return tt2_set_error(TT2_E_HIP, "tt2_decode_graph_create: out of host memory");
  int rc = capture_steps(d, 1, s, &g->graph, &g->exec);
  if (rc == TT2_OK && steps > 1) {
    rc = capture_steps(d, steps, s, &g->graph_n, &g->exec_n);
    g->steps = steps;
  }
  if (rc != TT2_OK) {
    tt2_decode_graph_destroy(g);
    return rc;
  }
  *out = g;
  return TT2_OK;
}

extern "C" int tt2_decode_graph_create(const tt2_decode_desc* d, hipStream_t s, tt2_decode_graph_t* out) {
  return tt2_decode_graph_create_n(d, 1, s, out);
}

extern "C" int tt2_decode_graph_launch(tt2_decode_graph_t g, int32_t n_steps, hipStream_t s) {
  if (!g || !g->exec) return tt2_set_error(TT2_E_INVALID, "tt2_decode_graph_launch: null graph");
  int i = 0;
  if (g->exec_n)
    for (; i + g->steps <= n_steps; i += g->steps) {
      const hipError_t e = hipGraphLaunch(g->exec_n, s);
      if (e != hipSuccess) return tt2_check_launch(e, "tt2_decode_graph_launch");
    }
  for (; i < n_steps; ++i) {
    const hipError_t e = hipGraphLaunch(g->exec, s);
    if (e != hipSuccess) return tt2_check_launch(e, "tt2_decode_graph_launch");
  }
  return TT2_OK;
}

extern "C" int tt2_decode_graph_destroy(tt2_decode_graph_t g) {
  if (!g) return TT2_OK;
  hipError_t e = hipSuccess;
  if (g->exec_n) e = hipGraphExecDestroy(g->exec_n);
  if (g->graph_n && e == hipSuccess) e = hipGraphDestroy(g->graph_n);
  if (g->exec && e == hipSuccess) e = hipGraphExecDestroy(g->exec);
  if (g->graph && e == hipSuccess) e = hipGraphDestroy(g->graph);
  delete g;
  return tt2_check_launch(e, "tt2_decode_graph_destroy");
}
