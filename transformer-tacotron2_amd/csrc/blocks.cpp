// blocks.cpp -- block-level entry points of the C ABI: each block of the
// encoder -> decoder -> post-net path as one call, a fixed sequence of the library's
// kernels (tt2_gemm, tt2_attn_*, tt2_layernorm_*, tt2_batchnorm_*, tt2_tts_loss) on the
// caller's stream.  A host in any language drives a layer with three calls
// (self-attention, cross-attention, FFN sublayers) and owns every buffer.
//
// Each block body runs twice: a dry pass that only sizes its scratch (carve offsets and
// the largest split-K slab any of its GEMMs needs), then the real pass with the slab
// region at the start of the caller's workspace and the scratch buffers after it.  The
// tt2_*_workspace_size functions are the dry pass alone, so sizes and use never drift.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "tt2_capi.h"
#include "tt2_internal.h"

namespace {

constexpr int SEED_SITE_FFN_OUT = 1;   // the FFN's output dropout is site + 1

// Sizing passes run the block body with this stand-in for every pointer argument: optional
// outputs then count as present (the largest scratch), and a dry pass never dereferences it.
void* const kAny = reinterpret_cast<void*>(256);
float* const kAnyF = reinterpret_cast<float*>(256);

struct Ctx {
  const tt2_desc* d;
  hipStream_t s;
  bool dry;
  char* base;       // scratch (after the slab region)
  size_t off;
  float* slab;      // split-K slabs shared by the block's GEMMs (stream-ordered reuse)
  size_t slab_bytes, slab_need;
  void* take(size_t n) {
    void* p = dry ? nullptr : base + off;
    off += (n + 255) / 256 * 256;
    return p;
  }
};

size_t esz(int dt) { return dt == TT2_DT_F32 ? 4 : 2; }

#define TT2_TRY(x)                 \
  do {                             \
    const int rc_ = (x);           \
    if (rc_ != TT2_OK) return rc_; \
  } while (0)

// Dry pass for sizes, then the real pass (see the file comment).
template <class F>
int run_block(const tt2_desc* d, void* ws, size_t ws_bytes, hipStream_t s, size_t* size_out, F&& body) {
  if (!d) return tt2_set_error(TT2_E_INVALID, "tt2 block: null descriptor");
  if (d->dtype != TT2_DT_BF16 && d->dtype != TT2_DT_F32)
    return tt2_set_error(TT2_E_INVALID, "tt2 block: dtype must be TT2_DT_BF16 or TT2_DT_F32");
  Ctx dry{d, s, true, nullptr, 0, nullptr, 0, 0};
  TT2_TRY(body(dry));
  const size_t slab = (dry.slab_need + 255) / 256 * 256, total = slab + dry.off;
  if (size_out) {
    *size_out = total;
    return TT2_OK;
  }
  if (total && (!ws || ws_bytes < total))
    return tt2_set_error(TT2_E_INVALID, "tt2 block: workspace smaller than its tt2_*_workspace_size()");
  Ctx c{d, s, false, reinterpret_cast<char*>(ws) + slab, 0, reinterpret_cast<float*>(ws), slab, 0};
  return body(c);
}

template <class F>
size_t block_size(const tt2_desc* d, F&& body) {
  size_t n = 0;
  return run_block(d, nullptr, 0, nullptr, &n, body) == TT2_OK ? n : 0;
}

// v7 (256 x 128, warp-specialised) takes the GEMM: split-K heuristics follow tt2/engine.py
bool wide(int dt, int m, std::initializer_list<int> inner) {
  if (dt != TT2_DT_BF16 || m <= 32) return false;
  for (int v : inner)
    if (v % 8) return false;
  return true;
}
int act_splits(int m, int n, int k, bool w) {
  if (w) {
    const int tiles = ((m + 255) / 256) * ((n + 127) / 128);
    if (tiles >= 128 || k < 1024 || m <= 32) return 1;
    return std::max(1, std::min({8, 256 / tiles, k / 512}));
  }
  const int tiles = ((m + 127) / 128) * ((n + 127) / 128);
  if (tiles >= 192 || k < 1024 || m <= 32) return 1;
  return std::max(1, std::min({8, 512 / tiles, k / 512}));
}
int w_splits(int n_out, int n_in, int k, bool w) {
  if (w) {
    const int tiles = ((n_out + 255) / 256) * ((n_in + 127) / 128);
    return std::max(1, std::min({16, 256 / tiles, k / 512}));
  }
  const int tiles = ((n_out + 127) / 128) * ((n_in + 127) / 128);
  if (tiles >= 256) return 1;
  return std::max(1, std::min({32, 512 / tiles, k / 256}));
}

tt2_gemm_args gargs(const void* a, const void* b, void* c, int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc,
                    int dt_in, int dt_out) {
  tt2_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.a = a; g.b = b; g.c = c;
  g.m = m; g.n = n; g.k = k;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.dtype_in = dt_in; g.dtype_out = dt_out;
  g.alpha = 1.f; g.gate_scale = 1.f; g.drop_scale = 1.f;
  g.splits = 1;
  return g;
}

int gemm(Ctx& c, tt2_gemm_args g) {
  if (g.splits > 1) {
    const size_t need = tt2_gemm_workspace_size(&g);
    if (c.dry) {
      c.slab_need = std::max(c.slab_need, need);
      return TT2_OK;
    }
    g.workspace = c.slab;
    g.ws_bytes = c.slab_bytes;
  }
  return c.dry ? TT2_OK : tt2_gemm(&g, c.s);
}

void drop_into(const tt2_desc* d, uint32_t site, const uint32_t*& seed, uint32_t& s_site, uint32_t& thr,
               float& scale) {
  seed = nullptr; s_site = 0; thr = 0; scale = 1.f;
  if (!d->training || d->dropout <= 0.f) return;
  seed = d->seed;
  s_site = site;
  thr = (uint32_t)std::min(4294967295.0, double(d->dropout) * 4294967296.0);
  scale = 1.f / (1.f - d->dropout);
}

// y[m, n] = x[m, k] W[n, k]^T (+ bias) (act) (drop)
int linear(Ctx& c, const void* x, int64_t ldx, const void* w, const float* bias, void* y, int64_t ldy, int m, int n,
           int k, int act = 0, uint32_t site = 0, bool use_drop = false, int dt_out = -1) {
  const int dt = c.d->dtype;
  tt2_gemm_args g = gargs(x, w, y, m, n, k, ldx, k, ldy, dt, dt_out < 0 ? dt : dt_out);
  g.bias = bias;
  g.act = act;
  if (use_drop) drop_into(c.d, site, g.drop_seed, g.drop_site, g.drop_thr, g.drop_scale);
  g.splits = act_splits(m, n, k, wide(dt, m, {(int)k}));
  return gemm(c, g);
}

// out[m, n_in] = dy[m, n_out] W[n_out, n_in] (+ beta * out) (* gate != 0 ? gate_scale : 0)
int dgrad(Ctx& c, const void* dy, int64_t ldy, const void* w, void* out, int64_t ldo, int m, int n_in, int n_out,
          float beta = 0.f, const void* gate = nullptr, float gate_scale = 1.f) {
  const int dt = c.d->dtype;
  tt2_gemm_args g = gargs(dy, w, out, m, n_in, n_out, ldy, n_in, ldo, dt, dt);
  g.trans_b = 1;
  g.beta = beta;
  if (gate) {
    g.gate = gate; g.ldg = ldo; g.gate_dtype = dt; g.gate_scale = gate_scale;
  }
  g.splits = act_splits(m, n_in, n_out, wide(dt, m, {n_out, n_in}));
  return gemm(c, g);
}

// gw[n_out, n_in] (f32) = dy[m, n_out]^T x[m, n_in]; gb[n_out] = sum_m dy (optional)
int wgrad(Ctx& c, const void* dy, int64_t ldy, const void* x, int64_t ldx, float* gw, float* gb, int n_out, int n_in,
          int m) {
  const int dt = c.d->dtype;
  tt2_gemm_args g = gargs(dy, x, gw, n_out, n_in, m, ldy, ldx, n_in, dt, TT2_DT_F32);
  g.trans_a = 1; g.trans_b = 1;
  const bool fused = gb && dt == TT2_DT_BF16 && n_out % 8 == 0 && n_in % 8 == 0;
  if (fused) g.a_ksum = gb;
  g.splits = w_splits(n_out, n_in, m, wide(dt, n_out, {n_out, n_in}));
  TT2_TRY(gemm(c, g));
  if (gb && !fused) {
    const size_t need = tt2_colsum_workspace_size(m, n_out);
    void* ws = c.take(need);
    if (!c.dry) TT2_TRY(tt2_colsum(dy, dt, ldy, m, n_out, gb, 0.f, ws, need, c.s));
  }
  return TT2_OK;
}

tt2_ln_args ln_args(const tt2_desc* d, const void* x, const void* branch, const float* g, const float* b, float* mean,
                    float* rstd, uint32_t site) {
  tt2_ln_args a;
  std::memset(&a, 0, sizeof(a));
  a.x = x; a.branch = branch; a.gamma = g; a.beta = b; a.mean = mean; a.rstd = rstd;
  a.m = d->batch * d->tq; a.c = d->d_model; a.dtype = d->dtype; a.eps = d->eps;
  drop_into(d, site, a.drop_seed, a.drop_site, a.drop_thr, a.drop_scale);
  return a;
}

// backward of y = LN(x + drop(branch)): dx, dbranch, dgamma / dbeta (+ the producing linear's bias gradient)
int ln_bwd(Ctx& c, tt2_ln_args a, const void* dy, void* dx, void* dbranch, float* dg, float* db, float* dbias) {
  a.dy = dy; a.dx = dx; a.dbranch = dbranch; a.dgamma = dg; a.dbeta = db; a.dbias = dbias; a.grad_beta = 0.f;
  const size_t need = tt2_layernorm_bwd_workspace_size(&a);
  a.workspace = c.take(need);
  a.ws_bytes = need;
  return c.dry ? TT2_OK : tt2_layernorm_bwd(&a, c.s);
}

// ------------------------------------------------------------ attention sublayer
struct AttnSaved {   // carve of `saved` (same order in fwd and bwd)
  char *q, *kv, *att, *o;
  float *lse, *mean, *rstd;
  size_t total;
};
AttnSaved attn_saved(const tt2_desc* d, char* base) {
  AttnSaved s{};
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + off : nullptr;
    off += (n + 255) / 256 * 256;
    return p;
  };
  const size_t e = esz(d->dtype), D = d->d_model, mq = (size_t)d->batch * d->tq, mk = (size_t)d->batch * d->tk;
  if (d->cross) {
    s.q = take(mq * D * e);
    s.kv = take(mk * 2 * D * e);
  } else {
    s.q = take(mq * 3 * D * e);   // fused [q | k | v] rows
    s.kv = nullptr;
  }
  s.att = take(mq * D * e);
  s.o = take(mq * D * e);
  s.lse = reinterpret_cast<float*>(take((size_t)d->batch * d->n_heads * d->tq * sizeof(float)));
  s.mean = reinterpret_cast<float*>(take(mq * sizeof(float)));
  s.rstd = reinterpret_cast<float*>(take(mq * sizeof(float)));
  s.total = off;
  return s;
}

int attn_check(const tt2_desc* d) {
  if (d->d_model != 512 || d->n_heads * 64 != d->d_model)
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_block: d_model 512 with heads of width 64");
  if (d->batch <= 0 || d->tq <= 0 || (d->cross && d->tk <= 0))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_block: batch, tq (and tk for cross) must be > 0");
  return TT2_OK;
}

tt2_attn_args sdpa_args(const tt2_desc* d, const AttnSaved& s) {
  const int D = d->d_model;
  const size_t e = esz(d->dtype);
  tt2_attn_args a;
  std::memset(&a, 0, sizeof(a));
  const int tk = d->cross ? d->tk : d->tq;
  if (d->cross) {
    a.q = s.q; a.k = s.kv; a.v = s.kv + D * e;
    a.q_ld = D; a.k_ld = 2 * D; a.v_ld = 2 * D;
  } else {
    a.q = s.q; a.k = s.q + D * e; a.v = s.q + 2 * D * e;
    a.q_ld = 3 * D; a.k_ld = 3 * D; a.v_ld = 3 * D;
  }
  a.key_len = d->k_len;
  a.batch = d->batch; a.heads = d->n_heads; a.head_dim = 64; a.tq = d->tq; a.tk = tk;
  a.causal = d->causal; a.dtype = d->dtype; a.scale = 0.125f;
  a.lse = s.lse;
  return a;
}

}  // namespace

extern "C" size_t tt2_attn_block_saved_size(const tt2_desc* d) {
  return d && attn_check(d) == TT2_OK ? attn_saved(d, nullptr).total : 0;
}

static int attn_fwd_body(Ctx& c, const void* x, const void* mem, const void* w_in, const float* b_in,
                         const void* w_out, const float* b_out, const float* ln_g, const float* ln_b, void* y,
                         void* saved) {
  const tt2_desc* d = c.d;
  TT2_TRY(attn_check(d));
  const AttnSaved s = attn_saved(d, reinterpret_cast<char*>(saved));
  const int D = d->d_model, mq = d->batch * d->tq, mk = d->batch * d->tk;
  const size_t e = esz(d->dtype);
  if (d->cross) {
    TT2_TRY(linear(c, x, D, w_in, b_in, s.q, D, mq, D, D));
    TT2_TRY(linear(c, mem, D, reinterpret_cast<const char*>(w_in) + (size_t)D * D * e, b_in + D, s.kv, 2 * D, mk,
                   2 * D, D));
  } else {
    TT2_TRY(linear(c, x, D, w_in, b_in, s.q, 3 * D, mq, 3 * D, D));
  }
  if (!c.dry) {
    tt2_attn_args a = sdpa_args(d, s);
    a.o_out = s.att;
    a.o_ld = D;
    TT2_TRY(tt2_attn_fwd(&a, c.s));
  }
  TT2_TRY(linear(c, s.att, D, w_out, b_out, s.o, D, mq, D, D));
  if (c.dry) return TT2_OK;
  tt2_ln_args la = ln_args(d, x, s.o, ln_g, ln_b, s.mean, s.rstd, d->site);
  la.y = y;
  return tt2_layernorm_fwd(&la, c.s);
}

extern "C" int tt2_attn_block_fwd(const tt2_desc* d, const void* x, const void* mem, const void* w_in,
                                  const float* b_in, const void* w_out, const float* b_out, const float* ln_g,
                                  const float* ln_b, void* y, void* saved, void* workspace, size_t ws_bytes,
                                  hipStream_t stream) {
  if (!x || !w_in || !b_in || !w_out || !b_out || !ln_g || !ln_b || !y || !saved || (d && d->cross && !mem))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_block_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return attn_fwd_body(c, x, mem, w_in, b_in, w_out, b_out, ln_g, ln_b, y, saved);
  });
}

static int attn_bwd_body(Ctx& c, const void* x, const void* mem, const void* w_in, const void* w_out,
                         const float* ln_g, const float* ln_b, const void* saved, const void* dy, void* dx,
                         void* dmem, float* dw_in, float* db_in, float* dw_out, float* db_out, float* dln_g,
                         float* dln_b) {
  const tt2_desc* d = c.d;
  TT2_TRY(attn_check(d));
  const AttnSaved s = attn_saved(d, const_cast<char*>(reinterpret_cast<const char*>(saved)));
  const int D = d->d_model, mq = d->batch * d->tq, mk = d->batch * d->tk;
  const size_t e = esz(d->dtype);
  char* g_br = reinterpret_cast<char*>(c.take((size_t)mq * D * e));
  char* g_att = reinterpret_cast<char*>(c.take((size_t)mq * D * e));
  char* g_q = reinterpret_cast<char*>(c.take((size_t)mq * (d->cross ? 1 : 3) * D * e));
  char* g_kv = d->cross ? reinterpret_cast<char*>(c.take((size_t)mk * 2 * D * e)) : nullptr;
  float* delta = reinterpret_cast<float*>(c.take((size_t)d->batch * d->n_heads * d->tq * sizeof(float)));
  // LN: dx = residual-stream gradient, g_br = drop'(dx); db_out = column sums of g_br
  TT2_TRY(ln_bwd(c, ln_args(d, x, s.o, ln_g, ln_b, s.mean, s.rstd, d->site), dy, dx, g_br, dln_g, dln_b, db_out));
  TT2_TRY(wgrad(c, g_br, D, s.att, D, dw_out, nullptr, D, D, mq));
  TT2_TRY(dgrad(c, g_br, D, w_out, g_att, D, mq, D, D));
  if (!c.dry) {
    tt2_attn_args a = sdpa_args(d, s);
    a.o = s.att; a.o_ld = D; a.dout = g_att; a.do_ld = D; a.delta = delta;
    if (d->cross) {
      a.dq = g_q; a.dq_ld = D; a.dk = g_kv; a.dv = g_kv + D * e; a.dk_ld = 2 * D; a.dv_ld = 2 * D;
    } else {
      a.dq = g_q; a.dk = g_q + D * e; a.dv = g_q + 2 * D * e; a.dq_ld = a.dk_ld = a.dv_ld = 3 * D;
    }
    TT2_TRY(tt2_attn_bwd(&a, c.s));
  }
  if (d->cross) {
    TT2_TRY(wgrad(c, g_q, D, x, D, dw_in, db_in, D, D, mq));
    TT2_TRY(wgrad(c, g_kv, 2 * D, mem, D, dw_in + (size_t)D * D, db_in + D, 2 * D, D, mk));
    TT2_TRY(dgrad(c, g_q, D, w_in, dx, D, mq, D, D, 1.f));
    TT2_TRY(dgrad(c, g_kv, 2 * D, reinterpret_cast<const char*>(w_in) + (size_t)D * D * e, dmem, D, mk, D, 2 * D));
  } else {
    TT2_TRY(wgrad(c, g_q, 3 * D, x, D, dw_in, db_in, 3 * D, D, mq));
    TT2_TRY(dgrad(c, g_q, 3 * D, w_in, dx, D, mq, D, 3 * D, 1.f));
  }
  return TT2_OK;
}

extern "C" size_t tt2_attn_block_workspace_size(const tt2_desc* d) {
  // the larger of the forward's and the backward's needs
  const size_t f = block_size(d, [&](Ctx& c) {
    return attn_fwd_body(c, kAny, kAny, kAny, kAnyF, kAny, kAnyF, kAnyF, kAnyF, kAny, kAny);
  });
  const size_t b = block_size(d, [&](Ctx& c) {
    return attn_bwd_body(c, kAny, kAny, kAny, kAny, kAnyF, kAnyF, kAny, kAny, kAny, kAny, kAnyF, kAnyF, kAnyF,
                         kAnyF, kAnyF, kAnyF);
  });
  return std::max(f, b);
}

extern "C" int tt2_attn_block_bwd(const tt2_desc* d, const void* x, const void* mem, const void* w_in,
                                  const void* w_out, const float* ln_g, const float* ln_b, const void* saved,
                                  const void* dy, void* dx, void* dmem, float* dw_in, float* db_in, float* dw_out,
                                  float* db_out, float* dln_g, float* dln_b, void* workspace, size_t ws_bytes,
                                  hipStream_t stream) {
  if (!x || !w_in || !w_out || !ln_g || !ln_b || !saved || !dy || !dx || !dw_in || !db_in || !dw_out || !db_out ||
      !dln_g || !dln_b || (d && d->cross && (!mem || !dmem)))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_block_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return attn_bwd_body(c, x, mem, w_in, w_out, ln_g, ln_b, saved, dy, dx, dmem, dw_in, db_in, dw_out, db_out,
                         dln_g, dln_b);
  });
}

// ------------------------------------------------------------------ FFN sublayer
namespace {
struct FfnSaved {
  char *h, *f;
  float *mean, *rstd;
  size_t total;
};
FfnSaved ffn_saved(const tt2_desc* d, char* base) {
  FfnSaved s{};
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + off : nullptr;
    off += (n + 255) / 256 * 256;
    return p;
  };
  const size_t e = esz(d->dtype), m = (size_t)d->batch * d->tq;
  s.h = take(m * d->d_ffn * e);
  s.f = take(m * d->d_model * e);
  s.mean = reinterpret_cast<float*>(take(m * sizeof(float)));
  s.rstd = reinterpret_cast<float*>(take(m * sizeof(float)));
  s.total = off;
  return s;
}
int ffn_check(const tt2_desc* d) {
  if (d->d_model != 512 || d->d_ffn <= 0 || d->d_ffn % 8 || d->batch <= 0 || d->tq <= 0)
    return tt2_set_error(TT2_E_INVALID, "tt2_ffn: d_model 512, d_ffn a multiple of 8, batch, tq > 0");
  return TT2_OK;
}
float drop_gate_scale(const tt2_desc* d) { return d->training && d->dropout > 0.f ? 1.f / (1.f - d->dropout) : 1.f; }

int ffn_fwd_body(Ctx& c, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                 const float* ln_g, const float* ln_b, void* y, void* saved) {
  const tt2_desc* d = c.d;
  TT2_TRY(ffn_check(d));
  const FfnSaved s = ffn_saved(d, reinterpret_cast<char*>(saved));
  const int D = d->d_model, F = d->d_ffn, m = d->batch * d->tq;
  TT2_TRY(linear(c, x, D, w1, b1, s.h, F, m, F, D, 1, d->site, true));
  TT2_TRY(linear(c, s.h, F, w2, b2, s.f, D, m, D, F));
  if (c.dry) return TT2_OK;
  tt2_ln_args la = ln_args(d, x, s.f, ln_g, ln_b, s.mean, s.rstd, d->site + SEED_SITE_FFN_OUT);
  la.y = y;
  return tt2_layernorm_fwd(&la, c.s);
}

int ffn_bwd_body(Ctx& c, const void* x, const void* w1, const void* w2, const float* ln_g, const float* ln_b,
                 const void* saved, const void* dy, void* dx, float* dw1, float* db1, float* dw2, float* db2,
                 float* dln_g, float* dln_b) {
  const tt2_desc* d = c.d;
  TT2_TRY(ffn_check(d));
  const FfnSaved s = ffn_saved(d, const_cast<char*>(reinterpret_cast<const char*>(saved)));
  const int D = d->d_model, F = d->d_ffn, m = d->batch * d->tq;
  const size_t e = esz(d->dtype);
  char* g_br = reinterpret_cast<char*>(c.take((size_t)m * D * e));
  char* g_h = reinterpret_cast<char*>(c.take((size_t)m * F * e));
  TT2_TRY(ln_bwd(c, ln_args(d, x, s.f, ln_g, ln_b, s.mean, s.rstd, d->site + SEED_SITE_FFN_OUT), dy, dx, g_br,
                 dln_g, dln_b, db2));
  TT2_TRY(wgrad(c, g_br, D, s.h, F, dw2, nullptr, D, F, m));
  // relu' and the hidden dropout: the saved h is drop(relu(.)), zero exactly where either dropped it
  TT2_TRY(dgrad(c, g_br, D, w2, g_h, F, m, F, D, 0.f, s.h, drop_gate_scale(d)));
  TT2_TRY(wgrad(c, g_h, F, x, D, dw1, db1, F, D, m));
  return dgrad(c, g_h, F, w1, dx, D, m, D, F, 1.f);
}
}  // namespace

extern "C" size_t tt2_ffn_saved_size(const tt2_desc* d) {
  return d && ffn_check(d) == TT2_OK ? ffn_saved(d, nullptr).total : 0;
}
extern "C" size_t tt2_ffn_workspace_size(const tt2_desc* d) {
  const size_t f = block_size(d, [&](Ctx& c) {
    return ffn_fwd_body(c, kAny, kAny, kAnyF, kAny, kAnyF, kAnyF, kAnyF, kAny, kAny);
  });
  const size_t b = block_size(d, [&](Ctx& c) {
    return ffn_bwd_body(c, kAny, kAny, kAny, kAnyF, kAnyF, kAny, kAny, kAny, kAnyF, kAnyF, kAnyF, kAnyF, kAnyF,
                        kAnyF);
  });
  return std::max(f, b);
}
extern "C" int tt2_ffn_fwd(const tt2_desc* d, const void* x, const void* w1, const float* b1, const void* w2,
                           const float* b2, const float* ln_g, const float* ln_b, void* y, void* saved,
                           void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !w1 || !b1 || !w2 || !b2 || !ln_g || !ln_b || !y || !saved)
    return tt2_set_error(TT2_E_INVALID, "tt2_ffn_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr,
                   [&](Ctx& c) { return ffn_fwd_body(c, x, w1, b1, w2, b2, ln_g, ln_b, y, saved); });
}
extern "C" int tt2_ffn_bwd(const tt2_desc* d, const void* x, const void* w1, const void* w2, const float* ln_g,
                           const float* ln_b, const void* saved, const void* dy, void* dx, float* dw1, float* db1,
                           float* dw2, float* db2, float* dln_g, float* dln_b, void* workspace, size_t ws_bytes,
                           hipStream_t stream) {
  if (!x || !w1 || !w2 || !ln_g || !ln_b || !saved || !dy || !dx || !dw1 || !db1 || !dw2 || !db2 || !dln_g || !dln_b)
    return tt2_set_error(TT2_E_INVALID, "tt2_ffn_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return ffn_bwd_body(c, x, w1, w2, ln_g, ln_b, saved, dy, dx, dw1, db1, dw2, db2, dln_g, dln_b);
  });
}

// ------------------------------------------------------------------------ linear
namespace {
int lin_check(const tt2_desc* d) {
  if (d->batch <= 0 || d->tq <= 0 || d->c_in <= 0 || d->c_out <= 0)
    return tt2_set_error(TT2_E_INVALID, "tt2_linear: batch, tq, c_in, c_out must be > 0");
  return TT2_OK;
}
int linear_bwd_body(Ctx& c, const void* x, const void* w, const void* dy, void* dx, float* dw, float* db) {
  const tt2_desc* d = c.d;
  TT2_TRY(lin_check(d));
  const int m = d->batch * d->tq;
  TT2_TRY(wgrad(c, dy, d->c_out, x, d->c_in, dw, db, d->c_out, d->c_in, m));
  return dx ? dgrad(c, dy, d->c_out, w, dx, d->c_in, m, d->c_in, d->c_out) : TT2_OK;
}
}  // namespace

extern "C" size_t tt2_linear_workspace_size(const tt2_desc* d) {
  const size_t f = block_size(d, [&](Ctx& c) {
    TT2_TRY(lin_check(c.d));
    return linear(c, kAny, c.d->c_in, kAny, kAnyF, kAny, c.d->c_out, c.d->batch * c.d->tq, c.d->c_out, c.d->c_in);
  });
  const size_t b = block_size(d, [&](Ctx& c) {
    return linear_bwd_body(c, kAny, kAny, kAny, kAny, kAnyF, kAnyF);
  });
  return std::max(f, b);
}
extern "C" int tt2_linear_fwd(const tt2_desc* d, const void* x, const void* w, const float* b, void* y,
                              void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !w || !y) return tt2_set_error(TT2_E_INVALID, "tt2_linear_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    TT2_TRY(lin_check(c.d));
    return linear(c, x, c.d->c_in, w, b, y, c.d->c_out, c.d->batch * c.d->tq, c.d->c_out, c.d->c_in);
  });
}
extern "C" int tt2_linear_bwd(const tt2_desc* d, const void* x, const void* w, const void* dy, void* dx, float* dw,
                              float* db, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !w || !dy || !dw) return tt2_set_error(TT2_E_INVALID, "tt2_linear_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr,
                   [&](Ctx& c) { return linear_bwd_body(c, x, w, dy, dx, dw, db); });
}

// ----------------------------------------------------------------------- add + LN
extern "C" size_t tt2_add_ln_saved_size(const tt2_desc* d) {
  return d ? 2 * (((size_t)d->batch * d->tq * sizeof(float) + 255) / 256 * 256) : 0;
}
extern "C" size_t tt2_add_ln_workspace_size(const tt2_desc* d) {
  return block_size(d, [&](Ctx& c) {
    return ln_bwd(c, ln_args(c.d, kAny, kAny, kAnyF, kAnyF, kAnyF, kAnyF, 0), kAny, kAny, kAny, kAnyF, kAnyF,
                  nullptr);
  });
}
static void add_ln_stats(const tt2_desc* d, void* saved, float*& mean, float*& rstd) {
  mean = reinterpret_cast<float*>(saved);
  rstd = reinterpret_cast<float*>(reinterpret_cast<char*>(saved) + tt2_add_ln_saved_size(d) / 2);
}
extern "C" int tt2_add_ln_fwd(const tt2_desc* d, const void* x, const void* branch, const float* ln_g,
                              const float* ln_b, void* y, void* saved, hipStream_t stream) {
  if (!d || !x || !ln_g || !ln_b || !y || !saved) return tt2_set_error(TT2_E_INVALID, "tt2_add_ln_fwd: null argument");
  if (d->d_model != 512) return tt2_set_error(TT2_E_INVALID, "tt2_add_ln: d_model must be 512");
  float *mean, *rstd;
  add_ln_stats(d, saved, mean, rstd);
  tt2_ln_args a = ln_args(d, x, branch, ln_g, ln_b, mean, rstd, d->site);
  a.y = y;
  return tt2_layernorm_fwd(&a, stream);
}
extern "C" int tt2_add_ln_bwd(const tt2_desc* d, const void* x, const void* branch, const float* ln_g,
                              const void* saved, const void* dy, void* dx, void* dbranch, float* dln_g, float* dln_b,
                              void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !ln_g || !saved || !dy || !dx || !dln_g || !dln_b || (branch && !dbranch))
    return tt2_set_error(TT2_E_INVALID, "tt2_add_ln_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    if (c.d->d_model != 512) return tt2_set_error(TT2_E_INVALID, "tt2_add_ln: d_model must be 512");
    float *mean, *rstd;
    add_ln_stats(c.d, const_cast<void*>(saved), mean, rstd);
    return ln_bwd(c, ln_args(c.d, x, branch, ln_g, nullptr, mean, rstd, c.d->site), dy, dx, dbranch, dln_g, dln_b,
                  nullptr);
  });
}

// ------------------------------------------------------------ conv1d + BN + act
namespace {
struct ConvSaved {
  char* y;
  float *mean, *rstd;
  size_t total;
};
ConvSaved conv_saved(const tt2_desc* d, char* base) {
  ConvSaved s{};
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + off : nullptr;
    off += (n + 255) / 256 * 256;
    return p;
  };
  s.y = take((size_t)d->batch * d->tq * d->c_out * esz(d->dtype));
  s.mean = reinterpret_cast<float*>(take((size_t)d->c_out * sizeof(float)));
  s.rstd = reinterpret_cast<float*>(take((size_t)d->c_out * sizeof(float)));
  s.total = off;
  return s;
}
int conv_check(const tt2_desc* d) {
  const int e = d->dtype == TT2_DT_F32 ? 4 : 8;
  if (d->batch <= 0 || d->tq <= 0 || d->c_in <= 0 || d->c_out <= 0 || d->kernel <= 0 || d->kernel % 2 == 0 ||
      d->c_in % e || d->c_out % e)
    return tt2_set_error(TT2_E_INVALID, "tt2_conv1d_bn_act: odd kernel, channels multiples of 16 B");
  return TT2_OK;
}
tt2_bn_args bn_args(const tt2_desc* d, const ConvSaved& s, const float* g, const float* b) {
  tt2_bn_args a;
  std::memset(&a, 0, sizeof(a));
  a.y = s.y; a.gamma = g; a.beta = b; a.mean = s.mean; a.rstd = s.rstd;
  a.m = d->batch * d->tq; a.c = d->c_out; a.act = d->act; a.dtype = d->dtype; a.out_dtype = d->dtype;
  a.training = d->training; a.eps = d->eps; a.momentum = d->momentum;
  drop_into(d, d->site, a.drop_seed, a.drop_site, a.drop_thr, a.drop_scale);
  return a;
}
int conv_fwd_body(Ctx& c, const void* x, const void* w, const float* b, const float* bn_g, const float* bn_b,
                  float* run_mean, float* run_var, const void* res, int res_dtype, void* out, void* saved) {
  const tt2_desc* d = c.d;
  TT2_TRY(conv_check(d));
  const ConvSaved s = conv_saved(d, reinterpret_cast<char*>(saved));
  const int m = d->batch * d->tq, K = d->kernel, ci = d->c_in, co = d->c_out;
  tt2_gemm_args g = gargs(x, w, s.y, m, co, K * ci, ci, (int64_t)K * ci, co, d->dtype, d->dtype);
  g.bias = b;
  g.a_conv_t = d->tq; g.a_conv_c = ci; g.a_conv_pad = (K - 1) / 2;
  g.splits = act_splits(m, co, K * ci, wide(d->dtype, m, {K * ci}) && d->tq >= 64 && ci >= 64);
  TT2_TRY(gemm(c, g));
  tt2_bn_args a = bn_args(d, s, bn_g, bn_b);
  a.run_mean = run_mean; a.run_var = run_var; a.out = out;
  a.res = res; a.res_dtype = res_dtype; a.res_ld = co;
  const size_t need = tt2_batchnorm_workspace_size(&a);
  a.workspace = c.take(need);
  a.ws_bytes = need;
  return c.dry ? TT2_OK : tt2_batchnorm_fwd(&a, c.s);
}
int conv_bwd_body(Ctx& c, const void* x, const void* w, const float* bn_g, const float* bn_b, const void* saved,
                  const void* dout, void* dx, float* dw, float* db, float* dbn_g, float* dbn_b) {
  const tt2_desc* d = c.d;
  TT2_TRY(conv_check(d));
  const ConvSaved s = conv_saved(d, const_cast<char*>(reinterpret_cast<const char*>(saved)));
  const int m = d->batch * d->tq, K = d->kernel, ci = d->c_in, co = d->c_out, pad = (K - 1) / 2;
  const size_t e = esz(d->dtype);
  char* gy = reinterpret_cast<char*>(c.take((size_t)m * co * e));
  char* wflip = reinterpret_cast<char*>(c.take((size_t)ci * K * co * e));
  tt2_bn_args a = bn_args(d, s, bn_g, bn_b);
  a.training = 1;
  a.dout = dout; a.dout_dtype = d->dtype; a.dy = gy; a.dgamma = dbn_g; a.dbeta = dbn_b;
  const size_t need = tt2_batchnorm_workspace_size(&a);
  a.workspace = c.take(need);
  a.ws_bytes = need;
  if (!c.dry) TT2_TRY(tt2_batchnorm_bwd(&a, c.s));
  {   // dW [co][K*ci] = gy^T im2col(x)
    tt2_gemm_args g = gargs(gy, x, dw, co, K * ci, m, co, ci, (int64_t)K * ci, d->dtype, TT2_DT_F32);
    g.trans_a = 1; g.trans_b = 1;
    g.b_conv_t = d->tq; g.b_conv_c = ci; g.b_conv_pad = pad;
    const bool fused = db && d->dtype == TT2_DT_BF16 && co % 8 == 0;
    if (fused) g.a_ksum = db;
    g.splits = w_splits(co, K * ci, m, wide(d->dtype, co, {co, K * ci}) && d->tq >= 64 && ci >= 64);
    TT2_TRY(gemm(c, g));
    if (db && !fused) {
      const size_t nc = tt2_colsum_workspace_size(m, co);
      void* ws = c.take(nc);
      if (!c.dry) TT2_TRY(tt2_colsum(gy, d->dtype, co, m, co, db, 0.f, ws, nc, c.s));
    }
  }
  if (!dx) return TT2_OK;
  if (!c.dry) TT2_TRY(tt2_conv_weight_flip(w, wflip, co, ci, K, d->dtype, c.s));
  // dx [m][ci] = im2col(gy) wflip^T, wflip [ci][K*co]
  tt2_gemm_args g = gargs(gy, wflip, dx, m, ci, K * co, co, (int64_t)K * co, ci, d->dtype, d->dtype);
  g.a_conv_t = d->tq; g.a_conv_c = co; g.a_conv_pad = pad;
  g.splits = act_splits(m, ci, K * co, wide(d->dtype, m, {K * co}) && d->tq >= 64 && co >= 64);
  return gemm(c, g);
}
}  // namespace

extern "C" size_t tt2_conv1d_bn_act_saved_size(const tt2_desc* d) {
  return d && conv_check(d) == TT2_OK ? conv_saved(d, nullptr).total : 0;
}
extern "C" size_t tt2_conv1d_bn_act_workspace_size(const tt2_desc* d) {
  const size_t f = block_size(d, [&](Ctx& c) {
    return conv_fwd_body(c, kAny, kAny, kAnyF, kAnyF, kAnyF, kAnyF, kAnyF, kAny, c.d->dtype, kAny, kAny);
  });
  const size_t b = block_size(d, [&](Ctx& c) {
    return conv_bwd_body(c, kAny, kAny, kAnyF, kAnyF, kAny, kAny, kAny, kAnyF, kAnyF, kAnyF, kAnyF);
  });
  return std::max(f, b);
}
extern "C" int tt2_conv1d_bn_act_fwd(const tt2_desc* d, const void* x, const void* w, const float* b,
                                     const float* bn_g, const float* bn_b, float* run_mean, float* run_var,
                                     const void* res, int32_t res_dtype, void* out, void* saved, void* workspace,
                                     size_t ws_bytes, hipStream_t stream) {
  if (!x || !w || !bn_g || !bn_b || !out || !saved || !run_mean || !run_var)
    return tt2_set_error(TT2_E_INVALID, "tt2_conv1d_bn_act_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return conv_fwd_body(c, x, w, b, bn_g, bn_b, run_mean, run_var, res, res_dtype, out, saved);
  });
}
extern "C" int tt2_conv1d_bn_act_bwd(const tt2_desc* d, const void* x, const void* w, const float* bn_g,
                                     const float* bn_b, const void* saved, const void* dout, void* dx, float* dw,
                                     float* db, float* dbn_g, float* dbn_b, void* workspace, size_t ws_bytes,
                                     hipStream_t stream) {
  if (!x || !w || !bn_g || !bn_b || !saved || !dout || !dw || !dbn_g || !dbn_b)
    return tt2_set_error(TT2_E_INVALID, "tt2_conv1d_bn_act_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return conv_bwd_body(c, x, w, bn_g, bn_b, saved, dout, dx, dw, db, dbn_g, dbn_b);
  });
}

// ------------------------------------------------------------------------- heads
namespace {
int heads_check(const tt2_desc* d) {
  if (d->batch <= 0 || d->tq <= 0 || d->n_mels <= 0 || d->heads_ld < d->n_mels + 1 || d->d_model % 8)
    return tt2_set_error(TT2_E_INVALID, "tt2_heads: n_mels > 0, heads_ld >= n_mels + 1");
  return TT2_OK;
}
int heads_bwd_body(Ctx& c, const void* x, const void* w, const float* g_heads, void* dx, float* dw, float* db) {
  const tt2_desc* d = c.d;
  TT2_TRY(heads_check(d));
  const int m = d->batch * d->tq, nh = d->n_mels + 1, D = d->d_model;
  // the f32 head gradient in the compute dtype; its row stride stays heads_ld
  void* gh = c.take((size_t)m * d->heads_ld * esz(d->dtype));
  if (!c.dry) TT2_TRY(tt2_cast2d(g_heads, TT2_DT_F32, d->heads_ld, gh, d->dtype, d->heads_ld, m, nh, c.s));
  TT2_TRY(wgrad(c, gh, d->heads_ld, x, D, dw, db, nh, D, m));
  return dx ? dgrad(c, gh, d->heads_ld, w, dx, D, m, D, nh) : TT2_OK;
}
}  // namespace

extern "C" size_t tt2_heads_workspace_size(const tt2_desc* d) {
  return block_size(d, [&](Ctx& c) {
    return heads_bwd_body(c, kAny, kAny, kAnyF, kAny, kAnyF, kAnyF);
  });
}
extern "C" int tt2_heads_fwd(const tt2_desc* d, const void* x, const void* w, const float* b, float* heads,
                             void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !w || !heads) return tt2_set_error(TT2_E_INVALID, "tt2_heads_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    TT2_TRY(heads_check(c.d));
    return linear(c, x, c.d->d_model, w, b, heads, c.d->heads_ld, c.d->batch * c.d->tq, c.d->n_mels + 1,
                  c.d->d_model, 0, 0, false, TT2_DT_F32);
  });
}
extern "C" int tt2_heads_bwd(const tt2_desc* d, const void* x, const void* w, const float* g_heads, void* dx,
                             float* dw, float* db, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!x || !w || !g_heads || !dw) return tt2_set_error(TT2_E_INVALID, "tt2_heads_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr,
                   [&](Ctx& c) { return heads_bwd_body(c, x, w, g_heads, dx, dw, db); });
}

// -------------------------------------------------------------------------- loss
namespace {
int loss_body(Ctx& c, const float* heads, const float* mel_after, const float* target, float* loss_out,
              float* g_heads, void* g_after) {
  const tt2_desc* d = c.d;
  if (d->batch <= 0 || d->tq <= 0 || d->n_mels <= 0 || d->heads_ld < d->n_mels + 1)
    return tt2_set_error(TT2_E_INVALID, "tt2_loss: batch, tq, n_mels > 0, heads_ld >= n_mels + 1");
  const size_t m = (size_t)d->batch * d->tq;
  // the forward still runs the fused kernel, which writes gradients: they go to scratch
  float* gh = g_heads ? g_heads : reinterpret_cast<float*>(c.take(m * d->heads_ld * sizeof(float)));
  void* ga = g_after ? g_after : c.take(m * d->n_mels * esz(d->dtype));
  tt2_loss_args a;
  std::memset(&a, 0, sizeof(a));
  a.heads = heads; a.mel_after = mel_after; a.target = target; a.mel_len = d->mel_len;
  a.loss_out = loss_out; a.g_heads = gh; a.g_after = ga;
  a.heads_ld = d->heads_ld; a.batch = d->batch; a.t = d->tq; a.n_mels = d->n_mels; a.grad_dtype = d->dtype;
  a.pos_weight = d->pos_weight; a.grad_scale = d->grad_scale;
  a.separate_grads = 1;
  a.workspace = c.take(tt2_loss_workspace_size());
  a.ws_bytes = tt2_loss_workspace_size();
  return c.dry ? TT2_OK : tt2_tts_loss(&a, c.s);
}
}  // namespace

extern "C" size_t tt2_loss_block_workspace_size(const tt2_desc* d) {
  // the forward's gradient scratch is the larger need
  return block_size(d, [&](Ctx& c) { return loss_body(c, kAnyF, kAnyF, kAnyF, kAnyF, nullptr, nullptr); });
}
extern "C" int tt2_loss_fwd(const tt2_desc* d, const float* heads, const float* mel_after, const float* target,
                            float* loss_out, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (!d || !heads || !mel_after || !target || !loss_out || !d->mel_len)
    return tt2_set_error(TT2_E_INVALID, "tt2_loss_fwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return loss_body(c, heads, mel_after, target, loss_out, nullptr, nullptr);
  });
}
extern "C" int tt2_loss_bwd(const tt2_desc* d, const float* heads, const float* mel_after, const float* target,
                            float* loss_out, float* g_heads, void* g_after, void* workspace, size_t ws_bytes,
                            hipStream_t stream) {
  if (!d || !heads || !mel_after || !target || !loss_out || !g_heads || !g_after || !d->mel_len)
    return tt2_set_error(TT2_E_INVALID, "tt2_loss_bwd: null argument");
  return run_block(d, workspace, ws_bytes, stream, nullptr, [&](Ctx& c) {
    return loss_body(c, heads, mel_after, target, loss_out, g_heads, g_after);
  });
}
