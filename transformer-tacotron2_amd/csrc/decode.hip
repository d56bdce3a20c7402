// decode.hip -- the autoregressive decode step, gfx950.
//
// One decode step per utterance of the batch: a single query row per (batch,
// head) against (i) the layer's self-attention KV cache [B][T_max][K|V] holding
// positions 0..t, and (ii) the encoder memory's precomputed cross K/V.  The step
// index t lives in DEVICE memory and every kernel here reads it, so the whole
// step (prenet -> 6 layers -> heads -> emit) is captured once as a hipGraph and
// replayed T times with no host round trip.
//
// attn_decode: workgroup = one (batch, head), 8 waves split the keys into
// contiguous eighths; each wave takes 32 keys per iteration (8 lanes x 16-B per
// 64-wide head row, for K and for V; all 8 loads of a lane issued before the
// first use, so an iteration costs one memory round trip), keeps an online
// softmax, and the eight partial (max, sum, o[64]) are merged through LDS.
// Latency-bound at decode sizes; HBM-bound on the cache at long t.
#include <math.h>

#include "tt2_capi.h"
#include "tt2_internal.h"
#include "tt2_common.h"

namespace {
constexpr int NT = 256;
constexpr int D = 64;
constexpr float LOG2E = 1.4426950408889634f;

template <typename T> TT2_DEV void load8f(const T* p, float (&v)[8]);
template <> TT2_DEV void load8f(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> TT2_DEV void load8f(const f16* p, float (&v)[8]) {
  const f16x8 x = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> TT2_DEV void load8f(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}

struct DecArgs {
  const void* q; const void* k; const void* v; void* out;
  int64_t q_ld, k_bstride, k_ld, v_bstride, v_ld, o_ld;
  const int32_t* key_len;   // per-batch number of keys (cross attention) or null
  const int32_t* t_ptr;     // self attention: keys = *t_ptr + 1
  const int32_t* stop_len;  // optional [B]: utterance b is finished once *step >= stop_len[b]
  const int32_t* step;
  int tk, H, B;
  float scale;
  const void* wo; int64_t wo_ld; float* slab;   // fused output projection (wo != null)
  const void* wq; int64_t wq_ld; const float* bq;   // fused query projection (wq != null; q = its input)
  // fused residual combine + LayerNorm of the projection input (ln_part != null): x[b] =
  // LN(q[b] + ln_bias + sum_s ln_part[s][b]) (ln_combine_row), written to ln_out by head 0
  const float* ln_part; const float* ln_bias; const float* ln_gamma; const float* ln_beta; void* ln_out;
  float ln_eps;
};

// q-prologue (wq != null): this head's 64 query values from the projection input row x[b]
// (H*64 wide): wave w computes output rows 8w .. 8w+7 (NW = 8), eight lanes per row; load i
// of lane c covers k = 64 i + 8 c .. + 7, so each wave instruction reads 8 whole 128-B row
// segments (lanes 64 consecutive k each touched 64 lines per instruction: 3.8 us of the
// launch); all 8 loads issued before the first FMA; the eight partials of a row meet by xor
// shuffles.  Result (f32, + bias) in sq[64].
// The projection weights are loaded first (qproj_w: they do not depend on x, so their latency
// overlaps the fused LayerNorm prologue); sx: the input row already in LDS (f32 values of T,
// that prologue), or null (x read from q).
template <typename T>
using T8 = T __attribute__((ext_vector_type(8)));
// the raw rows (converted at their use in qproj, so no wait for them is placed before the
// loads that follow: they are issued first thing in the kernel)
template <typename T, int NW>
TT2_DEV void qproj_w(const DecArgs& a, int h, T8<T> (&wraw)[8]) {
  static_assert(NW == 8, "one wave per 8 query rows");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 7, g = lane >> 3;
  const int r = h * D + 8 * w + g;   // output feature
  const T* wr = reinterpret_cast<const T*>(a.wq) + (int64_t)r * a.wq_ld + 8 * c;
#pragma unroll
  for (int i = 0; i < 8; ++i) wraw[i] = *reinterpret_cast<const T8<T>*>(wr + 64 * i);
}
template <typename T, int NW>
TT2_DEV void qproj(const DecArgs& a, int b, int h, float* sq, const float* sx, const T8<T> (&wraw)[8]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 7, g = lane >> 3;
  const int r = h * D + 8 * w + g;   // output feature
  const T* x = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_ld + 8 * c;
  float xv[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (sx) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[i][j] = sx[64 * i + 8 * c + j];
    } else {
      load8f(x + 64 * i, xv[i]);
    }
  }
  float p = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) p += xv[i][j] * (float)wraw[i][j];
  p += __shfl_xor(p, 1, 64);
  p += __shfl_xor(p, 2, 64);
  p += __shfl_xor(p, 4, 64);
  if (c == 0) sq[8 * w + g] = p + (a.bq ? a.bq[r] : 0.f);
}

// slab[(h*B + b)*H*64 + n] = sum_j o[j] * Wo[n][h*64 + j] for the H*64 output columns.
// Eight lanes cover one 128-B row of Wo's head slice (lane & 7 = 16-B chunk), so a wave
// instruction reads 8 whole rows; every lane issues its 8 row loads before the first FMA;
// the 8 chunk partials of a row meet by xor shuffles and leave through LDS as one
// coalesced row of the slab.  o: this lane's 8 elements of the head output (chunk lane & 7).
// pre: this wave's first 8 rows, loaded by oproj_prefetch at the start of the kernel (behind the
// first keys, so no earlier wait drains them): the projection then costs no memory round trip
// of its own when H * 64 == NW * 64 (one row block per wave)
template <typename T, int NW>
TT2_DEV void oproj_prefetch(const DecArgs& a, int h, T8<T> (&pre)[8]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 7, g = lane >> 3;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    pre[i] = *reinterpret_cast<const T8<T>*>(reinterpret_cast<const T*>(a.wo) + (int64_t)(w * 64 + 8 * i + g) * a.wo_ld +
                                              h * D + 8 * c);
}
template <typename T, int NW>
TT2_DEV void oproj_slab(const DecArgs& a, int b, int h, const float (&o)[8], float* sres, const T8<T> (&pre)[8]) {
  const int N = a.H * D, lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 7, g = lane >> 3;
  for (int r0 = w * 64; r0 < N; r0 += NW * 64) {
    float wv[8][8];
    if (sizeof(T) == 2 && r0 == w * 64) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) wv[i][j] = (float)pre[i][j];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        load8f(reinterpret_cast<const T*>(a.wo) + (int64_t)(r0 + 8 * i + g) * a.wo_ld + h * D + 8 * c, wv[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) p += o[j] * wv[i][j];
      p += __shfl_xor(p, 1, 64);
      p += __shfl_xor(p, 2, 64);
      p += __shfl_xor(p, 4, 64);
      if (c == 0) sres[r0 + 8 * i + g] = p;
    }
  }
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += NW * 64) a.slab[((int64_t)h * a.B + b) * N + n] = sres[n];
}

template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode_kernel(DecArgs a) {
  constexpr int U = 4;   // 8-key groups per wave per iteration: 2*U 16-B loads in flight per lane
  __shared__ float sm[NW], sl[NW], so[NW][D], sfin[D], sres[512], sq[D], sx[512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int dc = lane & 7, kg = lane >> 3;   // 8-dim chunk, key slot within an 8-key group
  // fused prologue (ln_part): wave 0 combines + normalises the projection input row into sx
  // (f32 values of T) and head 0's workgroup writes it to ln_out
  auto ln_prologue = [&]() {
    if (w != 0) return;
    float o[8];
    ln_combine_row<8, T>(reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_ld, a.ln_part + (int64_t)b * 512,
                         (int64_t)a.B * 512, a.ln_bias, a.ln_gamma, a.ln_beta, a.ln_eps, lane, o);
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 y;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y[j] = from_f32<T>(o[j]);
      sx[lane * 8 + j] = (float)y[j];
    }
    if (h == 0) *reinterpret_cast<t8*>(reinterpret_cast<T*>(a.ln_out) + (int64_t)b * 512 + lane * 8) = y;
  };
  // the weights first: they depend on nothing the kernel reads (step, stop, key counts), so their
  // memory round trip overlaps those scalar loads instead of following them
  T8<T> wpre[8];   // 16-bit types only: the f32 (parity-mode) kernel has no registers to spare
  if constexpr (sizeof(T) == 2) {
    // only waves that own a row block (w * 64 < H * 64): with fewer heads than waves the
    // rows past N do not exist (oproj_slab's loop then skips the wave too)
    if (a.wo && w * 64 < a.H * D) oproj_prefetch<T, NW>(a, h, wpre);
  }
  T8<T> wq[8];
  if (a.wq) qproj_w<T, NW>(a, h, wq);
  if (a.stop_len && *a.step >= a.stop_len[b]) {
    if (a.ln_part) ln_prologue();   // the row stays defined for the sublayers after this one
    // a finished utterance: its frames past the stop are discarded, so skip the key stream
    if (a.out && threadIdx.x < D)
      reinterpret_cast<T*>(a.out)[(int64_t)b * a.o_ld + h * D + threadIdx.x] = from_f32<T>(0.f);
    if (a.wo)
      for (int n = threadIdx.x; n < a.H * D; n += NW * 64) a.slab[((int64_t)h * a.B + b) * a.H * D + n] = 0.f;
    return;
  }
  int nk = a.tk;
  if (a.t_ptr) nk = min(nk, *a.t_ptr + 1);
  if (a.key_len) nk = min(nk, a.key_len[b]);
  nk = max(nk, 0);
  const float c = a.scale * LOG2E;
  // contiguous per-wave key ranges, multiples of 8 keys
  const int per = ((nk + NW - 1) / NW + 7) & ~7;
  const int k0 = w * per, k1 = min(nk, k0 + per);
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)b * a.k_bstride + h * D + dc * 8;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)b * a.v_bstride + h * D + dc * 8;
  // two register buffers of raw K / V rows: the loads of iteration i + 1 are issued before
  // iteration i's arithmetic, so a wave's key range costs one memory round trip plus its
  // arithmetic instead of one round trip per iteration
  typedef T t8 __attribute__((ext_vector_type(8)));
  t8 kr[2][U], vr[2][U];
  // every load of an iteration at once (clamped to the last valid key: branch-free)
  auto load_keys = [&](int kb, int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = min(kb + 8 * u + kg, k1 - 1);
      kr[buf][u] = *reinterpret_cast<const t8*>(K + (int64_t)key * a.k_ld);
      vr[buf][u] = *reinterpret_cast<const t8*>(V + (int64_t)key * a.v_ld);
    }
  };
  // the first iteration's keys do not depend on the query: in flight during its projection
  if (k0 < k1) load_keys(k0, 0);
  float qv[8];
  if (a.wq) {
    if (a.ln_part) {   // the projection input row: residual combine + LayerNorm, rounded to T
      ln_prologue();
      __syncthreads();
    }
    qproj<T, NW>(a, b, h, sq, a.ln_part ? sx : nullptr, wq);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[j] = sq[dc * 8 + j];
  } else {
    load8f(reinterpret_cast<const T*>(a.q) + (int64_t)b * a.q_ld + h * D + dc * 8, qv);
  }
  float m = -INFINITY, l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // one iteration on register buffer BUF (compile-time, so the buffers stay in registers)
  auto iter = [&](auto BUFC, int kb) {
    constexpr int BUF = decltype(BUFC)::value;
    if (kb + 8 * U < k1) load_keys(kb + 8 * U, BUF ^ 1);
    float kv[U][8], vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        kv[u][j] = (float)kr[BUF][u][j];
        vv[u][j] = (float)vr[BUF][u][j];
      }
    float s[U];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float x = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) x += qv[j] * kv[u][j];
      x += __shfl_xor(x, 1, 64);
      x += __shfl_xor(x, 2, 64);
      x += __shfl_xor(x, 4, 64);
      s[u] = kb + 8 * u + kg < k1 ? x * c : -INFINITY;
      mx = fmaxf(mx, s[u]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);          // finite: the group's first key is always valid
    const float alpha = exp2f(m - mn);      // m = -inf -> 0
    l *= alpha;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] *= alpha;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p = exp2f(s[u] - mn);     // masked -> 0
      l += p;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += p * vv[u][j];
    }
    m = mn;
  };
  for (int kb = k0; kb < k1; kb += 16 * U) {
    iter(std::integral_constant<int, 0>{}, kb);
    if (kb + 8 * U < k1) iter(std::integral_constant<int, 1>{}, kb + 8 * U);
  }
  // combine the 8 key slots (same m across the wave)
#pragma unroll
  for (int off = 8; off < 64; off <<= 1) {
    l += __shfl_xor(l, off, 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] += __shfl_xor(o[j], off, 64);
  }
  if (lane == 0) { sm[w] = m; sl[w] = l; }
  if (lane < 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) so[w][lane * 8 + j] = o[j];
  __syncthreads();
  if (threadIdx.x < D) {
    const int d = threadIdx.x;
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < NW; ++i) M = fmaxf(M, sm[i]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const float f = sm[i] == -INFINITY ? 0.f : exp2f(sm[i] - M);
      L += sl[i] * f;
      O += so[i][d] * f;
    }
    const float r = L > 0.f ? O / L : 0.f;
    if (a.out) reinterpret_cast<T*>(a.out)[(int64_t)b * a.o_ld + h * D + d] = from_f32<T>(r);
    sfin[d] = r;
  }
  if (a.wo) {
    __syncthreads();
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = sfin[8 * (lane & 7) + j];
    oproj_slab<T, NW>(a, b, h, o, sres, wpre);
  }
}

// cache[b][*t][0:n] = src[b][0:n]
template <typename T>
__global__ void kv_append_kernel(const T* src, int64_t src_ld, T* cache, int64_t c_bstride, int64_t c_ld, int n,
                                 int B, const int32_t* t_ptr) {
  const int t = *t_ptr;
  if ((int64_t)t * c_ld >= c_bstride) return;   // t >= t_max: past the cache, nothing to append
  const int64_t total = (int64_t)B * n;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int b = (int)(i / n), c = (int)(i % n);
    cache[(int64_t)b * c_bstride + (int64_t)t * c_ld + c] = src[(int64_t)b * src_ld + c];
  }
}

// heads [B, hld] f32 -> mel_seq[b][t][:], stop_seq[b][t], prev frame (T); then t += 1, seed += 1
template <typename T>
__global__ void decode_emit_kernel(const float* heads, int64_t hld, int B, int NM, int tmax, float* mel_seq,
                                   float* stop_seq, T* prev, int32_t* t_ptr, uint32_t* seed, const float* stop_bias,
                                   int32_t* stop_len, float stop_thr) {
  const int t = *t_ptr;
  for (int i = threadIdx.x; i < B * (NM + 1); i += blockDim.x) {
    const int b = i / (NM + 1), c = i % (NM + 1);
    const float v = heads[(int64_t)b * hld + c];
    if (t < tmax) {
      if (c < NM) {
        const float vm = (stop_len && stop_len[b] <= t) ? 0.f : v;   // zero frames after the stop
        mel_seq[((int64_t)b * tmax + t) * NM + c] = vm;
        prev[(int64_t)b * NM + c] = from_f32<T>(vm);
      } else {
        const float vs = stop_bias ? v + stop_bias[(int64_t)b * tmax + t] : v;
        stop_seq[(int64_t)b * tmax + t] = vs;
        if (stop_len && vs >= stop_thr && stop_len[b] > t) stop_len[b] = t + 1;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && t < tmax) {   // the counter saturates at t_max
    t_ptr[0] = t + 1;
    if (seed) seed[0] += 1u;
  }
}

}  // namespace

extern "C" int tt2_attn_decode(const tt2_attn_decode_args* p, hipStream_t s) {
  if (p->head_dim != D) return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: head_dim must be 64");
  const int esz = p->dtype == TT2_DT_F32 ? 4 : 2;
  const int64_t lds[] = {p->q_ld, p->k_ld, p->v_ld, p->k_bstride, p->v_bstride};
  for (int64_t ld : lds)
    if ((ld * esz) % 16) return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: strides must be 16-B multiples");
  DecArgs a;
  a.q = p->q; a.k = p->k; a.v = p->v; a.out = p->out;
  a.q_ld = p->q_ld; a.k_bstride = p->k_bstride; a.k_ld = p->k_ld; a.v_bstride = p->v_bstride; a.v_ld = p->v_ld;
  a.o_ld = p->o_ld; a.key_len = p->key_len; a.t_ptr = p->t_ptr; a.tk = p->tk; a.H = p->heads; a.scale = p->scale;
  a.stop_len = p->stop_len;
  a.step = p->step ? p->step : p->t_ptr;
  a.B = p->batch;
  a.wo = p->wo; a.wo_ld = p->wo_ld; a.slab = p->slab;
  a.wq = p->wq; a.wq_ld = p->wq_ld; a.bq = p->bq;
  a.ln_part = p->ln_part; a.ln_bias = p->ln_bias; a.ln_gamma = p->ln_gamma; a.ln_beta = p->ln_beta;
  a.ln_out = p->ln_out; a.ln_eps = p->ln_eps;
  if (a.ln_part && (!a.wq || p->heads != 8 || !p->ln_bias || !p->ln_gamma || !p->ln_beta || !p->ln_out ||
                    p->q_ld != 512 || p->dtype == TT2_DT_F32))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: the fused LayerNorm prologue needs the fused query "
                                       "projection, 8 heads, bias / gamma / beta / ln_out and a packed bf16 / f16 q");
  if (a.wq && ((p->wq_ld * esz) % 16 || p->heads * D != 512))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: the fused query projection needs a 16-B wq_ld and "
                                       "heads * head_dim == 512");
  if (a.wo && (!a.slab || (p->wo_ld * esz) % 16 || p->heads * D > 512))
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: the fused projection needs slab, a 16-B wo_ld and "
                                       "heads * head_dim <= 512");
  if (!a.out && !a.wo) return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: null out");
  if (a.stop_len && !a.step) return tt2_set_error(TT2_E_INVALID, "tt2_attn_decode: stop_len needs step or t_ptr");
  dim3 g(p->batch * p->heads);
  // 8 waves per (batch, head): each wave takes 1/8 of the keys, 32 keys per iteration
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL((attn_decode_kernel<bf16, 8>), g, dim3(8 * 64), 0, s, a);
  else if (p->dtype == TT2_DT_F16) hipLaunchKernelGGL((attn_decode_kernel<f16, 8>), g, dim3(8 * 64), 0, s, a);
  else hipLaunchKernelGGL((attn_decode_kernel<float, 8>), g, dim3(8 * 64), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_attn_decode");
}

extern "C" int tt2_kv_append(const void* src, int64_t src_ld, void* cache, int64_t c_bstride, int64_t c_ld, int n,
                             int batch, const int32_t* t_ptr, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)batch * n;
  const int g = (int)((total + NT - 1) / NT);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(kv_append_kernel<bf16>, dim3(g), dim3(NT), 0, s, (const bf16*)src, src_ld, (bf16*)cache,
                       c_bstride, c_ld, n, batch, t_ptr);
  else
    hipLaunchKernelGGL(kv_append_kernel<float>, dim3(g), dim3(NT), 0, s, (const float*)src, src_ld, (float*)cache,
                       c_bstride, c_ld, n, batch, t_ptr);
  return tt2_check_launch(hipGetLastError(), "tt2_kv_append");
}

extern "C" int tt2_decode_emit(const float* heads, int64_t heads_ld, int batch, int n_mels, int t_max,
                               float* mel_seq, float* stop_seq, void* prev, int prev_dtype, int32_t* t_ptr,
                               uint32_t* seed, const float* stop_bias, int32_t* stop_len, float stop_thr,
                               hipStream_t s) {
  if (prev_dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(decode_emit_kernel<bf16>, dim3(1), dim3(NT), 0, s, heads, heads_ld, batch, n_mels, t_max,
                       mel_seq, stop_seq, (bf16*)prev, t_ptr, seed, stop_bias, stop_len, stop_thr);
  else if (prev_dtype == TT2_DT_F16)
    hipLaunchKernelGGL(decode_emit_kernel<f16>, dim3(1), dim3(NT), 0, s, heads, heads_ld, batch, n_mels, t_max,
                       mel_seq, stop_seq, (f16*)prev, t_ptr, seed, stop_bias, stop_len, stop_thr);
  else
    hipLaunchKernelGGL(decode_emit_kernel<float>, dim3(1), dim3(NT), 0, s, heads, heads_ld, batch, n_mels, t_max,
                       mel_seq, stop_seq, (float*)prev, t_ptr, seed, stop_bias, stop_len, stop_thr);
  return tt2_check_launch(hipGetLastError(), "tt2_decode_emit");
}
