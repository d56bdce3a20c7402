// attention.hip -- fused scaled-dot-product attention, head dim 64 (gfx950).
//
// One kernel family serves the three attention blocks of the path
// (SURVEY 8(a) a3 encoder self-attention, a6 decoder causal self-attention,
// a7 encoder-decoder cross-attention): Q/K/V are read in place from the fused
// projection outputs (row stride + head offset), masks are a per-batch key
// length and an optional causal flag, and the score matrix is never written to
// HBM (online softmax over 64-key tiles held in LDS).
//
// Forward: workgroup = 4 waves = 64 query rows of one (batch, head); each wave
// owns 16 rows.  S = Q K^T and O += P V run on MFMA 16x16 (bf16 16x16x32 or
// exact-f32 16x16x4).  Row max / row sum are wave shuffles over the 16 lanes
// that hold one row's columns.  The per-row log-sum-exp (log2 domain, scores
// pre-multiplied by scale*log2(e)) is saved for the backward; a row with no
// visible key stores +inf so every recomputed probability is exactly 0 and the
// output row is 0 (SURVEY 8(b) mask convention).
//
// Backward (no atomics, bitwise reproducible): attn_bwd_dq walks key tiles per
// query block (dQ), attn_bwd_dkdv walks query tiles per key block (dK, dV);
// both recompute P from the saved LSE.  delta = rowsum(dO * O) comes from
// attn_bwd_prep (f32 / v1 path) or from the v3 dQ kernel, which runs first.
#include <math.h>

#include <type_traits>

#include "tt2_capi.h"
#include "tt2_internal.h"
#include "tt2_common.h"

namespace {

constexpr int D = 64;     // head dim
constexpr int BQ = 64;    // query rows per workgroup
constexpr int BKV = 64;   // keys per tile
constexpr int NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

template <typename T> struct LdsLd { static constexpr int V = D + Chunk<T>::N; };

// 8 contiguous elements from global (row pointer already offset), zero if !ok
template <typename T> TT2_DEV void frag_g(Frag8<T>& f, const T* p, bool ok);
template <> TT2_DEV void frag_g(Frag8<bf16>& f, const bf16* p, bool ok) {
  if (ok) f.v = *reinterpret_cast<const bf16x8*>(p);
  else { union { uint4 u; bf16x8 v; } z; z.u = make_uint4(0, 0, 0, 0); f.v = z.v; }
}
template <> TT2_DEV void frag_g(Frag8<float>& f, const float* p, bool ok) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = ok ? p[j] : 0.f;
}

// [64 rows][64] tile of a strided global matrix -> LDS (rows >= nrows zeroed)
template <typename T>
TT2_DEV void tile_to_lds(T* s, const T* g, int64_t ld, int row0, int nrows, int tid) {
  constexpr int E = Chunk<T>::N;
  constexpr int CPR = D / E;
  constexpr int LD = LdsLd<T>::V;
#pragma unroll
  for (int c = tid; c < 64 * CPR; c += NT) {
    const int r = c / CPR, cc = c % CPR;
    ChunkV<T> v = (row0 + r < nrows) ? ld_chunk<T>(g + (int64_t)(row0 + r) * ld + cc * E) : zero_chunk<T>();
    st_chunk<T>(s + r * LD + cc * E, v);
  }
}

struct AttnArgs {
  const void* q; const void* k; const void* v; const void* o; const void* dout;
  void* out; void* dq; void* dk; void* dv;
  float* lse; float* delta;
  int64_t q_ld, k_ld, v_ld, o_ld, do_ld, dq_ld, dk_ld, dv_ld;
  const int32_t* key_len;
  int B, H, Tq, Tk, causal;
  float scale;
};

TT2_DEV int key_limit(const AttnArgs& a, int b) {
  int kl = a.Tk;
  if (a.key_len) kl = min(kl, a.key_len[b]);
  return kl < 0 ? 0 : kl;
}

// ----------------------------------------------------------------- forward
template <typename T>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(AttnArgs a) {
  constexpr int LD = LdsLd<T>::V;
  __shared__ __attribute__((aligned(16))) T sK[BKV * LD];
  __shared__ __attribute__((aligned(16))) T sV[BKV * LD];
  __shared__ __attribute__((aligned(16))) T sP[4 * 16 * LD];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int q0 = blockIdx.x * BQ;
  const int row_l = lane & 15, hq = lane >> 4;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D;
  T* O = reinterpret_cast<T*>(a.out) + (int64_t)b * a.Tq * a.o_ld + h * D;

  // Q fragments: row q0 + 16w + (lane&15), d = 32*kk + 8*(lane>>4) + j
  Frag8<T> fq[2];
  {
    const int qr = q0 + 16 * w + row_l;
    const bool ok = qr < a.Tq;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) frag_g(fq[kk], Q + (int64_t)(ok ? qr : 0) * a.q_ld + 32 * kk + 8 * hq, ok);
  }
  const float c = a.scale * LOG2E;
  float m_r[4], l_r[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m_r[r] = -INFINITY; l_r[r] = 0.f; }
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int klim = key_limit(a, b);
  int kend = klim;
  if (a.causal) kend = min(kend, q0 + BQ);
  T* myP = sP + w * 16 * LD;

  for (int k0 = 0; k0 < kend; k0 += BKV) {
    __syncthreads();
    tile_to_lds<T>(sK, K, a.k_ld, k0, a.Tk, tid);
    tile_to_lds<T>(sV, V, a.v_ld, k0, a.Tk, tid);
    __syncthreads();

    f32x4 s[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      s[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        Frag8<T> fk;
        frag_row(fk, sK + (16 * jb + row_l) * LD + 32 * kk + 8 * hq);
        mma16(fq[kk], fk, s[jb]);
      }
    }
    // scale + mask; lane holds S[row 4*hq + r][key 16*jb + (lane&15)]
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mt[r] = -INFINITY;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int key = k0 + 16 * jb + row_l;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qr = q0 + 16 * w + 4 * hq + r;
        float x = s[jb][r] * c;
        if (key >= klim || (a.causal && key > qr)) x = -INFINITY;
        s[jb][r] = x;
        mt[r] = fmaxf(mt[r], x);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m_r[r], max16(mt[r]));
      const float base = mn == -INFINITY ? 0.f : mn;
      const float alpha = exp2f(m_r[r] - base);  // m_r = -inf -> 0
      float rs = 0.f;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const float p = exp2f(s[jb][r] - base);
        s[jb][r] = p;
        rs += p;
      }
      l_r[r] = l_r[r] * alpha + sum16(rs);
      m_r[r] = mn;
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) o[jd][r] *= alpha;
    }
    // P -> LDS (wave private), then O += P V
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) myP[(4 * hq + r) * LD + 16 * jb + row_l] = from_f32<T>(s[jb][r]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<T> fp;
      frag_row(fp, myP + row_l * LD + 32 * kk + 8 * hq);
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        Frag8<T> fv;
        frag_col(fv, sV, LD, 32 * kk + 8 * hq, 16 * jd, lane);
        mma16(fp, fv, o[jd]);
      }
    }
  }

  // finalize
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 16 * w + 4 * hq + r;
    if (qr >= a.Tq) continue;
    const float inv = l_r[r] > 0.f ? 1.f / l_r[r] : 0.f;
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) O[(int64_t)qr * a.o_ld + 16 * jd + row_l] = from_f32<T>(o[jd][r] * inv);
    if (row_l == 0)
      a.lse[(int64_t)bh * a.Tq + qr] = l_r[r] > 0.f ? m_r[r] + log2f(l_r[r]) : INFINITY;
  }
}

// ---------------------------------------------------------------- backward
// delta[bh, t] = sum_d dO[t, h*64 + d] * O[t, h*64 + d]; one wave per (b, t) row, all heads.
template <typename T>
__global__ __launch_bounds__(NT) void attn_bwd_prep_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // b * Tq + t
  if (row >= a.B * a.Tq) return;
  const int b = row / a.Tq, t = row % a.Tq;
  const T* O = reinterpret_cast<const T*>(a.o) + (int64_t)row * a.o_ld;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)row * a.do_ld;
  for (int h0 = 0; h0 < a.H; h0 += 8) {
    // lane covers head h0 + lane/8, elements 8*(lane%8) .. +8
    const int h = h0 + (lane >> 3);
    float s = 0.f;
    if (h < a.H) {
      const int off = h * D + 8 * (lane & 7);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += to_f32(O[off + j]) * to_f32(dO[off + j]);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((lane & 7) == 0 && h < a.H) a.delta[((int64_t)b * a.H + h) * a.Tq + t] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int LD = LdsLd<T>::V;
  __shared__ __attribute__((aligned(16))) T sK[BKV * LD];
  __shared__ __attribute__((aligned(16))) T sV[BKV * LD];
  __shared__ __attribute__((aligned(16))) T sP[4 * 16 * LD];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int q0 = blockIdx.x * BQ;
  const int row_l = lane & 15, hq = lane >> 4;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)b * a.Tq * a.do_ld + h * D;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D;
  T* dQ = reinterpret_cast<T*>(a.dq) + (int64_t)b * a.Tq * a.dq_ld + h * D;

  Frag8<T> fq[2], fdo[2];
  {
    const int qr = q0 + 16 * w + row_l;
    const bool ok = qr < a.Tq;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag_g(fq[kk], Q + (int64_t)(ok ? qr : 0) * a.q_ld + 32 * kk + 8 * hq, ok);
      frag_g(fdo[kk], dO + (int64_t)(ok ? qr : 0) * a.do_ld + 32 * kk + 8 * hq, ok);
    }
  }
  float lse[4], dl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 16 * w + 4 * hq + r;
    lse[r] = qr < a.Tq ? a.lse[(int64_t)bh * a.Tq + qr] : INFINITY;
    dl[r] = qr < a.Tq ? a.delta[(int64_t)bh * a.Tq + qr] : 0.f;
  }
  const float c = a.scale * LOG2E;
  f32x4 dq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int klim = key_limit(a, b);
  int kend = klim;
  if (a.causal) kend = min(kend, q0 + BQ);
  T* myP = sP + w * 16 * LD;

  for (int k0 = 0; k0 < kend; k0 += BKV) {
    __syncthreads();
    tile_to_lds<T>(sK, K, a.k_ld, k0, a.Tk, tid);
    tile_to_lds<T>(sV, V, a.v_ld, k0, a.Tk, tid);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      s[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        Frag8<T> fk, fv;
        frag_row(fk, sK + (16 * jb + row_l) * LD + 32 * kk + 8 * hq);
        frag_row(fv, sV + (16 * jb + row_l) * LD + 32 * kk + 8 * hq);
        mma16(fq[kk], fk, s[jb]);
        mma16(fdo[kk], fv, dp[jb]);
      }
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int key = k0 + 16 * jb + row_l;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qr = q0 + 16 * w + 4 * hq + r;
        float p = exp2f(s[jb][r] * c - lse[r]);
        if (key >= klim || (a.causal && key > qr)) p = 0.f;
        const float ds = p * (dp[jb][r] - dl[r]);
        myP[(4 * hq + r) * LD + 16 * jb + row_l] = from_f32<T>(ds);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<T> fds;
      frag_row(fds, myP + row_l * LD + 32 * kk + 8 * hq);
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        Frag8<T> fk;
        frag_col(fk, sK, LD, 32 * kk + 8 * hq, 16 * jd, lane);
        mma16(fds, fk, dq[jd]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 16 * w + 4 * hq + r;
    if (qr >= a.Tq) continue;
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) dQ[(int64_t)qr * a.dq_ld + 16 * jd + row_l] = from_f32<T>(dq[jd][r] * a.scale);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void attn_bwd_dkdv_kernel(AttnArgs a) {
  constexpr int LD = LdsLd<T>::V;
  __shared__ __attribute__((aligned(16))) T sQ[BQ * LD];
  __shared__ __attribute__((aligned(16))) T sdO[BQ * LD];
  __shared__ __attribute__((aligned(16))) T sP[4 * 16 * LD];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int k0 = blockIdx.x * BKV;
  const int row_l = lane & 15, hq = lane >> 4;
  const T* Q = reinterpret_cast<const T*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (int64_t)b * a.Tq * a.do_ld + h * D;
  const T* K = reinterpret_cast<const T*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D;
  const T* V = reinterpret_cast<const T*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D;
  T* dK = reinterpret_cast<T*>(a.dk) + (int64_t)b * a.Tk * a.dk_ld + h * D;
  T* dV = reinterpret_cast<T*>(a.dv) + (int64_t)b * a.Tk * a.dv_ld + h * D;

  const int klim = key_limit(a, b);
  // this wave's keys: k0 + 16w + (lane&15) as MFMA rows
  Frag8<T> fk[2], fv[2];
  {
    const int kr = k0 + 16 * w + row_l;
    const bool ok = kr < a.Tk;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag_g(fk[kk], K + (int64_t)(ok ? kr : 0) * a.k_ld + 32 * kk + 8 * hq, ok);
      frag_g(fv[kk], V + (int64_t)(ok ? kr : 0) * a.v_ld + 32 * kk + 8 * hq, ok);
    }
  }
  const float c = a.scale * LOG2E;
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { dk[j] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[j] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  T* myP = sP + w * 16 * LD;
  const bool block_live = k0 < klim;
  const int qstart = (a.causal ? (k0 / BQ) * BQ : 0);

  for (int q0 = qstart; block_live && q0 < a.Tq; q0 += BQ) {
    __syncthreads();
    tile_to_lds<T>(sQ, Q, a.q_ld, q0, a.Tq, tid);
    tile_to_lds<T>(sdO, dO, a.do_ld, q0, a.Tq, tid);
    __syncthreads();
    // lane holds S^T[key 4*hq + r][query 16*jb + (lane&15)]
    float lse[4], dl[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int qc = q0 + 16 * jb + row_l;
      lse[jb] = qc < a.Tq ? a.lse[(int64_t)bh * a.Tq + qc] : INFINITY;
      dl[jb] = qc < a.Tq ? a.delta[(int64_t)bh * a.Tq + qc] : 0.f;
    }
    f32x4 s[4], dp[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      s[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        Frag8<T> fqq, fdd;
        frag_row(fqq, sQ + (16 * jb + row_l) * LD + 32 * kk + 8 * hq);
        frag_row(fdd, sdO + (16 * jb + row_l) * LD + 32 * kk + 8 * hq);
        mma16(fk[kk], fqq, s[jb]);
        mma16(fv[kk], fdd, dp[jb]);
      }
    }
    float pv[4][4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int qc = q0 + 16 * jb + row_l;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * w + 4 * hq + r;
        float p = exp2f(s[jb][r] * c - lse[jb]);
        if (key >= klim || (a.causal && key > qc) || qc >= a.Tq) p = 0.f;
        pv[jb][r] = p;
        myP[(4 * hq + r) * LD + 16 * jb + row_l] = from_f32<T>(p);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // dV += P^T dO
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<T> fp;
      frag_row(fp, myP + row_l * LD + 32 * kk + 8 * hq);
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        Frag8<T> fd;
        frag_col(fd, sdO, LD, 32 * kk + 8 * hq, 16 * jd, lane);
        mma16(fp, fd, dv[jd]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // dS^T = P^T (dP^T - delta) -> LDS, dK += dS^T Q
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        myP[(4 * hq + r) * LD + 16 * jb + row_l] = from_f32<T>(pv[jb][r] * (dp[jb][r] - dl[jb]));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<T> fds;
      frag_row(fds, myP + row_l * LD + 32 * kk + 8 * hq);
#pragma unroll
      for (int jd = 0; jd < 4; ++jd) {
        Frag8<T> fqq;
        frag_col(fqq, sQ, LD, 32 * kk + 8 * hq, 16 * jd, lane);
        mma16(fds, fqq, dk[jd]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kr = k0 + 16 * w + 4 * hq + r;
    if (kr >= a.Tk) continue;
#pragma unroll
    for (int jd = 0; jd < 4; ++jd) {
      dK[(int64_t)kr * a.dk_ld + 16 * jd + row_l] = from_f32<T>(dk[jd][r] * a.scale);
      dV[(int64_t)kr * a.dv_ld + 16 * jd + row_l] = from_f32<T>(dv[jd][r]);
    }
  }
}

// =====================================================================================
// v3 kernels (bf16): v_mfma_f32_32x32x16_bf16 with "swapped" products.  Every product
// puts the streamed dimension (keys in dQ / forward, queries in dK-dV) on the MFMA rows
// and the wave's own 32 rows (queries, or keys) on the lane:
//   forward  S^T = K Q^T      O^T  += V^T  P^T
//   dQ       S^T = K Q^T, dP^T = V dO^T,   dQ^T += K^T dS^T
//   dK, dV   S   = Q K^T, dP  = dO V^T,    dV^T += dO^T P,  dK^T += Q^T dS
// The 32x32 accumulator then holds, per lane, 16 streamed rows crow(r, hi) =
// (r&3) + 8(r>>2) + 4hi of ONE own row, and those 16 values ARE the B operand of the
// next product once its A operand is read transposed (ds_read_b64_tr_b16) from rows
// base + {4hi + 0..3} and base + {8 + 4hi + 0..3}.  P and dS never leave registers,
// softmax statistics are per lane (one xor-32 shuffle per tile), and each LDS fragment
// feeds a 32-row MFMA (32 FLOP per LDS byte: the LDS array is not the bound).
// Tiles are 64 rows x 64 bf16 in LDS with the chunk swizzle below, double-buffered and
// register-staged (global loads for tile t+1 in flight while tile t computes).
// =====================================================================================
typedef float f32x16 __attribute__((ext_vector_type(16)));

TT2_DEV void mma32(const bf16x8& a, const bf16x8& b, f32x16& c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
TT2_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 16-B chunk c of tile row r lives at slot c ^ swz(r), swz(r) = h((r >> 1) & 7) with
// h(x) = ((x & 1) << 2) | (x >> 1).  Row reads (ds_read_b128: 16 distinct rows mod 16
// per lane group) and 4-row transposed reads (ds_read_b64_tr_b16: rows 4i..4i+3 x one
// 4-chunk half per 32-lane group) are both bank-conflict-free.
TT2_DEV int swz(int r) {
  const int x = (r >> 1) & 7;
  return ((x & 1) << 2) | (x >> 1);
}
TT2_DEV int toff(int r, int col) { return r * D + ((((col >> 3) ^ swz(r))) << 3) + (col & 7); }

template <int NTH> struct Stage3 { static constexpr int PER = 64 * 8 / NTH; };

// Buffer view of one (batch, head) slice of a [T rows][ld] bf16 matrix: rows >= T fall
// outside num_records and load as zeros (no per-row branches or exec masking).
struct RowBuf {
  __amdgpu_buffer_rsrc_t rs;
  int ldb;   // row stride in bytes
};
TT2_DEV RowBuf row_buf(const bf16* base, int64_t ld, int T) {
  RowBuf r;
  r.ldb = (int)(ld * 2);
  const int bytes = T > 0 ? (T - 1) * r.ldb + D * 2 : 0;
  r.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(base), (short)0, bytes, 0x00020000);
  return r;
}
TT2_DEV uint4 buf_ld16(const RowBuf& b, int row, int chunk) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(b.rs, row * b.ldb + chunk * 16, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

template <int NTH>
TT2_DEV void g2r3(uint4 (&r)[Stage3<NTH>::PER], const RowBuf& g, int row0, int tid) {
#pragma unroll
  for (int i = 0; i < Stage3<NTH>::PER; ++i) {
    const int c = tid + NTH * i;
    r[i] = buf_ld16(g, row0 + (c >> 3), c & 7);
  }
}
template <int NTH>
TT2_DEV void r2s3(const uint4 (&r)[Stage3<NTH>::PER], bf16* s, int tid) {
#pragma unroll
  for (int i = 0; i < Stage3<NTH>::PER; ++i) {
    const int c = tid + NTH * i, rr = c >> 3, cc = c & 7;
    *reinterpret_cast<uint4*>(s + rr * D + ((cc ^ swz(rr)) << 3)) = r[i];
  }
}
// A operand rows: X[row][16 st + 8 hi + j]
TT2_DEV bf16x8 rowfrag(const bf16* t, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(t + row * D + ((chunk ^ swz(row)) << 3));
}
// A operand X^T[d = 32 db + (lane & 31)][k = 8 hi + j], k <-> tile row base + 8(j>>2) + 4hi + (j&3)
TT2_DEV bf16x8 trfrag(const bf16* t, int base, int db, int lane) {
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const int hi = lane >> 5, q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1;
  const int col = 32 * db + 16 * g + 4 * p;
  const int r0 = base + 4 * hi + q;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + toff(r0, col)));
  short4v up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + toff(r0 + 8, col)));
  union { short4v s[2]; bf16x8 v; } u;
  u.s[0] = lo;
  u.s[1] = up;
  return u.v;
}
// own-row fragments: X[row][16 st + 8 hi + j], st = 0..3 (zeros past the last row)
TT2_DEV void own_frags(bf16x8 (&f)[4], const RowBuf& X, int row, int hi) {
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    union { uint4 u; bf16x8 v; } x;
    x.u = buf_ld16(X, row, 2 * st + hi);
    f[st] = x.v;
  }
}
// value of lane l ^ 32 combined with lane l's: v_permlane32_swap instead of ds_bpermute
TT2_DEV float xor32_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
TT2_DEV float xor32_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
TT2_DEV int crow(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }
// store the lane's 16 accumulator rows (d = 32 db + crow) of one output row
TT2_DEV void store_rowT(bf16* row, const f32x16 (&acc)[2], float sc, int hi) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      bf16x4 x;
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = (bf16)(acc[db][4 * rr + i] * sc);
      *reinterpret_cast<bf16x4*>(row + 32 * db + 8 * rr + 4 * hi) = x;
    }
}
TT2_DEV void zero16(f32x16& x) {
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0.f;
}

// s_waitcnt vmcnt(0) as the builtin (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15), which the
// compiler's wait-count pass sees: registers loaded before a tile loop are then known complete.
// Without it the pass carried those loads' pending state around the loop and made each MFMA that
// reads them wait for the NEXT tile's prefetch loads issued just before (vmcnt(3)..vmcnt(0)),
// which put the prefetch's whole memory latency in front of every tile's first MFMAs.
#define TT2_VMCNT0() __builtin_amdgcn_s_waitcnt(0x0F70)

// in-kernel timeline hooks of the v3 forward (tools/attn_stamps.hip defines them; empty here)
#ifndef ATTN_STAMP
#define ATTN_STAMP(slot)
#endif

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_fwd3_kernel(AttnArgs a) {
  constexpr int NTH = NW * 64, PER = Stage3<NTH>::PER, QB = 32 * NW;
  __shared__ __attribute__((aligned(16))) bf16 sK[2][64 * D];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][64 * D];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ql = lane & 31, hi = lane >> 5;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;   // x = (batch, head): block index on y
  const int qblk = a.causal ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y;   // heavy blocks first
  const int q0 = qblk * QB, qw = q0 + 32 * w, qv = qw + ql;
  ATTN_STAMP(0)
  const RowBuf Q = row_buf(reinterpret_cast<const bf16*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D, a.q_ld, a.Tq);
  const RowBuf K = row_buf(reinterpret_cast<const bf16*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D, a.k_ld, a.Tk);
  const RowBuf V = row_buf(reinterpret_cast<const bf16*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D, a.v_ld, a.Tk);
  bf16* O = reinterpret_cast<bf16*>(a.out) + (int64_t)b * a.Tq * a.o_ld + h * D;

  bf16x8 fq[4];
  own_frags(fq, Q, qv, hi);
  // (no TT2_VMCNT0 here: with the forward's gated MFMAs ungated it measured 0.7-0.9 us slower
  // per launch)
  const float c = a.scale * LOG2E;
  float m_r = -INFINITY, l_r = 0.f;
  f32x16 o[2];
  zero16(o[0]);
  zero16(o[1]);

  const int klim = key_limit(a, b);
  int kend = klim;
  if (a.causal) kend = min(kend, q0 + QB);
  const int ntile = kend > 0 ? (kend + 63) / 64 : 0;
  uint4 rk[PER], rv[PER];
  if (ntile > 0) {
    g2r3<NTH>(rk, K, 0, tid);
    g2r3<NTH>(rv, V, 0, tid);
    r2s3<NTH>(rk, sK[0], tid);
    r2s3<NTH>(rv, sV[0], tid);
  }
  __syncthreads();
  ATTN_STAMP(1)
  // one 64-key tile; BUF is compile-time so every LDS address is lane base + immediate
  auto tile = [&](auto BUFC, int t) {
    constexpr int BUF = decltype(BUFC)::value;
    const int k0 = 64 * t;
    const bool more = t + 1 < ntile;
    if (more) {
      g2r3<NTH>(rk, K, k0 + 64, tid);
      g2r3<NTH>(rv, V, k0 + 64, tid);
    }
    const bf16* cK = sK[BUF];
    const bf16* cV = sV[BUF];
    // wave-uniform: the wave has a query row (the last block of a head is partly past Tq:
    // 800 queries give 6.25 blocks of 128) and some key of the tile is visible
    if (qw < a.Tq && !(a.causal && k0 > qw + 31)) {
      f32x16 s[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        zero16(s[kb]);
#pragma unroll
        for (int st = 0; st < 4; ++st) mma32(rowfrag(cK, 32 * kb + ql, 2 * st + hi), fq[st], s[kb]);
      }
      if (k0 + 64 > klim || (a.causal && k0 + 63 > qw)) {
        // visible keys: key <= lim (one compare + select per score, no branches)
        const int lim = (a.causal ? min(klim - 1, qv) : klim - 1) - k0 - 4 * hi;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[kb][r] = 32 * kb + crow(r, 0) > lim ? -INFINITY : s[kb][r];
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
      mx = xor32_max(mx);
      ATTN_STAMP(2 + 4 * t)
      const float mn = fmaxf(m_r, mx * c);
      const float base = mn == -INFINITY ? 0.f : mn;
      if (__any(mn != m_r)) {   // exact: skipped lanes would multiply by 1
        const float alpha = fast_exp2(m_r - base);
        l_r *= alpha;
#pragma unroll
        for (int db = 0; db < 2; ++db) o[db] *= alpha;
      }
      m_r = mn;
      bf16x8 pf[2][2];
      float rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(s[kb][r], c, -base));
          rs += p;
          pf[kb][r >> 3][r & 7] = (bf16)p;
        }
      l_r += rs;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int db = 0; db < 2; ++db) mma32(trfrag(cV, 32 * kb + 16 * hh, db, lane), pf[kb][hh], o[db]);
    }
    ATTN_STAMP(3 + 4 * t)
    if (more) {
      r2s3<NTH>(rk, sK[BUF ^ 1], tid);
      r2s3<NTH>(rv, sV[BUF ^ 1], tid);
    }
    ATTN_STAMP(4 + 4 * t)
    __syncthreads();
    ATTN_STAMP(5 + 4 * t)
  };
  for (int t = 0; t < ntile; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntile) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  const float l = xor32_sum(l_r);
  if (qv < a.Tq) {
    store_rowT(O + (int64_t)qv * a.o_ld, o, l > 0.f ? 1.f / l : 0.f, hi);
    if (hi == 0) a.lse[(int64_t)bh * a.Tq + qv] = l > 0.f ? m_r + log2f(l) : INFINITY;
  }
}

// dQ: wave = 32 queries (query on the lane), workgroup walks 64-key tiles in two
// 32-key halves.
template <int NW>
// dQ body (also the fused dQ + dK/dV launch): workgroup (bx, by) of a (B*H, ny) grid; smem
// holds sK[2][64 D] and sV[2][64 D]; publish: store delta = rowsum(dO * O) for a later dK/dV
TT2_DEV void attn_bwd_dq3_body(const AttnArgs& a, int bx, int by, int ny, char* smem, bool publish) {
  constexpr int NTH = NW * 64, PER = Stage3<NTH>::PER, QB = 32 * NW;
  bf16 (*sK)[64 * D] = reinterpret_cast<bf16 (*)[64 * D]>(smem);
  bf16 (*sV)[64 * D] = reinterpret_cast<bf16 (*)[64 * D]>(smem + 2 * 64 * D * sizeof(bf16));
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ql = lane & 31, hi = lane >> 5;
  const int bh = bx, b = bh / a.H, h = bh % a.H;   // x = (batch, head): block index on y
  const int qblk = a.causal ? ny - 1 - by : by;
  const int q0 = qblk * QB, qw = q0 + 32 * w, qv = qw + ql;
  const RowBuf Q = row_buf(reinterpret_cast<const bf16*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D, a.q_ld, a.Tq);
  const RowBuf dO =
      row_buf(reinterpret_cast<const bf16*>(a.dout) + (int64_t)b * a.Tq * a.do_ld + h * D, a.do_ld, a.Tq);
  const RowBuf K = row_buf(reinterpret_cast<const bf16*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D, a.k_ld, a.Tk);
  const RowBuf V = row_buf(reinterpret_cast<const bf16*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D, a.v_ld, a.Tk);
  bf16* dQ = reinterpret_cast<bf16*>(a.dq) + (int64_t)b * a.Tq * a.dq_ld + h * D;

  const bool qok = qv < a.Tq;
  bf16x8 fq[4], fdo[4], fo[4];
  own_frags(fq, Q, qv, hi);
  own_frags(fdo, dO, qv, hi);
  // delta = rowsum(dO * O) of this lane's query row, computed here (the two lane halves hold
  // 32 dims each) and published for the dK / dV kernel that runs next on the stream
  const RowBuf Ob = row_buf(reinterpret_cast<const bf16*>(a.o) + (int64_t)b * a.Tq * a.o_ld + h * D, a.o_ld, a.Tq);
  own_frags(fo, Ob, qv, hi);
  const float lse = qok ? a.lse[(int64_t)bh * a.Tq + qv] : INFINITY;
  TT2_VMCNT0();   // Q / dO / O fragments and the LSE are final before the tile loop
  float dsum = 0.f;
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += (float)fdo[st][j] * (float)fo[st][j];
  dsum += __shfl_xor(dsum, 32, 64);
  const float dl = qok ? dsum : 0.f;
  if (publish && qok && hi == 0) a.delta[(int64_t)bh * a.Tq + qv] = dsum;
  const float c = a.scale * LOG2E;
  f32x16 dq[2];
  zero16(dq[0]);
  zero16(dq[1]);

  const int klim = key_limit(a, b);
  int kend = klim;
  if (a.causal) kend = min(kend, q0 + QB);
  const int ntile = kend > 0 ? (kend + 63) / 64 : 0;
  uint4 rk[PER], rv[PER];
  if (ntile > 0) {
    g2r3<NTH>(rk, K, 0, tid);
    g2r3<NTH>(rv, V, 0, tid);
    r2s3<NTH>(rk, sK[0], tid);
    r2s3<NTH>(rv, sV[0], tid);
  }
  __syncthreads();
  auto tile = [&](auto BUFC, int t) {
    constexpr int BUF = decltype(BUFC)::value;
    const int k0 = 64 * t;
    const bool more = t + 1 < ntile;
    if (more) {
      g2r3<NTH>(rk, K, k0 + 64, tid);
      g2r3<NTH>(rv, V, k0 + 64, tid);
    }
    const bf16* cK = sK[BUF];
    const bf16* cV = sV[BUF];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int kb0 = k0 + 32 * kb;
      if (qw >= a.Tq || (a.causal && kb0 > qw + 31)) continue;   // wave-uniform (no query row, or masked)
      f32x16 s, dp;
      zero16(s);
      zero16(dp);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        mma32(rowfrag(cK, 32 * kb + ql, 2 * st + hi), fq[st], s);
        mma32(rowfrag(cV, 32 * kb + ql, 2 * st + hi), fdo[st], dp);
      }
      float p[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) p[r] = fast_exp2(fmaf(s[r], c, -lse));
      if (kb0 + 32 > klim || (a.causal && kb0 + 31 > qw)) {   // wave-uniform: mask edge tiles only
        const int lim = (a.causal ? min(klim - 1, qv) : klim - 1) - kb0 - 4 * hi;
#pragma unroll
        for (int r = 0; r < 16; ++r) p[r] = crow(r, 0) > lim ? 0.f : p[r];
      }
      bf16x8 dsf[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) dsf[r >> 3][r & 7] = (bf16)(p[r] * (dp[r] - dl));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int db = 0; db < 2; ++db) mma32(trfrag(cK, 32 * kb + 16 * hh, db, lane), dsf[hh], dq[db]);
    }
    if (more) {
      r2s3<NTH>(rk, sK[BUF ^ 1], tid);
      r2s3<NTH>(rv, sV[BUF ^ 1], tid);
    }
    __syncthreads();
  };
  for (int t = 0; t < ntile; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntile) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  if (qok) store_rowT(dQ + (int64_t)qv * a.dq_ld, dq, a.scale, hi);
}

// dK, dV: wave = 32 keys (key on the lane), workgroup walks 64-query tiles in two
// 32-query halves.
template <int NW>
// dK / dV body: workgroup (bx, by) of a (B*H, key blocks) grid; smem holds sQ[2][64 D],
// sdO[2][64 D], sL[2][64], sDl[2][64]; reads delta (published by the dQ pass or attn_bwd_prep)
// self_delta: compute delta = rowsum(dO * O) of each staged query tile here (from the dO
// chunks already in registers and the matching O chunks) instead of reading a.delta
TT2_DEV void attn_bwd_dkdv3_body(const AttnArgs& a, int bx, int by, char* smem, bool self_delta) {
  constexpr int NTH = NW * 64, PER = Stage3<NTH>::PER, KB = 32 * NW;
  bf16 (*sQ)[64 * D] = reinterpret_cast<bf16 (*)[64 * D]>(smem);
  bf16 (*sdO)[64 * D] = reinterpret_cast<bf16 (*)[64 * D]>(smem + 2 * 64 * D * sizeof(bf16));
  float (*sL)[64] = reinterpret_cast<float (*)[64]>(smem + 4 * 64 * D * sizeof(bf16));
  float (*sDl)[64] = reinterpret_cast<float (*)[64]>(smem + 4 * 64 * D * sizeof(bf16) + 2 * 64 * sizeof(float));
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kl = lane & 31, hi = lane >> 5;
  const int bh = bx, b = bh / a.H, h = bh % a.H;   // x = (batch, head): block index on y
  const int k0 = by * KB, kw = k0 + 32 * w, kv = kw + kl;   // causal: low blocks (heaviest) first
  const RowBuf Q = row_buf(reinterpret_cast<const bf16*>(a.q) + (int64_t)b * a.Tq * a.q_ld + h * D, a.q_ld, a.Tq);
  const RowBuf dO =
      row_buf(reinterpret_cast<const bf16*>(a.dout) + (int64_t)b * a.Tq * a.do_ld + h * D, a.do_ld, a.Tq);
  const RowBuf K = row_buf(reinterpret_cast<const bf16*>(a.k) + (int64_t)b * a.Tk * a.k_ld + h * D, a.k_ld, a.Tk);
  const RowBuf V = row_buf(reinterpret_cast<const bf16*>(a.v) + (int64_t)b * a.Tk * a.v_ld + h * D, a.v_ld, a.Tk);
  bf16* dK = reinterpret_cast<bf16*>(a.dk) + (int64_t)b * a.Tk * a.dk_ld + h * D;
  bf16* dV = reinterpret_cast<bf16*>(a.dv) + (int64_t)b * a.Tk * a.dv_ld + h * D;
  const float* LSE = a.lse + (int64_t)bh * a.Tq;
  const float* DL = a.delta + (int64_t)bh * a.Tq;
  const RowBuf Ob = row_buf(reinterpret_cast<const bf16*>(a.o) + (int64_t)b * a.Tq * a.o_ld + h * D, a.o_ld, a.Tq);

  bf16x8 fk[4], fv[4];
  own_frags(fk, K, kv, hi);
  own_frags(fv, V, kv, hi);
  TT2_VMCNT0();   // the K / V fragments are final before the tile loop (see TT2_VMCNT0)
  const float c = a.scale * LOG2E;
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    zero16(dk[db]);
    zero16(dv[db]);
  }
  const int klim = key_limit(a, b);
  const int qstart = a.causal ? (k0 / 64) * 64 : 0;
  const int ntile = k0 < klim && a.Tq > qstart ? (a.Tq - qstart + 63) / 64 : 0;
  uint4 rq[PER], rd[PER], ro[PER];
  // the next tile's LSE / delta are loaded with its Q / dO rows (stats_load) and stored to LDS
  // with them (stats): loaded at the store, they cost a memory round trip at every tile's end
  float lse_n = INFINITY, dl_n = 0.f;
  auto stats_load = [&](int qb) {
    if (tid < 64) {
      const int q = qb + tid;
      lse_n = q < a.Tq ? LSE[q] : INFINITY;
      if (!self_delta) dl_n = q < a.Tq ? DL[q] : 0.f;
    }
  };
  auto stats = [&](int buf, int qb) {
    (void)qb;
    if (tid < 64) {
      sL[buf][tid] = lse_n;
      if (!self_delta) sDl[buf][tid] = dl_n;
    }
    if (self_delta) {   // chunk c = tid + NTH i is row c >> 3, 8 columns; the row's 8 chunks sit in 8 lanes
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        union { uint4 u; bf16x8 v; } x, y;
        x.u = rd[i];
        y.u = ro[i];
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d += (float)x.v[j] * (float)y.v[j];
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        if ((tid & 7) == 0) sDl[buf][(tid + NTH * i) >> 3] = d;
      }
    }
  };
  if (ntile > 0) {
    g2r3<NTH>(rq, Q, qstart, tid);
    g2r3<NTH>(rd, dO, qstart, tid);
    if (self_delta) g2r3<NTH>(ro, Ob, qstart, tid);
    stats_load(qstart);
    r2s3<NTH>(rq, sQ[0], tid);
    r2s3<NTH>(rd, sdO[0], tid);
    stats(0, qstart);
  }
  __syncthreads();
  auto tile = [&](auto BUFC, int t) {
    constexpr int BUF = decltype(BUFC)::value;
    const int q0 = qstart + 64 * t;
    const bool more = t + 1 < ntile;
    if (more) {
      g2r3<NTH>(rq, Q, q0 + 64, tid);
      g2r3<NTH>(rd, dO, q0 + 64, tid);
      if (self_delta) g2r3<NTH>(ro, Ob, q0 + 64, tid);
      stats_load(q0 + 64);
    }
    const bf16* cQ = sQ[BUF];
    const bf16* cD = sdO[BUF];
    const float* cL = sL[BUF];
    const float* cDl = sDl[BUF];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int qb0 = q0 + 32 * qb;
      if (kw >= klim || (a.causal && qb0 + 31 < kw)) continue;   // wave-uniform
      f32x16 s, dp;
      zero16(s);
      zero16(dp);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        mma32(rowfrag(cQ, 32 * qb + kl, 2 * st + hi), fk[st], s);
        mma32(rowfrag(cD, 32 * qb + kl, 2 * st + hi), fv[st], dp);
      }
      float p[16], dl[16];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int qi = 32 * qb + 8 * rr + 4 * hi;
        const f32x4 L = *reinterpret_cast<const f32x4*>(cL + qi);
        const f32x4 Dl = *reinterpret_cast<const f32x4*>(cDl + qi);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[4 * rr + i] = fast_exp2(fmaf(s[4 * rr + i], c, -L[i]));
          dl[4 * rr + i] = Dl[i];
        }
      }
      if (kw + 32 > klim || (a.causal && qb0 < kw + 31)) {   // wave-uniform: mask edge tiles only
        // masked: query q < kv (causal) or every query when kv >= klim
        const int qlo = (kv >= klim ? 1 << 20 : (a.causal ? kv - qb0 : -1)) - 4 * hi;   // visible iff crow >= qlo
#pragma unroll
        for (int r = 0; r < 16; ++r) p[r] = crow(r, 0) < qlo ? 0.f : p[r];
      }
      bf16x8 pf[2], dsf[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pf[r >> 3][r & 7] = (bf16)p[r];
        dsf[r >> 3][r & 7] = (bf16)(p[r] * (dp[r] - dl[r]));
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          mma32(trfrag(cD, 32 * qb + 16 * hh, db, lane), pf[hh], dv[db]);
          mma32(trfrag(cQ, 32 * qb + 16 * hh, db, lane), dsf[hh], dk[db]);
        }
    }
    if (more) {
      r2s3<NTH>(rq, sQ[BUF ^ 1], tid);
      r2s3<NTH>(rd, sdO[BUF ^ 1], tid);
      stats(BUF ^ 1, q0 + 64);
    }
    __syncthreads();
  };
  for (int t = 0; t < ntile; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntile) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  if (kv < a.Tk) {
    store_rowT(dK + (int64_t)kv * a.dk_ld, dk, a.scale, hi);
    store_rowT(dV + (int64_t)kv * a.dv_ld, dv, 1.f, hi);
  }
}

constexpr int ATTN_BWD3_SMEM = 4 * 64 * D * sizeof(bf16) + 4 * 64 * sizeof(float);   // the larger (dK / dV) body

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dq3_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 64 * D * sizeof(bf16)];
  attn_bwd_dq3_body<NW>(a, blockIdx.x, blockIdx.y, gridDim.y, smem, true);
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dkdv3_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[ATTN_BWD3_SMEM];
  attn_bwd_dkdv3_body<NW>(a, blockIdx.x, blockIdx.y, smem, false);
}

// dQ and dK / dV in one launch (each computes delta itself): y < nkb are the key blocks, the
// rest the query blocks, so the (few, long) dK / dV workgroups of a short key range run
// beside the dQ workgroups instead of after them on a mostly idle chip
template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_fused3_kernel(AttnArgs a, int nkb) {
  __shared__ __attribute__((aligned(16))) char smem[ATTN_BWD3_SMEM];
  if ((int)blockIdx.y < nkb) attn_bwd_dkdv3_body<NW>(a, blockIdx.x, blockIdx.y, smem, true);
  else attn_bwd_dq3_body<NW>(a, blockIdx.x, (int)blockIdx.y - nkb, (int)gridDim.y - nkb, smem, false);
}

AttnArgs to_args(const tt2_attn_args* p) {
  AttnArgs a;
  a.q = p->q; a.k = p->k; a.v = p->v; a.o = p->o; a.dout = p->dout;
  a.out = p->o_out; a.dq = p->dq; a.dk = p->dk; a.dv = p->dv;
  a.lse = p->lse; a.delta = p->delta;
  a.q_ld = p->q_ld; a.k_ld = p->k_ld; a.v_ld = p->v_ld; a.o_ld = p->o_ld; a.do_ld = p->do_ld;
  a.dq_ld = p->dq_ld; a.dk_ld = p->dk_ld; a.dv_ld = p->dv_ld;
  a.key_len = p->key_len;
  a.B = p->batch; a.H = p->heads; a.Tq = p->tq; a.Tk = p->tk; a.causal = p->causal;
  a.scale = p->scale;
  return a;
}

int validate(const tt2_attn_args* p) {
  if (p->head_dim != D) return tt2_set_error(TT2_E_INVALID, "tt2_attn: head_dim must be 64");
  const int esz = p->dtype == TT2_DT_BF16 ? 2 : 4;
  const int64_t lds[] = {p->q_ld, p->k_ld, p->v_ld};
  for (int64_t ld : lds)
    if ((ld * esz) % 16) return tt2_set_error(TT2_E_INVALID, "tt2_attn: leading dims must be 16-B multiples");
  return TT2_OK;
}

}  // namespace

// v3 grids are (batch*heads, row blocks): dispatch walks every (batch, head) of one
// row block before the next, so under a causal mask the heaviest blocks go first
// chip-wide (forward / dQ blocks are reversed in-kernel; dK-dV block 0 is heaviest).
// variant: 0 auto (bf16 -> v3, f32 -> v1), 1 v1, 2 v3 with 2 waves/workgroup, 3 v3 with 4.
int v3_waves(const tt2_attn_args* p, int rows, bool fwd) {
  if (p->dtype != TT2_DT_BF16 || p->variant == 1) return 0;
  if (p->variant == 2) return 2;
  if (p->variant == 3) return 4;
  // auto: the forward shares each K/V tile across 4 waves (128 queries) while that
  // still gives two workgroups per CU; the backward kernels (buffer-unrolled loops)
  // measure fastest with 4-wave workgroups at every shape of the workload.
  const int64_t wg4 = (int64_t)((rows + 127) / 128) * p->batch * p->heads;
  return !fwd || wg4 >= 512 ? 4 : 2;
}

// ------------------------------------------------------------ diagnostics
// Attention probabilities of a forward already run (alignment diagnostics, SURVEY 8(f)
// row 3): P[bh][q][j] = exp2(s * scale * log2e - lse[bh][q]) from the saved log2-LSE,
// 0 where masked.  One workgroup per (batch*head, query row); off the training path.
template <typename T>
__global__ __launch_bounds__(NT) void attn_probs_kernel(AttnArgs a, float* probs) {
  __shared__ float sq[D];
  const int bh = blockIdx.y, qi = blockIdx.x;
  const int b = bh / a.H, h = bh % a.H;
  const T* Q = reinterpret_cast<const T*>(a.q) + ((int64_t)b * a.Tq + qi) * a.q_ld + h * D;
  if (threadIdx.x < D) sq[threadIdx.x] = to_f32(Q[threadIdx.x]);
  __syncthreads();
  const float lse = a.lse[(int64_t)bh * a.Tq + qi];
  const int klim = key_limit(a, b);
  const float c = a.scale * LOG2E;
  float* out = probs + ((int64_t)bh * a.Tq + qi) * a.Tk;
  for (int j = threadIdx.x; j < a.Tk; j += NT) {
    float v = 0.f;
    if (j < klim && (!a.causal || j <= qi)) {
      const T* Kr = reinterpret_cast<const T*>(a.k) + ((int64_t)b * a.Tk + j) * a.k_ld + h * D;
      float dot = 0.f;
#pragma unroll 8
      for (int d = 0; d < D; ++d) dot += sq[d] * to_f32(Kr[d]);
      v = exp2f(dot * c - lse);
    }
    out[j] = v;
  }
}

extern "C" int tt2_attn_probs(const tt2_attn_args* p, float* probs, hipStream_t s) {
  if (int rc = validate(p)) return rc;
  if (!p->lse || !probs) return tt2_set_error(TT2_E_INVALID, "tt2_attn_probs: lse / probs required");
  if (p->batch * p->tq * p->tk == 0) return TT2_OK;
  AttnArgs a = to_args(p);
  const dim3 g(p->tq, p->batch * p->heads);
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(attn_probs_kernel<bf16>, g, dim3(NT), 0, s, a, probs);
  else hipLaunchKernelGGL(attn_probs_kernel<float>, g, dim3(NT), 0, s, a, probs);
  return tt2_check_launch(hipGetLastError(), "tt2_attn_probs");
}

extern "C" int tt2_attn_fwd(const tt2_attn_args* p, hipStream_t s) {
  if (int rc = validate(p)) return rc;
  if (!p->o_out || !p->lse) return tt2_set_error(TT2_E_INVALID, "tt2_attn_fwd: out/lse required");
  if (p->batch * p->tq == 0) return TT2_OK;
  AttnArgs a = to_args(p);
  const int nw = v3_waves(p, p->tq, true);
  if (nw == 4) {
    hipLaunchKernelGGL(attn_fwd3_kernel<4>, dim3(p->batch * p->heads, (p->tq + 127) / 128), dim3(256), 0, s, a);
  } else if (nw == 2) {
    hipLaunchKernelGGL(attn_fwd3_kernel<2>, dim3(p->batch * p->heads, (p->tq + 63) / 64), dim3(128), 0, s, a);
  } else {
    dim3 grid((p->tq + BQ - 1) / BQ, p->batch * p->heads);
    if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(attn_fwd_kernel<bf16>, grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(NT), 0, s, a);
  }
  return tt2_check_launch(hipGetLastError(), "tt2_attn_fwd");
}

extern "C" int tt2_attn_bwd(const tt2_attn_args* p, hipStream_t s) {
  if (int rc = validate(p)) return rc;
  if (!p->dq || !p->dk || !p->dv || !p->delta || !p->lse || !p->o || !p->dout)
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_bwd: missing buffer");
  if (p->batch * p->tq == 0) return TT2_OK;
  AttnArgs a = to_args(p);
  const int BH = p->batch * p->heads;
  dim3 gprep((p->batch * p->tq + 3) / 4);
  if (p->dtype == TT2_DT_BF16) {
    const int nq = v3_waves(p, p->tq, false), nk = v3_waves(p, p->tk, false);
    // the v3 dQ kernel computes delta = rowsum(dO * O) itself (and stores it for dK / dV).
    // Non-causal: dQ and dK / dV workgroups in one launch (the causal case gained nothing
    // from the same fusion)
    if (nq == 4 && nk == 4 && !p->causal) {
      // parts: both halves (the dK / dV blocks compute delta themselves, the dQ blocks do not
      // publish it), or one of them alone
      const int nkb = p->parts == 1 ? 0 : (p->tk + 127) / 128, nqb = p->parts == 2 ? 0 : (p->tq + 127) / 128;
      hipLaunchKernelGGL(attn_bwd_fused3_kernel<4>, dim3(BH, nkb + nqb), dim3(256), 0, s, a, nkb);
      return tt2_check_launch(hipGetLastError(), "tt2_attn_bwd");
    }
    if (p->parts != 0)
      return tt2_set_error(TT2_E_INVALID, "tt2_attn_bwd: parts needs the non-causal bf16 launch (4-wave v3)");
    if (nq == 0) hipLaunchKernelGGL(attn_bwd_prep_kernel<bf16>, gprep, dim3(NT), 0, s, a);
    if (nq == 4) hipLaunchKernelGGL(attn_bwd_dq3_kernel<4>, dim3(BH, (p->tq + 127) / 128), dim3(256), 0, s, a);
    else if (nq == 2) hipLaunchKernelGGL(attn_bwd_dq3_kernel<2>, dim3(BH, (p->tq + 63) / 64), dim3(128), 0, s, a);
    else hipLaunchKernelGGL(attn_bwd_dq_kernel<bf16>, dim3((p->tq + BQ - 1) / BQ, BH), dim3(NT), 0, s, a);
    if (nk == 4) hipLaunchKernelGGL(attn_bwd_dkdv3_kernel<4>, dim3(BH, (p->tk + 127) / 128), dim3(256), 0, s, a);
    else if (nk == 2) hipLaunchKernelGGL(attn_bwd_dkdv3_kernel<2>, dim3(BH, (p->tk + 63) / 64), dim3(128), 0, s, a);
    else hipLaunchKernelGGL(attn_bwd_dkdv_kernel<bf16>, dim3((p->tk + BKV - 1) / BKV, BH), dim3(NT), 0, s, a);
  } else {
    if (p->parts != 0) return tt2_set_error(TT2_E_INVALID, "tt2_attn_bwd: parts needs bf16");
    hipLaunchKernelGGL(attn_bwd_prep_kernel<float>, gprep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<float>, dim3((p->tq + BQ - 1) / BQ, BH), dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<float>, dim3((p->tk + BKV - 1) / BKV, BH), dim3(NT), 0, s, a);
  }
  return tt2_check_launch(hipGetLastError(), "tt2_attn_bwd");
}
