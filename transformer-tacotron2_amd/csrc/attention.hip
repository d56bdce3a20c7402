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
// attn_bwd_prep.
#include <math.h>

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

extern "C" int tt2_attn_fwd(const tt2_attn_args* p, hipStream_t s) {
  if (int rc = validate(p)) return rc;
  if (!p->o_out || !p->lse) return tt2_set_error(TT2_E_INVALID, "tt2_attn_fwd: out/lse required");
  if (p->batch * p->tq == 0) return TT2_OK;
  AttnArgs a = to_args(p);
  dim3 grid((p->tq + BQ - 1) / BQ, p->batch * p->heads);
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(attn_fwd_kernel<bf16>, grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_attn_fwd");
}

extern "C" int tt2_attn_bwd(const tt2_attn_args* p, hipStream_t s) {
  if (int rc = validate(p)) return rc;
  if (!p->dq || !p->dk || !p->dv || !p->delta || !p->lse || !p->o || !p->dout)
    return tt2_set_error(TT2_E_INVALID, "tt2_attn_bwd: missing buffer");
  if (p->batch * p->tq == 0) return TT2_OK;
  AttnArgs a = to_args(p);
  dim3 gprep((p->batch * p->tq + 3) / 4);
  dim3 gq((p->tq + BQ - 1) / BQ, p->batch * p->heads);
  dim3 gk((p->tk + BKV - 1) / BKV, p->batch * p->heads);
  if (p->dtype == TT2_DT_BF16) {
    hipLaunchKernelGGL(attn_bwd_prep_kernel<bf16>, gprep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<bf16>, gq, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<bf16>, gk, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_prep_kernel<float>, gprep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<float>, gq, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<float>, gk, dim3(NT), 0, s, a);
  }
  return tt2_check_launch(hipGetLastError(), "tt2_attn_bwd");
}
