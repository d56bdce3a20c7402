// misc.hip -- the HBM-bound pieces of the path (gfx950): row reductions,
// bias gradients, embedding, scaled positional encoding, teacher-forcing input,
// casts, the fused TTS loss (+ its input gradients), weight repacks and the
// fused Adam/clip optimizer step.  All grid-stride, 16-B vectorised where the
// row width allows, deterministic (fixed-order partial sums, no float atomics
// except the embedding scatter).
#include <math.h>

#include <algorithm>

#include "tt2_capi.h"
#include "tt2_internal.h"
#include "tt2_common.h"

namespace {
constexpr int NT = 256;

int grid_for(int64_t total, int per = NT) {
  int64_t b = (total + per - 1) / per;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

TT2_DEV float ldf(const void* p, int64_t i, int dt) {
  if (dt == TT2_F16) return (float)reinterpret_cast<const f16*>(p)[i];
  return dt == TT2_BF16 ? (float)reinterpret_cast<const bf16*>(p)[i] : reinterpret_cast<const float*>(p)[i];
}
TT2_DEV void stf(void* p, int64_t i, int dt, float v) {
  if (dt == TT2_F16) reinterpret_cast<f16*>(p)[i] = (f16)v;
  else if (dt == TT2_BF16) reinterpret_cast<bf16*>(p)[i] = (bf16)v;
  else reinterpret_cast<float*>(p)[i] = v;
}

// dst[c] = beta * dst[c] + sum_r src[r * ld + c]   (fixed order)
// block = 16 columns x 16 row groups (short dependent chains); LDS combine in a fixed order.
constexpr int RR_COLS = 16;
// block = CW columns x (NT / CW) row groups, CW = min(16, cols rounded up to a power of
// two): narrow reductions (the Adam norm's 1024 x 1 partials) use every lane.  Each lane
// sums its rows two at a time; the group sums combine in a fixed order (two levels).
__global__ __launch_bounds__(NT) void reduce_rows_kernel(const float* src, int rows, int cols, int64_t ld, float* dst,
                                                         float beta, int cw) {
  __shared__ float red[NT];
  const int G = NT / cw;
  const int cl = threadIdx.x % cw, g = threadIdx.x / cw;
  const int c = blockIdx.x * cw + cl;
  float s0 = 0.f, s1 = 0.f;
  if (c < cols) {
    int r = g;
    for (; r + G < rows; r += 2 * G) {
      s0 += src[(int64_t)r * ld + c];
      s1 += src[(int64_t)(r + G) * ld + c];
    }
    if (r < rows) s0 += src[(int64_t)r * ld + c];
  }
  red[threadIdx.x] = s0 + s1;
  __syncthreads();
  // level 1: 16 partial sums per column over strided groups; level 2: lane g == 0
  const int P = G < 16 ? G : 16;
  float t1 = 0.f;
  if (g < P)
    for (int k = g; k < G; k += P) t1 += red[k * cw + cl];
  __syncthreads();
  if (g < P) red[g * cw + cl] = t1;
  __syncthreads();
  if (g == 0 && c < cols) {
    float t = 0.f;
    for (int k = 0; k < P; ++k) t += red[k * cw + cl];
    dst[c] = beta != 0.f ? beta * dst[c] + t : t;
  }
}

// partial column sums of a [M, N] matrix: part[blockIdx.y][n] over rows [y*rows_per, ...).
// block = 64 columns (8 lanes x 8 columns, 16-B loads) x 32 row lanes; LDS combine.
template <typename T>
__global__ __launch_bounds__(NT) void colsum_partial_kernel(const T* x, int64_t ld, int M, int N, int rows_per,
                                                            int vec, float* part) {
  __shared__ float red[32][65];
  const int cg = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int n0 = blockIdx.x * 64 + cg * 8;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (vec && n0 + 8 <= N) {
    for (int r = r0 + rg; r < r1; r += 32) {
      const T* p = x + (int64_t)r * ld + n0;
      ChunkV<T> c0 = ld_chunk<T>(p);
      if (Chunk<T>::N == 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += to_f32(c0.e[j % Chunk<T>::N]);
      } else {
        ChunkV<T> c1 = ld_chunk<T>(p + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[j] += to_f32(c0.e[j]); acc[4 + j] += to_f32(c1.e[j]); }
      }
    }
  } else {
    for (int r = r0 + rg; r < r1; r += 32)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (n0 + j < N) acc[j] += to_f32(x[(int64_t)r * ld + n0 + j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cg * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int n = blockIdx.x * 64 + threadIdx.x;
    float s = 0.f;
    for (int r = 0; r < 32; ++r) s += red[r][threadIdx.x];
    if (n < N) part[(int64_t)blockIdx.y * N + n] = s;
  }
}

// number of row chunks for a colsum over [m, n]: ~1024 blocks total, >= 32 rows each
int colsum_chunks(int m, int n) {
  const int cb = (n + 63) / 64;
  int r = 1024 / cb;
  if (r < 1) r = 1;
  const int max_r = (m + 31) / 32;
  if (r > max_r) r = max_r;
  return r < 1 ? 1 : r;
}

// ------------------------------------------------------------ embedding
template <typename T>
__global__ void embed_fwd_kernel(const int64_t* ids, const T* table, T* out, int M, int C, int V) {
  const int64_t total = (int64_t)M * C;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int m = (int)(i / C), c = (int)(i % C);
    const int64_t id = ids[m];
    out[i] = (id >= 0 && id < V) ? table[id * C + c] : from_f32<T>(0.f);
  }
}

// Gather form, deterministic (no atomics): workgroup (v, column block of 512) writes table row
// v's gradient = sum over the rows m with ids[m] == v of dout[m], added in increasing m (the same
// bits every run, whatever the collisions).  The ids are taken in chunks of EB_CHUNK rows: each
// of the 8 waves ballots its slice of the chunk, the matching rows are compacted into an LDS
// list in row order (wave offsets from the per-wave counts), then every thread adds its column of
// those rows with EB_UNROLL loads in flight.  Rows == pad_idx (and out-of-range ids) get no
// gradient; every table row is written, not accumulated.
constexpr int EB_NT = 512, EB_CHUNK = 4096, EB_UNROLL = 8;
template <typename T>
__global__ __launch_bounds__(EB_NT) void embed_bwd_kernel(const int64_t* ids, const T* dout, float* dtable, int M,
                                                          int C, int V, int pad_idx) {
  __shared__ int list[EB_CHUNK];
  __shared__ int wcnt[EB_NT / 64];
  const int v = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * EB_NT + threadIdx.x;
  constexpr int PERW = EB_CHUNK / (EB_NT / 64);   // rows per wave per chunk
  float acc = 0.f;
  if (v != pad_idx) {
    for (int base = 0; base < M; base += EB_CHUNK) {
      const int r0 = base + w * PERW;
      uint64_t masks[PERW / 64];
      int n = 0;
#pragma unroll
      for (int i = 0; i < PERW / 64; ++i) {
        const int m = r0 + 64 * i + lane;
        masks[i] = __ballot(m < M && ids[m] == (int64_t)v);
        n += __builtin_popcountll(masks[i]);
      }
      if (lane == 0) wcnt[w] = n;
      __syncthreads();
      int off = 0, total = 0;
#pragma unroll
      for (int k = 0; k < EB_NT / 64; ++k) {
        off += k < w ? wcnt[k] : 0;
        total += wcnt[k];
      }
#pragma unroll
      for (int i = 0; i < PERW / 64; ++i) {
        const uint64_t below = lane ? (masks[i] & (~0ull >> (64 - lane))) : 0ull;
        if ((masks[i] >> lane) & 1ull) list[off + __builtin_popcountll(below)] = r0 + 64 * i + lane;
        off += __builtin_popcountll(masks[i]);
      }
      __syncthreads();
      if (c < C) {
        int i = 0;
        for (; i + EB_UNROLL <= total; i += EB_UNROLL) {
          float x[EB_UNROLL];
#pragma unroll
          for (int u = 0; u < EB_UNROLL; ++u) x[u] = to_f32(dout[(int64_t)list[i + u] * C + c]);
#pragma unroll
          for (int u = 0; u < EB_UNROLL; ++u) acc += x[u];
        }
        for (; i < total; ++i) acc += to_f32(dout[(int64_t)list[i] * C + c]);
      }
      __syncthreads();   // the list is rebuilt for the next chunk
    }
  }
  if (c < C) dtable[(int64_t)v * C + c] = acc;
}

// ------------------------------------------------------ positional encoding
// out = drop(x + alpha * pe[t]),  t = row % T
template <typename T>
__global__ void pe_fwd_kernel(const T* x, const float* alpha, const float* pe, T* out, int M, int C, int Tlen,
                              int t_off, const int32_t* t_ptr, DropDesc drop) {
  const int64_t total = (int64_t)M * C;
  const float al = *alpha;
  if (t_ptr) t_off += *t_ptr;
  const uint32_t seed = drop.thr ? *drop.seed : 0u;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int m = (int)(i / C), c = (int)(i % C);
    const int t = m % Tlen + t_off;
    float v = to_f32(x[i]) + al * pe[(int64_t)t * C + c];
    if (drop.thr) v = drop_apply(drop, seed, (uint32_t)i, v);
    out[i] = from_f32<T>(v);
  }
}
// 8 elements per thread (C % 8 == 0, bf16 / f32): 16-B loads, 32-bit chunk indexing, the
// dropout bits of the chunk from drop_bits8, nontemporal stores
template <typename T>
__global__ __launch_bounds__(NT) void pe_fwd8_kernel(const T* x, const float* alpha, const float* pe, T* out, int M,
                                                     int C, int Tlen, int t_off, const int32_t* t_ptr, DropDesc drop) {
  const int cpr = C >> 3, nchunk = M * cpr;
  const float al = *alpha;
  if (t_ptr) t_off += *t_ptr;
  const uint32_t seed = drop.thr ? *drop.seed : 0u;
  for (int q = blockIdx.x * NT + threadIdx.x; q < nchunk; q += gridDim.x * NT) {
    const int m = q / cpr, c0 = (q - m * cpr) * 8, t = m % Tlen + t_off;
    const uint32_t i0 = (uint32_t)m * C + c0;
    float v[8];
    if constexpr (sizeof(T) == 2) {
      const bf16x8 xv = *reinterpret_cast<const bf16x8*>(x + i0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)xv[j];
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(x + i0), b = *reinterpret_cast<const f32x4*>(x + i0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
    }
    const f32x4 p0 = *reinterpret_cast<const f32x4*>(pe + (int64_t)t * C + c0);
    const f32x4 p1 = *reinterpret_cast<const f32x4*>(pe + (int64_t)t * C + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += al * p0[j]; v[4 + j] += al * p1[j]; }
    if (drop.thr) drop_apply8(drop, seed, i0, v);
    if constexpr (sizeof(T) == 2) {
      bf16 o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
      __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(o), reinterpret_cast<u32x4*>(out + i0));
    } else {
      __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(out + i0));
      __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(out + i0) + 1);
    }
  }
}

// dx = drop'(dout); part[block] = sum dx * pe
// dx = drop(dout) and a per-block partial of dalpha = sum(dx * pe[t]).  8-element
// chunks (C % 8 == 0): 16-B loads, 32-bit chunk indexing.
template <typename T>
__global__ __launch_bounds__(NT) void pe_bwd_kernel(const T* dout, const float* pe, T* dx, float* part, int M, int C,
                                                    int Tlen, DropDesc drop) {
  __shared__ float red[NT / 64];
  const int cpr = C >> 3, nchunk = M * cpr;
  const uint32_t seed = drop.thr ? *drop.seed : 0u;
  float s = 0.f;
  for (int q = blockIdx.x * NT + threadIdx.x; q < nchunk; q += gridDim.x * NT) {
    const int m = q / cpr, c0 = (q - m * cpr) * 8;
    const int t = m % Tlen;
    const int64_t i0 = (int64_t)m * C + c0;
    float g[8];
    if constexpr (sizeof(T) == 2) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(dout + i0);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (float)v[j];
    } else {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(dout + i0), hi = *reinterpret_cast<const f32x4*>(dout + i0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { g[j] = lo[j]; g[4 + j] = hi[j]; }
    }
    if (drop.thr) drop_apply8(drop, seed, (uint32_t)i0, g);
    const f32x4 p0 = *reinterpret_cast<const f32x4*>(pe + (int64_t)t * C + c0);
    const f32x4 p1 = *reinterpret_cast<const f32x4*>(pe + (int64_t)t * C + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) s += g[j] * p0[j] + g[4 + j] * p1[j];
    if constexpr (sizeof(T) == 2) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)g[j];
      *reinterpret_cast<bf16x8*>(dx + i0) = o;
    } else {
      *reinterpret_cast<f32x4*>(dx + i0) = f32x4{g[0], g[1], g[2], g[3]};
      *reinterpret_cast<f32x4*>(dx + i0 + 4) = f32x4{g[4], g[5], g[6], g[7]};
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

// ------------------------------------------------------ teacher forcing input
// out[b*T + t, c] = t == 0 ? 0 : mel[b, t-1, c]
template <typename T>
__global__ void shift_right_kernel(const float* mel, T* out, int B, int Tlen, int C) {
  const int64_t total = (int64_t)B * Tlen * C;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t m = i / C;
    const int t = (int)(m % Tlen);
    out[i] = from_f32<T>(t == 0 ? 0.f : mel[i - C]);
  }
}

__global__ void cast2d_kernel(const void* src, int sdt, int64_t sld, void* dst, int ddt, int64_t dld, int M, int N) {
  const int64_t total = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int m = (int)(i / N), n = (int)(i % N);
    stf(dst, (int64_t)m * dld + n, ddt, ldf(src, (int64_t)m * sld + n, sdt));
  }
}

// ------------------------------------------------------------------- loss
// heads [M, hld] f32: cols 0..79 mel_before, col 80 stop logit.  after [M, 80] f32.
// Writes: part[block][4] = (sum sq before, sum sq after, sum bce, 0);
//         g_heads[m, 0..79] = d/dbefore (direct + residual from after), g_heads[m, 80] = d/dstop,
//         g_heads[m, 81..hld) = 0; g_after[m, c] (T) = d/dafter.
template <typename T>
__global__ __launch_bounds__(NT) void loss_kernel(const float* heads, int64_t hld, const float* after,
                                                  const float* target, const int32_t* mel_len, int B, int Tlen,
                                                  int NM, float pos_weight, float gscale, float* g_heads, T* g_after, float* part,
                                                  int separate, int vec4) {
  __shared__ float red[3][NT / 64];
  int nvalid = 0;
  for (int b = 0; b < B; ++b) nvalid += min(max(mel_len[b], 0), Tlen);
  const float inv_n = nvalid > 0 ? gscale / nvalid : 0.f;
  const float inv_nm = inv_n / NM;
  const int M = B * Tlen;
  const int64_t total = vec4 ? 0 : (int64_t)M * hld;
  float sb = 0.f, sa = 0.f, ss = 0.f;
  if (vec4) {   // 4 columns per thread (hld, NM % 4 == 0, 16-B aligned rows): 32-bit indexing, vector loads
    const int cpr = (int)(hld >> 2), nchunk = M * cpr;
    for (int q = blockIdx.x * NT + threadIdx.x; q < nchunk; q += gridDim.x * NT) {
      const int m = q / cpr, c0 = (q - m * cpr) * 4;
      const int b = m / Tlen, t = m - b * Tlen;
      const int len = mel_len[b];
      const bool valid = t < len;
      const f32x4 hv = *reinterpret_cast<const f32x4*>(heads + (int64_t)m * hld + c0);
      f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
      if (c0 + 4 <= NM) {
        const int64_t j = (int64_t)m * NM + c0;
        const f32x4 tg = *reinterpret_cast<const f32x4*>(target + j), af = *reinterpret_cast<const f32x4*>(after + j);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float db = hv[k] - tg[k], da = af[k] - tg[k];
          float ga = 0.f;
          if (valid) {
            sb += db * db;
            sa += da * da;
            g[k] = 2.f * db * inv_nm;
            ga = 2.f * da * inv_nm;
          }
          g_after[j + k] = from_f32<T>(ga);
          if (!separate) g[k] += ga;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (c0 + k != NM || !valid) continue;
          const float x = hv[k];
          const float y = (t == len - 1) ? 1.f : 0.f;
          const float lsp = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
          const float lsn = fminf(-x, 0.f) - log1pf(expf(-fabsf(x)));
          ss += -(pos_weight * y * lsp + (1.f - y) * lsn);
          const float sg = 1.f / (1.f + expf(-x));
          g[k] = (pos_weight * y * (sg - 1.f) + (1.f - y) * sg) * inv_n;
        }
      }
      *reinterpret_cast<f32x4*>(g_heads + (int64_t)m * hld + c0) = g;
    }
  }
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int m = (int)(i / hld), c = (int)(i % hld);
    const int b = m / Tlen, t = m % Tlen;
    const int len = mel_len[b];
    const bool valid = t < len;
    float g = 0.f;
    if (c < NM) {
      const int64_t j = (int64_t)m * NM + c;
      const float db = heads[i] - target[j];
      const float da = after[j] - target[j];
      float ga = 0.f;
      if (valid) {
        sb += db * db;
        sa += da * da;
        g = 2.f * db * inv_nm;
        ga = 2.f * da * inv_nm;
      }
      g_after[j] = from_f32<T>(ga);
      if (!separate) g += ga;  // mel_after = mel_before + postnet(mel_before): residual path
    } else if (c == NM) {
      const float x = heads[i];
      const float y = (t == len - 1) ? 1.f : 0.f;
      if (valid) {
        // BCEWithLogits(pos_weight): l = -[pw*y*log s(x) + (1-y)*log(1-s(x))]
        const float lsp = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));   // log sigmoid(x)
        const float lsn = fminf(-x, 0.f) - log1pf(expf(-fabsf(x)));  // log sigmoid(-x)
        ss += -(pos_weight * y * lsp + (1.f - y) * lsn);
        const float sg = 1.f / (1.f + expf(-x));
        g = (pos_weight * y * (sg - 1.f) + (1.f - y) * sg) * inv_n;
      }
    }
    g_heads[i] = g;
  }
  sb = wave_sum(sb); sa = wave_sum(sa); ss = wave_sum(ss);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = sb; red[1][w] = sa; red[2][w] = ss; }
  __syncthreads();
  if (threadIdx.x < 3) {
    float t = 0.f;
    for (int k = 0; k < NT / 64; ++k) t += red[threadIdx.x][k];
    part[blockIdx.x * 4 + threadIdx.x] = t;
  }
}

// one wave: lane l sums partial rows l, l + 64, ... (loads issued together), then lane 0
// adds the 64 lane sums in lane order (fixed order: reproducible)
__global__ void loss_finalize_kernel(const float* part, int nblocks, const int32_t* mel_len, int B, int Tlen, int NM,
                                     float* out) {
  __shared__ float red[3][64];
  const int l = threadIdx.x;
  float a[3] = {0.f, 0.f, 0.f};
  for (int i = l; i < nblocks; i += 64) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(part + i * 4);
    a[0] += v[0]; a[1] += v[1]; a[2] += v[2];
  }
  red[0][l] = a[0]; red[1][l] = a[1]; red[2][l] = a[2];
  __syncthreads();
  if (l != 0) return;
  int nvalid = 0;
  for (int b = 0; b < B; ++b) nvalid += min(max(mel_len[b], 0), Tlen);
  float s[3] = {0.f, 0.f, 0.f};
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 64; ++i) s[k] += red[k][i];
  const float n = nvalid > 0 ? (float)nvalid : 1.f;
  out[1] = s[0] / (n * NM);
  out[2] = s[1] / (n * NM);
  out[3] = s[2] / n;
  out[0] = out[1] + out[2] + out[3];
}

// ------------------------------------------------------------ weight repack
// conv dgrad weight: wd[ci][tap'][co] = w[co][K-1-tap'][ci] -- per tap a [Cout x Cin] ->
// [Cin x Cout] transpose through a 64 x 64 LDS tile: reads coalesced along ci, writes along co.
template <typename T>
TT2_DEV void conv_wflip_tile(const T* w, T* wd, int Cout, int Cin, int K, int bx, int by, int tap) {
  __shared__ T tile[64][65];
  const int ci0 = bx * 64, co0 = by * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int r = ty; r < 64; r += NT / 64) {
    const int co = co0 + r, ci = ci0 + tx;
    if (co < Cout && ci < Cin) tile[r][tx] = w[((int64_t)co * K + tap) * Cin + ci];
  }
  __syncthreads();
  const int tp = K - 1 - tap;
#pragma unroll 4
  for (int r = ty; r < 64; r += NT / 64) {
    const int ci = ci0 + r, co = co0 + tx;
    if (co < Cout && ci < Cin) wd[((int64_t)ci * K + tp) * Cout + co] = tile[tx][r];
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void conv_wflip_kernel(const T* w, T* wd, int Cout, int Cin, int K) {
  conv_wflip_tile<T>(w, wd, Cout, Cin, K, blockIdx.x, blockIdx.y, blockIdx.z);
}

// every conv layer's flip in one launch: workgroup b belongs to the job whose item range
// [first[j], first[j + 1]) holds it; items are (tap, co block, ci block) in that order
struct WflipBatch {
  tt2_wflip_job job[TT2_WFLIP_MAX];
  int first[TT2_WFLIP_MAX + 1];
  int n;
};
template <typename T>
__global__ __launch_bounds__(NT) void conv_wflip_batch_kernel(WflipBatch B) {
  int j = 0;
  while (j + 1 < B.n && (int)blockIdx.x >= B.first[j + 1]) ++j;
  const tt2_wflip_job& J = B.job[j];
  const int it = blockIdx.x - B.first[j], nbx = (J.cin + 63) / 64, nby = (J.cout + 63) / 64;
  conv_wflip_tile<T>(reinterpret_cast<const T*>(J.w), reinterpret_cast<T*>(J.wd), J.cout, J.cin, J.k, it % nbx,
                     (it / nbx) % nby, it / (nbx * nby));
}

// nn.Conv1d weight [Cout][Cin][K] -> tap-major [Cout][K][Cin]: per output channel a
// [Cin x K] -> [K x Cin] transpose (weights are small; one thread per element, writes coalesced)
template <typename T>
__global__ __launch_bounds__(NT) void conv_wpack_kernel(const T* w, T* wp, int Cout, int Cin, int K) {
  const int64_t total = (int64_t)Cout * Cin * K;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int ci = (int)(i % Cin);
    const int64_t r = i / Cin;
    const int tap = (int)(r % K), co = (int)(r / K);
    wp[i] = w[((int64_t)co * Cin + ci) * K + tap];
  }
}

// ------------------------------------------------------------------ Adam
__global__ __launch_bounds__(NT) void sumsq_kernel(const float* g, int64_t n, float* part) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  const int64_t n4 = n / 4;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const f32x4 v = g4[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

struct AdamArgs {
  float* p; const float* g; float* m; float* v; bf16* shadow;
  int64_t n;
  const float* sumsq;   // clip: global squared gradient norm (device scalar) or null
  int32_t* step;        // device step counter (read; bumped by tt2_step_bump)
  const int32_t* gate;  // null, or: update only while *gate != 0 (tt2_adam_gate)
  float lr, beta1, beta2, eps, wd, clip, warmup, d_model_rsqrt;
  int noam;
};

TT2_DEV void adam_one(const AdamArgs& a, int64_t i, float g, float lr, float step_size, float bc2_sqrt) {
  float p = a.p[i];
  if (a.wd != 0.f) p -= lr * a.wd * p;  // decoupled (AdamW) weight decay
  const float m = a.beta1 * a.m[i] + (1.f - a.beta1) * g;
  const float v = a.beta2 * a.v[i] + (1.f - a.beta2) * g * g;
  a.m[i] = m;
  a.v[i] = v;
  p -= step_size * m / (sqrtf(v) / bc2_sqrt + a.eps);
  a.p[i] = p;
  if (a.shadow) a.shadow[i] = (bf16)p;
}

// one thread updates 4 consecutive parameters (n is a multiple of 16: slots are 16-aligned)
__global__ __launch_bounds__(NT) void adam_kernel(AdamArgs a) {
  if (a.gate && *a.gate == 0) return;   // a deferred update that already ran (or none pending)
  const int step = *a.step + 1;
  float scale = 1.f;
  if (a.clip > 0.f && a.sumsq) {
    const float nrm = sqrtf(*a.sumsq);
    if (nrm > a.clip) scale = a.clip / (nrm + 1e-6f);
  }
  float lr = a.lr;
  if (a.noam) lr = a.lr * a.d_model_rsqrt * fminf(rsqrtf((float)step), step * powf(a.warmup, -1.5f));
  const float bc1 = 1.f - powf(a.beta1, (float)step);
  const float bc2 = 1.f - powf(a.beta2, (float)step);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const int64_t n4 = a.n / 4;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const f32x4 g = reinterpret_cast<const f32x4*>(a.g)[i];
    const f32x4 p = reinterpret_cast<const f32x4*>(a.p)[i];
    const f32x4 m = reinterpret_cast<const f32x4*>(a.m)[i];
    const f32x4 v = reinterpret_cast<const f32x4*>(a.v)[i];
    f32x4 po, mo, vo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = g[j] * scale;
      float pj = p[j];
      if (a.wd != 0.f) pj -= lr * a.wd * pj;
      mo[j] = a.beta1 * m[j] + (1.f - a.beta1) * gj;
      vo[j] = a.beta2 * v[j] + (1.f - a.beta2) * gj * gj;
      po[j] = pj - step_size * mo[j] / (sqrtf(vo[j]) / bc2_sqrt + a.eps);
    }
    // nontemporal: every lane's 16 B (8 B for the shadow) continue its neighbours' into
    // whole lines, which stream to memory instead of being written back at the kernel's end
    __builtin_nontemporal_store(po, reinterpret_cast<f32x4*>(a.p) + i);
    __builtin_nontemporal_store(mo, reinterpret_cast<f32x4*>(a.m) + i);
    __builtin_nontemporal_store(vo, reinterpret_cast<f32x4*>(a.v) + i);
    if (a.shadow) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      bf16x4 sh;
#pragma unroll
      for (int j = 0; j < 4; ++j) sh[j] = (bf16)po[j];
      __builtin_nontemporal_store(*reinterpret_cast<const u32x2*>(&sh), reinterpret_cast<u32x2*>(a.shadow) + i);
    }
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)NT + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * NT)
    adam_one(a, i, a.g[i] * scale, lr, step_size, bc2_sqrt);
}

__global__ void step_bump_kernel(int32_t* step, uint32_t* seed) {
  if (threadIdx.x == 0) {
    if (step) step[0] += 1;
    if (seed) seed[0] += 1u;
  }
}

__global__ void adam_gate_kernel(int32_t* gate, int32_t* step, int op) {
  if (threadIdx.x == 0) {
    if (op == 1) {
      gate[0] = 1;
    } else if (gate[0] != 0) {
      if (step) step[0] += 1;
      gate[0] = 0;
    }
  }
}

}  // namespace

// =============================================================== C ABI
extern "C" int tt2_reduce_rows(const tt2_reduce_args* p, hipStream_t s) {
  if (p->cols <= 0) return TT2_OK;
  int cw = 1;
  while (cw < p->cols && cw < RR_COLS) cw <<= 1;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((p->cols + cw - 1) / cw), dim3(NT), 0, s, p->src, p->rows, p->cols,
                     p->ld, p->dst, p->beta, cw);
  return tt2_check_launch(hipGetLastError(), "tt2_reduce_rows");
}

extern "C" size_t tt2_colsum_workspace_size(int m, int n) {
  return (size_t)colsum_chunks(m, n) * n * sizeof(float);
}

extern "C" int tt2_colsum(const void* x, int dtype, int64_t ld, int m, int n, float* dst, float beta, void* ws,
                          size_t ws_bytes, hipStream_t s) {
  if (n <= 0) return TT2_OK;
  if (ws_bytes < tt2_colsum_workspace_size(m, n)) return tt2_set_error(TT2_E_INVALID, "tt2_colsum: workspace");
  const int R = colsum_chunks(m, n);
  const int rows_per = (m + R - 1) / R;
  float* part = reinterpret_cast<float*>(ws);
  const int esz = dtype == TT2_DT_BF16 ? 2 : 4;
  const int vec = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && ((ld * esz) % 16 == 0);
  dim3 g((n + 63) / 64, R);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, g, dim3(NT), 0, s, (const bf16*)x, ld, m, n, rows_per, vec, part);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, g, dim3(NT), 0, s, (const float*)x, ld, m, n, rows_per, vec,
                       part);
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((n + RR_COLS - 1) / RR_COLS), dim3(NT), 0, s, part, R, n, (int64_t)n,
                     dst, beta, RR_COLS);
  return tt2_check_launch(hipGetLastError(), "tt2_colsum");
}

extern "C" int tt2_embedding_fwd(const int64_t* ids, const void* table, void* out, int m, int c, int vocab,
                                 int dtype, hipStream_t s) {
  const int g = grid_for((int64_t)m * c);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(embed_fwd_kernel<bf16>, dim3(g), dim3(NT), 0, s, ids, (const bf16*)table, (bf16*)out, m, c, vocab);
  else
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3(g), dim3(NT), 0, s, ids, (const float*)table, (float*)out, m, c,
                       vocab);
  return tt2_check_launch(hipGetLastError(), "tt2_embedding_fwd");
}

extern "C" int tt2_embedding_bwd(const int64_t* ids, const void* dout, float* dtable, int m, int c, int vocab,
                                 int pad_idx, int dtype, hipStream_t s) {
  if (vocab <= 0 || c <= 0) return TT2_OK;
  const dim3 g(vocab, (c + EB_NT - 1) / EB_NT);   // every table row written: no memset
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(embed_bwd_kernel<bf16>, g, dim3(EB_NT), 0, s, ids, (const bf16*)dout, dtable, m, c, vocab,
                       pad_idx);
  else
    hipLaunchKernelGGL(embed_bwd_kernel<float>, g, dim3(EB_NT), 0, s, ids, (const float*)dout, dtable, m, c,
                       vocab, pad_idx);
  return tt2_check_launch(hipGetLastError(), "tt2_embedding_bwd");
}

extern "C" int tt2_posenc_fwd(const tt2_pe_args* p, hipStream_t s) {
  DropDesc d{p->drop_seed, p->drop_site, p->drop_thr, p->drop_scale};
  const bool v8 = p->c % 8 == 0 && (int64_t)p->m * p->c < (1ll << 31) &&
                  reinterpret_cast<uintptr_t>(p->x) % 16 == 0 && reinterpret_cast<uintptr_t>(p->out) % 16 == 0;
  if (v8) {
    const int g8 = grid_for((int64_t)p->m * p->c / 8);
    if (p->dtype == TT2_DT_BF16)
      hipLaunchKernelGGL(pe_fwd8_kernel<bf16>, dim3(g8), dim3(NT), 0, s, (const bf16*)p->x, p->alpha, p->pe,
                         (bf16*)p->out, p->m, p->c, p->t, p->t_offset, p->t_ptr, d);
    else
      hipLaunchKernelGGL(pe_fwd8_kernel<float>, dim3(g8), dim3(NT), 0, s, (const float*)p->x, p->alpha, p->pe,
                         (float*)p->out, p->m, p->c, p->t, p->t_offset, p->t_ptr, d);
    return tt2_check_launch(hipGetLastError(), "tt2_posenc_fwd");
  }
  const int g = grid_for((int64_t)p->m * p->c);
  if (p->dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(pe_fwd_kernel<bf16>, dim3(g), dim3(NT), 0, s, (const bf16*)p->x, p->alpha, p->pe,
                       (bf16*)p->out, p->m, p->c, p->t, p->t_offset, p->t_ptr, d);
  else
    hipLaunchKernelGGL(pe_fwd_kernel<float>, dim3(g), dim3(NT), 0, s, (const float*)p->x, p->alpha, p->pe,
                       (float*)p->out, p->m, p->c, p->t, p->t_offset, p->t_ptr, d);
  return tt2_check_launch(hipGetLastError(), "tt2_posenc_fwd");
}

extern "C" size_t tt2_posenc_bwd_workspace_size(void) { return TT2_PE_BWD_BLOCKS * sizeof(float); }

extern "C" int tt2_posenc_bwd(const tt2_pe_args* p, hipStream_t s) {
  if (!p->workspace || p->ws_bytes < tt2_posenc_bwd_workspace_size())
    return tt2_set_error(TT2_E_INVALID, "tt2_posenc_bwd: workspace");
  if (p->c % 8 || (int64_t)p->m * p->c >= (1ll << 31))
    return tt2_set_error(TT2_E_INVALID, "tt2_posenc_bwd: C must be a multiple of 8 and M*C < 2^31");
  DropDesc d{p->drop_seed, p->drop_site, p->drop_thr, p->drop_scale};
  float* part = reinterpret_cast<float*>(p->workspace);
  if (p->dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(pe_bwd_kernel<bf16>, dim3(TT2_PE_BWD_BLOCKS), dim3(NT), 0, s, (const bf16*)p->dout, p->pe,
                       (bf16*)p->dx, part, p->m, p->c, p->t, d);
  else
    hipLaunchKernelGGL(pe_bwd_kernel<float>, dim3(TT2_PE_BWD_BLOCKS), dim3(NT), 0, s, (const float*)p->dout, p->pe,
                       (float*)p->dx, part, p->m, p->c, p->t, d);
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(1), dim3(NT), 0, s, part, TT2_PE_BWD_BLOCKS, 1, (int64_t)1,
                     p->dalpha, 0.f, 1);
  return tt2_check_launch(hipGetLastError(), "tt2_posenc_bwd");
}

extern "C" int tt2_shift_right(const float* mel, void* out, int batch, int t, int c, int dtype, hipStream_t s) {
  const int g = grid_for((int64_t)batch * t * c);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(shift_right_kernel<bf16>, dim3(g), dim3(NT), 0, s, mel, (bf16*)out, batch, t, c);
  else
    hipLaunchKernelGGL(shift_right_kernel<float>, dim3(g), dim3(NT), 0, s, mel, (float*)out, batch, t, c);
  return tt2_check_launch(hipGetLastError(), "tt2_shift_right");
}

extern "C" int tt2_cast2d(const void* src, int src_dtype, int64_t src_ld, void* dst, int dst_dtype, int64_t dst_ld,
                          int m, int n, hipStream_t s) {
  if ((int64_t)m * n == 0) return TT2_OK;
  hipLaunchKernelGGL(cast2d_kernel, dim3(grid_for((int64_t)m * n)), dim3(NT), 0, s, src, src_dtype, src_ld, dst,
                     dst_dtype, dst_ld, m, n);
  return tt2_check_launch(hipGetLastError(), "tt2_cast2d");
}

extern "C" size_t tt2_loss_workspace_size(void) { return TT2_LOSS_BLOCKS * 4 * sizeof(float); }

extern "C" int tt2_tts_loss(const tt2_loss_args* p, hipStream_t s) {
  if (p->n_mels + 1 > p->heads_ld) return tt2_set_error(TT2_E_INVALID, "tt2_tts_loss: heads_ld too small");
  if (!p->workspace || p->ws_bytes < tt2_loss_workspace_size())
    return tt2_set_error(TT2_E_INVALID, "tt2_tts_loss: workspace");
  float* part = reinterpret_cast<float*>(p->workspace);
  auto al16 = [](const void* q) { return reinterpret_cast<uintptr_t>(q) % 16 == 0; };
  const int vec4 = p->heads_ld % 4 == 0 && p->n_mels % 4 == 0 && al16(p->heads) && al16(p->g_heads) &&
                   al16(p->mel_after) && al16(p->target);
  if (p->grad_dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(loss_kernel<bf16>, dim3(TT2_LOSS_BLOCKS), dim3(NT), 0, s, p->heads, p->heads_ld,
                       p->mel_after, p->target, p->mel_len, p->batch, p->t, p->n_mels, p->pos_weight, p->grad_scale, p->g_heads,
                       (bf16*)p->g_after, part, p->separate_grads, vec4);
  else
    hipLaunchKernelGGL(loss_kernel<float>, dim3(TT2_LOSS_BLOCKS), dim3(NT), 0, s, p->heads, p->heads_ld,
                       p->mel_after, p->target, p->mel_len, p->batch, p->t, p->n_mels, p->pos_weight, p->grad_scale, p->g_heads,
                       (float*)p->g_after, part, p->separate_grads, vec4);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, s, part, TT2_LOSS_BLOCKS, p->mel_len, p->batch,
                     p->t, p->n_mels, p->loss_out);
  return tt2_check_launch(hipGetLastError(), "tt2_tts_loss");
}

extern "C" int tt2_conv_weight_flip(const void* w, void* wd, int cout, int cin, int k, int dtype, hipStream_t s) {
  if (cout <= 0 || cin <= 0 || k <= 0) return TT2_OK;
  const dim3 g((cin + 63) / 64, (cout + 63) / 64, k);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(conv_wflip_kernel<bf16>, g, dim3(NT), 0, s, (const bf16*)w, (bf16*)wd, cout, cin, k);
  else
    hipLaunchKernelGGL(conv_wflip_kernel<float>, g, dim3(NT), 0, s, (const float*)w, (float*)wd, cout, cin, k);
  return tt2_check_launch(hipGetLastError(), "tt2_conv_weight_flip");
}

extern "C" int tt2_conv_weight_flip_batch(const tt2_wflip_job* jobs, int32_t n, int32_t dtype, hipStream_t s) {
  if (n <= 0) return TT2_OK;
  if (n > TT2_WFLIP_MAX || !jobs) return tt2_set_error(TT2_E_INVALID, "tt2_conv_weight_flip_batch: 1..16 jobs");
  WflipBatch B{};
  B.n = n;
  for (int j = 0; j < n; ++j) {
    const tt2_wflip_job& J = jobs[j];
    if (J.cout <= 0 || J.cin <= 0 || J.k <= 0 || !J.w || !J.wd || J.w == J.wd)
      return tt2_set_error(TT2_E_INVALID, "tt2_conv_weight_flip_batch: bad job");
    B.job[j] = J;
    B.first[j + 1] = B.first[j] + ((J.cin + 63) / 64) * ((J.cout + 63) / 64) * J.k;
  }
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(conv_wflip_batch_kernel<bf16>, dim3(B.first[n]), dim3(NT), 0, s, B);
  else
    hipLaunchKernelGGL(conv_wflip_batch_kernel<float>, dim3(B.first[n]), dim3(NT), 0, s, B);
  return tt2_check_launch(hipGetLastError(), "tt2_conv_weight_flip_batch");
}

extern "C" int tt2_conv_weight_pack(const void* w, void* wp, int32_t cout, int32_t cin, int32_t k, int32_t dtype,
                                    hipStream_t s) {
  if (cout <= 0 || cin <= 0 || k <= 0) return TT2_OK;
  if (!w || !wp || w == wp) return tt2_set_error(TT2_E_INVALID, "tt2_conv_weight_pack: null or in-place");
  const int64_t total = (int64_t)cout * cin * k;
  const int g = (int)std::min<int64_t>((total + NT - 1) / NT, 4096);
  if (dtype == TT2_DT_BF16)
    hipLaunchKernelGGL(conv_wpack_kernel<bf16>, dim3(g), dim3(NT), 0, s, (const bf16*)w, (bf16*)wp, cout, cin, k);
  else if (dtype == TT2_DT_F32)
    hipLaunchKernelGGL(conv_wpack_kernel<float>, dim3(g), dim3(NT), 0, s, (const float*)w, (float*)wp, cout, cin, k);
  else
    return tt2_set_error(TT2_E_INVALID, "tt2_conv_weight_pack: dtype");
  return tt2_check_launch(hipGetLastError(), "tt2_conv_weight_pack");
}

extern "C" size_t tt2_adam_workspace_size(void) { return (TT2_ADAM_NORM_BLOCKS + 16) * sizeof(float); }

extern "C" int tt2_adam_step(const tt2_adam_args* p, hipStream_t s) {
  AdamArgs a{};
  a.p = p->params; a.g = p->grads; a.m = p->exp_avg; a.v = p->exp_avg_sq; a.shadow = (bf16*)p->shadow_bf16;
  a.n = p->n; a.step = p->step; a.gate = p->gate;
  a.lr = p->lr; a.beta1 = p->beta1; a.beta2 = p->beta2; a.eps = p->eps; a.wd = p->weight_decay;
  a.clip = p->clip_norm; a.warmup = p->warmup; a.noam = p->noam;
  a.d_model_rsqrt = p->d_model > 0 ? 1.f / sqrtf((float)p->d_model) : 1.f;
  if ((reinterpret_cast<uintptr_t>(p->params) | reinterpret_cast<uintptr_t>(p->grads) |
       reinterpret_cast<uintptr_t>(p->exp_avg) | reinterpret_cast<uintptr_t>(p->exp_avg_sq)) % 16 ||
      reinterpret_cast<uintptr_t>(p->shadow_bf16) % 8)
    return tt2_set_error(TT2_E_INVALID, "tt2_adam_step: buffers must be 16-B aligned");
  if (p->clip_norm > 0.f) {
    if (!p->workspace || p->ws_bytes < tt2_adam_workspace_size())
      return tt2_set_error(TT2_E_INVALID, "tt2_adam_step: workspace");
    if (p->norm_parts && p->norm_nparts <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_adam_step: norm_nparts");
    float* part = reinterpret_cast<float*>(p->workspace);
    float* total = part + TT2_ADAM_NORM_BLOCKS;
    if (!p->norm_parts)
      hipLaunchKernelGGL(sumsq_kernel, dim3(TT2_ADAM_NORM_BLOCKS), dim3(NT), 0, s, p->grads, p->n, part);
    hipLaunchKernelGGL(reduce_rows_kernel, dim3(1), dim3(NT), 0, s, p->norm_parts ? p->norm_parts : part,
                       p->norm_parts ? p->norm_nparts : TT2_ADAM_NORM_BLOCKS, 1, (int64_t)1, total, 0.f, 1);
    a.sumsq = total;
  }
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(p->n / 4)), dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_adam_step");
}

extern "C" int tt2_sumsq_parts(const float* g, int64_t n, float* parts, int32_t nparts, hipStream_t s) {
  if (!g || !parts || nparts <= 0 || n < 0 || (reinterpret_cast<uintptr_t>(g) % 16))
    return tt2_set_error(TT2_E_INVALID, "tt2_sumsq_parts: g 16-B aligned, parts, nparts > 0");
  hipLaunchKernelGGL(sumsq_kernel, dim3(nparts), dim3(NT), 0, s, g, n, parts);
  return tt2_check_launch(hipGetLastError(), "tt2_sumsq_parts");
}

extern "C" int tt2_adam_gate(int32_t* gate, int32_t* step, int32_t op, hipStream_t s) {
  if (!gate || (op != 0 && op != 1)) return tt2_set_error(TT2_E_INVALID, "tt2_adam_gate: gate, op 0 or 1");
  hipLaunchKernelGGL(adam_gate_kernel, dim3(1), dim3(64), 0, s, gate, step, (int)op);
  return tt2_check_launch(hipGetLastError(), "tt2_adam_gate");
}

extern "C" int tt2_step_bump(int32_t* step, uint32_t* seed, hipStream_t s) {
  if (!step && !seed) return TT2_OK;
  hipLaunchKernelGGL(step_bump_kernel, dim3(1), dim3(64), 0, s, step, seed);
  return tt2_check_launch(hipGetLastError(), "tt2_step_bump");
}

// ------------------------------------------------------------ DP exchange stand-in
// A kernel with the footprint of one rank's share of an N-rank ring all-reduce of a bucket
// (measurement of the DP schedule on one GPU, tt2/dist.py StandinGradSync): `wgs` work groups
// (RCCL's channels) copy `bytes` from the bucket into a scratch buffer (the reduce-scatter /
// all-gather traffic through HBM), then each holds its CU until `ticks` of the device wall clock
// have passed since it started (the time the ring waits on its xGMI links).  Every wave exits:
// the wait is bounded by the clock, not by a flag.
__global__ __launch_bounds__(256) void comm_standin_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                           int64_t n16, uint64_t ticks, uint64_t* rec) {
  const uint64_t t0 = wall_clock64();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (rec && threadIdx.x == 0) {   // this work group's {start, end} on the wall clock
    rec[2 * blockIdx.x] = t0;
    rec[2 * blockIdx.x + 1] = wall_clock64();
  }
}

extern "C" int tt2_comm_standin(const void* src, void* scratch, size_t bytes, double seconds, int32_t wgs,
                                uint64_t* rec, hipStream_t s) {
  if (!src || !scratch || wgs <= 0 || wgs > 1024 || seconds < 0 || seconds > 1.0 ||
      (reinterpret_cast<uintptr_t>(src) % 16) || (reinterpret_cast<uintptr_t>(scratch) % 16))
    return tt2_set_error(TT2_E_INVALID, "tt2_comm_standin: 16-B aligned src / scratch, 0 < wgs <= 1024, "
                                        "0 <= seconds <= 1");
  static int khz = 0;
  if (!khz) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) {
      khz = 0;
      return tt2_set_error(TT2_E_HIP, "tt2_comm_standin: no wall clock rate");
    }
  }
  const uint64_t ticks = (uint64_t)(seconds * khz * 1e3);
  hipLaunchKernelGGL(comm_standin_kernel, dim3(wgs), dim3(256), 0, s, reinterpret_cast<const u32x4*>(src),
                     reinterpret_cast<u32x4*>(scratch), (int64_t)(bytes / 16), ticks, rec);
  return tt2_check_launch(hipGetLastError(), "tt2_comm_standin");
}
