// norm.hip -- fused residual + dropout + LayerNorm, and training/eval BatchNorm
// with fused activation + dropout (+ residual), forward and backward (gfx950).
//
// LayerNorm (post-LN sublayer end):
//   s = x + drop(branch);  y = (s - mean(s)) * rstd * gamma + beta
// one wave per 512-wide row (8 values per lane, 16-B vector loads).  The
// backward recomputes s from the saved x and branch (no s buffer) and emits
// ds (the residual-stream gradient) and drop-masked ds (the branch gradient),
// plus per-workgroup gamma/beta partial sums reduced by tt2_reduce_rows.
//
// BatchNorm1d over rows (SURVEY 8(a) a1 encoder convs, a9 post-net):
//   train: per-chunk (mean, M2) partials -> Chan combine -> mean, rstd, running
//   stats update (unbiased var, momentum); eval: running stats.
//   z = act((y - mean) * rstd * gamma + beta); out = drop(z) (+ res)
// The backward recomputes z from y (saved) and the statistics.
#include <math.h>
#include <stdlib.h>

#include "tt2_capi.h"
#include "tt2_internal.h"
#include "tt2_common.h"

namespace {

constexpr int NT = 256;

template <typename T> TT2_DEV void ld8(const T* p, float (&v)[8]);
template <> TT2_DEV void ld8(const bf16* p, float (&v)[8]) {
  bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> TT2_DEV void ld8(const f16* p, float (&v)[8]) {
  f16x8 x = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> TT2_DEV void ld8(const float* p, float (&v)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
template <typename T> TT2_DEV void st8(T* p, const float (&v)[8]);
template <> TT2_DEV void st8(bf16* p, const float (&v)[8]) {
  bf16x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
  *reinterpret_cast<bf16x8*>(p) = x;
}
template <> TT2_DEV void st8(f16* p, const float (&v)[8]) {
  f16x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (f16)v[j];
  *reinterpret_cast<f16x8*>(p) = x;
}
template <> TT2_DEV void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
// Nontemporal form for the training kernels' full-tensor outputs: the rows stream out as
// they are produced instead of sitting dirty in L2 until the end-of-kernel write-back.
template <typename T> TT2_DEV void st8nt(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(p));
    __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(p) + 1);
  } else {
    T x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (T)v[j];
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(x), reinterpret_cast<u32x4*>(p));
  }
}

// --------------------------------------------------------------- LayerNorm
// A deferred LayerNorm-backward finalize: column sums of part[nb][3][C] into (dg, db, dd).
struct LnFin {
  const float* part;
  float* dg; float* db; float* dd;
  float gb;
  int nb;   // 0 = nothing to finalize
};

struct LnArgs {
  const void* x; const void* branch; const void* dy;
  void* y; void* dx; void* dbranch;
  const float* gamma; const float* beta;
  float* mean; float* rstd;
  float* part;  // bwd: [gridDim.x][3][C] (dgamma, dbeta, dbias) partial sums
  float* dgamma; float* dbeta; float* dbias;
  float grad_beta;
  int M, C;
  float eps;
  DropDesc drop;
  LnFin fin;   // bwd: an earlier deferred call's finalize, done in this launch's spare waves
};

template <typename T> TT2_DEV void unpack8(const uint4 (&u)[sizeof(T) / 2], float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    union { uint4 q; bf16x8 b; } c;
    c.q = u[0];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)c.b[j];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = __uint_as_float((&u[0].x)[j]); v[4 + j] = __uint_as_float((&u[1].x)[j]); }
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(LnArgs a) {
  constexpr int NV = sizeof(T) / 2;   // 16-B vectors per 8 elements
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.M) return;
  const int c0 = lane * 8;
  const int64_t off = (int64_t)row * a.C + c0;
  // every load of the row first (x, branch, gamma, beta, the dropout seed): one round trip
  // (a branch-dependent load behind the x unpack used to cost a second one)
  const bool has_br = a.branch != nullptr;
  const uint4* X = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.x) + off);
  const uint4* BR = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(has_br ? a.branch : a.x) + off);
  uint4 xr[NV], brr[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) { xr[v] = X[v]; brr[v] = BR[v]; }
  const f32x4 g0 = *reinterpret_cast<const f32x4*>(a.gamma + c0), g1 = *reinterpret_cast<const f32x4*>(a.gamma + c0 + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.beta + c0), b1 = *reinterpret_cast<const f32x4*>(a.beta + c0 + 4);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  float s[8], br[8];
  unpack8<T>(xr, s);
  if (has_br) {
    unpack8<T>(brr, br);
    if (a.drop.thr) drop_apply8(a.drop, seed, (uint32_t)off, br);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += br[j];
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) sum += s[j];
  const float mean = wave_sum(sum) / a.C;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { const float d = s[j] - mean; sq += d * d; }
  const float rstd = rsqrtf(wave_sum(sq) / a.C + a.eps);
  float y[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    y[j] = (s[j] - mean) * rstd * g0[j] + b0[j];
    y[4 + j] = (s[4 + j] - mean) * rstd * g1[j] + b1[j];
  }
  st8nt(reinterpret_cast<T*>(a.y) + off, y);
  if (lane == 0 && a.mean) { a.mean[row] = mean; a.rstd[row] = rstd; }
}

// Decode-step residual combine + LayerNorm: y = LN(x + bias + sum_s part[s]) over the
// 512 columns of a row, where part holds the raw partial sums of a skinny split-K
// projection ([S][M][512] f32).  One wave per row, every load (x, the S slabs, bias,
// gamma, beta) issued before the first reduction: one memory round trip.
#ifndef LNC_ROWS
#define LNC_ROWS 1   // rows (waves) per work group: one row per CU reads its 8 slabs faster than 4 (r06zp)
#endif
template <int S, typename T>
__global__ __launch_bounds__(64 * LNC_ROWS) void ln_combine_kernel(const T* x, const float* part, const float* bias,
                                                                   const float* gamma, const float* beta, T* y, int M,
                                                                   float eps) {
  constexpr int C = 512;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LNC_ROWS + (threadIdx.x >> 6);
  if (row >= M) return;
  float o[8];
  ln_combine_row<S, T>(x + (int64_t)row * C, part + (int64_t)row * C, (int64_t)M * C, bias, gamma, beta, eps, lane,
                       o);
  st8(y + (int64_t)row * C + lane * 8, o);
}

// Backward: 8 waves per workgroup, one 512-wide row per wave at a time, software-
// pipelined: the raw x / branch / dy chunks of the wave's next row are loaded before the
// current row is reduced, so every wave always has a row of loads in flight.  The
// dropout keep-mask of an element is hashed once and used for both s = x + drop(br)
// and dbranch = drop(ds).  Per-workgroup (dgamma, dbeta, dbias) column partials go to
// part[block][3][C]; ln_bwd_finalize sums them (fixed order: bitwise reproducible).
// 12 waves: 17.0-17.5 us at 12800 x 512 against 18.0-18.5 with 8 and 18.0 with 16
// (tools/norm_ab.py, gpurun_out/r05ln)
constexpr int LNB_NT = 768;
template <typename T> struct LnRow { uint4 x[sizeof(T) / 2], dy[sizeof(T) / 2], br[sizeof(T) / 2]; float mean, rstd; };

template <typename T>
TT2_DEV void ln_row_load(LnRow<T>& r, const LnArgs& a, int row, int c0) {
  constexpr int NV = sizeof(T) / 2;   // 16-B vectors per 8 elements
  const int64_t off = (int64_t)row * a.C + c0;
  const uint4* X = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.x) + off);
  const uint4* DY = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dy) + off);
#pragma unroll
  for (int v = 0; v < NV; ++v) { r.x[v] = X[v]; r.dy[v] = DY[v]; }
  if (a.branch) {
    const uint4* BR = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.branch) + off);
#pragma unroll
    for (int v = 0; v < NV; ++v) r.br[v] = BR[v];
  }
  r.mean = a.mean[row];
  r.rstd = a.rstd[row];
}


// One wave sums output o (= which * C + c) of a deferred finalize over the nb partial rows
// (4 loads in flight per lane, then a DPP wave sum): a fixed order, shared by the chained
// and the standalone finalize.
TT2_DEV void ln_fin_col(const LnFin& f, int C, int o, int lane) {
  const int which = o / C, c = o - which * C;
  float* dst = which == 0 ? f.dg : (which == 1 ? f.db : f.dd);
  if (!dst) return;
  const float* src = f.part + (int64_t)which * C + c;
  const int64_t rs = 3 * (int64_t)C;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int r = lane;
  for (; r + 192 < f.nb; r += 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += src[(r + 64 * u) * rs];
  }
  for (; r < f.nb; r += 64) acc[0] += src[r * rs];
  const float v = wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
  if (lane == 0) dst[c] = f.gb != 0.f ? f.gb * dst[c] + v : v;
}

__global__ __launch_bounds__(LNB_NT) void ln_fin_kernel(LnFin f, int C) {
  const int o = blockIdx.x * (LNB_NT / 64) + (threadIdx.x >> 6);
  if (o < 3 * C) ln_fin_col(f, C, o, threadIdx.x & 63);
}

template <typename T>
__global__ __launch_bounds__(LNB_NT) void ln_bwd_kernel(LnArgs a) {
  constexpr int HW = LNB_NT / 128;   // half the waves
  __shared__ float red[3][HW][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * 8;
  float g[8];
  {
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(a.gamma + c0), g1 = *reinterpret_cast<const f32x4*>(a.gamma + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { g[j] = g0[j]; g[4 + j] = g1[j]; }
  }
  float pg[8], pb[8], pd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pg[j] = pb[j] = pd[j] = 0.f;
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  const int stride = gridDim.x * (LNB_NT / 64);
  int row = blockIdx.x * (LNB_NT / 64) + w;
  LnRow<T> cur, nxt;
  if (row < a.M) ln_row_load<T>(cur, a, row, c0);
  for (; row < a.M; row += stride) {
    if (row + stride < a.M) ln_row_load<T>(nxt, a, row + stride, c0);
    const int64_t off = (int64_t)row * a.C + c0;
    float s[8], dy[8], keep[8];
    unpack8<T>(cur.x, s);
    unpack8<T>(cur.dy, dy);
    {
      const uint32_t kb = a.drop.thr ? drop_bits8(seed, a.drop.site, (uint32_t)off, a.drop.thr) : 0xFFu;
      const float sc = a.drop.thr ? a.drop.scale : 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) keep[j] = (kb >> j) & 1u ? sc : 0.f;
    }
    if (a.branch) {
      float br[8];
      unpack8<T>(cur.br, br);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += br[j] * keep[j];
    }
    float c1 = 0.f, c2 = 0.f, xh[8], gd[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xh[j] = (s[j] - cur.mean) * cur.rstd;
      gd[j] = g[j] * dy[j];
      c1 += gd[j];
      c2 += gd[j] * xh[j];
      pg[j] += dy[j] * xh[j];
      pb[j] += dy[j];
    }
    c1 = wave_sum(c1) / a.C;
    c2 = wave_sum(c2) / a.C;
    float ds[8], db[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ds[j] = cur.rstd * (gd[j] - c1 - xh[j] * c2);
      db[j] = ds[j] * keep[j];
      pd[j] += db[j];
    }
    st8nt(reinterpret_cast<T*>(a.dx) + off, ds);
    if (a.dbranch) st8nt(reinterpret_cast<T*>(a.dbranch) + off, db);
    cur = nxt;
  }
  // the waves' partials: the upper half into LDS rows, the lower half adds its own, then rows summed
  if (w >= HW) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][w - HW][c0 + j] = pg[j]; red[1][w - HW][c0 + j] = pb[j]; red[2][w - HW][c0 + j] = pd[j]; }
  }
  __syncthreads();
  if (w < HW) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][w][c0 + j] += pg[j]; red[1][w][c0 + j] += pb[j]; red[2][w][c0 + j] += pd[j]; }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * a.C; i += LNB_NT) {
    const int which = i / a.C, c = i % a.C;
    float v = red[which][0][c] + red[which][1][c] + red[which][2][c] + red[which][3][c];
#pragma unroll
    for (int h = 4; h < HW; ++h) v += red[which][h][c];
    a.part[((int64_t)blockIdx.x * 3 + which) * a.C + c] = v;
  }
  if (a.fin.nb) {   // the previous LayerNorm's column sums, spread over every workgroup's waves
    const int per = (3 * a.C + gridDim.x - 1) / gridDim.x;
    for (int i = w; i < per; i += LNB_NT / 64) {
      const int o = blockIdx.x * per + i;
      if (o < 3 * a.C) ln_fin_col(a.fin, a.C, o, lane);
    }
  }
}

// grid (C / 16, 3): 16 columns of partial array y per block, 16 row groups of 16
// lanes; each lane sums nb/16 partial rows with independent loads in flight.
__global__ __launch_bounds__(256) void ln_bwd_finalize(LnArgs a, int nb) {
  __shared__ float sm[16][17];
  const int which = blockIdx.y;
  float* dst = which == 0 ? a.dgamma : (which == 1 ? a.dbeta : a.dbias);
  if (!dst) return;
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  const float* src = a.part + (int64_t)which * a.C + c;
  const int64_t rs = 3 * (int64_t)a.C;   // stride between partial rows
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int r = rg;
  for (; r + 48 < nb; r += 64) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += src[(r + 16 * u) * rs];
  }
  for (; r < nb; r += 16) acc[0] += src[r * rs];
  sm[rg][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (rg == 0) {
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) v += sm[g][cl];
    dst[c] = a.grad_beta != 0.f ? a.grad_beta * dst[c] + v : v;
  }
}

// --------------------------------------------------------------- BatchNorm
struct BnArgs {
  const void* y; const void* dout; const void* res;
  void* out; void* dy;
  const float* gamma; const float* beta;
  float* mean; float* rstd;
  float* run_mean; float* run_var;
  float* part;  // train stats: [R][2][C] (chunk mean, chunk M2); bwd: [R][2][C] sums
  float* dgamma; float* dbeta;
  int64_t res_ld;
  int M, C, R, rows_per, act, out_dt, res_dt, training;
  float eps, momentum;
  DropDesc drop;
  // SyncBatchNorm exchange (tt2_batchnorm_{fwd,bwd}_{stats,apply}): [W][3][C] rank slots
  // (this rank's moments or sums and its row count, zeros in the others; all-reduced by the
  // caller) + [2][C]
  float* sync;
  int W, rank;
  int64_t Mtot;   // rows behind the statistics: M (SyncBN: the exchanged counts, see inv_m)
  const float* inv_m;   // SyncBN backward apply: 1 / (sum of the ranks' rows), written by bn_bwd_sync_kernel
};

// (fast_tanh, act_f, act_grad_from_out: tt2_common.h, shared with the GEMM's fused BatchNorm sums)

// All BatchNorm kernels work on 8-column groups (16-B loads/stores; C % 8 == 0).
// Statistics: one workgroup per chunk of rows_per rows; CG = C/8 column groups x
// (256/CG) row lanes.  Chunk moments use a per-column shift (the chunk's first row)
// so sum / sum-of-squares keep full precision; chunks are combined exactly in double.

TT2_DEV void ld8v(const void* p, int64_t off, int dt, float (&v)[8]) {
  if (dt == TT2_BF16) ld8(reinterpret_cast<const bf16*>(p) + off, v);
  else ld8(reinterpret_cast<const float*>(p) + off, v);
}

template <typename T>
__global__ __launch_bounds__(NT) void bn_stats_kernel(BnArgs a) {
  __shared__ float red[2][NT][8];
  const int CG = a.C >> 3, nrl = NT / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int r0 = blockIdx.x * a.rows_per, r1 = min(a.M, r0 + a.rows_per);
  const T* y = reinterpret_cast<const T*>(a.y);
  float k[8], s1[8], s2[8];
  ld8(y + (int64_t)r0 * a.C + cg * 8, k);
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (rl < nrl) {
    for (int r = r0 + rl; r < r1; r += nrl) {
      float v[8];
      ld8(y + (int64_t)r * a.C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - k[j];
        s1[j] += d;
        s2[j] += d * d;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
  __syncthreads();
  if (threadIdx.x < CG) {
    const float n = (float)(r1 - r0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float S1 = 0.f, S2 = 0.f;
      for (int l = 0; l < nrl; ++l) { S1 += red[0][l * CG + cg][j]; S2 += red[1][l * CG + cg][j]; }
      const int c = cg * 8 + j;
      a.part[((int64_t)blockIdx.x * 2 + 0) * a.C + c] = k[j] + S1 / n;
      a.part[((int64_t)blockIdx.x * 2 + 1) * a.C + c] = fmaxf(S2 - S1 * S1 / n, 0.f);
    }
  }
}

// Chunk combine of 64 columns per workgroup: thread (column cl = t % 64, group g = t / 64)
// walks chunks r = g, g + 4, ... (4 loads in flight), then the 4 group partials are added in
// order.  Exact two-pass combine of the chunk moments (no per-chunk division): mean =
// sum n_c mean_c / n, then M2 = sum M2_c + n_c (mean_c - mean)^2, accumulated in double.  The
// standalone finalize (grid ceil(C / 64)) and the apply kernels that finalize their own column
// block (bn_apply_fin_kernel) run this same code, so both give the same statistics.
constexpr int BNC_COLS = 64, BNC_G = NT / BNC_COLS;
// bn_fin64 / bn_bsum64 combine exactly red[0..3] in a fixed order (the standalone finalize's
// summation order, which the fused apply must reproduce bit for bit)
static_assert(BNC_G == 4, "bn_fin64 / bn_bsum64 sum four chunk groups");
struct BnFinScratch { double red[BNC_G][BNC_COLS]; double mu[BNC_COLS]; float mean[BNC_COLS], rstd[BNC_COLS]; };

// forward: mean / rstd of column block cb into S.mean / S.rstd; write: also a.mean / a.rstd and
// the running statistics (or, SyncBN, this rank's slots)
TT2_DEV void bn_fin64(const BnArgs& a, int cb, BnFinScratch& S, bool write) {
  const int cl = threadIdx.x % BNC_COLS, g = threadIdx.x / BNC_COLS;
  const int c = cb * BNC_COLS + cl;
  const bool ok = c < a.C;
  const int cc = ok ? c : 0;
  auto nrows = [&](int r) { return (double)min(a.rows_per, a.M - r * a.rows_per); };
  auto pm = [&](int r, int w) { return a.part[((int64_t)r * 2 + w) * a.C + cc]; };
  double acc = 0.0;
  int r = g;
  for (; r + 3 * BNC_G < a.R; r += 4 * BNC_G) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = pm(r + u * BNC_G, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += nrows(r + u * BNC_G) * v[u];
  }
  for (; r < a.R; r += BNC_G) acc += nrows(r) * pm(r, 0);
  S.red[g][cl] = acc;
  __syncthreads();
  if (g == 0) S.mu[cl] = (((S.red[0][cl] + S.red[1][cl]) + S.red[2][cl]) + S.red[3][cl]) / a.M;
  __syncthreads();
  const double mu = S.mu[cl];
  acc = 0.0;
  r = g;
  for (; r + 3 * BNC_G < a.R; r += 4 * BNC_G) {
    float m1[4], m2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { m1[u] = pm(r + u * BNC_G, 0); m2[u] = pm(r + u * BNC_G, 1); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double d = m1[u] - mu;
      acc += m2[u] + nrows(r + u * BNC_G) * d * d;
    }
  }
  for (; r < a.R; r += BNC_G) {
    const double d = pm(r, 0) - mu;
    acc += pm(r, 1) + nrows(r) * d * d;
  }
  __syncthreads();
  S.red[g][cl] = acc;
  __syncthreads();
  if (g != 0) return;
  const double m2 = ((S.red[0][cl] + S.red[1][cl]) + S.red[2][cl]) + S.red[3][cl];
  const double n = a.M;
  const double var = m2 / n;
  S.mean[cl] = (float)mu;
  S.rstd[cl] = (float)(1.0 / sqrt(var + a.eps));
  if (!write || !ok) return;
  if (a.sync) {   // this rank's (mean, M2, rows) into its slot; the other ranks' slots zero
    for (int r2 = 0; r2 < a.W; ++r2) {
      a.sync[((int64_t)r2 * 3 + 0) * a.C + c] = r2 == a.rank ? (float)mu : 0.f;
      a.sync[((int64_t)r2 * 3 + 1) * a.C + c] = r2 == a.rank ? (float)m2 : 0.f;
      a.sync[((int64_t)r2 * 3 + 2) * a.C + c] = r2 == a.rank ? (float)a.M : 0.f;
    }
    return;
  }
  a.mean[c] = S.mean[cl];
  a.rstd[c] = S.rstd[cl];
  if (a.run_mean) {
    const double unb = n > 1 ? m2 / (n - 1) : var;
    a.run_mean[c] = (float)((1.0 - a.momentum) * a.run_mean[c] + a.momentum * mu);
    a.run_var[c] = (float)((1.0 - a.momentum) * a.run_var[c] + a.momentum * unb);
  }
}

__global__ __launch_bounds__(NT) void bn_finalize_kernel(BnArgs a) {
  __shared__ BnFinScratch S;
  if (!a.training) {   // eval: the running statistics
    const int c = blockIdx.x * BNC_COLS + threadIdx.x;
    if (threadIdx.x < BNC_COLS && c < a.C) {
      a.mean[c] = a.run_mean[c];
      a.rstd[c] = rsqrtf(a.run_var[c] + a.eps);
    }
    return;
  }
  bn_fin64(a, blockIdx.x, S, true);
}

// SyncBatchNorm: combine the W exchanged rank moments in rank order, exactly as
// bn_finalize_kernel combines chunks, weighted by each rank's row count n_r (ranks may hold
// different numbers of rows): N = sum n_r, mean = sum n_r mean_r / N,
// M2 = sum M2_r + n_r (mean_r - mean)^2.  Slots are [W][3][C]: (mean, M2, n) per rank.
__global__ __launch_bounds__(NT) void bn_sync_finalize_kernel(BnArgs a) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= a.C) return;
  double n = 0.0, mu = 0.0;
  for (int r = 0; r < a.W; ++r) {
    const double nr = (double)a.sync[((int64_t)r * 3 + 2) * a.C + c];
    n += nr;
    mu += nr * (double)a.sync[((int64_t)r * 3 + 0) * a.C + c];
  }
  mu /= n;
  double m2 = 0.0;
  for (int r = 0; r < a.W; ++r) {
    const double d = (double)a.sync[((int64_t)r * 3 + 0) * a.C + c] - mu;
    m2 += (double)a.sync[((int64_t)r * 3 + 1) * a.C + c] + (double)a.sync[((int64_t)r * 3 + 2) * a.C + c] * d * d;
  }
  const double var = m2 / n;
  a.mean[c] = (float)mu;
  a.rstd[c] = (float)(1.0 / sqrt(var + a.eps));
  if (a.run_mean) {
    const double unb = n > 1 ? m2 / (n - 1) : var;
    a.run_mean[c] = (float)((1.0 - a.momentum) * a.run_mean[c] + a.momentum * mu);
    a.run_var[c] = (float)((1.0 - a.momentum) * a.run_var[c] + a.momentum * unb);
  }
}

// SyncBatchNorm backward: the global column sums (sum dpre, sum dpre * xhat) from the W
// exchanged rank slots, in rank order, into the [2][C] region after the slots, and
// 1 / N (N = sum of the ranks' row counts, as f32: the value bn_bwd_apply_kernel forms from
// Mtot on one rank, so one SyncBN rank reproduces plain BatchNorm bit for bit) after them
__global__ __launch_bounds__(NT) void bn_bwd_sync_kernel(BnArgs a) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= a.C) return;
  float s1 = 0.f, s2 = 0.f, n = 0.f;
  for (int r = 0; r < a.W; ++r) {
    s1 += a.sync[((int64_t)r * 3 + 0) * a.C + c];
    s2 += a.sync[((int64_t)r * 3 + 1) * a.C + c];
    n += a.sync[((int64_t)r * 3 + 2) * a.C + c];
  }
  a.sync[((int64_t)a.W * 3 + 0) * a.C + c] = s1;
  a.sync[((int64_t)a.W * 3 + 1) * a.C + c] = s2;
  if (c == 0) a.sync[((int64_t)a.W * 3 + 2) * a.C] = 1.f / n;
}

// per-column constants of 8 consecutive columns
TT2_DEV void col8(const float* p, int c0, float (&v)[8]) {
  const f32x4 lo = *reinterpret_cast<const f32x4*>(p + c0), hi = *reinterpret_cast<const f32x4*>(p + c0 + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
}

template <typename T>
__global__ __launch_bounds__(NT) void bn_apply_kernel(BnArgs a) {
  const int CG = a.C >> 3;
  const int nq = a.M * CG;
  const T* y = reinterpret_cast<const T*>(a.y);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  for (int q = blockIdx.x * NT + threadIdx.x; q < nq; q += gridDim.x * NT) {
    const int m = q / CG, c0 = (q - m * CG) * 8;
    const int64_t i0 = (int64_t)m * a.C + c0;
    float v[8], mu[8], rs[8], g[8], b[8];
    ld8(y + i0, v);
    col8(a.mean, c0, mu); col8(a.rstd, c0, rs); col8(a.gamma, c0, g); col8(a.beta, c0, b);
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = act_f(a.act, (v[j] - mu[j]) * rs[j] * g[j] + b[j]);
    if (a.drop.thr) drop_apply8(a.drop, seed, (uint32_t)i0, z);
    if (a.res) {
      float r[8];
      ld8v(a.res, (int64_t)m * a.res_ld + c0, a.res_dt, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] += r[j];
    }
    if (a.out_dt == TT2_BF16) st8nt(reinterpret_cast<bf16*>(a.out) + i0, z);
    else st8nt(reinterpret_cast<float*>(a.out) + i0, z);
  }
}

// dpre = d(pre-activation BN output): recompute z from y.
// keep: the element's dropout factor (0 or 1 / (1 - p); 1 without dropout)
TT2_DEV float bn_dpre(const BnArgs& a, float keep, float xh, float g, float b, float doutv) {
  const float z = act_f(a.act, xh * g + b);
  return doutv * keep * act_grad_from_out(a.act, z);
}
// the dropout factors of elements i0 .. i0 + 7 (drop_bits8: 4-5 hashes for 8 elements)
TT2_DEV void bn_keep8(const BnArgs& a, uint32_t seed, int64_t i0, float (&k)[8]) {
  const uint32_t bits = a.drop.thr ? drop_bits8(seed, a.drop.site, (uint32_t)i0, a.drop.thr) : 0xFFu;
  const float sc = a.drop.thr ? a.drop.scale : 1.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = (bits >> j) & 1u ? sc : 0.f;
}

template <typename T, typename TD>
__global__ __launch_bounds__(NT) void bn_bwd_stats_kernel(BnArgs a) {
  __shared__ float red[2][NT][8];
  const int CG = a.C >> 3, nrl = NT / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int c0 = cg * 8;
  const int r0 = blockIdx.x * a.rows_per, r1 = min(a.M, r0 + a.rows_per);
  const T* y = reinterpret_cast<const T*>(a.y);
  const TD* dout = reinterpret_cast<const TD*>(a.dout);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  float s1[8], s2[8], mu[8], rs[8], g[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  col8(a.mean, c0, mu); col8(a.rstd, c0, rs); col8(a.gamma, c0, g); col8(a.beta, c0, b);
  if (rl < nrl) {
    for (int r = r0 + rl; r < r1; r += nrl) {
      const int64_t i0 = (int64_t)r * a.C + c0;
      float v[8], d[8], kp[8];
      ld8(y + i0, v);
      ld8(dout + i0, d);
      bn_keep8(a, seed, i0, kp);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (v[j] - mu[j]) * rs[j];
        const float dp = bn_dpre(a, kp[j], xh, g[j], b[j], d[j]);
        s1[j] += dp;
        s2[j] += dp * xh;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
  __syncthreads();
  if (threadIdx.x < CG) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float S1 = 0.f, S2 = 0.f;
      for (int l = 0; l < nrl; ++l) { S1 += red[0][l * CG + cg][j]; S2 += red[1][l * CG + cg][j]; }
      a.part[((int64_t)blockIdx.x * 2 + 0) * a.C + c0 + j] = S1;
      a.part[((int64_t)blockIdx.x * 2 + 1) * a.C + c0 + j] = S2;
    }
  }
}

// backward: the chunk sums (sum dpre, sum dpre * xhat) of column block cb, in bn_fin64's order,
// into db / dg (LDS); write: also a.dbeta / a.dgamma (this rank's parameter gradients) and the
// SyncBN slots
struct BnBsumScratch { float red[2][BNC_G][BNC_COLS]; float db[BNC_COLS], dg[BNC_COLS]; };
TT2_DEV void bn_bsum64(const BnArgs& a, int cb, BnBsumScratch& S, bool write) {
  const int cl = threadIdx.x % BNC_COLS, g = threadIdx.x / BNC_COLS;
  const int c = cb * BNC_COLS + cl;
  const int cc = c < a.C ? c : 0;
  float s1 = 0.f, s2 = 0.f;
  int r = g;
  for (; r + 3 * BNC_G < a.R; r += 4 * BNC_G) {
    float v1[4], v2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v1[u] = a.part[((int64_t)(r + u * BNC_G) * 2 + 0) * a.C + cc];
      v2[u] = a.part[((int64_t)(r + u * BNC_G) * 2 + 1) * a.C + cc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += v1[u]; s2 += v2[u]; }
  }
  for (; r < a.R; r += BNC_G) {
    s1 += a.part[((int64_t)r * 2 + 0) * a.C + cc];
    s2 += a.part[((int64_t)r * 2 + 1) * a.C + cc];
  }
  S.red[0][g][cl] = s1;
  S.red[1][g][cl] = s2;
  __syncthreads();
  if (g != 0) return;
  const float t1 = ((S.red[0][0][cl] + S.red[0][1][cl]) + S.red[0][2][cl]) + S.red[0][3][cl];
  const float t2 = ((S.red[1][0][cl] + S.red[1][1][cl]) + S.red[1][2][cl]) + S.red[1][3][cl];
  S.db[cl] = t1;
  S.dg[cl] = t2;
  if (!write || c >= a.C) return;
  a.dbeta[c] = t1;    // this rank's parameter gradients (the DP all-reduce sums them)
  a.dgamma[c] = t2;
  if (a.sync) {
    for (int r2 = 0; r2 < a.W; ++r2) {
      a.sync[((int64_t)r2 * 3 + 0) * a.C + c] = r2 == a.rank ? t1 : 0.f;
      a.sync[((int64_t)r2 * 3 + 1) * a.C + c] = r2 == a.rank ? t2 : 0.f;
      a.sync[((int64_t)r2 * 3 + 2) * a.C + c] = r2 == a.rank ? (float)a.M : 0.f;
    }
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_finalize_kernel(BnArgs a) {
  __shared__ BnBsumScratch S;
  bn_bsum64(a, blockIdx.x, S, true);
}

// one 8-column group of the backward apply (shared by bn_bwd_apply_kernel and the fused
// bn_bwd_apply_fin_kernel, so both compile the same expression: SyncBN at one rank stays
// bit-identical to plain BatchNorm)
TT2_DEV void bn_dy8(const BnArgs& a, const float (&v)[8], const float (&d)[8], const float (&kp)[8],
                    const float (&mu)[8], const float (&rs)[8], const float (&g)[8], const float (&b)[8],
                    const float (&db)[8], const float (&dg)[8], float invM, float (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float xh = (v[j] - mu[j]) * rs[j];
    const float dp = bn_dpre(a, kp[j], xh, g[j], b[j], d[j]);
    o[j] = a.training ? g[j] * rs[j] * (dp - db[j] * invM - xh * dg[j] * invM) : g[j] * rs[j] * dp;
  }
}

template <typename T, typename TD>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnArgs a) {
  const int CG = a.C >> 3;
  const int nq = a.M * CG;
  const T* y = reinterpret_cast<const T*>(a.y);
  const TD* dout = reinterpret_cast<const TD*>(a.dout);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  const float invM = a.inv_m ? *a.inv_m : 1.f / (float)a.Mtot;
  for (int q = blockIdx.x * NT + threadIdx.x; q < nq; q += gridDim.x * NT) {
    const int m = q / CG, c0 = (q - m * CG) * 8;
    const int64_t i0 = (int64_t)m * a.C + c0;
    float v[8], d[8], mu[8], rs[8], g[8], b[8], db[8], dg[8], o[8];
    ld8(y + i0, v);
    ld8(dout + i0, d);
    col8(a.mean, c0, mu); col8(a.rstd, c0, rs); col8(a.gamma, c0, g); col8(a.beta, c0, b);
    if (a.training) { col8(a.dbeta, c0, db); col8(a.dgamma, c0, dg); }
    float kp[8];
    bn_keep8(a, seed, i0, kp);
    bn_dy8(a, v, d, kp, mu, rs, g, b, db, dg, invM, o);
    st8nt(reinterpret_cast<T*>(a.dy) + i0, o);
  }
}

// Training apply with the finalize folded in: workgroup (column block x, row block y)
// first combines the chunk statistics of its 64 columns (bn_fin64 / bn_bsum64: the
// standalone finalize's code and order, ≈ 25 KB of chunk partials per workgroup), row block
// 0 writing mean / rstd / running statistics (forward) or dbeta / dgamma (backward), then
// applies them to its rows: one launch fewer per BatchNorm pass on the step's critical path.
// Threads: 8 column groups x 32 row lanes.
#ifndef BN_FUSED_FIN
#define BN_FUSED_FIN 1
#endif
TT2_DEV void bn_rows_of(const BnArgs& a, int& r0, int& r1) {
  const int per = (a.M + gridDim.y - 1) / gridDim.y;
  r0 = blockIdx.y * per;
  r1 = min(a.M, r0 + per);
}

template <typename T>
__global__ __launch_bounds__(NT) void bn_apply_fin_kernel(BnArgs a) {
  __shared__ BnFinScratch S;
  bn_fin64(a, blockIdx.x, S, blockIdx.y == 0);
  __syncthreads();
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * BNC_COLS + cg * 8;
  if (c0 >= a.C) return;
  int r0, r1;
  bn_rows_of(a, r0, r1);
  const T* y = reinterpret_cast<const T*>(a.y);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  float mu[8], rs[8], g[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { mu[j] = S.mean[cg * 8 + j]; rs[j] = S.rstd[cg * 8 + j]; }
  col8(a.gamma, c0, g); col8(a.beta, c0, b);
  for (int m = r0 + rl; m < r1; m += NT / 8) {
    const int64_t i0 = (int64_t)m * a.C + c0;
    float v[8];
    ld8(y + i0, v);
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = act_f(a.act, (v[j] - mu[j]) * rs[j] * g[j] + b[j]);
    if (a.drop.thr) drop_apply8(a.drop, seed, (uint32_t)i0, z);
    if (a.res) {
      float r[8];
      ld8v(a.res, (int64_t)m * a.res_ld + c0, a.res_dt, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] += r[j];
    }
    if (a.out_dt == TT2_BF16) st8nt(reinterpret_cast<bf16*>(a.out) + i0, z);
    else st8nt(reinterpret_cast<float*>(a.out) + i0, z);
  }
}

// FIN = false: the sums are already final in a.dbeta / a.dgamma (SyncBatchNorm: the exchanged
// global sums) and are only staged; the rest is the same code, so SyncBN at one rank stays
// bit-identical to plain BatchNorm
template <typename T, typename TD, bool FIN>
__global__ __launch_bounds__(NT) void bn_bwd_apply_fin_kernel(BnArgs a) {
  __shared__ BnBsumScratch S;
  if constexpr (FIN) {
    bn_bsum64(a, blockIdx.x, S, blockIdx.y == 0);
  } else if (threadIdx.x < BNC_COLS) {
    const int c = blockIdx.x * BNC_COLS + threadIdx.x;
    S.db[threadIdx.x] = c < a.C ? a.dbeta[c] : 0.f;
    S.dg[threadIdx.x] = c < a.C ? a.dgamma[c] : 0.f;
  }
  __syncthreads();
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * BNC_COLS + cg * 8;
  if (c0 >= a.C) return;
  int r0, r1;
  bn_rows_of(a, r0, r1);
  const T* y = reinterpret_cast<const T*>(a.y);
  const TD* dout = reinterpret_cast<const TD*>(a.dout);
  const uint32_t seed = a.drop.thr ? *a.drop.seed : 0u;
  const float invM = a.inv_m ? *a.inv_m : 1.f / (float)a.Mtot;   // (bn_bwd_apply_kernel's form)
  float mu[8], rs[8], g[8], b[8], db[8], dg[8];
  col8(a.mean, c0, mu); col8(a.rstd, c0, rs); col8(a.gamma, c0, g); col8(a.beta, c0, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) { db[j] = S.db[cg * 8 + j]; dg[j] = S.dg[cg * 8 + j]; }
  for (int m = r0 + rl; m < r1; m += NT / 8) {
    const int64_t i0 = (int64_t)m * a.C + c0;
    float v[8], d[8], o[8], kp[8];
    ld8(y + i0, v);
    ld8(dout + i0, d);
    bn_keep8(a, seed, i0, kp);
    bn_dy8(a, v, d, kp, mu, rs, g, b, db, dg, invM, o);
    st8nt(reinterpret_cast<T*>(a.dy) + i0, o);
  }
}

void bn_bwd_apply_fin(const BnArgs& a, bool bf, bool dbf, bool fin, dim3 grid, hipStream_t s) {
#define TT2_BNF(T_, TD_)                                                                           \
  if (fin) hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<T_, TD_, true>), grid, dim3(NT), 0, s, a);  \
  else hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<T_, TD_, false>), grid, dim3(NT), 0, s, a);
  if (bf && dbf) { TT2_BNF(bf16, bf16) }
  else if (bf) { TT2_BNF(bf16, float) }
  else if (dbf) { TT2_BNF(float, bf16) }
  else { TT2_BNF(float, float) }
#undef TT2_BNF
}

// (column blocks, row blocks) of the fused applies: about 512 workgroups, >= 32 rows each
dim3 bn_fin_grid(int m, int c) {
  const int ncb = (c + BNC_COLS - 1) / BNC_COLS;
  return dim3(ncb, std::max(1, std::min((m + 31) / 32, 512 / ncb)));
}

int grid_for(int64_t total) {
  int64_t b = (total + NT - 1) / NT;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

extern "C" int tt2_layernorm_fwd(const tt2_ln_args* p, hipStream_t s) {
  if (p->c != 512) return tt2_set_error(TT2_E_INVALID, "tt2_layernorm: C must be 512");
  LnArgs a{};
  a.x = p->x; a.branch = p->branch; a.y = p->y;
  a.gamma = p->gamma; a.beta = p->beta; a.mean = p->mean; a.rstd = p->rstd;
  a.M = p->m; a.C = p->c; a.eps = p->eps;
  a.drop = DropDesc{p->drop_seed, p->drop_site, p->drop_thr, p->drop_scale};
  if (p->m == 0) return TT2_OK;
  dim3 g((p->m + 3) / 4);
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(ln_fwd_kernel<bf16>, g, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(ln_fwd_kernel<float>, g, dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_layernorm_fwd");
}

extern "C" int tt2_ln_combine(const void* x, const float* part, int32_t splits, const float* bias,
                              const float* gamma, const float* beta, void* y, int32_t m, int32_t c, float eps,
                              int32_t dtype, hipStream_t s) {
  if (c != 512) return tt2_set_error(TT2_E_INVALID, "tt2_ln_combine: c must be 512");
  if (!x || !part || !bias || !gamma || !beta || !y) return tt2_set_error(TT2_E_INVALID, "tt2_ln_combine: null");
  if (dtype != TT2_DT_BF16 && dtype != TT2_DT_F16) return tt2_set_error(TT2_E_INVALID, "tt2_ln_combine: bf16 / f16");
  if (m <= 0) return TT2_OK;
  const dim3 g((m + LNC_ROWS - 1) / LNC_ROWS), b(64 * LNC_ROWS);
#define TT2_LNC(S)                                                                                             \
  if (dtype == TT2_DT_F16)                                                                                     \
    hipLaunchKernelGGL((ln_combine_kernel<S, f16>), g, b, 0, s, (const f16*)x, part, bias, gamma, beta,        \
                       (f16*)y, m, eps);                                                                       \
  else                                                                                                         \
    hipLaunchKernelGGL((ln_combine_kernel<S, bf16>), g, b, 0, s, (const bf16*)x, part, bias, gamma, beta,      \
                       (bf16*)y, m, eps);
  switch (splits) {
    case 1: TT2_LNC(1) break;
    case 2: TT2_LNC(2) break;
    case 4: TT2_LNC(4) break;
    case 8: TT2_LNC(8) break;
    case 16: TT2_LNC(16) break;
    default: return tt2_set_error(TT2_E_INVALID, "tt2_ln_combine: splits must be 1, 2, 4, 8 or 16");
  }
#undef TT2_LNC
  return tt2_check_launch(hipGetLastError(), "tt2_ln_combine");
}

static int ln_bwd_blocks(int m) {
  // at most one workgroup per CU, 16+ rows each (512 / 1024 / 128 work groups: 19.0-19.3 / 23.6 /
  // 21.5 us against 17.9-18.2 us at 12800 x 512, tools/norm_ab.py, gpurun_out/r05hp)
  return min(256, (m + 15) / 16);
}

static LnFin ln_fin_of(const tt2_ln_args* q) {
  return LnFin{reinterpret_cast<const float*>(q->workspace), q->dgamma, q->dbeta, q->dbias, q->grad_beta,
               ln_bwd_blocks(q->m)};
}

extern "C" size_t tt2_layernorm_bwd_workspace_size(const tt2_ln_args* p) {
  return (size_t)ln_bwd_blocks(p->m) * 3 * p->c * sizeof(float);
}

extern "C" int tt2_layernorm_bwd(const tt2_ln_args* p, hipStream_t s) {
  if (p->c != 512) return tt2_set_error(TT2_E_INVALID, "tt2_layernorm: C must be 512");
  if (!p->workspace || p->ws_bytes < tt2_layernorm_bwd_workspace_size(p))
    return tt2_set_error(TT2_E_INVALID, "tt2_layernorm_bwd: workspace too small");
  if (p->dbias && !p->branch) return tt2_set_error(TT2_E_INVALID, "tt2_layernorm_bwd: dbias needs a branch");
  LnArgs a{};
  a.x = p->x; a.branch = p->branch; a.dy = p->dy; a.dx = p->dx; a.dbranch = p->dbranch;
  a.gamma = p->gamma; a.beta = p->beta; a.mean = p->mean; a.rstd = p->rstd;
  a.part = reinterpret_cast<float*>(p->workspace);
  a.dgamma = p->dgamma; a.dbeta = p->dbeta; a.dbias = p->dbias; a.grad_beta = p->grad_beta;
  a.M = p->m; a.C = p->c; a.eps = p->eps;
  a.drop = DropDesc{p->drop_seed, p->drop_site, p->drop_thr, p->drop_scale};
  if (const tt2_ln_args* q = p->finalize_prev) {
    if (!q->defer_finalize || q->c != p->c || !q->workspace)
      return tt2_set_error(TT2_E_INVALID, "tt2_layernorm_bwd: finalize_prev must be a deferred call with the same c");
    if (q->workspace == p->workspace && q->m > 0)
      return tt2_set_error(TT2_E_INVALID, "tt2_layernorm_bwd: finalize_prev's workspace is overwritten by this call");
    if (q->m > 0) a.fin = ln_fin_of(q);
  }
  if (p->m == 0) {   // nothing of our own; still complete the chained finalize
    if (a.fin.nb) hipLaunchKernelGGL(ln_fin_kernel, dim3((3 * p->c + LNB_NT / 64 - 1) / (LNB_NT / 64)), dim3(LNB_NT), 0, s, a.fin, p->c);
    return tt2_check_launch(hipGetLastError(), "tt2_layernorm_bwd");
  }
  const int nb = ln_bwd_blocks(p->m);
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(ln_bwd_kernel<bf16>, dim3(nb), dim3(LNB_NT), 0, s, a);
  else hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(LNB_NT), 0, s, a);
  if (!p->defer_finalize) {
    a.fin = LnFin{};
    hipLaunchKernelGGL(ln_bwd_finalize, dim3(p->c / 16, 3), dim3(256), 0, s, a, nb);
  }
  return tt2_check_launch(hipGetLastError(), "tt2_layernorm_bwd");
}

extern "C" int tt2_layernorm_bwd_finalize(const tt2_ln_args* p, hipStream_t s) {
  if (!p->defer_finalize || !p->workspace) return tt2_set_error(TT2_E_INVALID, "tt2_layernorm_bwd_finalize: not a deferred call");
  if (p->m == 0) return TT2_OK;
  hipLaunchKernelGGL(ln_fin_kernel, dim3((3 * p->c + LNB_NT / 64 - 1) / (LNB_NT / 64)), dim3(LNB_NT), 0, s, ln_fin_of(p), p->c);
  return tt2_check_launch(hipGetLastError(), "tt2_layernorm_bwd_finalize");
}

// rows per statistics chunk: at most TT2_BN_ROWS_PER_CHUNK, fewer for short inputs
// so there are >= ~256 chunk workgroups (one per CU) when the rows allow it
static int bn_rows_per(int m) {
  int rp = TT2_BN_ROWS_PER_CHUNK;
  while (rp > 8 && (m + rp - 1) / rp < 256) rp >>= 1;
  return rp;
}

static BnArgs bn_args(const tt2_bn_args* p) {
  BnArgs a{};
  a.y = p->y; a.dout = p->dout; a.res = p->res; a.out = p->out; a.dy = p->dy;
  a.gamma = p->gamma; a.beta = p->beta; a.mean = p->mean; a.rstd = p->rstd;
  a.run_mean = p->run_mean; a.run_var = p->run_var;
  a.part = reinterpret_cast<float*>(p->workspace);
  a.dgamma = p->dgamma; a.dbeta = p->dbeta;
  a.M = p->m; a.C = p->c; a.act = p->act; a.out_dt = p->out_dtype; a.res_dt = p->res_dtype;
  a.res_ld = p->res_ld > 0 ? p->res_ld : p->c;
  a.training = p->training;
  a.eps = p->eps; a.momentum = p->momentum;
  // stats_rows > 0: the workspace already holds the chunk moments (tt2_gemm col_stats)
  a.rows_per = p->stats_rows > 0 ? p->stats_rows : bn_rows_per(p->m);
  a.R = (p->m + a.rows_per - 1) / a.rows_per;
  a.drop = DropDesc{p->drop_seed, p->drop_site, p->drop_thr, p->drop_scale};
  a.W = 1;
  a.Mtot = p->m;
  return a;
}

extern "C" size_t tt2_batchnorm_workspace_size(const tt2_bn_args* p) {
  const int rp = p->stats_rows > 0 ? p->stats_rows : bn_rows_per(p->m);
  const size_t R = (p->m + rp - 1) / rp;
  return R * 2 * p->c * sizeof(float);
}

static int bn_check(const tt2_bn_args* p, const char* what) {
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (p->c % 8 || p->c / 8 > NT) return tt2_set_error(TT2_E_INVALID, what);
  if (p->res && p->res_ld % 8) return tt2_set_error(TT2_E_INVALID, what);
  if (!al(p->y) || !al(p->out) || !al(p->res) || !al(p->dout) || !al(p->dy) || !al(p->gamma) || !al(p->beta) ||
      !al(p->mean) || !al(p->rstd) || !al(p->dgamma) || !al(p->dbeta))
    return tt2_set_error(TT2_E_INVALID, what);
  return TT2_OK;
}

extern "C" int tt2_batchnorm_fwd(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return TT2_OK;
  if (p->training && (!p->workspace || p->ws_bytes < tt2_batchnorm_workspace_size(p)))
    return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_fwd: workspace too small");
  if (bn_check(p, "tt2_batchnorm_fwd: C % 8, C <= 2048, res_ld % 8 and 16-B aligned buffers required"))
    return TT2_E_INVALID;
  BnArgs a = bn_args(p);
  const bool bf = p->dtype == TT2_DT_BF16;
  if (p->training && p->stats_rows <= 0) {
    if (bf) hipLaunchKernelGGL(bn_stats_kernel<bf16>, dim3(a.R), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(a.R), dim3(NT), 0, s, a);
  }
  if (BN_FUSED_FIN && p->training) {   // the finalize inside the apply
    if (bf) hipLaunchKernelGGL(bn_apply_fin_kernel<bf16>, bn_fin_grid(p->m, p->c), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(bn_apply_fin_kernel<float>, bn_fin_grid(p->m, p->c), dim3(NT), 0, s, a);
    return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_fwd");
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((p->c + BNC_COLS - 1) / BNC_COLS), dim3(NT), 0, s, a);
  const int g = grid_for((int64_t)p->m * p->c / 8);
  if (bf) hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(g), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(g), dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_fwd");
}

extern "C" int tt2_batchnorm_bwd(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return TT2_OK;
  if (!p->workspace || p->ws_bytes < tt2_batchnorm_workspace_size(p))
    return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_bwd: workspace too small");
  if (bn_check(p, "tt2_batchnorm_bwd: C % 8, C <= 2048 and 16-B aligned buffers required")) return TT2_E_INVALID;
  BnArgs a = bn_args(p);
  const bool bf = p->dtype == TT2_DT_BF16;
  const bool dbf = p->dout_dtype == TT2_DT_BF16;
#define TT2_BN_DISPATCH(KER, grid)                                                              \
  if (bf && dbf) hipLaunchKernelGGL((KER<bf16, bf16>), grid, dim3(NT), 0, s, a);                \
  else if (bf) hipLaunchKernelGGL((KER<bf16, float>), grid, dim3(NT), 0, s, a);                 \
  else if (dbf) hipLaunchKernelGGL((KER<float, bf16>), grid, dim3(NT), 0, s, a);                \
  else hipLaunchKernelGGL((KER<float, float>), grid, dim3(NT), 0, s, a);
  if (p->stats_rows <= 0) { TT2_BN_DISPATCH(bn_bwd_stats_kernel, dim3(a.R)) }   // else: tt2_gemm bn_bwd's sums
  if (BN_FUSED_FIN && p->training) {   // the finalize inside the apply
    bn_bwd_apply_fin(a, bf, dbf, true, bn_fin_grid(p->m, p->c), s);
    return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_bwd");
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((p->c + BNC_COLS - 1) / BNC_COLS), dim3(NT), 0, s, a);
  const int ga = grid_for((int64_t)p->m * p->c / 8);
  TT2_BN_DISPATCH(bn_bwd_apply_kernel, dim3(ga))
#undef TT2_BN_DISPATCH
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_bwd");
}

// ------------------------------------------------------------ SyncBatchNorm phases
// The caller SUM-all-reduces the first W * 3 * C floats of sync_buf between the phases
// (tt2/dist.py BnSync: RCCL in the captured step, or torch.distributed).  Every rank then
// holds the same slots and computes the same global statistics in the same order.
extern "C" size_t tt2_batchnorm_sync_size(const tt2_bn_args* p) {
  const int w = p->sync_world > 0 ? p->sync_world : 1;
  return ((size_t)(3 * w + 2) * p->c + 4) * sizeof(float);   // + 1 / N (padded to 16 B)
}

static int bn_sync_check(const tt2_bn_args* p, const char* what) {
  if (bn_check(p, what)) return TT2_E_INVALID;
  if (!p->training || p->sync_world < 1 || p->sync_rank < 0 || p->sync_rank >= p->sync_world || !p->sync_buf ||
      (reinterpret_cast<uintptr_t>(p->sync_buf) & 15) || !p->workspace ||
      p->ws_bytes < tt2_batchnorm_workspace_size(p))
    return tt2_set_error(TT2_E_INVALID, what);
  return TT2_OK;
}

static BnArgs bn_sync_args(const tt2_bn_args* p) {
  BnArgs a = bn_args(p);
  a.sync = p->sync_buf;
  a.W = p->sync_world;
  a.rank = p->sync_rank;
  a.Mtot = 1;   // unused: the exchanged statistics carry each rank's row count (bn_*sync*_kernel, inv_m)
  return a;
}

extern "C" int tt2_batchnorm_fwd_stats(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_fwd_stats: m must be > 0");
  if (bn_sync_check(p, "tt2_batchnorm_fwd_stats: training, 1 <= sync_world, 0 <= sync_rank < sync_world, "
                       "16-B aligned sync_buf, workspace and the tt2_batchnorm_fwd layout rules required"))
    return TT2_E_INVALID;
  const BnArgs a = bn_sync_args(p);
  if (p->stats_rows <= 0) {
    if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(bn_stats_kernel<bf16>, dim3(a.R), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(a.R), dim3(NT), 0, s, a);
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((p->c + BNC_COLS - 1) / BNC_COLS), dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_fwd_stats");
}

extern "C" int tt2_batchnorm_fwd_apply(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_fwd_apply: m must be > 0");
  if (bn_sync_check(p, "tt2_batchnorm_fwd_apply: the tt2_batchnorm_fwd_stats arguments required"))
    return TT2_E_INVALID;
  const BnArgs a = bn_sync_args(p);
  hipLaunchKernelGGL(bn_sync_finalize_kernel, dim3((p->c + NT - 1) / NT), dim3(NT), 0, s, a);
  const int g = grid_for((int64_t)p->m * p->c / 8);
  if (p->dtype == TT2_DT_BF16) hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(g), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(g), dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_fwd_apply");
}

#define TT2_BN_DISPATCH2(KER, grid, args)                                                       \
  if (bf && dbf) hipLaunchKernelGGL((KER<bf16, bf16>), grid, dim3(NT), 0, s, args);             \
  else if (bf) hipLaunchKernelGGL((KER<bf16, float>), grid, dim3(NT), 0, s, args);              \
  else if (dbf) hipLaunchKernelGGL((KER<float, bf16>), grid, dim3(NT), 0, s, args);             \
  else hipLaunchKernelGGL((KER<float, float>), grid, dim3(NT), 0, s, args);

extern "C" int tt2_batchnorm_bwd_stats(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_bwd_stats: m must be > 0");
  if (bn_sync_check(p, "tt2_batchnorm_bwd_stats: the tt2_batchnorm_fwd_stats arguments required"))
    return TT2_E_INVALID;
  const BnArgs a = bn_sync_args(p);
  const bool bf = p->dtype == TT2_DT_BF16, dbf = p->dout_dtype == TT2_DT_BF16;
  if (p->stats_rows <= 0) { TT2_BN_DISPATCH2(bn_bwd_stats_kernel, dim3(a.R), a) }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((p->c + BNC_COLS - 1) / BNC_COLS), dim3(NT), 0, s, a);
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_bwd_stats");
}

extern "C" int tt2_batchnorm_bwd_apply(const tt2_bn_args* p, hipStream_t s) {
  if (p->m <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_batchnorm_bwd_apply: m must be > 0");
  if (bn_sync_check(p, "tt2_batchnorm_bwd_apply: the tt2_batchnorm_fwd_stats arguments required"))
    return TT2_E_INVALID;
  BnArgs a = bn_sync_args(p);
  hipLaunchKernelGGL(bn_bwd_sync_kernel, dim3((p->c + NT - 1) / NT), dim3(NT), 0, s, a);
  a.dbeta = a.sync + (int64_t)a.W * 3 * a.C;   // the apply reads the global sums and 1 / N
  a.dgamma = a.dbeta + a.C;
  a.inv_m = a.dgamma + a.C;
  const bool bf = p->dtype == TT2_DT_BF16, dbf = p->dout_dtype == TT2_DT_BF16;
  if (BN_FUSED_FIN) {   // plain BatchNorm's apply code with the exchanged sums staged (one rank: bitwise equal)
    bn_bwd_apply_fin(a, bf, dbf, false, bn_fin_grid(p->m, p->c), s);
    return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_bwd_apply");
  }
  const int ga = grid_for((int64_t)p->m * p->c / 8);
  TT2_BN_DISPATCH2(bn_bwd_apply_kernel, dim3(ga), a)
  return tt2_check_launch(hipGetLastError(), "tt2_batchnorm_bwd_apply");
}
#undef TT2_BN_DISPATCH2
