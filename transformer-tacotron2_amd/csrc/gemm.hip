// gemm.hip -- MFMA GEMM with fused epilogues and implicit-im2col operands.
//
//   C[m, n] = epi( alpha * sum_k A(m, k) * B(n, k) )
//
// A(m,k) is K-contiguous (A[m*lda + k]) or M-contiguous (A[k*lda + m]);
// likewise B(n,k).  That covers every product of the training step:
//   linear fwd   Y  = X  W^T      (A K-contig, B K-contig)
//   linear dgrad dX = dY W        (A K-contig, B N-contig)
//   linear wgrad dW = dY^T X      (A M-contig, B N-contig)
// and the Conv1d(k5) layers as implicit GEMMs: with channels-last activations
// x[(b*T + t)*C + c] and weights packed [Cout][tap][Cin], the im2col row of
// output frame (b,t) is the overlapping window x[(b*T+t-pad)*C ...], i.e. an
// operand with ld = C and a per-chunk validity test 0 <= t + tap - pad < T.
//
// Tiling: 128x128 output tile, BK = 32, 256 threads = 4 waves (2 x 2), each wave
// 64x64 = 4x4 MFMA 16x16 blocks.  Global -> registers -> LDS double buffer with
// the next tile's loads in flight during the current tile's MFMAs (one barrier
// per K step).  K-contiguous tiles are read with 16-B ds_read, M/N-contiguous
// tiles with ds_read_b64_tr_b16 (gfx950 transposing LDS read).
// Split-K (gridDim.z > 1) writes raw f32 partial slabs to the workspace and a
// second kernel (gemm_splitk_reduce) sums them in a fixed order (bitwise
// reproducible) and applies the epilogue.
#include "tt2_common.h"
#include "tt2_capi.h"
#include "tt2_internal.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

struct EpiParams {
  void* c; int64_t ldc; int c_dt;
  const float* bias;
  const void* res; int64_t ldr; int res_dt;
  const void* gate; int64_t ldg; int gate_dt; float gate_scale;
  float alpha, beta;
  int act;
  DropDesc drop;
  int n_log;  // logical N for dropout index (m * n_log + n)
  int vec;    // every row of C/res/gate/bias is 16-B aligned at 8-column boundaries
  float* ksum; float ksum_beta;   // fused row sums of op(A) over k (v2, M-contiguous A)
  int main_only;                  // split-K: skip the reduce launch (measurement hook)
};

TT2_DEV float ld_any(const void* p, int64_t i, int dt) {
  return dt == TT2_BF16 ? (float)reinterpret_cast<const bf16*>(p)[i] : reinterpret_cast<const float*>(p)[i];
}
TT2_DEV void st_any(void* p, int64_t i, int dt, float v) {
  if (dt == TT2_BF16) reinterpret_cast<bf16*>(p)[i] = (bf16)v;
  else reinterpret_cast<float*>(p)[i] = v;
}

TT2_DEV float epi_value(const EpiParams& e, uint32_t seed, int m, int n, float v) {
  v *= e.alpha;
  if (e.bias) v += e.bias[n];
  if (e.res) v += ld_any(e.res, (int64_t)m * e.ldr + n, e.res_dt);
  if (e.act == ACT_RELU) v = fmaxf(v, 0.f);
  else if (e.act == ACT_TANH) v = tanhf(v);
  if (e.gate) v = ld_any(e.gate, (int64_t)m * e.ldg + n, e.gate_dt) != 0.f ? v * e.gate_scale : 0.f;
  if (e.drop.thr) v = drop_apply(e.drop, seed, (uint32_t)((int64_t)m * e.n_log + n), v);
  if (e.beta != 0.f) v += e.beta * ld_any(e.c, (int64_t)m * e.ldc + n, e.c_dt);
  return v;
}

struct OpDesc {
  const void* p;
  int64_t ld;
  int outer_max, inner_max;   // bounds of the outer (strided) and inner (contiguous) index
  int conv_t, conv_c, conv_pad;
};

// Load one 16-B chunk at (outer, inner) with bounds/conv masking.
template <typename T>
TT2_DEV ChunkV<T> load_op_chunk(const OpDesc& d, int outer, int inner) {
  constexpr int E = Chunk<T>::N;
  const T* base = reinterpret_cast<const T*>(d.p);
  if (outer >= d.outer_max || inner >= d.inner_max) return zero_chunk<T>();
  if (d.conv_t > 0) {
    const int t = outer % d.conv_t;
    const int ts = t + inner / d.conv_c - d.conv_pad;
    if (ts < 0 || ts >= d.conv_t) return zero_chunk<T>();
    // chunks never straddle taps (conv_c % E == 0, checked on the host)
    return ld_chunk<T>(base + (int64_t)outer * d.ld + inner - (int64_t)d.conv_pad * d.conv_c);
  }
  const T* p = base + (int64_t)outer * d.ld + inner;
  if (inner + E <= d.inner_max) return ld_chunk<T>(p);
  ChunkV<T> c = zero_chunk<T>();
  for (int e = 0; e < E; ++e)
    if (inner + e < d.inner_max) c.e[e] = p[e];
  return c;
}

// LDS tile geometry for one operand.
//  KC (K-contiguous): tile[128][BK + pad], row = m (or n)
//  MC (M-contiguous): tile[BK][128 + pad], row = k
template <typename T, bool KC> struct TileGeo;
template <typename T> struct TileGeo<T, true> {
  static constexpr int LD = BK + Chunk<T>::N;   // +16 B per row
  static constexpr int ELEMS = 128 * LD;
  static constexpr int CPR = BK / Chunk<T>::N;   // chunks per row
};
template <typename T> struct TileGeo<T, false> {
  static constexpr int LD = 128 + Chunk<T>::N;
  static constexpr int ELEMS = BK * LD;
  static constexpr int CPR = 128 / Chunk<T>::N;
};

template <typename T> struct NCh { static constexpr int V = 128 * BK / Chunk<T>::N / NT; };

// global tile -> registers.  tile_r0: first m/n of the tile; k0: first k.
template <typename T, bool KC>
TT2_DEV void g2r(ChunkV<T> (&r)[NCh<T>::V], const OpDesc& d, int tile_r0, int k0, int tid) {
  using G = TileGeo<T, KC>;
#pragma unroll
  for (int i = 0; i < NCh<T>::V; ++i) {
    const int c = tid + NT * i;
    const int row = c / G::CPR, cc = c % G::CPR;
    if (KC) r[i] = load_op_chunk<T>(d, tile_r0 + row, k0 + cc * Chunk<T>::N);
    else r[i] = load_op_chunk<T>(d, k0 + row, tile_r0 + cc * Chunk<T>::N);
  }
}
template <typename T, bool KC>
TT2_DEV void r2s(const ChunkV<T> (&r)[NCh<T>::V], T* tile, int tid) {
  using G = TileGeo<T, KC>;
#pragma unroll
  for (int i = 0; i < NCh<T>::V; ++i) {
    const int c = tid + NT * i;
    const int row = c / G::CPR, cc = c % G::CPR;
    st_chunk<T>(tile + row * G::LD + cc * Chunk<T>::N, r[i]);
  }
}

// fragment for rows [r0, r0+16) of the tile (r = m or n), k in [0, 32)
template <typename T, bool KC>
TT2_DEV void s2f(Frag8<T>& f, const T* tile, int r0, int lane) {
  using G = TileGeo<T, KC>;
  if (KC) frag_row(f, tile + (r0 + (lane & 15)) * G::LD + 8 * (lane >> 4));
  else frag_col(f, tile, G::LD, 8 * (lane >> 4), r0, lane);
}

template <typename T, bool AK, bool BKC>
__global__ __launch_bounds__(NT) void gemm_kernel(OpDesc A, OpDesc B, EpiParams E, int M, int N, int K,
                                                  int k_split, float* ws) {
  using GA = TileGeo<T, AK>;
  using GB = TileGeo<T, BKC>;
  __shared__ __attribute__((aligned(16))) T smem[2 * (GA::ELEMS + GB::ELEMS)];
  constexpr int STAGE = GA::ELEMS + GB::ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kb = blockIdx.z * k_split;
  const int ke = min(K, kb + k_split);
  // bound the k dimension of both operands to this split
  if (AK) A.inner_max = ke; else A.outer_max = ke;
  if (BKC) B.inner_max = ke; else B.outer_max = ke;
  const int nkt = (ke - kb + BK - 1) / BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  ChunkV<T> ra[NCh<T>::V], rb[NCh<T>::V];
  g2r<T, AK>(ra, A, m0, kb, tid);
  g2r<T, BKC>(rb, B, n0, kb, tid);
  r2s<T, AK>(ra, smem, tid);
  r2s<T, BKC>(rb, smem + GA::ELEMS, tid);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      g2r<T, AK>(ra, A, m0, kb + (kt + 1) * BK, tid);
      g2r<T, BKC>(rb, B, n0, kb + (kt + 1) * BK, tid);
    }
    Frag8<T> fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) s2f<T, AK>(fa[i], smem + cur * STAGE, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) s2f<T, BKC>(fb[j], smem + cur * STAGE + GA::ELEMS, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mma16(fa[i], fb[j], acc[i][j]);
    if (more) {
      r2s<T, AK>(ra, smem + (cur ^ 1) * STAGE, tid);
      r2s<T, BKC>(rb, smem + (cur ^ 1) * STAGE + GA::ELEMS, tid);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[m0 + wm*64 + 16i + 4*(lane>>4) + r][n0 + wn*64 + 16j + (lane&15)]
  const uint32_t seed = E.drop.thr ? *E.drop.seed : 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 64 + 16 * j + (lane & 15);
        if (m < M && n < N) {
          if (ws) ws[((int64_t)blockIdx.z * M + m) * N + n] = acc[i][j][r];
          else st_any(E.c, (int64_t)m * E.ldc + n, E.c_dt, epi_value(E, seed, m, n, acc[i][j][r]));
        }
      }
}

__global__ void gemm_splitk_reduce(const float* ws, int splits, EpiParams E, int M, int N) {
  const int64_t total = (int64_t)M * N;
  const uint32_t seed = E.drop.thr ? *E.drop.seed : 0u;
  if (E.ksum) {   // [splits][M] k-sum partials after the C slabs, fixed split order
    const float* kp = ws + splits * total;
    for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
      float v = 0.f;
      for (int z = 0; z < splits; ++z) v += kp[z * (int64_t)M + m];
      E.ksum[m] = E.ksum_beta != 0.f ? E.ksum_beta * E.ksum[m] + v : v;
    }
  }
  if ((N & 3) == 0) {
    // 4 consecutive columns per thread (16-B partial-slab loads), fixed split order
    const int64_t t4 = total / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < t4; i += (int64_t)gridDim.x * blockDim.x) {
      // two accumulators, 4 slab loads in flight per step (fixed order per element)
      f32x4 v = reinterpret_cast<const f32x4*>(ws)[i], w = f32x4{0.f, 0.f, 0.f, 0.f};
      int z = 1;
      for (; z + 3 < splits; z += 4) {
        const f32x4 a0 = reinterpret_cast<const f32x4*>(ws + z * total)[i];
        const f32x4 a1 = reinterpret_cast<const f32x4*>(ws + (z + 1) * total)[i];
        const f32x4 a2 = reinterpret_cast<const f32x4*>(ws + (z + 2) * total)[i];
        const f32x4 a3 = reinterpret_cast<const f32x4*>(ws + (z + 3) * total)[i];
        v += a0 + a2;
        w += a1 + a3;
      }
      for (; z < splits; ++z) v += reinterpret_cast<const f32x4*>(ws + z * total)[i];
      v += w;
      const int m = (int)(4 * i / N), n = (int)(4 * i % N);
#pragma unroll
      for (int j = 0; j < 4; ++j) st_any(E.c, (int64_t)m * E.ldc + n + j, E.c_dt, epi_value(E, seed, m, n + j, v[j]));
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[z * total + i];
    const int m = (int)(i / N), n = (int)(i % N);
    st_any(E.c, (int64_t)m * E.ldc + n, E.c_dt, epi_value(E, seed, m, n, v));
  }
}

template <typename T, bool AK, bool BKC>
hipError_t launch_t(const OpDesc& A, const OpDesc& B, const EpiParams& E, int M, int N, int K, int splits,
                    float* ws, hipStream_t s) {
  int k_split = K;
  if (splits > 1) {
    k_split = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    splits = (K + k_split - 1) / k_split;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((gemm_kernel<T, AK, BKC>), grid, dim3(NT), 0, s, A, B, E, M, N, K, k_split,
                     splits > 1 ? ws : nullptr);
  if (splits > 1 && !E.main_only) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256; int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}

// =====================================================================================
// v2 (bf16): BK = 64, LDS-DMA staging (global_load_lds_dwordx4: each lane's 16-B chunk
// lands at lds_base + 16*lane), two LDS stages, one barrier per K-tile, XOR swizzles
// applied on the per-lane GLOBAL source address so the lane-linear LDS image reads
// conflict-free with ds_read_b128 (K-contiguous tiles) and ds_read_b64_tr_b16
// (M/N-contiguous tiles).  Out-of-range / conv-padding chunks load from a zero page.
// Epilogue: accumulators -> LDS (f32) -> 16-B vectorised epilogue + stores.
// =====================================================================================
constexpr int BK2 = 64;
constexpr int TILE_BYTES = 128 * BK2 * 2;               // 16 KB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;             // A + B
constexpr int EPI_LD = 132;                             // f32 words per staged C row (pad: conflict-free)
constexpr int SMEM2 = (2 * STAGE_BYTES > 128 * EPI_LD * 4) ? 2 * STAGE_BYTES : 128 * EPI_LD * 4;

__device__ __attribute__((aligned(64))) uint4 g_zero_page[64];

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// swizzle of the 16-B chunk index for an M/N-contiguous tile row k (256-B rows)
TT2_DEV int mc_swz(int k) { return ((k & 3) << 1) ^ (((k >> 3) & 1) << 3); }

// Per-lane LDS-DMA source: the chunk's address, or the zero page when the chunk is out
// of range (or reads conv padding).  Branch-free per lane (a select), so the DMA issue
// is not wrapped in exec-mask branches; the conv test is behind a uniform branch.
TT2_DEV const void* chunk_src(const OpDesc& d, int outer, int inner) {
  bool ok = (outer < d.outer_max) & (inner < d.inner_max);
  int64_t off = (int64_t)outer * d.ld + inner;
  if (d.conv_t > 0) {
    const int ts = outer % d.conv_t + inner / d.conv_c - d.conv_pad;
    ok = ok & (ts >= 0) & (ts < d.conv_t);
    off -= (int64_t)d.conv_pad * d.conv_c;
  }
  const void* p = reinterpret_cast<const bf16*>(d.p) + off;
  return ok ? p : (const void*)g_zero_page;
}

// issue this wave's 4 of the 16 LDS-DMA instructions of one 128 x 64 operand tile
template <bool KC>
TT2_DEV void issue_tile(const OpDesc& d, char* lds_tile, int r0, int k0, int lane, int wave) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int inst = wave * 4 + i;
    const void* src;
    if (KC) {
      const int row = inst * 8 + (lane >> 3);
      const int gc = (lane & 7) ^ (row & 7);
      src = chunk_src(d, r0 + row, k0 + gc * 8);
    } else {
      const int kr = inst * 4 + (lane >> 4);
      const int gc = (lane & 15) ^ mc_swz(kr);
      src = chunk_src(d, k0 + kr, r0 + gc * 8);
    }
    __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(lds_tile + inst * 1024), 16, 0, 0);
  }
}

// fragment (8 consecutive k of row r0 + (lane&15)) for k-step kk (0/1) of the 64-deep tile
template <bool KC>
TT2_DEV void frag2(Frag8<bf16>& f, const char* tile, int r0, int kk, int lane) {
  if (KC) {
    const int row = r0 + (lane & 15);
    const int h = 4 * kk + (lane >> 4);
    f.v = *reinterpret_cast<const bf16x8*>(tile + row * 128 + ((h ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c = (r0 + 4 * p) >> 3;
    typedef __attribute__((address_space(3))) short4v lds_s4;
    const int k_lo = 32 * kk + 8 * g + q;
    const int k_hi = k_lo + 4;
    const char* a0 = tile + k_lo * 256 + ((c ^ mc_swz(k_lo)) << 4) + ((p & 1) << 3);
    const char* a1 = tile + k_hi * 256 + ((c ^ mc_swz(k_hi)) << 4) + ((p & 1) << 3);
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a1));
    union { short s[8]; bf16x8 v; } u;
    u.s[0] = lo[0]; u.s[1] = lo[1]; u.s[2] = lo[2]; u.s[3] = lo[3];
    u.s[4] = hi[0]; u.s[5] = hi[1]; u.s[6] = hi[2]; u.s[7] = hi[3];
    f.v = u.v;
  }
}

// 8 consecutive elements of a row from a bf16 or f32 tensor (16-B aligned)
TT2_DEV void ld8_any(const void* p, int64_t off, int dt, float (&o)[8]) {
  if (dt == TT2_BF16) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)x[j];
  } else {
    const float* q = reinterpret_cast<const float*>(p) + off;
    const f32x4 a = *reinterpret_cast<const f32x4*>(q), b = *reinterpret_cast<const f32x4*>(q + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
  }
}

// Chunk epilogue: 8 consecutive outputs of row m starting at column n0.  Full,
// aligned chunks (E.vec) take 16-B loads/stores with every option tested once
// per chunk; edge chunks fall back to the per-element path.
TT2_DEV void epi_store8(const EpiParams& E, uint32_t seed, int m, int n0, int N, const float (&v)[8]) {
  const int64_t off = (int64_t)m * E.ldc + n0;
  if (E.vec && n0 + 8 <= N) {
    float o[8], t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j] * E.alpha;
    if (E.bias) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(E.bias + n0), b = *reinterpret_cast<const f32x4*>(E.bias + n0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[j] += a[j]; o[4 + j] += b[j]; }
    }
    if (E.res) {
      ld8_any(E.res, (int64_t)m * E.ldr + n0, E.res_dt, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += t[j];
    }
    if (E.act == ACT_RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    } else if (E.act == ACT_TANH) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = tanhf(o[j]);
    }
    if (E.gate) {
      ld8_any(E.gate, (int64_t)m * E.ldg + n0, E.gate_dt, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = t[j] != 0.f ? o[j] * E.gate_scale : 0.f;
    }
    if (E.drop.thr) {
      const uint32_t base = (uint32_t)((int64_t)m * E.n_log + n0);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = drop_apply(E.drop, seed, base + j, o[j]);
    }
    if (E.beta != 0.f) {
      ld8_any(E.c, off, E.c_dt, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += E.beta * t[j];
    }
    if (E.c_dt == TT2_BF16) {
      bf16x8 x;
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (bf16)o[j];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(E.c) + off) = x;
    } else {
      float* c = reinterpret_cast<float*>(E.c) + off;
      *reinterpret_cast<f32x4*>(c) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(c + 4) = f32x4{o[4], o[5], o[6], o[7]};
    }
    return;
  }
  for (int j = 0; j < 8; ++j)
    if (n0 + j < N) st_any(E.c, off + j, E.c_dt, epi_value(E, seed, m, n0 + j, v[j]));
}

template <bool AK, bool BKC>
__global__ __launch_bounds__(NT, 2) void gemm2_kernel(OpDesc A, OpDesc B, EpiParams E, int M, int N, int K,
                                                      int k_split, float* ws, int ntm, int ntn) {
  __shared__ __attribute__((aligned(1024))) char smem[SMEM2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: blocks b and b+8 share an XCD, so give each XCD a
  // contiguous run of tiles (walking n for a fixed m: the A row panel stays in that L2).
  const int nt = ntm * ntn;
  const int bid = blockIdx.x;
  const int q = nt / 8, rr = nt % 8, x = bid % 8;
  const int tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + bid / 8;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int kb = blockIdx.y * k_split;
  const int ke = min(K, kb + k_split);
  if (AK) A.inner_max = ke; else A.outer_max = ke;
  if (BKC) B.inner_max = ke; else B.outer_max = ke;
  const int nkt = (ke - kb + BK2 - 1) / BK2;
  const bool do_ks = !AK && E.ksum && (tile % ntn) == 0;   // one n-tile per m-tile sums A over k
  float ks[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_tile<AK>(A, smem, m0, kb, lane, wave);
  issue_tile<BKC>(B, smem + TILE_BYTES, n0, kb, lane, wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const char* sa = smem + (kt & 1) * STAGE_BYTES;
    const char* sb = sa + TILE_BYTES;
#ifndef TT2_ABL_NO_LOAD
    if (kt + 1 < nkt) {
      char* na = smem + ((kt + 1) & 1) * STAGE_BYTES;
      issue_tile<AK>(A, na, m0, kb + (kt + 1) * BK2, lane, wave);
      issue_tile<BKC>(B, na + TILE_BYTES, n0, kb + (kt + 1) * BK2, lane, wave);
    }
#endif
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<bf16> fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) frag2<AK>(fa[i], sa, wm * 64 + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) frag2<BKC>(fb[j], sb, wn * 64 + 16 * j, kk, lane);
#ifdef TT2_ABL_NO_MFMA
#pragma unroll
      for (int i = 0; i < 4; ++i) { asm volatile("" :: "v"(fa[i].v)); asm volatile("" :: "v"(fb[i].v)); }
#else
#ifdef TT2_G2_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mma16(fa[i], fb[j], acc[i][j]);
#ifdef TT2_G2_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
#endif
    }
    if (!AK && do_ks) {
      // rows 4*(tid>>4) .. +3 of the [64 k][128 m] A image, m-chunk tid & 15
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kr = 4 * (tid >> 4) + r;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(sa + kr * 256 + (((tid & 15) ^ mc_swz(kr)) << 4));
#pragma unroll
        for (int j = 0; j < 8; ++j) ks[j] += (float)v[j];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (!AK && do_ks) {
    // reduce over the 16 k-groups: lanes l, l^16, l^32, l^48, then the 4 waves via LDS
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ks[j] += __shfl_xor(ks[j], 16, 64);
      ks[j] += __shfl_xor(ks[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(wave * 16 + lane) * 8 + j] = ks[j];
    }
    __syncthreads();
    if (tid < 128) {
      const int cc = tid >> 3, j = tid & 7, m = m0 + tid;
      const float v = (red[(0 * 16 + cc) * 8 + j] + red[(1 * 16 + cc) * 8 + j]) +
                      (red[(2 * 16 + cc) * 8 + j] + red[(3 * 16 + cc) * 8 + j]);
      if (m < M) {
        if (ws) ws[(int64_t)gridDim.y * M * N + (int64_t)blockIdx.y * M + m] = v;
        else E.ksum[m] = E.ksum_beta != 0.f ? E.ksum_beta * E.ksum[m] + v : v;
      }
    }
    __syncthreads();
  }
#ifdef TT2_ABL_NO_EPI
  if (acc[0][0][0] == 1234.5f && acc[3][3][3] == 1234.5f) reinterpret_cast<float*>(E.c)[tid] = acc[1][1][1];
  return;
#endif

  // stage C (f32) through LDS: row-major [128][EPI_LD]
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * 64 + 16 * i + 4 * (lane >> 4) + r) * EPI_LD + wn * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const uint32_t seed = (!ws && E.drop.thr) ? *E.drop.seed : 0u;
#pragma unroll 2
  for (int it = 0; it < 8; ++it) {
    const int id = tid + NT * it;
    const int row = id >> 4, c8 = (id & 15) * 8;
    const int m = m0 + row, n = n0 + c8;
    if (m >= M || n >= N) continue;
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8 + 4);
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
#ifdef TT2_ABL_NO_STORE
    if (v[0] != 1234.5f) continue;
#endif
    if (ws) {
      float* w = ws + ((int64_t)blockIdx.y * M + m) * N + n;
      if (n + 8 <= N && (N % 4) == 0) {
        *reinterpret_cast<f32x4*>(w) = lo;
        *reinterpret_cast<f32x4*>(w + 4) = hi;
      } else {
        for (int j = 0; j < 8; ++j)
          if (n + j < N) w[j] = v[j];
      }
    } else {
      epi_store8(E, seed, m, n, N, v);
    }
  }
}

// =====================================================================================
// v3 (bf16): the v2 operand images and swizzles, but a STAGES-deep LDS ring with the
// next STAGES-1 K tiles in flight across the barrier (counted `s_waitcnt vmcnt` +
// raw s_barrier, never a full drain inside the loop), BM = 128 or 256 rows
// (256 = 8 waves, K-contiguous A only), and branch-light per-lane addressing: each
// lane keeps its chunk pointers / conv tap-time state and advances them by one K
// tile per iteration instead of recomputing divisions.
// =====================================================================================
struct LaneChunk {
  const bf16* p;   // address of this lane's chunk for the current K tile (unmasked)
  int outer, inner;
  int t, tap;      // conv bookkeeping (time of outer, tap of inner)
};

template <bool KC>
TT2_DEV void lane_chunk_init(LaneChunk& c, const OpDesc& d, int inst, int lane, int r0, int k0) {
  if (KC) {
    const int row = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (row & 7);
    c.outer = r0 + row;
    c.inner = k0 + gc * 8;
  } else {
    const int kr = inst * 4 + (lane >> 4);
    const int gc = (lane & 15) ^ mc_swz(kr);
    c.outer = k0 + kr;
    c.inner = r0 + gc * 8;
  }
  c.p = reinterpret_cast<const bf16*>(d.p) + (int64_t)c.outer * d.ld + c.inner;
  if (d.conv_t > 0) {
    c.p -= (int64_t)d.conv_pad * d.conv_c;
    c.t = c.outer % d.conv_t;
    c.tap = c.inner / d.conv_c;
  } else {
    c.t = 0;
    c.tap = 0;
  }
}

template <bool KC>
TT2_DEV void lane_chunk_advance(LaneChunk& c, const OpDesc& d) {
  if (KC) {
    c.inner += BK2;
    c.p += BK2;
    if (d.conv_t > 0) {   // inner = tap * C + ci: ci grows by 64 < C (C >= 80 when conv)
      int ci = c.inner - c.tap * d.conv_c;
      while (ci >= d.conv_c) { ci -= d.conv_c; ++c.tap; }
    }
  } else {
    c.outer += BK2;
    c.p += (int64_t)BK2 * d.ld;
    if (d.conv_t > 0) {
      c.t += BK2;
      while (c.t >= d.conv_t) c.t -= d.conv_t;
    }
  }
}

TT2_DEV const void* lane_chunk_src(const LaneChunk& c, const OpDesc& d) {
  bool ok = c.outer < d.outer_max && c.inner < d.inner_max;
  if (d.conv_t > 0) {
    const int ts = c.t + c.tap - d.conv_pad;
    ok = ok && ts >= 0 && ts < d.conv_t;
  }
  return ok ? (const void*)c.p : (const void*)g_zero_page;
}

template <int N> TT2_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BM_, int STAGES> struct G3 {
  static constexpr int WAVES = BM_ / 32;                 // 2 (n) x BM/64 (m)
  static constexpr int THREADS = WAVES * 64;
  static constexpr int A_BYTES = BM_ * BK2 * 2;
  static constexpr int B_BYTES = 128 * BK2 * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_INST = A_BYTES / 1024 / WAVES;  // LDS-DMA instructions per wave per tile
  static constexpr int B_INST = B_BYTES / 1024 / WAVES;
  static constexpr int INST = A_INST + B_INST;
  static constexpr int EPI = BM_ * EPI_LD * 4;
  static constexpr int SMEM = STAGES * STAGE > EPI ? STAGES * STAGE : EPI;
};

template <bool AK, bool BKC, int BM_, int STAGES>
__global__ __launch_bounds__((BM_ / 32) * 64) void gemm3_kernel(OpDesc A, OpDesc B, EpiParams E, int M,
                                                                         int N, int K, int k_split, float* ws,
                                                                         int ntm, int ntn) {
  using G = G3<BM_, STAGES>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = ntm * ntn;
  const int bid = blockIdx.x;
  const int q = nt / 8, rr = nt % 8, x = bid % 8;
  const int tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + bid / 8;
  const int m0 = (tile / ntn) * BM_, n0 = (tile % ntn) * BN;
  const int kb = blockIdx.y * k_split;
  const int ke = min(K, kb + k_split);
  if (AK) A.inner_max = ke; else A.outer_max = ke;
  if (BKC) B.inner_max = ke; else B.outer_max = ke;
  const int nkt = (ke - kb + BK2 - 1) / BK2;

  LaneChunk ca[G::A_INST], cb[G::B_INST];
#pragma unroll
  for (int i = 0; i < G::A_INST; ++i) lane_chunk_init<AK>(ca[i], A, wave * G::A_INST + i, lane, m0, kb);
#pragma unroll
  for (int i = 0; i < G::B_INST; ++i) lane_chunk_init<BKC>(cb[i], B, wave * G::B_INST + i, lane, n0, kb);

  auto issue = [&](int stage) {
    char* sa = smem + stage * G::STAGE;
    char* sb = sa + G::A_BYTES;
#pragma unroll
    for (int i = 0; i < G::A_INST; ++i) {
      __builtin_amdgcn_global_load_lds((gvoid_t*)lane_chunk_src(ca[i], A),
                                       (lvoid_t*)(sa + (wave * G::A_INST + i) * 1024), 16, 0, 0);
      lane_chunk_advance<AK>(ca[i], A);
    }
#pragma unroll
    for (int i = 0; i < G::B_INST; ++i) {
      __builtin_amdgcn_global_load_lds((gvoid_t*)lane_chunk_src(cb[i], B),
                                       (lvoid_t*)(sb + (wave * G::B_INST + i) * 1024), 16, 0, 0);
      lane_chunk_advance<BKC>(cb[i], B);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: tiles 0 .. STAGES-2 in flight
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nkt) issue(s);
  if (nkt > STAGES - 2) wait_vmcnt<(STAGES - 2) * G::INST>();
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nkt; ++kt) {
    const bool more = kt + STAGES - 1 < nkt;
    if (more) issue((kt + STAGES - 1) % STAGES);
    const char* sa = smem + (kt % STAGES) * G::STAGE;
    const char* sb = sa + G::A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Frag8<bf16> fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) frag2<AK>(fa[i], sa, wm * 64 + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) frag2<BKC>(fb[j], sb, wn * 64 + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mma16(fa[i], fb[j], acc[i][j]);
    }
    // tile kt+1 must have landed (this wave's part), and every wave must be done
    // reading tile kt before the NEXT iteration's issue overwrites its slot.
    if (more) wait_vmcnt<(STAGES - 2) * G::INST>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * 64 + 16 * i + 4 * (lane >> 4) + r) * EPI_LD + wn * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const uint32_t seed = (!ws && E.drop.thr) ? *E.drop.seed : 0u;
  constexpr int ITERS = BM_ * 16 / G::THREADS;
#pragma unroll 2
  for (int it = 0; it < ITERS; ++it) {
    const int id = tid + G::THREADS * it;
    const int row = id >> 4, c8 = (id & 15) * 8;
    const int m = m0 + row, n = n0 + c8;
    if (m >= M || n >= N) continue;
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8 + 4);
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    if (ws) {
      float* w = ws + ((int64_t)blockIdx.y * M + m) * N + n;
      if (n + 8 <= N && (N % 4) == 0) {
        *reinterpret_cast<f32x4*>(w) = lo;
        *reinterpret_cast<f32x4*>(w + 4) = hi;
      } else {
        for (int j = 0; j < 8; ++j)
          if (n + j < N) w[j] = v[j];
      }
    } else {
      epi_store8(E, seed, m, n, N, v);
    }
  }
}

template <bool AK, bool BKC, int BM_, int STAGES>
hipError_t launch3(const OpDesc& A, const OpDesc& B, const EpiParams& E, int M, int N, int K, int splits, float* ws,
                   hipStream_t s) {
  using G = G3<BM_, STAGES>;
  int k_split = K;
  if (splits > 1) {
    k_split = ((K + splits - 1) / splits + BK2 - 1) / BK2 * BK2;
    splits = (K + k_split - 1) / k_split;
  }
  const int ntm = (M + BM_ - 1) / BM_, ntn = (N + BN - 1) / BN;
  static bool attr_set = false;   // one-time opt-in to > 64 KB dynamic LDS
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm3_kernel<AK, BKC, BM_, STAGES>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, G::SMEM);
    attr_set = true;
  }
  dim3 grid(ntm * ntn, splits);
  hipLaunchKernelGGL((gemm3_kernel<AK, BKC, BM_, STAGES>), grid, dim3(G::THREADS), G::SMEM, s, A, B, E, M, N, K,
                     k_split, splits > 1 ? ws : nullptr, ntm, ntn);
  if (splits > 1 && !E.main_only) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256;
    int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}

// =====================================================================================
// skinny-M (decode, M <= 32) bf16: out[M, N] = X[M, K] W[N, K]^T.  The problem is a
// weight stream: every workgroup owns 16 output columns and streams their W rows
// straight to registers (no LDS round trip), the 4 waves split K, and one MFMA
// 16x16x32 per 16 rows x 16 columns x 32 k.  Cross-wave sums go through LDS.
// =====================================================================================
constexpr int SK_COLS = 16;

// Decode-step fusions carried by the skinny kernel (tt2_gemm_args a_ln_* / kv_*).
struct SkinnyFuse {
  const bf16* br; const float* gamma; const float* beta; bf16* h_out; float eps;   // LN prologue (gamma != 0)
  bf16* kv; const int32_t* kv_t; int kv_col0; int64_t kv_bstride, kv_ld;           // KV scatter (kv != 0)
};

constexpr int SK_LN_LD = 512 + 8;   // bf16 per LDS row of the normalised A (16-B pad)

__global__ __launch_bounds__(NT) void gemm_skinny_kernel(const bf16* X, int64_t ldx, const bf16* W, int64_t ldw,
                                                         EpiParams E, int M, int N, int K, SkinnyFuse F) {
  __shared__ float red[4][32][SK_COLS + 1];
  extern __shared__ __attribute__((aligned(16))) bf16 s_h[];   // [32][SK_LN_LD] when F.gamma (K == 512)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * SK_COLS;
  if (F.gamma) {
    // h = LN(x + br) for the (<= 32) rows: rows wave, wave + 4, ... with every load issued
    // before the first reduction; h goes to LDS (the A operand below) and, from one
    // workgroup, to F.h_out (the next residual)
    const int c0 = lane * 8;
    union U { uint4 u; bf16x8 v; } a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = min(wave + 4 * u, M - 1);
      a[u].u = *reinterpret_cast<const uint4*>(X + (int64_t)row * ldx + c0);
      b[u].u = *reinterpret_cast<const uint4*>(F.br + (int64_t)row * ldx + c0);
    }
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(F.gamma + c0), g1 = *reinterpret_cast<const f32x4*>(F.gamma + c0 + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(F.beta + c0), b1 = *reinterpret_cast<const f32x4*>(F.beta + c0 + 4);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = wave + 4 * u;
      if (row >= M) break;
      float v[8], sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[j] = (float)a[u].v[j] + (float)b[u].v[j]; sum += v[j]; }
      const float mu = wave_sum(sum) / K;
      float sq = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - mu; sq += d * d; }
      const float rs = rsqrtf(wave_sum(sq) / K + F.eps);
      bf16x8 h;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        h[j] = (bf16)((v[j] - mu) * rs * (j < 4 ? g0[j] : g1[j - 4]) + (j < 4 ? b0[j] : b1[j - 4]));
      *reinterpret_cast<bf16x8*>(s_h + row * SK_LN_LD + c0) = h;
      if (blockIdx.x == 0) *reinterpret_cast<bf16x8*>(F.h_out + (int64_t)row * K + c0) = h;
    }
    __syncthreads();
  }
  const int kq = ((K + 127) / 128) * 32;                 // per-wave K slice, multiple of 32
  const int kb = wave * kq, ke = min(K, kb + kq);
  const int r = lane & 15, g = lane >> 4;
  const int n = n0 + r;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const bool nok = n < N, r0ok = r < M, r1ok = r + 16 < M;
  const bf16* wrow = W + (int64_t)(nok ? n : 0) * ldw;
  const bf16* x0 = X + (int64_t)(r0ok ? r : 0) * ldx;
  const bf16* x1 = X + (int64_t)(r1ok ? r + 16 : 0) * ldx;
  union U { uint4 u; bf16x8 v; };
  for (int k = kb; k < ke; k += 32) {
    const int kk = k + 8 * g;
    const bool kok = kk < ke;
    U w, a0, a1;
    w.u = (nok && kok) ? *reinterpret_cast<const uint4*>(wrow + kk) : make_uint4(0, 0, 0, 0);
    if (F.gamma) {
      a0.u = (r0ok && kok) ? *reinterpret_cast<const uint4*>(s_h + r * SK_LN_LD + kk) : make_uint4(0, 0, 0, 0);
      a1.u = (r1ok && kok) ? *reinterpret_cast<const uint4*>(s_h + (r + 16) * SK_LN_LD + kk) : make_uint4(0, 0, 0, 0);
    } else {
      a0.u = (r0ok && kok) ? *reinterpret_cast<const uint4*>(x0 + kk) : make_uint4(0, 0, 0, 0);
      a1.u = (r1ok && kok) ? *reinterpret_cast<const uint4*>(x1 + kk) : make_uint4(0, 0, 0, 0);
    }
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, w.v, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, w.v, acc1, 0, 0, 0);
  }
  // acc layout: row 4*(lane>>4) + i, col lane & 15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[wave][4 * g + i][r] = acc0[i];
    red[wave][16 + 4 * g + i][r] = acc1[i];
  }
  __syncthreads();
  const uint32_t seed = E.drop.thr ? *E.drop.seed : 0u;
  for (int o = threadIdx.x; o < 32 * SK_COLS; o += NT) {
    const int row = o / SK_COLS, col = o % SK_COLS;
    const int m = row, nn = n0 + col;
    if (m < M && nn < N) {
      const float v = (red[0][row][col] + red[1][row][col]) + (red[2][row][col] + red[3][row][col]);
      const float o = epi_value(E, seed, m, nn, v);
      st_any(E.c, (int64_t)m * E.ldc + nn, E.c_dt, o);
      if (F.kv && nn >= F.kv_col0)
        F.kv[(int64_t)m * F.kv_bstride + (int64_t)(*F.kv_t) * F.kv_ld + (nn - F.kv_col0)] = (bf16)o;
    }
  }
}

template <bool AK, bool BKC>
hipError_t launch2(const OpDesc& A, const OpDesc& B, const EpiParams& E, int M, int N, int K, int splits, float* ws,
                   hipStream_t s) {
  int k_split = K;
  if (splits > 1) {
    k_split = ((K + splits - 1) / splits + BK2 - 1) / BK2 * BK2;
    splits = (K + k_split - 1) / k_split;
  }
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  dim3 grid(ntm * ntn, splits);
  hipLaunchKernelGGL((gemm2_kernel<AK, BKC>), grid, dim3(NT), 0, s, A, B, E, M, N, K, k_split,
                     splits > 1 ? ws : nullptr, ntm, ntn);
  if (splits > 1 && !E.main_only) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256;
    int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}


// =====================================================================================
// v4 (bf16, K-contiguous A): 256 x 256 output tile, 512 threads = 8 waves (2 M x 4 N),
// each wave 128 x 64 = 8 x 4 MFMA 16x16x32 blocks.  At 64 MFMA FLOP per staged byte
// x 2 this halves the L2 -> CU bytes per FLOP of the 128^2 tile, which is what bounds
// the 128^2 kernel (~70 GB/s per CU served from L2).  K runs in 32-deep "k-halves"
// through a 4-slot LDS ring (slot = A 256x32 + B 256x32 bf16 = 32 KB), filled by
// LDS-DMA three k-halves ahead of the one being multiplied; per k-half: counted
// vmcnt for this thread's copies of the current slot, one barrier, re-issue into the
// slot the previous k-half released, 12 fragment reads, 32 MFMAs.
// LDS images (swizzle on the per-lane global source, image lane-linear):
//   K-contiguous operand: [256 rows][4 chunks of 16 B], chunk c of row r at c ^ ((r>>1)&3)
//   N-contiguous B      : [32 k rows][32 chunks], chunk c of row k at c ^ mc_swz(k)
// both bank-conflict-free for their ds_read_b128 / ds_read_b64_tr_b16 patterns.
// =====================================================================================
constexpr int G4_NT = 512;
constexpr int G4_OPB = 256 * 32 * 2;               // 16 KB: one operand's k-half
constexpr int G4_SLOT = 2 * G4_OPB;                // 32 KB
constexpr int G4_SLOTS = 4;
constexpr int G4_EPI_LD = 260;                     // f32 words per staged C row
constexpr int G4_SMEM = (G4_SLOTS * G4_SLOT > 128 * G4_EPI_LD * 4) ? G4_SLOTS * G4_SLOT : 128 * G4_EPI_LD * 4;

// this wave's 2 of the 16 LDS-DMA instructions of one operand k-half
template <bool KC>
TT2_DEV void g4_issue(const OpDesc& d, char* lds, int r0, int k0, int lane, int wave) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = wave * 2 + i;
    const void* src;
    if (KC) {
      const int row = inst * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((row >> 1) & 3);
      src = chunk_src(d, r0 + row, k0 + lc * 8);
    } else {
      const int kr = inst * 2 + (lane >> 5);
      const int lc = (lane & 31) ^ mc_swz(kr);
      src = chunk_src(d, k0 + kr, r0 + lc * 8);
    }
    __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(lds + inst * 1024), 16, 0, 0);
  }
}

// 16 x 32 fragment (rows r0 + (lane&15)) of a k-half image
template <bool KC>
TT2_DEV bf16x8 g4_frag(const char* img, int r0, int lane) {
  if (KC) {
    const int row = r0 + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((((lane >> 4) ^ (row >> 1)) & 3) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c = (r0 + 4 * p) >> 3;
    const int k_lo = 8 * g + q, k_hi = k_lo + 4;
    typedef __attribute__((address_space(3))) short4v lds_s4;
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(img + k_lo * 512 + ((c ^ mc_swz(k_lo)) << 4) + ((p & 1) << 3)));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(img + k_hi * 512 + ((c ^ mc_swz(k_hi)) << 4) + ((p & 1) << 3)));
    union { short4v s[2]; bf16x8 v; } u;
    u.s[0] = lo;
    u.s[1] = hi;
    return u.v;
  }
}

TT2_DEV void g4_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <bool BKC>
__global__ __launch_bounds__(G4_NT, 1) void gemm4_kernel(OpDesc A, OpDesc B, EpiParams E, int M, int N, int K,
                                                         int k_split, float* ws, int ntm, int ntn) {
  __shared__ __attribute__((aligned(1024))) char smem[G4_SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int nt = ntm * ntn;
  const int bid = blockIdx.x;
  const int q8 = nt / 8, rr = nt % 8, x = bid % 8;
  const int tile = (x < rr ? x * (q8 + 1) : rr * (q8 + 1) + (x - rr) * q8) + bid / 8;
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;
  const int kb = blockIdx.y * k_split;
  const int ke = min(K, kb + k_split);
  A.inner_max = ke;
  if (BKC) B.inner_max = ke; else B.outer_max = ke;
  const int nkh = (ke - kb + 31) / 32;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int h = 0; h < 3; ++h)
    if (h < nkh) {
      g4_issue<true>(A, smem + h * G4_SLOT, m0, kb + 32 * h, lane, wave);
      g4_issue<BKC>(B, smem + h * G4_SLOT + G4_OPB, n0, kb + 32 * h, lane, wave);
    }
  for (int h = 0; h < nkh; ++h) {
    // this thread's copies of k-half h are done when at most the later ones are pending
    if (h + 2 < nkh) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (h + 1 < nkh) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g4_barrier();   // everyone's copies of h landed; everyone finished reading k-half h-1
    if (h + 3 < nkh) {
      char* s3 = smem + ((h + 3) & 3) * G4_SLOT;
      g4_issue<true>(A, s3, m0, kb + 32 * (h + 3), lane, wave);
      g4_issue<BKC>(B, s3 + G4_OPB, n0, kb + 32 * (h + 3), lane, wave);
    }
    const char* sa = smem + (h & 3) * G4_SLOT;
    const char* sb = sa + G4_OPB;
    bf16x8 fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = g4_frag<BKC>(sb, wc * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      Frag8<bf16> fa;
      fa.v = g4_frag<true>(sa, wr * 128 + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Frag8<bf16> fbj;
        fbj.v = fb[j];
        mma16(fa, fbj, acc[i][j]);
      }
    }
  }
  g4_barrier();   // all waves done with the ring before it becomes the C staging area

  // C through LDS in two 128-row passes (pass q: the waves with wr == q)
  float* cs = reinterpret_cast<float*>(smem);
  const uint32_t seed = (!ws && E.drop.thr) ? *E.drop.seed : 0u;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (wr == q) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[(16 * i + 4 * (lane >> 4) + r) * G4_EPI_LD + wc * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int id = tid + G4_NT * it;   // 128 rows x 32 chunks of 8
      const int row = id >> 5, c8 = (id & 31) * 8;
      const int m = m0 + 128 * q + row, n = n0 + c8;
      if (m >= M || n >= N) continue;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * G4_EPI_LD + c8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * G4_EPI_LD + c8 + 4);
      if (ws) {
        float* w = ws + ((int64_t)blockIdx.y * M + m) * N + n;
        if (n + 8 <= N && (N % 4) == 0) {
          *reinterpret_cast<f32x4*>(w) = lo;
          *reinterpret_cast<f32x4*>(w + 4) = hi;
        } else {
          const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          for (int j = 0; j < 8; ++j)
            if (n + j < N) w[j] = v[j];
        }
      } else {
        const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        epi_store8(E, seed, m, n, N, v);
      }
    }
    __syncthreads();
  }
}

template <bool BKC>
hipError_t launch4(const OpDesc& A, const OpDesc& B, const EpiParams& E, int M, int N, int K, int splits, float* ws,
                   hipStream_t s) {
  int k_split = K;
  if (splits > 1) {
    k_split = ((K + splits - 1) / splits + 31) / 32 * 32;
    splits = (K + k_split - 1) / k_split;
  }
  const int ntm = (M + 255) / 256, ntn = (N + 255) / 256;
  hipLaunchKernelGGL((gemm4_kernel<BKC>), dim3(ntm * ntn, splits), dim3(G4_NT), 0, s, A, B, E, M, N, K, k_split,
                     splits > 1 ? ws : nullptr, ntm, ntn);
  if (splits > 1 && !E.main_only) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256;
    int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}


// =====================================================================================
// v5 (bf16): the v2 tile (128 x 128, 4 waves of 64 x 64) with BK = 32 and a 3-slot
// LDS ring (16 KB per slot, two K steps in flight), and the C staging split in two
// 64-row passes: 48 KB of LDS per workgroup, so three workgroups share a CU (v2: two).
// More resident workgroups is what hides the per-K-step load latency of this tile
// (measured: every v2 GEMM of the step runs faster with more workgroups per CU).
// Images: K-contiguous [128 rows][4 chunks], chunk c of row r at c ^ ((r >> 1) & 3);
// M/N-contiguous [32 k][16 chunks], chunk c of row k at c ^ mc_swz(k).
// =====================================================================================
constexpr int G5_OPB = 128 * 32 * 2;     // 8 KB per operand per slot
constexpr int G5_SLOT = 2 * G5_OPB;       // 16 KB
constexpr int G5_EPI = 64 * EPI_LD * 4;   // 33.8 KB of C staging per pass
template <int SLOTS> struct G5 {
  static constexpr int SMEM = SLOTS * G5_SLOT > G5_EPI ? SLOTS * G5_SLOT : G5_EPI;
  static constexpr int WG_PER_CU = SLOTS == 3 ? 3 : 4;
};

template <bool KC>
TT2_DEV void g5_issue(const OpDesc& d, char* lds, int r0, int k0, int lane, int wave) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = wave * 2 + i;
    const void* src;
    if (KC) {
      const int row = inst * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((row >> 1) & 3);
      src = chunk_src(d, r0 + row, k0 + lc * 8);
    } else {
      const int kr = inst * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ mc_swz(kr);
      src = chunk_src(d, k0 + kr, r0 + lc * 8);
    }
    __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(lds + inst * 1024), 16, 0, 0);
  }
}

template <bool KC>
TT2_DEV void g5_frag(Frag8<bf16>& f, const char* img, int r0, int lane) {
  if (KC) {
    const int row = r0 + (lane & 15);
    f.v = *reinterpret_cast<const bf16x8*>(img + row * 64 + ((((lane >> 4) ^ (row >> 1)) & 3) << 4));
  } else {
    frag2<false>(f, img, r0, 0, lane);   // 256-B k rows, k 0..31
  }
}

template <bool AK, bool BKC, int SLOTS>
__global__ __launch_bounds__(NT, G5<SLOTS>::WG_PER_CU) void gemm5_kernel(OpDesc A, OpDesc B, EpiParams E, int M,
                                                                         int N, int K, int k_split, float* ws,
                                                                         int ntm, int ntn) {
  __shared__ __attribute__((aligned(1024))) char smem[G5<SLOTS>::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = ntm * ntn;
  const int bid = blockIdx.x;
  const int q8 = nt / 8, rr = nt % 8, x = bid % 8;
  const int tile = (x < rr ? x * (q8 + 1) : rr * (q8 + 1) + (x - rr) * q8) + bid / 8;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int kb = blockIdx.y * k_split;
  const int ke = min(K, kb + k_split);
  if (AK) A.inner_max = ke; else A.outer_max = ke;
  if (BKC) B.inner_max = ke; else B.outer_max = ke;
  const int nkt = (ke - kb + 31) / 32;
  const bool do_ks = !AK && E.ksum && (tile % ntn) == 0;
  float ks[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < SLOTS - 1; ++t)
    if (t < nkt) {
      g5_issue<AK>(A, smem + t * G5_SLOT, m0, kb + 32 * t, lane, wave);
      g5_issue<BKC>(B, smem + t * G5_SLOT + G5_OPB, n0, kb + 32 * t, lane, wave);
    }
  int slot = 0;
  for (int kt = 0; kt < nkt; ++kt) {
    if (SLOTS == 3 && kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");   // step kt landed everywhere; step kt-1's slot is free
    if (kt + SLOTS - 1 < nkt) {
      const int s2 = slot == 0 ? SLOTS - 1 : slot - 1;
      g5_issue<AK>(A, smem + s2 * G5_SLOT, m0, kb + 32 * (kt + SLOTS - 1), lane, wave);
      g5_issue<BKC>(B, smem + s2 * G5_SLOT + G5_OPB, n0, kb + 32 * (kt + SLOTS - 1), lane, wave);
    }
    const char* sa = smem + slot * G5_SLOT;
    const char* sb = sa + G5_OPB;
    Frag8<bf16> fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) g5_frag<AK>(fa[i], sa, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) g5_frag<BKC>(fb[j], sb, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mma16(fa[i], fb[j], acc[i][j]);
    if (!AK && do_ks) {
      // k rows 2*(tid>>4), +1 of the [32 k][128 m] A image, m-chunk tid & 15
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int kr = 2 * (tid >> 4) + r;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(sa + kr * 256 + (((tid & 15) ^ mc_swz(kr)) << 4));
#pragma unroll
        for (int j = 0; j < 8; ++j) ks[j] += (float)v[j];
      }
    }
    slot = slot == SLOTS - 1 ? 0 : slot + 1;
  }
  asm volatile("s_barrier" ::: "memory");   // ring free for the epilogue

  if (!AK && do_ks) {
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ks[j] += __shfl_xor(ks[j], 16, 64);
      ks[j] += __shfl_xor(ks[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(wave * 16 + lane) * 8 + j] = ks[j];
    }
    __syncthreads();
    if (tid < 128) {
      const int cc = tid >> 3, j = tid & 7, m = m0 + tid;
      const float v = (red[(0 * 16 + cc) * 8 + j] + red[(1 * 16 + cc) * 8 + j]) +
                      (red[(2 * 16 + cc) * 8 + j] + red[(3 * 16 + cc) * 8 + j]);
      if (m < M) {
        if (ws) ws[(int64_t)gridDim.y * M * N + (int64_t)blockIdx.y * M + m] = v;
        else E.ksum[m] = E.ksum_beta != 0.f ? E.ksum_beta * E.ksum[m] + v : v;
      }
    }
    __syncthreads();
  }

  float* cs = reinterpret_cast<float*>(smem);
  const uint32_t seed = (!ws && E.drop.thr) ? *E.drop.seed : 0u;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (wm == q) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[(16 * i + 4 * (lane >> 4) + r) * EPI_LD + wn * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 4; ++it) {
      const int id = tid + NT * it;   // 64 rows x 16 chunks of 8
      const int row = id >> 4, c8 = (id & 15) * 8;
      const int m = m0 + 64 * q + row, n = n0 + c8;
      if (m >= M || n >= N) continue;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * EPI_LD + c8 + 4);
      const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (ws) {
        float* w = ws + ((int64_t)blockIdx.y * M + m) * N + n;
        if (n + 8 <= N && (N % 4) == 0) {
          *reinterpret_cast<f32x4*>(w) = lo;
          *reinterpret_cast<f32x4*>(w + 4) = hi;
        } else {
          for (int j = 0; j < 8; ++j)
            if (n + j < N) w[j] = v[j];
        }
      } else {
        epi_store8(E, seed, m, n, N, v);
      }
    }
    __syncthreads();
  }
}

template <bool AK, bool BKC, int SLOTS>
hipError_t launch5(const OpDesc& A, const OpDesc& B, const EpiParams& E, int M, int N, int K, int splits, float* ws,
                   hipStream_t s) {
  int k_split = K;
  if (splits > 1) {
    k_split = ((K + splits - 1) / splits + 31) / 32 * 32;
    splits = (K + k_split - 1) / k_split;
  }
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm5_kernel<AK, BKC, SLOTS>), dim3(ntm * ntn, splits), dim3(NT), 0, s, A, B, E, M, N, K, k_split,
                     splits > 1 ? ws : nullptr, ntm, ntn);
  if (splits > 1 && !E.main_only) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256;
    int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" size_t tt2_gemm_workspace_size(const tt2_gemm_args* a) {
  if (a->splits <= 1) return 0;
  return (size_t)a->splits * a->m * (a->n + (a->a_ksum ? 1 : 0)) * sizeof(float);
}

// Kernel selection (also exported as tt2_gemm_plan): 1 v1 register-staged, 2 v2
// LDS-DMA 128^2, 3 skinny (M <= 32), 4-7 v3 pipelines, 8 v4 256^2, 9/10 v5 BK=32 ring
// (3 / 2 slots).  Returns -1 (error set) for an unsupported fusion request.
static int gemm_plan(const tt2_gemm_args* a) {
  const int var = a->kernel_variant;
  const int64_t a_inner = a->trans_a ? a->m : a->k, b_inner = a->trans_b ? a->n : a->k;
  const bool skinny = a->dtype_in == TT2_BF16 && a->m <= 32 && !a->trans_a && !a->trans_b && a->k % 8 == 0 &&
                      a->a_conv_t == 0 && a->splits <= 1 && (var == 0 || var == 3);
  if ((a->a_ln_gamma || a->kv_cache) && !skinny)
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: a_ln / kv fusions need the skinny path (bf16, m <= 32, NT)"), -1;
  if (a->a_ln_gamma && (a->k != 512 || a->lda != a->k || !a->a_ln_branch || !a->a_ln_beta || !a->a_ln_out))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: a_ln needs k == lda == 512, branch, beta and out"), -1;
  if (a->kv_cache && (!a->kv_t || a->dtype_out != TT2_BF16))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: kv scatter needs kv_t and a bf16 output"), -1;
  if (skinny) return 3;
  // LDS-DMA kernels: bf16, every 16-B chunk either fully inside or fully outside its row
  const bool v2 = a->dtype_in == TT2_BF16 && var != 1 && a_inner % 8 == 0 && b_inner % 8 == 0;
  if (a->a_ksum && !(v2 && (var < 4 || var == 9 || var == 10) && a->trans_a && a->a_conv_t == 0))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: a_ksum needs bf16, trans_a, no conv A, the LDS-DMA kernel"), -1;
  if (!v2) return 1;
  // v4: 256^2 tiles (K-contiguous A).  Auto only for GEMMs with a full chip of such
  // tiles and a long K (4096^3: +20 % over v2); the training step's d_model = 512
  // shapes measure faster on v2 (more CUs pulling operands), or variant 8 forces it.
  const bool big = (int64_t)((a->m + 255) / 256) * ((a->n + 255) / 256) >= 256 && a->k >= 1024;
  if (!a->trans_a && !a->a_ksum && (var == 8 || (var == 0 && big))) return 8;
  // v5 auto: the BK=32 / 2-slot / 4-workgroups-per-CU form for activation GEMMs with
  // enough 128^2 tiles to give every CU four (e.g. 12800 x 2048 x 512: +15 % fwd, +25 %
  // dgrad); fewer tiles pile four workgroups onto a fraction of the CUs: those stay on v2
  const int64_t tiles128 = (int64_t)((a->m + 127) / 128) * ((a->n + 127) / 128);
  if (var == 9) return 9;
  if (var == 10 || (var == 0 && !a->trans_a && !a->a_ksum && tiles128 >= 1024 && a->k <= 1024)) return 10;
  if (var >= 4 && var <= 7) return var;
  return 2;
}

extern "C" int tt2_gemm_plan(const tt2_gemm_args* a) { return gemm_plan(a); }

extern "C" int tt2_gemm(const tt2_gemm_args* a, hipStream_t stream) {
  if (a->m <= 0 || a->n <= 0) return TT2_OK;
  const int esz = a->dtype_in == TT2_BF16 ? 2 : 4;
  const int E = 16 / esz;
  auto misaligned = [&](const void* p, int64_t ld) {
    return (reinterpret_cast<uintptr_t>(p) % 16) != 0 || (ld * esz) % 16 != 0;
  };
  if (!a->a || !a->b || !a->c) return tt2_set_error(TT2_E_INVALID, "tt2_gemm: null operand");
  if (misaligned(a->a, a->lda) || misaligned(a->b, a->ldb))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: operands must be 16-B aligned with 16-B multiple leading dims");
  if (a->a_conv_t > 0 && (a->trans_a || a->a_conv_c % E != 0 || a->lda != a->a_conv_c))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: conv A needs K-contiguous A, lda == C, C % chunk == 0");
  if (a->b_conv_t > 0 && (!a->trans_b || a->b_conv_c % E != 0 || a->ldb != a->b_conv_c))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: conv B needs N-contiguous B, ldb == C, C % chunk == 0");
  if (a->splits > 1 && (!a->workspace || a->ws_bytes < tt2_gemm_workspace_size(a)))
    return tt2_set_error(TT2_E_INVALID, "tt2_gemm: split-K workspace too small");

  OpDesc A{a->a, a->lda, 0, 0, a->a_conv_t, a->a_conv_c, a->a_conv_pad};
  OpDesc B{a->b, a->ldb, 0, 0, a->b_conv_t, a->b_conv_c, a->b_conv_pad};
  if (!a->trans_a) { A.outer_max = a->m; A.inner_max = a->k; } else { A.outer_max = a->k; A.inner_max = a->m; }
  if (!a->trans_b) { B.outer_max = a->n; B.inner_max = a->k; } else { B.outer_max = a->k; B.inner_max = a->n; }
  if (a->k <= 0) return tt2_set_error(TT2_E_INVALID, "tt2_gemm: k must be > 0");

  EpiParams ep;
  ep.c = a->c; ep.ldc = a->ldc; ep.c_dt = a->dtype_out;
  ep.bias = a->bias;
  ep.res = a->res; ep.ldr = a->ldr; ep.res_dt = a->res_dtype;
  ep.gate = a->gate; ep.ldg = a->ldg; ep.gate_dt = a->gate_dtype; ep.gate_scale = a->gate_scale;
  ep.alpha = a->alpha; ep.beta = a->beta; ep.act = a->act;
  ep.drop = DropDesc{a->drop_seed, a->drop_site, a->drop_thr, a->drop_scale};
  if (ep.drop.thr && !ep.drop.seed) return tt2_set_error(TT2_E_INVALID, "tt2_gemm: dropout without seed");
  ep.n_log = a->n;
  ep.ksum = a->a_ksum;
  ep.ksum_beta = a->a_ksum_beta;
  ep.main_only = a->main_only;
  {
    // vectorised epilogue: rows of C / res / gate start 16-B aligned at every 8th column
    auto ok = [](const void* p, int64_t ld, int dt) {
      if (!p) return true;
      const int esz = dt == TT2_BF16 ? 2 : 4;
      return reinterpret_cast<uintptr_t>(p) % 16 == 0 && (ld * esz) % 16 == 0 && (8 * esz) % 16 == 0;
    };
    ep.vec = ok(a->c, a->ldc, a->dtype_out) && ok(a->res, a->ldr, a->res_dtype) &&
             ok(a->gate, a->ldg, a->gate_dtype) && (reinterpret_cast<uintptr_t>(a->bias) % 16 == 0);
  }
  float* ws = reinterpret_cast<float*>(a->workspace);
  const int sp = a->splits > 1 ? a->splits : 1;

  hipError_t err;
  const int plan = gemm_plan(a);
  if (plan < 0) return TT2_E_INVALID;   // message already set
  if (plan == 3) {   // skinny-M weight-streaming path (decode step)
    SkinnyFuse F{reinterpret_cast<const bf16*>(a->a_ln_branch), a->a_ln_gamma, a->a_ln_beta,
                 reinterpret_cast<bf16*>(a->a_ln_out), a->a_ln_eps, reinterpret_cast<bf16*>(a->kv_cache), a->kv_t,
                 a->kv_col0, a->kv_bstride, a->kv_ld};
    const size_t lds = a->a_ln_gamma ? 32 * SK_LN_LD * sizeof(bf16) : 0;
    hipLaunchKernelGGL(gemm_skinny_kernel, dim3((a->n + SK_COLS - 1) / SK_COLS), dim3(NT), lds, stream,
                       reinterpret_cast<const bf16*>(a->a), a->lda, reinterpret_cast<const bf16*>(a->b), a->ldb, ep,
                       a->m, a->n, a->k, F);
    return tt2_check_launch(hipGetLastError(), "tt2_gemm(skinny)");
  }
  if (plan == 8) {
    if (!a->trans_b) err = launch4<true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    else err = launch4<false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    return tt2_check_launch(err, "tt2_gemm(v4)");
  }
  if (plan == 9 || plan == 10) {
#define TT2_G5(S)                                                                                            \
    if (!a->trans_a && !a->trans_b) err = launch5<true, true, S>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);   \
    else if (!a->trans_a && a->trans_b) err = launch5<true, false, S>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
    else if (a->trans_a && !a->trans_b) err = launch5<false, true, S>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
    else err = launch5<false, false, S>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    if (plan == 9) { TT2_G5(3) } else { TT2_G5(2) }
#undef TT2_G5
    return tt2_check_launch(err, "tt2_gemm(v5)");
  }
  if (plan >= 4 && plan <= 7) {
    // v3 configurations: 4 = BM128/2 stages, 5 = BM128/3, 6 = BM256/3 (K-contiguous A), 7 = BM128/4
    const int var = plan;
#define TT2_G3(AK_, BK_)                                                                              \
    if (var == 6 && AK_) err = launch3<AK_, BK_, 256, 3>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
    else if (var == 5 || var == 6) err = launch3<AK_, BK_, 128, 3>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
    else if (var == 7) err = launch3<AK_, BK_, 128, 4>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
    else err = launch3<AK_, BK_, 128, 2>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    if (!a->trans_a && !a->trans_b) { TT2_G3(true, true) }
    else if (!a->trans_a && a->trans_b) { TT2_G3(true, false) }
    else if (a->trans_a && !a->trans_b) { TT2_G3(false, true) }
    else { TT2_G3(false, false) }
#undef TT2_G3
    return tt2_check_launch(err, "tt2_gemm(v3)");
  }
  if (plan == 2) {
    if (!a->trans_a && !a->trans_b) err = launch2<true, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    else if (!a->trans_a && a->trans_b) err = launch2<true, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    else if (a->trans_a && !a->trans_b) err = launch2<false, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    else err = launch2<false, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
    return tt2_check_launch(err, "tt2_gemm");
  }
#define TT2_GEMM_CASE(T)                                                                              \
  if (!a->trans_a && !a->trans_b) err = launch_t<T, true, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);   \
  else if (!a->trans_a && a->trans_b) err = launch_t<T, true, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
  else if (a->trans_a && !a->trans_b) err = launch_t<T, false, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
  else err = launch_t<T, false, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
  if (a->dtype_in == TT2_BF16) { TT2_GEMM_CASE(bf16) } else { TT2_GEMM_CASE(float) }
#undef TT2_GEMM_CASE
  return tt2_check_launch(err, "tt2_gemm");
}
