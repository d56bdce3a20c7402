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
  if (splits > 1) {
    const int64_t total = (int64_t)M * N;
    int64_t nb = (total + 255) / 256; int blocks = (int)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(blocks), dim3(256), 0, s, ws, splits, E, M, N);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" size_t tt2_gemm_workspace_size(const tt2_gemm_args* a) {
  if (a->splits <= 1) return 0;
  return (size_t)a->splits * a->m * a->n * sizeof(float);
}

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
  float* ws = reinterpret_cast<float*>(a->workspace);
  const int sp = a->splits > 1 ? a->splits : 1;

  hipError_t err;
#define TT2_GEMM_CASE(T)                                                                              \
  if (!a->trans_a && !a->trans_b) err = launch_t<T, true, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);   \
  else if (!a->trans_a && a->trans_b) err = launch_t<T, true, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
  else if (a->trans_a && !a->trans_b) err = launch_t<T, false, true>(A, B, ep, a->m, a->n, a->k, sp, ws, stream); \
  else err = launch_t<T, false, false>(A, B, ep, a->m, a->n, a->k, sp, ws, stream);
  if (a->dtype_in == TT2_BF16) { TT2_GEMM_CASE(bf16) } else { TT2_GEMM_CASE(float) }
#undef TT2_GEMM_CASE
  return tt2_check_launch(err, "tt2_gemm");
}
