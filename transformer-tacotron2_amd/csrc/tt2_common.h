// tt2_common.h -- device helpers shared by every libtt2 kernel (gfx950 only).
//
// Storage types: activations/weights are either bf16 (__bf16) or f32; every
// kernel is a template over the storage type T and accumulates in f32.
// MFMA: bf16 uses v_mfma_f32_16x16x32_bf16; f32 uses v_mfma_f32_16x16x4_f32
// (exact f32, used for the 1e-3 parity mode).  Both consume the SAME per-lane
// fragment: lane l holds 8 consecutive k of row (l & 15), k = 8*(l >> 4) + j.
// For f32 the 8 elements are issued as 8 x (16x16x4) steps; the k order inside
// a 32-deep step is a permutation, which is legal because both operands use it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16;   // the fp16 decode path
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#define TT2_DEV __device__ __forceinline__

// ---------------------------------------------------------------- conversions
TT2_DEV float to_f32(float x) { return x; }
TT2_DEV float to_f32(bf16 x) { return (float)x; }
TT2_DEV float to_f32(f16 x) { return (float)x; }
template <typename T> TT2_DEV T from_f32(float x);
template <> TT2_DEV float from_f32<float>(float x) { return x; }
template <> TT2_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }
template <> TT2_DEV f16 from_f32<f16>(float x) { return (f16)x; }

// 16-byte chunk of T: 8 bf16 or 4 f32.
template <typename T> struct Chunk { static constexpr int N = 16 / sizeof(T); };

// 8-element fragment of T (16 B for bf16, 32 B for f32)
template <typename T> struct Frag8;
template <> struct Frag8<bf16> { bf16x8 v; };
template <> struct Frag8<float> { float v[8]; };

TT2_DEV void mma16(const Frag8<bf16>& a, const Frag8<bf16>& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
TT2_DEV void mma16(const Frag8<float>& a, const Frag8<float>& b, f32x4& c) {
#pragma unroll
  for (int s = 0; s < 8; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], c, 0, 0, 0);
}

// Fragment from an LDS row (8 consecutive elements, 16-B aligned for bf16).
TT2_DEV void frag_row(Frag8<bf16>& f, const bf16* p) { f.v = *reinterpret_cast<const bf16x8*>(p); }
TT2_DEV void frag_row(Frag8<float>& f, const float* p) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f.v[0] = a[0]; f.v[1] = a[1]; f.v[2] = a[2]; f.v[3] = a[3];
  f.v[4] = b[0]; f.v[5] = b[1]; f.v[6] = b[2]; f.v[7] = b[3];
}

// Fragment from a column of an LDS tile stored [k][ld] (k-major):
// lane needs tile[k0 + j][col] for j = 0..7.
// bf16: two ds_read_b64_tr_b16 (each 16-lane group reads a 4-row x 16-col block;
// lane 4q+p supplies &tile[row q][col0 + 4p]; lane i receives column i).
TT2_DEV void frag_col(Frag8<bf16>& f, const bf16* tile, int ld, int k0, int col0, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const bf16* a0 = tile + (k0 + q) * ld + col0 + 4 * p;
  const bf16* a1 = tile + (k0 + 4 + q) * ld + col0 + 4 * p;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a1));
  union { short s[8]; bf16x8 v; } u;
  u.s[0] = lo[0]; u.s[1] = lo[1]; u.s[2] = lo[2]; u.s[3] = lo[3];
  u.s[4] = hi[0]; u.s[5] = hi[1]; u.s[6] = hi[2]; u.s[7] = hi[3];
  f.v = u.v;
}
TT2_DEV void frag_col(Frag8<float>& f, const float* tile, int ld, int k0, int col0, int lane) {
  const int col = col0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = tile[(k0 + j) * ld + col];
}

// ---------------------------------------------------------------- chunk I/O
// 16-byte global loads/stores of one chunk (caller guarantees alignment).
template <typename T> struct alignas(16) ChunkV { T e[Chunk<T>::N]; };

template <typename T> TT2_DEV ChunkV<T> ld_chunk(const T* p) {
  ChunkV<T> c;
  *reinterpret_cast<uint4*>(&c) = *reinterpret_cast<const uint4*>(p);
  return c;
}
template <typename T> TT2_DEV void st_chunk(T* p, const ChunkV<T>& c) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(&c);
}
template <typename T> TT2_DEV ChunkV<T> zero_chunk() {
  ChunkV<T> c;
  *reinterpret_cast<uint4*>(&c) = make_uint4(0, 0, 0, 0);
  return c;
}

// ---------------------------------------------------------------- dropout hash
// Bit-identical to oracle/tt2_oracle.py::dropout_keep (with drop_keep below).
TT2_DEV uint32_t drop_hash(uint32_t seed, uint32_t site, uint32_t idx) {
  uint32_t x = idx * 0x9E3779B1u + seed * 0x85EBCA77u + site * 0xC2B2AE3Du;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// Dropout descriptor passed by value to kernels.  thr == 0 disables it.
struct DropDesc {
  const uint32_t* seed;  // device pointer to the per-step seed
  uint32_t site;
  uint32_t thr;          // floor(p * 2^32)
  float scale;           // 1 / (1 - p)
};
// Keep test of flat element idx: 16 bits per element, two elements per hash (the pair
// idx >> 1; the even element takes the low half) against thr >> 16 = floor(p * 2^16).
TT2_DEV bool drop_keep(uint32_t seed, uint32_t site, uint32_t idx, uint32_t thr) {
  const uint32_t h = drop_hash(seed, site, idx >> 1);
  return ((idx & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= (thr >> 16);
}
TT2_DEV float drop_apply(const DropDesc& d, uint32_t seed, uint32_t idx, float v) {
  return drop_keep(seed, d.site, idx, d.thr) ? v * d.scale : 0.f;
}
// Keep bits of elements base .. base + 7 (bit j: element base + j) from 4 hashes (5 for an
// odd base): the same decisions as drop_keep.
TT2_DEV uint32_t drop_bits8(uint32_t seed, uint32_t site, uint32_t base, uint32_t thr) {
  const uint32_t t16 = thr >> 16, odd = base & 1u, p0 = base >> 1;
  uint32_t bits = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    if (q == 4 && !odd) break;
    const uint32_t h = drop_hash(seed, site, p0 + q);
    const int jl = 2 * q - (int)odd;   // element of the low half; jl + 1 takes the high half
    if (jl >= 0) bits |= (uint32_t)((h & 0xFFFFu) >= t16) << jl;
    if (jl + 1 < 8) bits |= (uint32_t)((h >> 16) >= t16) << (jl + 1);
  }
  return bits;
}
TT2_DEV void drop_apply8(const DropDesc& d, uint32_t seed, uint32_t base, float (&v)[8]) {
  const uint32_t b = drop_bits8(seed, d.site, base, d.thr);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (b >> j) & 1u ? v[j] * d.scale : 0.f;
}

// ---------------------------------------------------------------- reductions
// Full-wave sum without LDS: DPP within 16-lane rows (quad xor 1, quad xor 2,
// half-row mirror, row mirror), then v_permlane16_swap / v_permlane32_swap across
// rows.  Every lane ends with the total (same value in all lanes).
template <int CTRL> TT2_DEV float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
TT2_DEV float wave_sum(float v) {
  v += dpp_f32<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f32<0x141>(v);   // row_half_mirror
  v += dpp_f32<0x140>(v);   // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// 8 consecutive elements as f32
template <typename T> TT2_DEV void ld8f(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 x = *reinterpret_cast<const t8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
  }
}

// The decode step's residual combine + LayerNorm of one 512-wide row by one wave (lane =
// 8-column chunk c0 = 8 lane): y = LN(x + (bias + sum_s part[s])) with the slab sum in fixed
// order.  tt2_ln_combine and the cross-attention launch's fused prologue both call it, so
// the two round identically (and tt2_ffn_decode, through ln_combine_vals: the same arithmetic
// on values it loads itself).  part: this row's slab 0 (slabs part_stride floats apart).
// ln_combine_vals: v = this lane's 8 x (overwritten), p its 8 columns of each slab, bb / g / be
// bias, gamma, beta.
template <int S>
TT2_DEV void ln_combine_vals(float (&v)[8], const float (&p)[S][8], const float (&bb)[8], const float (&g)[8],
                             const float (&be)[8], float eps, float (&o)[8]) {
  constexpr int C = 512;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = bb[j];
#pragma unroll
    for (int s = 0; s < S; ++s) a += p[s][j];   // fixed order: reproducible
    v[j] += a;
    sum += v[j];
  }
  const float mean = wave_sum(sum) / C;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { const float d = v[j] - mean; sq += d * d; }
  const float rstd = rsqrtf(wave_sum(sq) / C + eps);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (v[j] - mean) * rstd * g[j] + be[j];
}
template <int S, typename T>
TT2_DEV void ln_combine_row(const T* x, const float* part, int64_t part_stride, const float* bias,
                            const float* gamma, const float* beta, float eps, int lane, float (&o)[8]) {
  const int c0 = lane * 8;
  float v[8], p[S][8], bb[8], g[8], be[8];
  ld8f(x + c0, v);
#pragma unroll
  for (int s = 0; s < S; ++s) ld8f(part + s * part_stride + c0, p[s]);
  ld8f(bias + c0, bb);
  ld8f(gamma + c0, g);
  ld8f(beta + c0, be);
  ln_combine_vals<S>(v, p, bb, g, be, eps, o);
}

TT2_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce across the 16 lanes that share (lane >> 4)
TT2_DEV float sum16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TT2_DEV float max16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

enum { TT2_F32 = 0, TT2_BF16 = 1, TT2_F16 = 2 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

// tanh through one v_exp_f32 and one v_rcp_f32 (ocml's tanhf is a long branchy sequence and
// the BatchNorm passes evaluate it per element, twice in the backward): |error| < 1e-6
TT2_DEV float fast_tanh(float x) {
  const float t = 1.f - __fdividef(2.f, __expf(2.f * fabsf(x)) + 1.f);
  return copysignf(t, x);
}
TT2_DEV float act_f(int act, float v) {
  return act == ACT_RELU ? fmaxf(v, 0.f) : (act == ACT_TANH ? fast_tanh(v) : v);
}
TT2_DEV float act_grad_from_out(int act, float z) {
  return act == ACT_RELU ? (z > 0.f ? 1.f : 0.f) : (act == ACT_TANH ? 1.f - z * z : 1.f);
}
