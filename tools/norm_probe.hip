// Bandwidth probe for the step's memory-bound normalisation passes (dev tool, GPU): column
// statistics of a 12800 x 512 bf16 matrix (the post-net BatchNorm statistics) in several
// work splits, the BatchNorm apply with per-column constants loaded per element or folded into
// one scale / shift, and pure streaming references (read 1, read 1 + write 1, read 3 + write 2),
// each as 20 launches replayed from a hipGraph, warm (one buffer set) and cold (24 sets
// rotated, 315 MB > the 256 MB MALL).
//   hipcc --offload-arch=gfx950 -O3 tools/norm_probe.hip -o /tmp/np && /tmp/np
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef __hip_bfloat16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int M = 12800, C = 512, CG = C / 8;

__device__ __forceinline__ void ld8(const bf16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = __uint_as_float(w[j] << 16); v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u); }
}
__device__ __forceinline__ void st8nt(bf16* p, const float (&v)[8]) {
  unsigned w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned lo = __float_as_uint(v[2 * j]) >> 16, hi = __float_as_uint(v[2 * j + 1]) & 0xffff0000u;
    w[j] = lo | hi;
  }
  __builtin_nontemporal_store(u32x4{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4*>(p));
}

__device__ __forceinline__ float ftanh(float x) {
  const float t = 1.f - __fdividef(2.f, __expf(2.f * fabsf(x)) + 1.f);
  return copysignf(t, x);
}

// column moments, rows_per rows per work group, 256 threads = 64 column groups x 4 row lanes,
// U rows' loads issued before they are summed (U = 1: the production loop)
template <int RP, int U>
__global__ __launch_bounds__(256) void stats_k(const bf16* y, float* part) {
  __shared__ float red[2][256][8];
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int r0 = blockIdx.x * RP;
  float k[8], s1[8], s2[8];
  ld8(y + (int64_t)r0 * C + cg * 8, k);
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  constexpr int IT = RP / 4;
  if constexpr (U == 1) {
    for (int r = r0 + rl; r < r0 + RP; r += 4) {
      float v[8];
      ld8(y + (int64_t)r * C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - k[j]; s1[j] += d; s2[j] += d * d; }
    }
  } else {
#pragma unroll
    for (int i0 = 0; i0 < IT; i0 += U) {
      uint4 raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) raw[u] = *reinterpret_cast<const uint4*>(y + (int64_t)(r0 + rl + 4 * (i0 + u)) * C + cg * 8);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const unsigned w[4] = {raw[u].x, raw[u].y, raw[u].z, raw[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = __uint_as_float(w[j] << 16) - k[2 * j], b = __uint_as_float(w[j] & 0xffff0000u) - k[2 * j + 1];
          s1[2 * j] += a; s2[2 * j] += a * a; s1[2 * j + 1] += b; s2[2 * j + 1] += b * b;
        }
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
      for (int l = 0; l < 4; ++l) { S1 += red[0][l * CG + cg][j]; S2 += red[1][l * CG + cg][j]; }
      part[((int64_t)blockIdx.x * 2 + 0) * C + cg * 8 + j] = k[j] + S1 / RP;
      part[((int64_t)blockIdx.x * 2 + 1) * C + cg * 8 + j] = S2;
    }
  }
}

// the production apply: four per-column constant vectors per element, grid-stride
__global__ __launch_bounds__(256) void apply_k(const bf16* y, const float* mu, const float* rs, const float* g,
                                               const float* b, bf16* out) {
  for (int q = blockIdx.x * 256 + threadIdx.x; q < M * CG; q += gridDim.x * 256) {
    const int m = q / CG, c0 = (q - m * CG) * 8;
    float v[8], z[8];
    ld8(y + (int64_t)m * C + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = ftanh((v[j] - mu[c0 + j]) * rs[c0 + j] * g[c0 + j] + b[c0 + j]);
    st8nt(out + (int64_t)m * C + c0, z);
  }
}
// folded scale / shift, R rows per thread of one column group, loads first
template <int R>
__global__ __launch_bounds__(256) void apply2_k(const bf16* y, const float* sc, const float* sh, bf16* out) {
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int c0 = cg * 8;
  float a[8], s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = sc[c0 + j]; s[j] = sh[c0 + j]; }
  const int r0 = blockIdx.x * 4 * R + rl;
  float v[R][8];
#pragma unroll
  for (int u = 0; u < R; ++u) ld8(y + (int64_t)(r0 + 4 * u) * C + c0, v[u]);
#pragma unroll
  for (int u = 0; u < R; ++u) {
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = ftanh(v[u][j] * a[j] + s[j]);
    st8nt(out + (int64_t)(r0 + 4 * u) * C + c0, z);
  }
}
// references
__global__ __launch_bounds__(256) void read1_k(const bf16* y, float* o) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  float v[8];
  ld8(y + i, v);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j];
  if (s == 1234.5f) o[0] = s;
}
__global__ __launch_bounds__(256) void copy_k(const bf16* y, bf16* o) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  float v[8];
  ld8(y + i, v);
  st8nt(o + i, v);
}
__global__ __launch_bounds__(256) void r3w2_k(const bf16* x, const bf16* y, const bf16* z, bf16* o, bf16* p) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  float a[8], b[8], c[8];
  ld8(x + i, a); ld8(y + i, b); ld8(z + i, c);
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] += b[j]; b[j] = a[j] * c[j]; }
  st8nt(o + i, a); st8nt(p + i, b);
}

int main() {
  const int NS = 24;
  const size_t E = (size_t)M * C;
  std::vector<bf16*> X(NS), Y(NS), Z(NS), O(NS), P(NS);
  for (int i = 0; i < NS; ++i) {
    CK(hipMalloc(&X[i], E * 2)); CK(hipMalloc(&Y[i], E * 2)); CK(hipMalloc(&Z[i], E * 2));
    CK(hipMemset(X[i], 0x3c, E * 2)); CK(hipMemset(Y[i], 0x3c, E * 2)); CK(hipMemset(Z[i], 0x3c, E * 2));
    if (i < 2) { CK(hipMalloc(&O[i], E * 2)); CK(hipMalloc(&P[i], E * 2)); }
  }
  float *part, *cst;
  CK(hipMalloc(&part, 1600 * 2 * C * 4)); CK(hipMalloc(&cst, 8 * C * 4)); CK(hipMemset(cst, 0, 8 * C * 4));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int cold = 0; cold < 2; ++cold) {
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int it = 0; it < 20; ++it) launch(cold ? it % NS : 0);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, s)); CK(hipGraphLaunch(ge, s)); CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      const double us = best * 1e3 / 20;
      printf("%-34s %s %8.2f us  %6.2f TB/s\n", name, cold ? "cold" : "warm", us, bytes / us / 1e6);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  };
  const double B1 = E * 2.0;
  run("read 1 (3200 wg)", B1, [&](int i) { read1_k<<<M * CG / 256, 256, 0, s>>>(X[i], part); });
  run("copy 1 -> 1", 2 * B1, [&](int i) { copy_k<<<M * CG / 256, 256, 0, s>>>(X[i], O[0]); });
  run("read 3 write 2", 5 * B1, [&](int i) { r3w2_k<<<M * CG / 256, 256, 0, s>>>(X[i], Y[i], Z[i], O[0], P[0]); });
  run("stats rp32 u1 (production, 400 wg)", B1, [&](int i) { stats_k<32, 1><<<M / 32, 256, 0, s>>>(X[i], part); });
  run("stats rp32 u8 (400 wg)", B1, [&](int i) { stats_k<32, 8><<<M / 32, 256, 0, s>>>(X[i], part); });
  run("stats rp32 u4 (400 wg)", B1, [&](int i) { stats_k<32, 4><<<M / 32, 256, 0, s>>>(X[i], part); });
  run("stats rp16 u4 (800 wg)", B1, [&](int i) { stats_k<16, 4><<<M / 16, 256, 0, s>>>(X[i], part); });
  run("stats rp8 u2 (1600 wg)", B1, [&](int i) { stats_k<8, 2><<<M / 8, 256, 0, s>>>(X[i], part); });
  run("stats rp64 u16 (200 wg)", B1, [&](int i) { stats_k<64, 16><<<M / 64, 256, 0, s>>>(X[i], part); });
  run("apply production (3200 wg)", 2 * B1, [&](int i) {
    apply_k<<<M * CG / 256, 256, 0, s>>>(X[i], cst, cst + C, cst + 2 * C, cst + 3 * C, O[0]); });
  run("apply folded r1 (3200 wg)", 2 * B1, [&](int i) { apply2_k<1><<<M / 4, 256, 0, s>>>(X[i], cst, cst + C, O[0]); });
  run("apply folded r2 (1600 wg)", 2 * B1, [&](int i) { apply2_k<2><<<M / 8, 256, 0, s>>>(X[i], cst, cst + C, O[0]); });
  run("apply folded r4 (800 wg)", 2 * B1, [&](int i) { apply2_k<4><<<M / 16, 256, 0, s>>>(X[i], cst, cst + C, O[0]); });
  CK(hipStreamSynchronize(s));
  return 0;
}
