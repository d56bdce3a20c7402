// LDS fill-rate probe (dev tool, GPU): how fast one CU moves GEMM operand tiles into LDS with
// v7's loader pattern (48 KB per 64-deep K step: 384 rows x 128 B, 8 rows per 1-KB wave
// instruction, 3-stage ring, step t + 2 issued and step t + 1 waited for at step t, one barrier
// per step), 4 loader waves issuing global_load_lds_dwordx4:
//   resident  the same 384 rows every tile (L2 hits after the first tile)
//   fresh     each tile a new 384-row block (96 MB rotated: MALL / HBM, as a GEMM's A operand
//             that the previous kernel wrote), 4 work groups per block on one XCD (v7 at N = 512)
//   fresh+Pn  the same with an L2 warm-up: one 4-byte LDS-DMA copy per 128-B line of the rows
//             step t + 2 + n will copy, issued beside step t + 2's copies (into a junk slot)
// 256 work groups (one per CU), 64 tiles x 8 steps each, event-timed; B/clk/CU at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/fill_probe.hip -o tools/bin/fill_probe && tools/bin/fill_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// A barrier without a memory fence (v7's form): __syncthreads() adds a workgroup-scope fence,
// which waits vmcnt(0) -- every LDS-DMA copy and register load in flight -- before each barrier,
// leaving one step in flight instead of the ring's two (the round-5 rows were taken that way).
#define BARRIER() do { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); } while (0)

constexpr int ROWS = 384, STEP = ROWS * 128, STAGES = 3, NSTEP = 8, LD = 1024, NBLK = 256;

// PF: 0 no warm-up, n > 0 warm the lines of step t + 2 + n; FRESH: rotate row blocks per tile
template <int PF, bool FRESH>
__global__ __launch_bounds__(256) void dma_k(const char* src, int tiles, int* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * STEP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NI = 12;
  const int b = blockIdx.x, blk0 = (b % 8) * 8 + (b / 8) / 4;   // 4 WGs per block, one XCD
  int st = 0;
  auto rows_of = [&](int step) {
    const int tile = step / NSTEP;
    const int blk = FRESH ? (blk0 + 64 * tile) % NBLK : blk0;
    return src + (int64_t)blk * ROWS * LD + (step % NSTEP) * 128;
  };
  auto issue = [&](int step) {
    const char* base = rows_of(step);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int inst = w * NI + i, row = inst * 8 + (lane >> 3);
      __builtin_amdgcn_global_load_lds((gvoid_t*)(base + (int64_t)row * LD + (lane & 7) * 16),
                                       (lvoid_t*)(lds + st * STEP + inst * 1024), 16, 0, 0);
    }
    st = st == STAGES - 1 ? 0 : st + 1;
  };
  __shared__ __attribute__((aligned(1024))) char junk[1024];   // the warm-up copies' discarded dwords
  auto warm = [&](int step) {   // one dword per 128-B line of the step's 384 rows: 2 copies per lane
    const char* base = rows_of(step);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = min(threadIdx.x + 256 * i, ROWS - 1);
      __builtin_amdgcn_global_load_lds((gvoid_t*)(base + (int64_t)row * LD), (lvoid_t*)(junk + (w & 3) * 256), 4, 0,
                                       0);
    }
  };
  const int total = tiles * NSTEP;
  issue(0);
  issue(1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  BARRIER();
  for (int t = 0; t < total; ++t) {
    if (t + 2 < total) {
      issue(t + 2);
      if constexpr (PF > 0) {
        if (t + 2 + PF < total) {
          warm(t + 2 + PF);
          asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        }
      } else {
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    BARRIER();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && (lds[5] == 123 || junk[3] == 99)) *sink = 1;
}

// Register-staged fill: each loader lane loads its 12 pieces of a step with
// global_load_dwordx4 into VGPRs (48 VGPRs per step) and writes them into the ring with
// ds_write_b128 once the step's stage is free; RS register sets, so step s is issued RS
// iterations before it is written (RS steps of bytes in flight, against 2 for the LDS-DMA ring,
// whose destination stage must be free at issue).  Step s goes into stage s % 3 at iteration s - 2
// (the stage step s - 3 held was released by the barrier ending iteration s - 3).
// HYB: steps alternate between the LDS-DMA ring protocol (even) and register staging (odd).
template <int RS, bool FRESH>
__global__ __launch_bounds__(256) void reg_k(const char* src, int tiles, int* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * STEP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NI = 12;
  const int b = blockIdx.x, blk0 = (b % 8) * 8 + (b / 8) / 4;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 r[RS][NI];
  auto rows_of = [&](int step) {
    const int tile = step / NSTEP;
    const int blk = FRESH ? (blk0 + 64 * tile) % NBLK : blk0;
    return src + (int64_t)blk * ROWS * LD + (step % NSTEP) * 128;
  };
  auto load = [&](int step, u32x4 (&d)[NI]) {
    const char* base = rows_of(step);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int inst = w * NI + i, row = inst * 8 + (lane >> 3);
      d[i] = *(const u32x4*)(base + (int64_t)row * LD + (lane & 7) * 16);
    }
  };
  auto store = [&](int step, const u32x4 (&d)[NI]) {
    char* dst = lds + (step % STAGES) * STEP;
#pragma unroll
    for (int i = 0; i < NI; ++i) *(u32x4*)(dst + (w * NI + i) * 1024 + lane * 16) = d[i];
  };
  const int total = tiles * NSTEP;   // a multiple of RS (the loop body is RS steps, straight-line,
                                     // so the compiler's wait counts track each set exactly)
  auto clampv = [&](int s) { return s < total ? s : total - 1; };   // loads past the end re-read the last step
  {
    u32x4 t0[NI];
    load(0, t0); store(0, t0);
    load(1, t0); store(1, t0);
  }
#pragma unroll
  for (int j = 0; j < RS; ++j) load(clampv(2 + j), r[j]);
  BARRIER();
  for (int t = 0; t < total; t += RS) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      store(t + j + 2, r[j]);   // stores past the end land in stages no step reads
      load(clampv(t + j + 2 + RS), r[j]);
      BARRIER();
    }
  }
  if (threadIdx.x == 0 && lds[5] == 123) *sink = 1;
}

// v7's operand mix: rows 0..255 (A, the activations) fresh per tile as above, rows 256..383 (B,
// the weights) the same rows every tile (L2 hits).  MODE 0: every piece by LDS-DMA (v7 today);
// 1: every piece through registers (one set, lead 1); 2: A (8 pieces per wave) through
// registers, B (4 pieces) by LDS-DMA issued two steps ahead.
template <int MODE>
__global__ __launch_bounds__(256) void mix_k(const char* src, int tiles, int* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * STEP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NA = 8, NB = 4;
  const int b = blockIdx.x, blk0 = (b % 8) * 8 + (b / 8) / 4;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const char* wsrc = src + (int64_t)NBLK * ROWS * LD - (int64_t)1024 * LD;   // B: a fixed 128-row block
  auto addr = [&](int step, int i) -> const char* {   // piece i of this wave: i < NA A, else B
    const int tile = step / NSTEP, kof = (step % NSTEP) * 128;
    if (i < NA) {
      const int blk = (blk0 + 64 * tile) % NBLK;
      const int row = (w * NA + i) * 8 + (lane >> 3);
      return src + (int64_t)blk * ROWS * LD + (int64_t)row * LD + kof + (lane & 7) * 16;
    }
    const int row = (w * NB + (i - NA)) * 8 + (lane >> 3);
    return wsrc + (int64_t)row * LD + kof + (lane & 7) * 16;
  };
  auto dst = [&](int step, int i) {   // A pieces at [0, 32 KB), B pieces at [32, 48 KB) of the stage
    const int inst = i < NA ? w * NA + i : 32 + w * NB + (i - NA);
    return lds + (step % STAGES) * STEP + inst * 1024;
  };
  constexpr int R0 = MODE == 2 ? 0 : NA;   // pieces [R0, 12) of a step by DMA when MODE == 2
  constexpr int NR = MODE == 0 ? 0 : MODE == 1 ? NA + NB : NA;   // pieces [0, NR) through registers
  u32x4 r[NA + NB];
  auto dma = [&](int step) {
#pragma unroll
    for (int i = NR; i < NA + NB; ++i)
      __builtin_amdgcn_global_load_lds((gvoid_t*)addr(step, i), (lvoid_t*)dst(step, i), 16, 0, 0);
  };
  auto load = [&](int step) {
#pragma unroll
    for (int i = 0; i < NR; ++i) r[i] = *(const u32x4*)addr(step, i);
  };
  auto store = [&](int step) {
#pragma unroll
    for (int i = 0; i < NR; ++i) *(u32x4*)(dst(step, i) + lane * 16) = r[i];
  };
  const int total = tiles * NSTEP;
  (void)R0;
  if constexpr (MODE == 0) {
    dma(0); dma(1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    BARRIER();
    for (int t = 0; t < total; ++t) {
      if (t + 2 < total) { dma(t + 2); asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BARRIER();
    }
  } else {
    load(0); store(0);
    load(1); store(1);
    if constexpr (MODE == 2) { dma(0); dma(1); }
    load(2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BARRIER();
    // per iteration: store A(t+2) (its register loads are younger than the B copies of step t+1,
    // so waiting for them also lands B(t+1), which the next iteration reads), then B(t+2) by
    // DMA, then A(t+3) into the registers
    for (int t = 0; t < total; ++t) {
      if (t + 2 < total) {
        store(t + 2);
        if constexpr (MODE == 2) dma(t + 2);
        load(t + 3 < total ? t + 3 : total - 1);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      BARRIER();
    }
  }
  if (threadIdx.x == 0 && lds[5] == 123) *sink = 1;
}

// v7's K loop without its epilogue: 4 loader waves fill the ring by LDS-DMA as dma_k (step t + 2
// issued at step t), 8 reader waves read the stage of step t as v7's MFMA waves do (16
// ds_read_b128 per wave per step = 128 KB per step per CU) and, with MF, issue v7's 32
// v_mfma_f32_16x16x32_bf16 per wave per step on what they read; one barrier per step.  RD = 0:
// the loaders alone in a 768-thread work group.  Shows how much the fragment reads slow the fill.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
template <bool RD, bool MF, bool FRESH, bool BUF = false>
__global__ __launch_bounds__(768, 1) void con_k(const char* src, int tiles, int* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * STEP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NI = 12;
  const int b = blockIdx.x, blk0 = (b % 8) * 8 + (b / 8) / 4;
  const int total = tiles * NSTEP;
  if (w >= 8) {   // loaders
    const int lw = w - 8;
    // BUF: buffer_load ... lds (SGPR resource + 32-bit lane offset) instead of global_load_lds
    // (64-bit lane address)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
    auto issue = [&](int step) {
      const int tile = step / NSTEP;
      const int blk = FRESH ? (blk0 + 64 * tile) % NBLK : blk0;
      const int64_t boff = (int64_t)blk * ROWS * LD + (step % NSTEP) * 128;
      const char* base = src + boff;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int inst = lw * NI + i, row = inst * 8 + (lane >> 3);
        if (BUF)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid_t*)(lds + (step % STAGES) * STEP + inst * 1024), 16,
                                                   (unsigned)(boff + row * LD + (lane & 7) * 16), 0, 0, 0);
        else
          __builtin_amdgcn_global_load_lds((gvoid_t*)(base + (int64_t)row * LD + (lane & 7) * 16),
                                           (lvoid_t*)(lds + (step % STAGES) * STEP + inst * 1024), 16, 0, 0);
      }
    };
    issue(0);
    issue(1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    BARRIER();
    for (int t = 0; t < total; ++t) {
      if (t + 2 < total) { issue(t + 2); asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BARRIER();
    }
    return;
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  BARRIER();
  for (int t = 0; t < total; ++t) {
    if (RD) {
      const char* st = lds + (t % STAGES) * STEP;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = *(const bf16x8_t*)(st + (((w * 8 + kk * 4 + i) * 1024) % (32 * 1024)) + lane * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          fb[j] = *(const bf16x8_t*)(st + 32 * 1024 + (((w * 8 + kk * 4 + j) * 1024) % (16 * 1024)) + lane * 16);
        if (MF) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][0][0] += (float)fa[i][0] + (float)fb[i][1];
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    BARRIER();
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += acc[i][j][0];
  if (sum == 123.f) *sink = 1;
}

int main() {
  const int WG = 256, TILES = 64;
  const size_t bytes = (size_t)NBLK * ROWS * LD;   // 96 MB
  char* src;
  int* sink;
  CK(hipMalloc(&src, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern) {
    float best = 1e9;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(e0));
      kern<<<WG, 256>>>(src, TILES, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    const double b = (double)WG * TILES * NSTEP * STEP;
    printf("%-12s %8.1f us  %6.2f TB/s  %5.1f B/clk/CU  %6.0f cyc/step\n", name, best * 1e3,
           b / (best * 1e-3) / 1e12, b / (best * 1e-3) / WG / 2.4e9, best * 1e-3 * 2.4e9 / (TILES * NSTEP));
  };
  run("resident", dma_k<0, false>);
  run("fresh", dma_k<0, true>);
  run("fresh+P1", dma_k<1, true>);
  run("fresh+P2", dma_k<2, true>);
  run("fresh+P4", dma_k<4, true>);
  run("fresh+P6", dma_k<6, true>);
  run("resident+P2", dma_k<2, false>);
  auto run768 = [&](const char* name, auto kern) {
    float best = 1e9;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(e0));
      kern<<<WG, 768>>>(src, TILES, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    const double b = (double)WG * TILES * NSTEP * STEP;
    printf("%-12s %8.1f us  %6.2f TB/s  %5.1f B/clk/CU  %6.0f cyc/step\n", name, best * 1e3,
           b / (best * 1e-3) / 1e12, b / (best * 1e-3) / WG / 2.4e9, best * 1e-3 * 2.4e9 / (TILES * NSTEP));
  };
  run768("v7 loaders", con_k<false, false, true>);
  run768("+reads", con_k<true, false, true>);
  run768("+reads+mfma", con_k<true, true, true>);
  run768("res +r+mfma", con_k<true, true, false>);
  run768("buf loaders", con_k<false, false, true, true>);
  run768("buf +r+mfma", con_k<true, true, true, true>);
  run768("buf res+r+mf", con_k<true, true, false, true>);
  run("mix dma", mix_k<0>);
  run("mix reg", mix_k<1>);
  run("mix hyb", mix_k<2>);
  run("reg1 fresh", reg_k<1, true>);
  run("reg2 fresh", reg_k<2, true>);
  run("reg3 fresh", reg_k<3, true>);
  run("reg2 resid", reg_k<2, false>);
  run("reg3 resid", reg_k<3, false>);
  return 0;
}
