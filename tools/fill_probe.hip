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
  __syncthreads();
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
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && (lds[5] == 123 || junk[3] == 99)) *sink = 1;
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
  return 0;
}
