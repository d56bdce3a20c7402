// In-kernel timeline of the v7 GEMM (dev tool): builds gemm.hip with its stamp hooks defined, runs a
// shape, and prints the average per-K-step split (s_memtime cycles, wave 0 of every
// workgroup): wait = vmcnt + barrier, issue = LDS-DMA issue, comp = fragment reads +
// MFMA issue, plus the epilogue and the spread of workgroup start times.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I transformer-tacotron2_amd/csrc \
//     tools/gemm_stamps.hip -o tools/bin/gemm_stamps
//   tools/bin/gemm_stamps m n k ta tb variant splits
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

// the stamp hooks gemm.hip leaves empty in the library build (wave 0 of every workgroup)
__device__ unsigned long long g_st[4096 * 64 * 4];
#define G7_STAMP(t, slot)                                                                            \
  if (threadIdx.x == 0 && (t) < 64)                                                                  \
    g_st[((size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 64 + (t)) * 4 + (slot)] = __builtin_amdgcn_s_memtime();
#define G7_RT(slot)                                                                                  \
  if (threadIdx.x == 0) g_st[(size_t)blockIdx.x * 64 * 4 + 63 * 4 + (slot)] = __builtin_amdgcn_s_memrealtime();
#include "../transformer-tacotron2_amd/csrc/gemm.hip"
#include "../transformer-tacotron2_amd/csrc/runtime.cpp"
// gemm.hip's grouped launch sizes a LayerNorm finalize with this (norm.hip); unused here
extern "C" size_t tt2_layernorm_bwd_workspace_size(const tt2_ln_args*) { return 0; }

int main(int argc, char** argv) {
  if (argc < 8) { fprintf(stderr, "usage: m n k ta tb variant splits\n"); return 2; }
  const int m = atoi(argv[1]), n = atoi(argv[2]), k = atoi(argv[3]), ta = atoi(argv[4]), tb = atoi(argv[5]);
  const int var = atoi(argv[6]), sp = atoi(argv[7]);
  const size_t na = (size_t)m * k, nb = (size_t)n * k, nc = (size_t)m * n;
  void *A, *B, *Cm, *W = nullptr;
  hipMalloc(&A, na * 2); hipMalloc(&B, nb * 2); hipMalloc(&Cm, nc * 4);
  hipMemset(A, 0x3c, na * 2); hipMemset(B, 0x3c, nb * 2);
  tt2_gemm_args g{};
  g.a = A; g.b = B; g.c = Cm; g.m = m; g.n = n; g.k = k;
  g.lda = ta ? m : k; g.ldb = tb ? n : k; g.ldc = n;
  g.trans_a = ta; g.trans_b = tb; g.dtype_in = TT2_BF16; g.dtype_out = ta ? TT2_F32 : TT2_BF16;
  g.alpha = 1.f; g.gate_scale = 1.f; g.splits = sp; g.kernel_variant = var; g.main_only = 1;
  if (sp > 1) { g.ws_bytes = tt2_gemm_workspace_size(&g); hipMalloc(&W, g.ws_bytes); g.workspace = W; }
  if (getenv("TT2_BIAS")) {   // the forward linears' epilogue (bias prefetched before the K loop)
    float* bias = nullptr;
    hipMalloc(&bias, (size_t)n * 4);
    hipMemset(bias, 0, (size_t)n * 4);
    g.bias = bias;
  }
  for (int i = 0; i < 5; ++i)
    if (tt2_gemm(&g, 0) != TT2_OK) { fprintf(stderr, "gemm: %s\n", tt2_last_error()); return 1; }
  hipDeviceSynchronize();
  std::vector<unsigned long long> st(4096 * 64 * 4);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_st), st.size() * 8);
  const int bm = (var >= 11 && var <= 14) ? 256 : 128, bn = var == 11 ? 256 : 128;  // v7 (13/14): 256 x 128
  int k_split = k, splits = 1;
  if (sp > 1) { k_split = ((k + sp - 1) / sp + 63) / 64 * 64; splits = (k + k_split - 1) / k_split; }
  const int nwg = ((m + bm - 1) / bm) * ((n + bn - 1) / bn) * splits;
  const int nkt = (k_split + 63) / 64;
  double w = 0, is = 0, c = 0, epi = 0, tot = 0, e_img = 0, e_bar = 0, e_st = 0; unsigned long long t0min = ~0ull, t0max = 0, tend = 0;
  int cnt = 0;
  for (int b = 0; b < nwg && b < 4096; ++b) {
    const unsigned long long* s = &st[(size_t)b * 64 * 4];
    const int steps = std::min(nkt, 63);
    for (int t = 0; t < steps; ++t) {
      const unsigned long long* r = s + t * 4;
      const unsigned long long next = s[(t + 1) * 4];
      if (var == 13 || var == 14) {   // v7 MFMA wave 0: [0] step start, [1] after the step's MFMAs
        c += (double)(r[1] - r[0]); w += (double)(next - r[1]);
      } else {
        w += (double)(r[1] - r[0]); is += (double)(r[2] - r[1]); c += (double)(next - r[2]);
      }
      ++cnt;
    }
    epi += (double)(s[steps * 4 + 3] - s[steps * 4]);
    e_img += (double)(s[steps * 4 + 1] - s[steps * 4]);
    e_bar += (double)(s[steps * 4 + 2] - s[steps * 4 + 1]);
    e_st += (double)(s[steps * 4 + 3] - s[steps * 4 + 2]);
    tot += (double)(s[steps * 4 + 3] - s[0]);
    t0min = std::min(t0min, s[0]); t0max = std::max(t0max, s[0]); tend = std::max(tend, s[steps * 4 + 3]);
  }
  // chip-wide timeline (s_memrealtime, 100 MHz) and one launch's event time
  unsigned long long rs = ~0ull, rs_max = 0, re_max = 0;
  for (int b = 0; b < nwg && b < 4096; ++b) {
    const unsigned long long* s = &st[(size_t)b * 64 * 4 + 63 * 4];
    rs = std::min(rs, s[0]); rs_max = std::max(rs_max, s[0]); re_max = std::max(re_max, s[1]);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 20; ++i) tt2_gemm(&g, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  printf("  realtime: WG start spread %.2f us, first start -> last exit %.2f us; back-to-back launch %.2f us\n",
         (rs_max - rs) / 100.0, (re_max - rs) / 100.0, ms * 1e3 / 20);
  printf("%dx%dx%d ta%d tb%d v%d sp%d: %d WGs x %d steps | per step: wait %.0f issue %.0f comp %.0f cyc | "
         "epilogue %.0f | WG total %.0f | start spread %llu | span %llu cyc\n",
         m, n, k, ta, tb, var, sp, nwg, nkt, w / cnt, is / cnt, c / cnt, epi / nwg, tot / nwg, t0max - t0min,
         tend - t0min);
  printf("  epilogue (LDS-image form): image write %.0f, barrier %.0f, stores %.0f cyc\n", e_img / nwg, e_bar / nwg,
         e_st / nwg);
  return 0;
}
