// In-kernel timeline of the v3 attention forward (dev tool): builds attention.hip with its
// stamp hooks defined (s_memtime per wave), runs the decoder's causal self-attention shape
// (B = 16, H = 8, 800 x 800, d 64) and prints, per query block, the average per-tile split of
// its waves: S + row max, softmax + PV issue, next-tile LDS write (its loads' wait), barrier.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I transformer-tacotron2_amd/csrc \
//     tools/attn_stamps.hip -o tools/bin/attn_stamps
#include <cstdio>
#include <cstdlib>
#include <vector>

// [query block y < 8][batch * head x < 256][wave < 4][slot < 64]
constexpr size_t ST_N = (size_t)8 * 256 * 4 * 64;
__device__ unsigned long long g_st[ST_N];
#define ATTN_STAMP(slot)                                                                              \
  if ((threadIdx.x & 63) == 0 && (slot) < 64 && blockIdx.x < 256 && blockIdx.y < 8 && (threadIdx.x >> 6) < 4) \
    g_st[(((size_t)blockIdx.y * 256 + blockIdx.x) * 4 + (threadIdx.x >> 6)) * 64 + (slot)] = __builtin_amdgcn_s_memtime();
#include "../transformer-tacotron2_amd/csrc/attention.hip"
#include "../transformer-tacotron2_amd/csrc/runtime.cpp"

int main(int argc, char** argv) {
  const int B = 16, H = 8, T = argc > 1 ? atoi(argv[1]) : 800, causal = argc > 2 ? atoi(argv[2]) : 1;
  const int d = 512;
  void *qkv, *out;
  float* lse;
  hipMalloc(&qkv, (size_t)B * T * 3 * d * 2);
  hipMalloc(&out, (size_t)B * T * d * 2);
  hipMalloc(&lse, (size_t)B * H * T * 4);
  std::vector<unsigned short> h((size_t)B * T * 3 * d);
  unsigned x = 1;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = 0x3c00 + ((x >> 16) & 0xff) - 0x80; }   // bf16 ~[0.5, 1.5)
  hipMemcpy(qkv, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  tt2_attn_args a{};
  a.q = qkv; a.k = (char*)qkv + d * 2; a.v = (char*)qkv + 2 * d * 2; a.o_out = out; a.lse = lse;
  a.q_ld = a.k_ld = a.v_ld = 3 * d; a.o_ld = d;
  a.batch = B; a.heads = H; a.head_dim = 64; a.tq = T; a.tk = T; a.causal = causal; a.dtype = TT2_DT_BF16;
  a.scale = 0.125f;
  if ((T + 127) / 128 > 8 || B * H > 256) { fprintf(stderr, "shape exceeds the stamp buffer\n"); return 2; }
  for (int i = 0; i < 5; ++i)
    if (tt2_attn_fwd(&a, 0) != TT2_OK) { fprintf(stderr, "attn: %s\n", tt2_last_error()); return 1; }
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 20; ++i) tt2_attn_fwd(&a, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(ST_N);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_st), st.size() * 8);
  const int nqb = (T + 127) / 128;
  printf("T %d causal %d: %.1f us per launch\n", T, causal, ms * 1e3 / 20);
  printf("qblk tiles | prologue | per tile: S+max  softmax+PV  ldswrite  barrier | total (cycles, wave avg over %d heads)\n", 128);
  for (int y = 0; y < nqb; ++y) {
    const int qblk = causal ? nqb - 1 - y : y;
    const int kend = causal ? std::min(T, qblk * 128 + 128) : T;
    const int nt = (kend + 63) / 64;
    double pro = 0, ph[4] = {0, 0, 0, 0}, tot = 0;
    int cnt = 0;
    for (int bx = 0; bx < 128; ++bx)
      for (int w = 0; w < 4; ++w) {
        const unsigned long long* s = &st[(((size_t)y * 256 + bx) * 4 + w) * 64];
        if (qblk * 128 + 32 * w >= T) continue;
        pro += (double)(s[1] - s[0]);
        unsigned long long prev = s[1];
        bool ok = true;
        for (int t = 0; t < nt && 5 + 4 * t < 64; ++t) {
          const bool vis = !(causal && 64 * t > qblk * 128 + 32 * w + 31);
          if (!vis) { prev = s[5 + 4 * t]; continue; }
          ph[0] += (double)(s[2 + 4 * t] - prev);
          ph[1] += (double)(s[3 + 4 * t] - s[2 + 4 * t]);
          ph[2] += (double)(s[4 + 4 * t] - s[3 + 4 * t]);
          ph[3] += (double)(s[5 + 4 * t] - s[4 + 4 * t]);
          prev = s[5 + 4 * t];
        }
        tot += (double)(prev - s[0]);
        ++cnt;
        (void)ok;
      }
    if (!cnt) continue;
    printf("%4d %5d | %8.0f | %8.0f %10.0f %9.0f %8.0f | %8.0f\n", qblk, nt, pro / cnt, ph[0] / cnt / nt, ph[1] / cnt / nt,
           ph[2] / cnt / nt, ph[3] / cnt / nt, tot / cnt);
  }
  return 0;
}
