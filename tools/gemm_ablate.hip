// Standalone GEMM ablation harness (dev tool): builds gemm.hip with one of the
// TT2_ABL_* switches and times the bf16 kernel (variant TT2_V, default v2) on the step's
// key shapes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I transformer-tacotron2_amd/csrc \
//     -DTT2_ABL_NO_EPI tools/gemm_ablate.hip -o /tmp/abl_noepi
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../transformer-tacotron2_amd/csrc/gemm.hip"
#include "../transformer-tacotron2_amd/csrc/runtime.cpp"

int main() {
  struct S { const char* name; int m, n, k, ta, tb; };
  std::vector<S> shapes = {{"ffn1 fwd", 12800, 2048, 512, 0, 0}, {"ffn2 fwd", 12800, 512, 2048, 0, 0},
                           {"o fwd", 12800, 512, 512, 0, 0}, {"ffn2 dgrad", 12800, 2048, 512, 0, 1},
                           {"sq 4096", 4096, 4096, 4096, 0, 0}};
  if (getenv("TT2_ENC"))   // the encoder's 2048-row shapes
    shapes = {{"enc o", 2048, 512, 512, 0, 0},      {"enc qkv", 2048, 1536, 512, 0, 0},
              {"enc ffn1", 2048, 2048, 512, 0, 0},  {"enc ffn2", 2048, 512, 2048, 0, 0},
              {"enc o dg", 2048, 512, 512, 0, 1},   {"enc ffn1 dg", 2048, 512, 2048, 0, 1},
              {"enc conv", 2048, 512, 2560, 0, 0}};
  const int splits = getenv("TT2_SPLITS") ? atoi(getenv("TT2_SPLITS")) : 1;
  void* ws = nullptr;
  hipMalloc(&ws, 256u << 20);
  for (auto& s : shapes) {
    size_t na = (size_t)s.m * s.k, nb = (size_t)s.n * s.k, nc = (size_t)s.m * s.n;
    void *A, *B, *Cm;
    hipMalloc(&A, na * 2); hipMalloc(&B, nb * 2); hipMalloc(&Cm, nc * 2);
    hipMemset(A, 0x3c, na * 2); hipMemset(B, 0x3c, nb * 2);
    tt2_gemm_args g{};
    g.a = A; g.b = B; g.c = Cm; g.m = s.m; g.n = s.n; g.k = s.k;
    g.lda = s.ta ? s.m : s.k; g.ldb = s.tb ? s.n : s.k; g.ldc = s.n;
    g.trans_a = s.ta; g.trans_b = s.tb; g.dtype_in = 1; g.dtype_out = 1; g.alpha = 1.f; g.gate_scale = 1.f;
    g.splits = splits; g.workspace = ws; g.ws_bytes = 256u << 20; g.kernel_variant = getenv("TT2_V") ? atoi(getenv("TT2_V")) : 2;
    for (int i = 0; i < 3; ++i) tt2_gemm(&g, 0);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int it = 20;
    hipEventRecord(e0, 0);
    for (int i = 0; i < it; ++i) tt2_gemm(&g, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / it;
    printf("%-12s %6dx%5dx%5d: %8.1f us %7.1f TF\n", s.name, s.m, s.n, s.k, us, 2.0 * s.m * s.n * s.k / us / 1e6);
    hipFree(A); hipFree(B); hipFree(Cm);
  }
  return 0;
}
