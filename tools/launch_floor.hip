// Launch-floor microbenchmark (dev tool): per-kernel cost of a hipGraph-replayed chain of
// small dependent kernels, by what each kernel does.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/lf && /tmp/lf
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

struct Big { float pad[120]; const float* a; float* b; };

__global__ void k_empty() {}
__global__ void k_copy(const float* a, float* b) { int i = blockIdx.x * blockDim.x + threadIdx.x; b[i] = a[i] + 1.f; }
__global__ void k_dep(const int* t, const float* a, float* b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; int tt = *t; b[i] = a[i + (tt & 1)] + 1.f; }
__global__ void k_dep3(const int* t, const float* a, float* b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; int tt = *t; float x = a[i + (tt & 1)];
  float y = a[(i + (int)x) & 0xffff]; b[i] = y + 1.f; }
__global__ void k_big(Big p) { int i = blockIdx.x * blockDim.x + threadIdx.x; p.b[i] = p.a[i] + p.pad[threadIdx.x & 63]; }

int main() {
  float *a, *b; int* t;
  CK(hipMalloc(&a, 1 << 24)); CK(hipMalloc(&b, 1 << 24)); CK(hipMalloc(&t, 64));
  CK(hipMemset(a, 0, 1 << 24)); CK(hipMemset(t, 0, 64));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int NK = 100;
  const char* names[] = {"empty", "copy", "dep2", "dep3", "bigarg"};
  for (int grid : {32, 256, 1024}) {
    for (int kind = 0; kind < 5; ++kind) {
      Big bp{}; bp.a = a; bp.b = b;
      auto launch = [&](hipStream_t st) {
        for (int i = 0; i < NK; ++i) {
          float* src = (i & 1) ? b : a; float* dst = (i & 1) ? a : b;
          switch (kind) {
            case 0: hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st); break;
            case 1: hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, st, src, dst); break;
            case 2: hipLaunchKernelGGL(k_dep, dim3(grid), dim3(256), 0, st, t, src, dst); break;
            case 3: hipLaunchKernelGGL(k_dep3, dim3(grid), dim3(256), 0, st, t, src, dst); break;
            case 4: bp.a = src; bp.b = dst; hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, st, bp); break;
          }
        }
      };
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      launch(s);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      const int R = 20;
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      // eager
      launch(s); CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < R; ++r) launch(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms2; CK(hipEventElapsedTime(&ms2, e0, e1));
      printf("grid %5d %-7s graph %6.2f us/kernel   eager %6.2f us/kernel\n", grid, names[kind],
             ms * 1e3 / (R * NK), ms2 * 1e3 / (R * NK));
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
