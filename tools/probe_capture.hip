// Diagnostic (GPU): which ways of timing a kernel node inside a captured hipGraph work on this
// runtime.  Prints the HIP status of each attempt and the replayed intervals.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(float* p, int n) {
  float v = p[threadIdx.x];
  for (int i = 0; i < n; ++i) v = v * 1.0000001f + 1e-7f;
  p[threadIdx.x] = v;
}

#define S(x) do { hipError_t e_ = (x); printf("%-60s -> %s\n", #x, hipGetErrorString(e_)); } while (0)

int main() {
  float* d;
  hipMalloc(&d, 4096);
  hipMemset(d, 0, 4096);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (unsigned flags : {(unsigned)hipEventDefault, (unsigned)hipEventDisableSystemFence}) {
    for (int mode : {0, 1}) {
      printf("== event flags %x, capture mode %s\n", flags, mode ? "thread-local" : "global");
      hipEvent_t a, b;
      S(hipEventCreateWithFlags(&a, flags));
      S(hipEventCreateWithFlags(&b, flags));
      hipGraph_t g = nullptr;
      S(hipStreamBeginCapture(s, mode ? hipStreamCaptureModeThreadLocal : hipStreamCaptureModeGlobal));
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, d, 100);
      S(hipEventRecordWithFlags(a, s, hipEventRecordExternal));
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, d, 200000);
      S(hipGetLastError());
      S(hipEventRecordWithFlags(b, s, hipEventRecordExternal));
      S(hipStreamEndCapture(s, &g));
      hipGraphExec_t x = nullptr;
      S(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
      for (int r = 0; r < 3 && x; ++r) {
        S(hipGraphLaunch(x, s));
        S(hipStreamSynchronize(s));
        float ms = -1;
        S(hipEventElapsedTime(&ms, a, b));
        printf("   replay %d: %.4f ms\n", r, ms);
      }
      // eager reference
      hipEventRecord(a, s);
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, d, 200000);
      hipEventRecord(b, s);
      hipStreamSynchronize(s);
      float ms = -1;
      hipEventElapsedTime(&ms, a, b);
      printf("   eager: %.4f ms\n", ms);
      if (x) hipGraphExecDestroy(x);
      if (g) hipGraphDestroy(g);
    }
  }
  return 0;
}
