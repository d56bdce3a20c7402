// runtime.cpp -- libtt2 runtime: error reporting and device init.
#include <hip/hip_runtime.h>
#include <mutex>
#include <string>

#include "tt2_capi.h"
#include "tt2_internal.h"

namespace {
thread_local std::string g_err;
std::once_flag g_once;
int g_init_status = TT2_OK;
}  // namespace

extern "C" const char* tt2_last_error(void) { return g_err.c_str(); }

extern "C" int tt2_version(void) { return 1; }

extern "C" int tt2_set_error(int code, const char* msg) {
  g_err = msg ? msg : "";
  return code;
}

extern "C" int tt2_check_launch(hipError_t err, const char* what) {
  if (err == hipSuccess) return TT2_OK;
  g_err = std::string(what) + ": " + hipGetErrorString(err);
  return TT2_E_LAUNCH;
}

int tt2_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    cache[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return cache[dev];
}

extern "C" int tt2_init(int device) {
  std::call_once(g_once, [&] {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
      g_init_status = tt2_set_error(TT2_E_HIP, hipGetErrorString(e));
      return;
    }
    std::string arch = prop.gcnArchName;
    if (arch.rfind("gfx950", 0) != 0) {
      g_init_status = tt2_set_error(TT2_E_HIP, ("libtt2 is built for gfx950 only, device is " + arch).c_str());
    }
  });
  return g_init_status;
}
