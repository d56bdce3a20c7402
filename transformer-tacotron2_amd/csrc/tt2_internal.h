// tt2_internal.h -- library-internal helpers (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime_api.h>

extern "C" {
int tt2_set_error(int code, const char* msg);
int tt2_check_launch(hipError_t err, const char* what);
}
// compute units of the current device (cached per device; 256 on an MI355X)
int tt2_cu_count();
