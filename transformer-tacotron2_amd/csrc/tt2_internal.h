// tt2_internal.h -- library-internal helpers (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime_api.h>

extern "C" {
int tt2_set_error(int code, const char* msg);
int tt2_check_launch(hipError_t err, const char* what);
}
// compute units of the current device (cached per device; 256 on an MI355X)
int tt2_cu_count();
// gemm.hip -- n zeroed arrival counters from the device's counter pool for one launch whose
// last-arriving workgroup resets each counter it completes; null when the pool cannot be
// allocated here (first use inside a stream capture): the caller takes its multi-launch path
int* tt2_fix_counters(int n, hipStream_t s);
