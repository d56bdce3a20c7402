// runtime.cpp -- libtt2 runtime: error reporting and device init.
#include <hip/hip_runtime.h>
#include <mutex>
#include <string>
#include <unordered_set>
#include <vector>

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

// ------------------------------------------------------------ capture hygiene
// Which of `streams` still holds captured work that the origin stream does not depend on.
// A stream forked into a capture (it waited on an event of a capturing stream) must be joined
// back (the origin waits on an event recorded after its last captured work) before the origin
// ends the capture; this reads both streams' current capture dependencies and walks the
// captured graph backwards from the origin's, so a missing join is reported by name instead of
// surfacing inside hipStreamEndCapture.
extern "C" int tt2_capture_joined(hipStream_t origin, const hipStream_t* streams, int32_t n, int32_t* status) {
  if (n < 0 || (n > 0 && (!streams || !status))) return tt2_set_error(TT2_E_INVALID, "tt2_capture_joined: args");
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(origin, &st, &id, &graph, &deps, &nd);
  if (e != hipSuccess) return tt2_check_launch(e, "tt2_capture_joined: origin capture info");
  if (st != hipStreamCaptureStatusActive)
    return tt2_set_error(TT2_E_INVALID, "tt2_capture_joined: the origin stream is not capturing");
  // every node the origin's next captured operation would (transitively) depend on
  std::unordered_set<hipGraphNode_t> anc;
  std::vector<hipGraphNode_t> todo(deps, deps + nd);
  std::vector<hipGraphNode_t> buf;
  while (!todo.empty()) {
    hipGraphNode_t x = todo.back();
    todo.pop_back();
    if (!x || !anc.insert(x).second) continue;
    size_t k = 0;
    if ((e = hipGraphNodeGetDependencies(x, nullptr, &k)) != hipSuccess)
      return tt2_check_launch(e, "tt2_capture_joined: node dependencies");
    if (!k) continue;
    buf.assign(k, nullptr);
    if ((e = hipGraphNodeGetDependencies(x, buf.data(), &k)) != hipSuccess)
      return tt2_check_launch(e, "tt2_capture_joined: node dependencies");
    todo.insert(todo.end(), buf.begin(), buf.begin() + k);
  }
  for (int32_t i = 0; i < n; ++i) {
    hipStreamCaptureStatus si = hipStreamCaptureStatusNone;
    unsigned long long sid = 0;
    const hipGraphNode_t* sd = nullptr;
    size_t sn = 0;
    if ((e = hipStreamGetCaptureInfo_v2(streams[i], &si, &sid, nullptr, &sd, &sn)) != hipSuccess)
      return tt2_check_launch(e, "tt2_capture_joined: stream capture info");
    if (si != hipStreamCaptureStatusActive || sid != id) {
      status[i] = si == hipStreamCaptureStatusInvalidated ? 3 : 0;   // 0: not in this capture
      continue;
    }
    int32_t v = 1;   // joined: every pending dependency of the stream is an origin ancestor
    for (size_t j = 0; j < sn; ++j)
      if (sd[j] && !anc.count(sd[j])) v = 2;
    status[i] = v;
  }
  return TT2_OK;
}
