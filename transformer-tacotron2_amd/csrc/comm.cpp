// comm.cpp -- the data-parallel gradient bucket of the C ABI: an in-place
// RCCL SUM all-reduce on the caller's stream, plus communicator helpers for hosts that
// do not run torch.distributed.  librccl is bound at the first call with dlopen, so
// libtt2 has no link-time RCCL dependency and shares the process's already-loaded
// librccl (torch's) when there is one.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "tt2_capi.h"
#include "tt2_internal.h"

namespace {

struct Rccl {
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetUniqueId) unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  std::string why;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
      const char* e = dlerror();
      r.why = e ? e : "dlopen(librccl) failed";
      return;
    }
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.unique_id = reinterpret_cast<decltype(r.unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
    r.err = reinterpret_cast<decltype(r.err)>(dlsym(h, "ncclGetErrorString"));
    if (!r.all_reduce || !r.unique_id || !r.init_rank || !r.destroy || !r.err) {
      r.why = "librccl lacks an nccl* entry point";
      r.all_reduce = nullptr;
    }
  });
  return r;
}

int fail(const Rccl& r, ncclResult_t res, const char* what) {
  std::string m = std::string(what) + ": " + (r.err ? r.err(res) : "rccl error");
  return tt2_set_error(TT2_E_HIP, m.c_str());
}

int ready(const Rccl& r) {
  if (r.all_reduce) return TT2_OK;
  const std::string m = "tt2 comm: RCCL unavailable (" + r.why + ")";
  return tt2_set_error(TT2_E_INVALID, m.c_str());
}

}  // namespace

extern "C" int tt2_allreduce_bucket(void* buf, size_t n, int32_t dtype, void* comm, hipStream_t stream) {
  if (n == 0) return TT2_OK;
  if (!buf || !comm) return tt2_set_error(TT2_E_INVALID, "tt2_allreduce_bucket: null buffer or communicator");
  ncclDataType_t t;
  if (dtype == TT2_DT_F32) t = ncclFloat32;
  else if (dtype == TT2_DT_BF16) t = ncclBfloat16;
  else if (dtype == TT2_DT_F16) t = ncclFloat16;
  else return tt2_set_error(TT2_E_INVALID, "tt2_allreduce_bucket: dtype");
  const Rccl& r = rccl();
  if (const int rc = ready(r); rc != TT2_OK) return rc;
  const ncclResult_t res = r.all_reduce(buf, buf, n, t, ncclSum, reinterpret_cast<ncclComm_t>(comm), stream);
  return res == ncclSuccess ? TT2_OK : fail(r, res, "tt2_allreduce_bucket");
}

extern "C" int tt2_comm_unique_id(void* id_out) {
  if (!id_out) return tt2_set_error(TT2_E_INVALID, "tt2_comm_unique_id: null");
  const Rccl& r = rccl();
  if (const int rc = ready(r); rc != TT2_OK) return rc;
  ncclUniqueId id;
  const ncclResult_t res = r.unique_id(&id);
  if (res != ncclSuccess) return fail(r, res, "tt2_comm_unique_id");
  std::memcpy(id_out, &id, sizeof(id));
  return TT2_OK;
}

extern "C" int tt2_comm_init(void** comm_out, int32_t nranks, const void* id, int32_t rank) {
  if (!comm_out || !id || nranks <= 0 || rank < 0 || rank >= nranks)
    return tt2_set_error(TT2_E_INVALID, "tt2_comm_init: arguments");
  const Rccl& r = rccl();
  if (const int rc = ready(r); rc != TT2_OK) return rc;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ncclResult_t res = r.init_rank(&c, nranks, uid, rank);
  if (res != ncclSuccess) return fail(r, res, "tt2_comm_init");
  *comm_out = c;
  return TT2_OK;
}

extern "C" int tt2_comm_destroy(void* comm) {
  if (!comm) return TT2_OK;
  const Rccl& r = rccl();
  if (const int rc = ready(r); rc != TT2_OK) return rc;
  const ncclResult_t res = r.destroy(reinterpret_cast<ncclComm_t>(comm));
  return res == ncclSuccess ? TT2_OK : fail(r, res, "tt2_comm_destroy");
}
