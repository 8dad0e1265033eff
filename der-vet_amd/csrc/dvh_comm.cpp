// dvh_comm.cpp -- the library's own RCCL communicator: the result all-gather of a sharded run.
//
// The reference solves its sensitivity cases one after the other (dervet/DERVET.py:75-83) and their windows one after
// the other (dervet/MicrogridScenario.py:310); here the windows of all cases are sharded over the GPUs of a node, one
// process per GPU, with no traffic during the solve, and ONE all-gather returns every window's result row to every
// rank.  That collective lives in the library (dvh_comm_init / dvh_gather_results), so a consumer without PyTorch can
// shard too; the launcher only has to carry the 128-byte unique id from rank 0 to the others.
//
// RCCL is opened at run time (dlopen of /opt/rocm/lib/librccl.so.1, or DVH_RCCL_LIB), not linked: a process that never
// forms a communicator does not load it, and a host without RCCL still loads the solver.  RTLD_DEEPBIND keeps the
// library's own symbols first when another RCCL is already in the process (PyTorch ships one): the two copies do not
// interpose on each other.  Both use the process's one HIP runtime, so the caller's streams are valid for either.
#include <dlfcn.h>
#include <stdlib.h>

#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/dervet_hip.h"
#include "dvh_internal.h"

namespace dvh {
namespace {

struct RcclApi {
  void* lib = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string err;  // why the library could not be opened (empty: opened)
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = getenv("DVH_RCCL_LIB");
    const char* cands[] = {env, "/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"};
    for (const char* c : cands) {
      if (!c || !*c) continue;
      api.lib = dlopen(c, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
      if (api.lib) break;
      api.err += std::string(c) + ": " + dlerror() + "; ";
    }
    if (!api.lib) {
      api.err = "RCCL could not be opened (" + api.err + "set DVH_RCCL_LIB)";
      return;
    }
    auto sym = [](void* lib, const char* name, auto& fn) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
      return fn != nullptr;
    };
    const bool ok = sym(api.lib, "ncclGetUniqueId", api.get_unique_id) &&
                    sym(api.lib, "ncclCommInitRank", api.comm_init_rank) &&
                    sym(api.lib, "ncclAllGather", api.all_gather) &&
                    sym(api.lib, "ncclCommDestroy", api.comm_destroy) &&
                    sym(api.lib, "ncclCommGetAsyncError", api.comm_async_error) &&
                    sym(api.lib, "ncclGetErrorString", api.error_string);
    if (!ok) {
      api.err = "RCCL library lacks the entry points the result gather needs";
      dlclose(api.lib);
      api.lib = nullptr;
    }
  });
  return api;
}

std::string rccl_msg(const RcclApi& a, const char* where, ncclResult_t r) {
  return std::string(where) + ": " + (a.error_string ? a.error_string(r) : "RCCL error") + " (" +
         std::to_string((int)r) + ")";
}

}  // namespace

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
};

int comm_unique_id(unsigned char* id, std::string* err) {
  static_assert(sizeof(ncclUniqueId) == kCommIdBytes, "unique id size");
  const RcclApi& a = rccl();
  if (!a.lib) {
    *err = a.err;
    return DVH_ERR_UNSUPPORTED;
  }
  ncclUniqueId u;
  const ncclResult_t r = a.get_unique_id(&u);
  if (r != ncclSuccess) {
    *err = rccl_msg(a, "ncclGetUniqueId", r);
    return DVH_ERR_HIP;
  }
  memcpy(id, &u, sizeof(u));
  return DVH_OK;
}

int comm_init(int device, int rank, int world, const unsigned char* id, Comm** out, std::string* err) {
  const RcclApi& a = rccl();
  if (!a.lib) {
    *err = a.err;
    return DVH_ERR_UNSUPPORTED;
  }
  if (hipSetDevice(device) != hipSuccess) {
    *err = "hipSetDevice failed before ncclCommInitRank";
    return DVH_ERR_HIP;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  Comm* c = new Comm;
  c->rank = rank;
  c->world = world;
  c->device = device;
  const ncclResult_t r = a.comm_init_rank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    *err = rccl_msg(a, "ncclCommInitRank", r);
    delete c;
    return DVH_ERR_HIP;
  }
  *out = c;
  return DVH_OK;
}

int comm_all_gather(Comm* c, const void* send, void* recv, size_t bytes, hipStream_t s, std::string* err) {
  const RcclApi& a = rccl();
  ncclResult_t async = ncclSuccess;
  if (a.comm_async_error(c->comm, &async) == ncclSuccess && async != ncclSuccess) {
    *err = rccl_msg(a, "communicator (asynchronous error)", async);
    return DVH_ERR_HIP;
  }
  const ncclResult_t r = a.all_gather(send, recv, bytes, ncclUint8, c->comm, s);
  if (r != ncclSuccess) {
    *err = rccl_msg(a, "ncclAllGather", r);
    return DVH_ERR_HIP;
  }
  return DVH_OK;
}

void comm_info(const Comm* c, int* rank, int* world) {
  *rank = c->rank;
  *world = c->world;
}

void comm_destroy(Comm* c) {
  if (!c) return;
  const RcclApi& a = rccl();
  if (a.lib && c->comm) a.comm_destroy(c->comm);
  delete c;
}

}  // namespace dvh
