// Gradient all-reduce over RCCL for the data-parallel PPO update (SURVEY §8(b) lgx_allreduce_grads;
// the multi-GPU gradient average of the rsl_rl update, §8(e)): one communicator per rank, the
// all-reduce issued directly on the caller's stream, so the update's own streams order it -- no
// collective-side stream and no event handshake per call.
//
// RCCL is resolved at run time from the library the caller names (the process's own RCCL, e.g.
// the one torch.distributed already loaded), so one RCCL instance serves both communicators and
// liblgx.so carries no link-time dependency on it.  A loaded RCCL is never unloaded again (its
// bootstrap and proxy threads live in it).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>

#include "lgx_internal.h"

namespace {

struct RcclApi {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

int rccl_open(const char* path, RcclApi& api) {
  void* h = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return lgx_fail(LGX_EINVAL, "lgx_comm: RCCL library not loadable");
  api.handle = h;
  api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(dlsym(h, "ncclAllReduce"));
  api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
  if (!api.get_unique_id || !api.comm_init_rank || !api.comm_destroy || !api.all_reduce || !api.error_string) {
    dlclose(h);
    api = RcclApi{};
    return lgx_fail(LGX_EINVAL, "lgx_comm: RCCL entry points missing from the library");
  }
  return 0;
}

int rccl_status(const RcclApi& api, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, api.error_string(r));
  return lgx_fail(LGX_EHIP, buf);
}

}  // namespace

struct lgx_comm {
  RcclApi api;
  ncclComm_t comm;
  int32_t nranks, rank, device;
};

extern "C" {

int lgx_comm_unique_id(const char* rccl_path, uint8_t id[LGX_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == LGX_COMM_ID_BYTES, "RCCL unique id size");
  if (!id) return lgx_fail(LGX_EINVAL, "lgx_comm_unique_id: null id");
  RcclApi api;
  int rc = rccl_open(rccl_path, api);
  if (rc) return rc;
  ncclUniqueId u;
  rc = rccl_status(api, api.get_unique_id(&u), "ncclGetUniqueId");
  if (!rc) memcpy(id, &u, sizeof u);
  // the library stays loaded (never dlclose'd once used): the unique id's bootstrap root thread
  // runs inside it until the ranks have connected in lgx_comm_create
  return rc;
}

int lgx_comm_create(const char* rccl_path, const uint8_t id[LGX_COMM_ID_BYTES], int32_t nranks, int32_t rank,
                    int32_t device, lgx_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
    return lgx_fail(LGX_EINVAL, "lgx_comm_create: bad arguments");
  *out = nullptr;
  lgx_comm* c = new (std::nothrow) lgx_comm();
  if (!c) return lgx_fail(LGX_ENOMEM, "lgx_comm_create: out of host memory");
  int rc = rccl_open(rccl_path, c->api);
  if (rc) { delete c; return rc; }
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return lgx_fail(LGX_EHIP, "lgx_comm_create: hipSetDevice failed");
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  rc = rccl_status(c->api, c->api.comm_init_rank(&c->comm, nranks, u, rank), "ncclCommInitRank");
  if (rc) { delete c; return rc; }
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return 0;
}

int lgx_comm_destroy(lgx_comm* c) {
  if (!c) return 0;
  const int rc = rccl_status(c->api, c->api.comm_destroy(c->comm), "ncclCommDestroy");
  delete c;
  return rc;
}

int lgx_allreduce_grads(lgx_comm* c, float* buf, size_t count, int32_t op, void* stream) {
  if (!c || (!buf && count) || (op != LGX_REDUCE_SUM && op != LGX_REDUCE_AVG))
    return lgx_fail(LGX_EINVAL, "lgx_allreduce_grads: bad arguments");
  if (!count) return 0;
  return rccl_status(c->api,
                     c->api.all_reduce(buf, buf, count, ncclFloat32, op == LGX_REDUCE_SUM ? ncclSum : ncclAvg,
                                       c->comm, static_cast<hipStream_t>(stream)),
                     "ncclAllReduce");
}

}  // extern "C"
