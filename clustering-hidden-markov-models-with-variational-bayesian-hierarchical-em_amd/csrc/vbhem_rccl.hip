// vbhem_rccl.hip -- include/vbhem_dist.h: the SUM all-reduce of the packed
// K-cluster statistics over RCCL (vbhem_compute_Statistics.m:44-50 summed across
// the G shards of the base HMMs), host C++.
//
// RCCL is bound at run time with dlopen/dlsym: a process that already holds an
// RCCL (PyTorch's bundled librccl.so, which its ProcessGroupNCCL uses) shares that
// instance -- one RCCL and one HIP runtime in the process -- and a process without
// one (a MATLAB host) loads librccl.so.1 from the ROCm install.  Only the types
// come from rccl.h.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "vbhem_dist.h"
#include "vbhem_estep.h"
#include "vbhem_internal.h"

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
  std::string where;
  bool ok = false;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // the instance already mapped into the process first, then the ROCm install
    const char *names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
    void *h = nullptr;
    for (const char *n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD)) != nullptr) {
        r.where = std::string(n) + " (already loaded)";
        break;
      }
    for (int x = 1; !h && x < 3; ++x)
      if ((h = dlopen(names[x], RTLD_NOW | RTLD_LOCAL)) != nullptr) r.where = names[x];
    if (!h) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce;
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char *what) {
  const Rccl &r = rccl();
  return vbhem::set_error(VBHEM_ERR_HIP, std::string(what) + ": " +
                                             (r.error_string ? r.error_string(e) : "RCCL error"));
}

int need_rccl() {
  if (rccl().ok) return VBHEM_OK;
  return vbhem::set_error(VBHEM_ERR_UNSUPPORTED, "RCCL (librccl.so) could not be loaded");
}

}  // namespace

namespace {
// the reduced statistics into their destination (mapped pinned host memory): a
// grid-stride copy, vector stores
__global__ __launch_bounds__(256) void stats_copy_kernel(double *dst, const double *src, size_t n) {
  for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < n; x += (size_t)gridDim.x * blockDim.x)
    dst[x] = src[x];
}
}  // namespace

extern "C" {

int vbhem_rccl_available(void) { return need_rccl(); }

int vbhem_rccl_unique_id(void *id) {
  if (!id) return vbhem::set_error(VBHEM_ERR_ARG, "vbhem_rccl_unique_id: null id");
  if (int rc = need_rccl()) return rc;
  ncclUniqueId u;
  const ncclResult_t e = rccl().get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(e, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return VBHEM_OK;
}

int vbhem_rccl_comm_init(int nranks, int rank, const void *id, int device, void **comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
    return vbhem::set_error(VBHEM_ERR_ARG, "vbhem_rccl_comm_init: bad arguments");
  if (int rc = need_rccl()) return rc;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return vbhem::set_error(VBHEM_ERR_HIP, "vbhem_rccl_comm_init: hipSetDevice failed");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t e = rccl().comm_init_rank(&c, nranks, u, rank);
  (void)hipSetDevice(prev);
  if (e != ncclSuccess) return rccl_fail(e, "ncclCommInitRank");
  *comm = c;
  return VBHEM_OK;
}

int vbhem_rccl_comm_destroy(void *comm) {
  if (!comm) return VBHEM_OK;
  if (int rc = need_rccl()) return rc;
  const ncclResult_t e = rccl().comm_destroy(static_cast<ncclComm_t>(comm));
  return e == ncclSuccess ? VBHEM_OK : rccl_fail(e, "ncclCommDestroy");
}

int vbhem_rccl_allreduce_sum(void *comm, double *buf, size_t n, void *stream) {
  if (!comm || (!buf && n)) return vbhem::set_error(VBHEM_ERR_ARG, "vbhem_rccl_allreduce_sum: bad arguments");
  if (n == 0) return VBHEM_OK;
  if (int rc = need_rccl()) return rc;
  const ncclResult_t e = rccl().all_reduce(buf, buf, n, ncclFloat64, ncclSum, static_cast<ncclComm_t>(comm),
                                           static_cast<hipStream_t>(stream));
  return e == ncclSuccess ? VBHEM_OK : rccl_fail(e, "ncclAllReduce");
}

int vbhem_rccl_allreduce_to(void *comm, double *buf, size_t n, double *out_dev, void *stream) {
  if (!out_dev && n) return vbhem::set_error(VBHEM_ERR_ARG, "vbhem_rccl_allreduce_to: null destination");
  if (int rc = vbhem_rccl_allreduce_sum(comm, buf, n, stream)) return rc;
  if (n == 0) return VBHEM_OK;
  const unsigned grid = (unsigned)std::min<size_t>(64, (n + 255) / 256);
  hipLaunchKernelGGL(stats_copy_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     out_dev, buf, n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? VBHEM_OK
                         : vbhem::set_error(VBHEM_ERR_HIP, std::string("stats_copy_kernel: ") + hipGetErrorString(e));
}

}  // extern "C"
