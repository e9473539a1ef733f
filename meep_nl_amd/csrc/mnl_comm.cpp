// mnl_comm.cpp -- RCCL implementation of mnl::Comm (see mnl_comm.hpp).
#include "mnl_comm.hpp"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>

namespace mnl {

int Comm::unique_id(void *out128) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

int Comm::init(int r, int n, const void *id128) {
  rank = r;
  nranks = n;
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t c;
  if (ncclCommInitRank(&c, n, id, r) != ncclSuccess) return -1;
  comm_ = c;
  if (hipMalloc(&dscratch_, 64 * sizeof(double)) != hipSuccess) return -1;
  return 0;
}

int Comm::group_start() { return ncclGroupStart() == ncclSuccess ? 0 : -1; }
int Comm::group_end() { return ncclGroupEnd() == ncclSuccess ? 0 : -1; }

int Comm::send(const double *buf, size_t n, int peer, void *stream) {
  return ncclSend(buf, n, ncclDouble, peer, (ncclComm_t)comm_, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}
int Comm::recv(double *buf, size_t n, int peer, void *stream) {
  return ncclRecv(buf, n, ncclDouble, peer, (ncclComm_t)comm_, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}

int Comm::allreduce_sum(double *host, int n, void *stream) {
  if (n > 64) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(dscratch_, host, n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
    return -1;
  if (ncclAllReduce(dscratch_, dscratch_, n, ncclDouble, ncclSum, (ncclComm_t)comm_, s) !=
      ncclSuccess)
    return -1;
  if (hipMemcpyAsync(host, dscratch_, n * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess)
    return -1;
  return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy((ncclComm_t)comm_);
  if (dscratch_) hipFree(dscratch_);
}

}  // namespace mnl
