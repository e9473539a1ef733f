// mnl_comm.hpp -- ghost-plane transport between z-slab ranks.
// Replaces the reference's MPI comms_manager (src/mympi.cpp:87-151): the
// per-half-step ghost exchange becomes grouped ncclSend/ncclRecv of whole
// contiguous ghost planes between slab neighbours over xGMI (RCCL mode).
// LOCAL mode runs several slabs of one grid inside one process on one GPU
// (one host thread per slab) with device-to-device copies and host barriers;
// it exercises the identical decomposition / exchange code without RCCL.
#pragma once
#include <cstddef>
#include <vector>

namespace mnl {

struct LocalHub;  // opaque, mnl_comm.cpp

class Comm {
 public:
  static int unique_id(void *out128);
  int init(int rank, int nranks, const void *id128);      // RCCL
  int init_local(int rank, int nranks, LocalHub *hub);     // in-process
  int group_start();
  int group_end(void *stream);
  int send(const double *buf, size_t n, int peer, void *stream);
  int recv(double *buf, size_t n, int peer, void *stream);
  // in-place sum over ranks of n host doubles (get_field, fluxes, array slices)
  int allreduce_sum(double *host, int n, void *stream);
  ~Comm();
  int rank = 0, nranks = 1;

 private:
  void *comm_ = nullptr;
  double *dscratch_ = nullptr;
  size_t dcap_ = 64;
  LocalHub *hub_ = nullptr;
  struct Op {
    double *dst;
    const double *src;
    size_t n;
    int peer;
  };
  std::vector<Op> sends_, recvs_;
};

LocalHub *local_hub_create(int nranks);
void local_hub_destroy(LocalHub *h);

}  // namespace mnl
