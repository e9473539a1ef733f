// mnl_comm.hpp -- thin RCCL wrapper (one communicator per fields object).
// Replaces the reference's MPI comms_manager (src/mympi.cpp:87-151): the
// per-half-step ghost exchange becomes grouped ncclSend/ncclRecv of whole
// ghost planes between z-slab neighbours over xGMI.
#pragma once
#include <cstddef>

namespace mnl {

class Comm {
 public:
  static int unique_id(void *out128);
  int init(int rank, int nranks, const void *id128);
  int group_start();
  int group_end();
  int send(const double *buf, size_t n, int peer, void *stream);
  int recv(double *buf, size_t n, int peer, void *stream);
  // in-place sum over ranks of n host doubles (small; used by get_field)
  int allreduce_sum(double *host, int n, void *stream);
  ~Comm();
  int rank = 0, nranks = 1;

 private:
  void *comm_ = nullptr;
  double *dscratch_ = nullptr;
};

}  // namespace mnl
