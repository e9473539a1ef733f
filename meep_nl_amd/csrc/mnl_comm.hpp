// mnl_comm.hpp -- ghost-plane transport between z-slab ranks.
// Replaces the reference's MPI comms_manager (src/mympi.cpp:87-151): the
// per-half-step ghost exchange becomes grouped ncclSend/ncclRecv of whole
// contiguous ghost planes between slab neighbours over xGMI (RCCL mode).
// IPC mode runs one process per slab where several processes share a GPU (RCCL
// refuses two ranks on one device): a POSIX shared-memory control block with a
// process-shared barrier, and one IPC-exported device staging buffer per rank
// that its neighbours copy from.  Same decomposition, streams and exchange
// sequence as RCCL mode; only the send/recv transport differs.
// LOCAL mode runs several slabs of one grid inside one process on one GPU
// (one host thread per slab) with device-to-device copies and host barriers.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mnl {

struct LocalHub;  // opaque, mnl_comm.cpp
struct IpcCtl;    // shared-memory control block, mnl_comm.cpp

class Comm {
 public:
  static int unique_id(void *out128);           // RCCL unique id
  static int ipc_id(void *out128, int nranks);  // creates the shared-memory segment
  static bool is_ipc_id(const void *id128);
  static int ipc_unlink(const void *id128);
  // RCCL, or IPC when id128 came from ipc_id()
  int init(int rank, int nranks, const void *id128);
  int init_local(int rank, int nranks, LocalHub *hub);  // in-process
  int group_start();
  int group_end(void *stream);
  int send(const double *buf, size_t n, int peer, void *stream);
  int recv(double *buf, size_t n, int peer, void *stream);
  // in-place sum over ranks of n host doubles (get_field, fluxes, array slices)
  int allreduce_sum(double *host, int n, void *stream);
  // logical OR of a per-rank error flag: every rank learns whether any failed
  // (called before a collective data step so no rank is left waiting in it)
  int agree_ok(bool ok, void *stream);
  const char *transport() const { return hub_ ? "local" : ipc_ ? "ipc" : "rccl"; }
  ~Comm();
  int rank = 0, nranks = 1;

 private:
  int init_ipc(const void *id128);
  int ipc_group_end(void *stream);
  int ipc_barrier();
  void ipc_abort();
  void *comm_ = nullptr;
  double *dscratch_ = nullptr;
  size_t dcap_ = 64;
  LocalHub *hub_ = nullptr;
  // IPC mode
  IpcCtl *ipc_ = nullptr;
  double *stage_ = nullptr;  // this rank's exported staging buffer
  size_t stage_cap_ = 0;     // doubles
  std::vector<double *> peer_base_;
  std::vector<uint64_t> peer_gen_;
  double ipc_timeout_s_ = 300.0;
  bool ipc_ready_ = false;  // every rank joined (setup barrier passed)
  bool ipc_peer_dead() const;
  struct Op {
    double *dst;
    const double *src;
    size_t n;
    int peer;
  };
  std::vector<Op> sends_, recvs_;
};

// detail of the last failed RCCL setup call of this thread ("" if none)
const char *comm_last_error();
LocalHub *local_hub_create(int nranks);
void local_hub_destroy(LocalHub *h);

}  // namespace mnl
