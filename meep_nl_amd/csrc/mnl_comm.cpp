// mnl_comm.cpp -- RCCL and in-process implementations of mnl::Comm.
#include "mnl_comm.hpp"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <mutex>

namespace mnl {

struct LocalHub {
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long long gen = 0;
  struct Post {
    int dst;
    const double *ptr;
    size_t n;
  };
  std::vector<std::vector<Post>> sends;
  std::vector<hipEvent_t> ev_send, ev_done;
  std::vector<std::vector<double>> red;

  explicit LocalHub(int nr) : n(nr), sends(nr), ev_send(nr, nullptr), ev_done(nr, nullptr), red(nr) {}
  ~LocalHub() {
    for (auto e : ev_send)
      if (e) (void)hipEventDestroy(e);
    for (auto e : ev_done)
      if (e) (void)hipEventDestroy(e);
  }
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    long long g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

LocalHub *local_hub_create(int nranks) { return new LocalHub(nranks); }
void local_hub_destroy(LocalHub *h) { delete h; }

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

int Comm::init_local(int r, int n, LocalHub *hub) {
  rank = r;
  nranks = n;
  hub_ = hub;
  if (!hub || hub->n != n) return -1;
  std::lock_guard<std::mutex> lk(hub->m);
  if (!hub->ev_send[r] &&
      hipEventCreateWithFlags(&hub->ev_send[r], hipEventDisableTiming) != hipSuccess)
    return -1;
  if (!hub->ev_done[r] &&
      hipEventCreateWithFlags(&hub->ev_done[r], hipEventDisableTiming) != hipSuccess)
    return -1;
  return 0;
}

int Comm::group_start() {
  if (hub_) {
    sends_.clear();
    recvs_.clear();
    return 0;
  }
  return ncclGroupStart() == ncclSuccess ? 0 : -1;
}

int Comm::group_end(void *stream) {
  if (!hub_) return ncclGroupEnd() == ncclSuccess ? 0 : -1;
  hipStream_t s = (hipStream_t)stream;
  LocalHub &H = *hub_;
  // 1. publish this rank's sends once their data is ready on its stream
  H.sends[rank].clear();
  for (auto &o : sends_) H.sends[rank].push_back({o.peer, o.src, o.n});
  if (hipEventRecord(H.ev_send[rank], s) != hipSuccess) return -1;
  H.barrier();
  // 2. pull every matching send (k-th recv from p <-> k-th send of p to me)
  std::vector<int> seen(nranks, 0);
  for (auto &r : recvs_) {
    int k = seen[r.peer]++, cnt = 0;
    const LocalHub::Post *hit = nullptr;
    for (auto &p : H.sends[r.peer])
      if (p.dst == rank && cnt++ == k) hit = &p;
    if (!hit || hit->n != r.n) return -1;
    if (hipStreamWaitEvent(s, H.ev_send[r.peer], 0) != hipSuccess) return -1;
    if (hipMemcpyAsync(r.dst, hit->ptr, r.n * sizeof(double), hipMemcpyDeviceToDevice, s) !=
        hipSuccess)
      return -1;
  }
  if (hipEventRecord(H.ev_done[rank], s) != hipSuccess) return -1;
  H.barrier();
  // 3. later writes to our send buffers wait for every peer's copies
  for (int p = 0; p < nranks; p++)
    if (p != rank && hipStreamWaitEvent(s, H.ev_done[p], 0) != hipSuccess) return -1;
  return 0;
}

int Comm::send(const double *buf, size_t n, int peer, void *stream) {
  if (hub_) {
    sends_.push_back({nullptr, buf, n, peer});
    return 0;
  }
  return ncclSend(buf, n, ncclDouble, peer, (ncclComm_t)comm_, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}
int Comm::recv(double *buf, size_t n, int peer, void *stream) {
  if (hub_) {
    recvs_.push_back({buf, nullptr, n, peer});
    return 0;
  }
  return ncclRecv(buf, n, ncclDouble, peer, (ncclComm_t)comm_, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}

int Comm::allreduce_sum(double *host, int n, void *stream) {
  if (n < 0) return -1;
  if (hub_) {
    LocalHub &H = *hub_;
    H.red[rank].assign(host, host + n);
    H.barrier();
    for (int i = 0; i < n; i++) {
      double acc = 0.0;
      for (int r = 0; r < nranks; r++) acc += H.red[r][i];
      host[i] = acc;
    }
    H.barrier();
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  if ((size_t)n > dcap_) {  // grow the device staging buffer (64 doubles at init)
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (dscratch_) (void)hipFree(dscratch_);
    dscratch_ = nullptr;
    if (hipMalloc(&dscratch_, (size_t)n * sizeof(double)) != hipSuccess) return -1;
    dcap_ = (size_t)n;
  }
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
  // events belong to the hub (it may be destroyed before or after us)
}

}  // namespace mnl
