// mnl_comm.cpp -- RCCL, IPC (processes sharing a GPU) and in-process
// implementations of mnl::Comm.
#include "mnl_comm.hpp"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cerrno>
#include <csignal>
#include <fcntl.h>
#include <mutex>
#include <sched.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

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

// ------------------------------------------------------------------ IPC mode
// One shared-memory segment per job (created by ipc_id on one rank, name passed
// to the others in the 128-byte id).  Each rank owns a slot: the IPC handle of
// its staging buffer (+ a generation bumped when it grows), the posts of its
// current exchange group and a reduction buffer.
static const char IPC_MAGIC[8] = {'M', 'N', 'L', 'I', 'P', 'C', '1', 0};
constexpr int IPC_MAXR = 16, IPC_MAXPOST = 96, IPC_RED = 8192;

struct IpcPost {
  int dst;
  int pad;
  uint64_t off, n;  // doubles
};
struct IpcSlot {
  hipIpcMemHandle_t h;
  uint64_t gen;
  int nposts;
  int pid;  // the rank's process (liveness checks of the waits)
  IpcPost posts[IPC_MAXPOST];
  double red[IPC_RED];
};
struct IpcCtl {
  std::atomic<int> arrived;
  std::atomic<int> gen;
  std::atomic<int> abort;
  std::atomic<int> nranks;
  IpcSlot slot[IPC_MAXR];
};
static_assert(std::atomic<int>::is_always_lock_free, "process-shared atomics need lock-free int");

bool Comm::is_ipc_id(const void *id128) {
  return id128 && memcmp(id128, IPC_MAGIC, sizeof(IPC_MAGIC)) == 0;
}

int Comm::ipc_id(void *out128, int nranks) {
  if (nranks < 1 || nranks > IPC_MAXR) return -1;
  static std::atomic<int> counter{0};
  char name[96];
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  snprintf(name, sizeof(name), "/mnl_ipc_%d_%d_%lx", (int)getpid(), counter++,
           (unsigned long)(ts.tv_nsec ^ (ts.tv_sec << 20)));
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return -1;
  if (ftruncate(fd, sizeof(IpcCtl)) != 0) {
    close(fd);
    shm_unlink(name);
    return -1;
  }
  close(fd);  // zero-filled by ftruncate: counters 0, nranks 0 (set by the first rank)
  memset(out128, 0, 128);
  memcpy(out128, IPC_MAGIC, sizeof(IPC_MAGIC));
  strncpy((char *)out128 + 8, name, 119);
  return 0;
}

int Comm::ipc_unlink(const void *id128) {
  if (!is_ipc_id(id128)) return -1;
  char name[128];
  memcpy(name, (const char *)id128 + 8, 120);
  name[119] = 0;
  return shm_unlink(name) == 0 ? 0 : -1;
}

int Comm::init_ipc(const void *id128) {
  if (nranks > IPC_MAXR) return -1;
  char name[128];
  memcpy(name, (const char *)id128 + 8, 120);
  name[119] = 0;
  int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return -1;
  void *p = mmap(nullptr, sizeof(IpcCtl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -1;
  ipc_ = (IpcCtl *)p;
  int expect = 0;
  if (!ipc_->nranks.compare_exchange_strong(expect, nranks) && expect != nranks) {
    ipc_abort();  // the peers would otherwise wait for this rank until their timeout
    return -1;
  }
  if (const char *t = getenv("MNL_IPC_TIMEOUT")) ipc_timeout_s_ = std::max(1.0, atof(t));
  peer_base_.assign(nranks, nullptr);
  peer_gen_.assign(nranks, 0);
  ipc_->slot[rank].pid = (int)getpid();
  if (ipc_barrier()) return -1;  // the setup barrier: bounded by MNL_IPC_TIMEOUT
  ipc_ready_ = true;              // later waits: as long as every peer process lives
  if (rank == 0) shm_unlink(name);  // every rank has it mapped: nothing leaks in /dev/shm
  return 0;
}

// a process that has exited: its pid is gone, or it is a zombie (exited, not yet reaped by a
// launcher that may itself be waiting on another rank) -- /proc/<pid>/stat state Z or X
static bool pid_exited(int pid) {
  if (kill(pid, 0) != 0 && errno == ESRCH) return true;
  char path[64], buf[512];
  snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE *f = fopen(path, "r");
  if (!f) return false;  // cannot tell: alive
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char *p = strrchr(buf, ')');  // the command name may hold spaces and parentheses
  return p && p[1] == ' ' && (p[2] == 'Z' || p[2] == 'X');
}

// a peer's process has exited
bool Comm::ipc_peer_dead() const {
  for (int r = 0; r < nranks; r++) {
    const int pid = ipc_->slot[r].pid;
    if (r == rank || pid <= 0) continue;
    if (pid_exited(pid)) return true;
  }
  return false;
}

void Comm::ipc_abort() {
  if (ipc_) ipc_->abort.store(1, std::memory_order_release);
}

int Comm::ipc_barrier() {
  IpcCtl &C = *ipc_;
  if (C.abort.load(std::memory_order_acquire)) return -1;
  const int g = C.gen.load(std::memory_order_acquire);
  if (C.arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == nranks) {
    C.arrived.store(0, std::memory_order_relaxed);
    C.gen.fetch_add(1, std::memory_order_release);
    return 0;
  }
  // Setup waits are bounded by MNL_IPC_TIMEOUT (default 300 s).  Once every rank has joined,
  // a wait ends when a peer's process exits (or turns zombie) -- liveness comes from the
  // peers' pids -- or after MNL_IPC_TIMEOUT when it is set, else after IPC_RUN_TIMEOUT_S (2 h):
  // a rank-0-only output or a whole-cell setup can legitimately keep the others waiting for a
  // long time, but a peer that is alive and stuck (a GPU hang inside a synchronize, a rank on
  // another code path) must not hang every other rank forever.
  constexpr double IPC_RUN_TIMEOUT_S = 7200.0;
  static const bool explicit_timeout = getenv("MNL_IPC_TIMEOUT") != nullptr;
  const double limit = (ipc_ready_ && !explicit_timeout) ? IPC_RUN_TIMEOUT_S : ipc_timeout_s_;
  auto t0 = std::chrono::steady_clock::now();
  long spins = 0;
  while (C.gen.load(std::memory_order_acquire) == g) {
    if (C.abort.load(std::memory_order_acquire)) return -1;
    if (++spins > 2000) {
      struct timespec d = {0, 20000};
      nanosleep(&d, nullptr);
      if ((spins & 1023) == 0) {
        if (ipc_ready_ && ipc_peer_dead()) {
          ipc_abort();  // a peer died: fail every rank instead of hanging
          return -1;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
            limit) {
          ipc_abort();  // a peer never joined or diverged: fail every rank
          return -1;
        }
      }
    } else {
      sched_yield();
    }
  }
  return 0;
}

int Comm::ipc_group_end(void *stream) {
  hipStream_t s = (hipStream_t)stream;
  IpcSlot &me = ipc_->slot[rank];
  auto bail = [&]() {
    ipc_abort();
    return -1;
  };
  size_t total = 0;
  for (auto &o : sends_) total += o.n;
  if ((int)sends_.size() > IPC_MAXPOST) return bail();
  if (total > stage_cap_) {  // peers finished reading the old buffer (last group's barrier)
    if (hipStreamSynchronize(s) != hipSuccess) return bail();
    if (stage_) (void)hipFree(stage_);
    stage_ = nullptr;
    size_t cap = std::max<size_t>(total + total / 4, 1 << 16);
    if (hipMalloc(&stage_, cap * sizeof(double)) != hipSuccess) return bail();
    if (hipIpcGetMemHandle(&me.h, stage_) != hipSuccess) return bail();
    stage_cap_ = cap;
    me.gen++;
  }
  size_t off = 0;
  me.nposts = 0;
  for (auto &o : sends_) {
    if (o.n && hipMemcpyAsync(stage_ + off, o.src, o.n * sizeof(double), hipMemcpyDeviceToDevice,
                              s) != hipSuccess)
      return bail();
    me.posts[me.nposts++] = {o.peer, 0, off, o.n};
    off += o.n;
  }
  if (hipStreamSynchronize(s) != hipSuccess) return bail();  // staged data is complete
  if (ipc_barrier()) return -1;
  std::vector<int> seen(nranks, 0);
  for (auto &r : recvs_) {
    const IpcSlot &ps = ipc_->slot[r.peer];
    int k = seen[r.peer]++, cnt = 0;
    const IpcPost *hit = nullptr;
    for (int i = 0; i < ps.nposts; i++)
      if (ps.posts[i].dst == rank && cnt++ == k) hit = &ps.posts[i];
    if (!hit || hit->n != r.n) return bail();
    if (peer_gen_[r.peer] != ps.gen) {  // (re)map the peer's staging buffer
      if (peer_base_[r.peer]) (void)hipIpcCloseMemHandle(peer_base_[r.peer]);
      peer_base_[r.peer] = nullptr;
      void *p = nullptr;
      if (hipIpcOpenMemHandle(&p, ps.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
        return bail();
      peer_base_[r.peer] = (double *)p;
      peer_gen_[r.peer] = ps.gen;
    }
    if (r.n && hipMemcpyAsync(r.dst, peer_base_[r.peer] + hit->off, r.n * sizeof(double),
                              hipMemcpyDeviceToDevice, s) != hipSuccess)
      return bail();
  }
  if (hipStreamSynchronize(s) != hipSuccess) return bail();
  return ipc_barrier();  // our staging buffer may be rewritten only after every peer copied
}

// ------------------------------------------------------------------ common
int Comm::unique_id(void *out128) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

static thread_local char g_comm_err[256] = "";
const char *comm_last_error() { return g_comm_err; }

int Comm::init(int r, int n, const void *id128) {
  rank = r;
  nranks = n;
  if (!id128) return -1;
  if (is_ipc_id(id128)) return init_ipc(id128);
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t c;
  const ncclResult_t rc = ncclCommInitRank(&c, n, id, r);
  if (rc != ncclSuccess) {
    snprintf(g_comm_err, sizeof g_comm_err, "ncclCommInitRank(rank %d of %d): %s", r, n,
             ncclGetErrorString(rc));
    return -1;
  }
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
  if (hub_ || ipc_) {
    sends_.clear();
    recvs_.clear();
    return 0;
  }
  return ncclGroupStart() == ncclSuccess ? 0 : -1;
}

int Comm::group_end(void *stream) {
  if (ipc_) return ipc_group_end(stream);
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
  if (hub_ || ipc_) {
    sends_.push_back({nullptr, buf, n, peer});
    return 0;
  }
  return ncclSend(buf, n, ncclDouble, peer, (ncclComm_t)comm_, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}
int Comm::recv(double *buf, size_t n, int peer, void *stream) {
  if (hub_ || ipc_) {
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
  if (ipc_) {  // same rank-order sum as the in-process hub, in chunks of the slot buffer
    for (int q = 0; q < n; q += IPC_RED) {
      const int m = std::min(IPC_RED, n - q);
      memcpy(ipc_->slot[rank].red, host + q, m * sizeof(double));
      if (ipc_barrier()) return -1;
      for (int i = 0; i < m; i++) {
        double acc = 0.0;
        for (int r = 0; r < nranks; r++) acc += ipc_->slot[r].red[i];
        host[q + i] = acc;
      }
      if (ipc_barrier()) return -1;
    }
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

int Comm::agree_ok(bool ok, void *stream) {
  double v = ok ? 0.0 : 1.0;
  if (allreduce_sum(&v, 1, stream)) return -1;
  return v == 0.0 ? 0 : -1;
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy((ncclComm_t)comm_);
  if (dscratch_) hipFree(dscratch_);
  for (auto p : peer_base_)
    if (p) (void)hipIpcCloseMemHandle(p);
  if (stage_) (void)hipFree(stage_);
  if (ipc_) munmap(ipc_, sizeof(IpcCtl));
  // events belong to the hub (it may be destroyed before or after us)
}

}  // namespace mnl
