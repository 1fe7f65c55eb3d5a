#include "rccl_comm.h"

#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace {

struct RcclApi {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclReduceScatter) reduceScatter = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) getErrorString = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
  decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommCount) commCount = nullptr;
};

RcclApi g_api;
std::mutex g_mu;

template <class F>
void sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_api.handle, name));
  if (!f) throw std::runtime_error(std::string("RCCL symbol not found: ") + name);
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const char* msg = g_api.getErrorString ? g_api.getErrorString(r) : "?";
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + msg);
  }
}

void require_loaded() {
  if (!g_api.handle) throw std::runtime_error("RCCL not loaded: call RcclComm.load(path) first");
}

}  // namespace

void RcclComm::load(const std::string& lib_path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.handle) return;
  void* h = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!h) throw std::runtime_error(std::string("dlopen(") + lib_path + ") failed: " + dlerror());
  g_api.handle = h;
  sym(g_api.getUniqueId, "ncclGetUniqueId");
  sym(g_api.commInitRank, "ncclCommInitRank");
  sym(g_api.commDestroy, "ncclCommDestroy");
  sym(g_api.allReduce, "ncclAllReduce");
  sym(g_api.broadcast, "ncclBroadcast");
  sym(g_api.reduce, "ncclReduce");
  sym(g_api.allGather, "ncclAllGather");
  sym(g_api.reduceScatter, "ncclReduceScatter");
  sym(g_api.groupStart, "ncclGroupStart");
  sym(g_api.groupEnd, "ncclGroupEnd");
  sym(g_api.getErrorString, "ncclGetErrorString");
  sym(g_api.getVersion, "ncclGetVersion");
  sym(g_api.getAsyncError, "ncclCommGetAsyncError");
  sym(g_api.commAbort, "ncclCommAbort");
  sym(g_api.commCount, "ncclCommCount");
}

bool RcclComm::loaded() { return g_api.handle != nullptr; }

int RcclComm::version() {
  require_loaded();
  int v = 0;
  check(g_api.getVersion(&v), "GetVersion");
  return v;
}

std::vector<char> RcclComm::unique_id() {
  require_loaded();
  ncclUniqueId id;
  check(g_api.getUniqueId(&id), "GetUniqueId");
  std::vector<char> out(sizeof(id.internal));
  std::memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

RcclComm::RcclComm(const std::vector<char>& uid, int nranks, int rank)
    : nranks_(nranks), rank_(rank) {
  require_loaded();
  ncclUniqueId id;
  if (uid.size() != sizeof(id.internal)) throw std::runtime_error("bad RCCL unique id size");
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  ncclComm_t c = nullptr;
  check(g_api.commInitRank(&c, nranks, id, rank), "CommInitRank");
  comm_.store(c);
}

RcclComm::~RcclComm() {
  try {
    destroy();
  } catch (...) {
  }
}

void RcclComm::destroy() {
  std::lock_guard<std::timed_mutex> lk(mu_);
  ncclComm_t c = comm_.exchange(nullptr);
  if (c) check(g_api.commDestroy(c), "CommDestroy");
}

// Failure detection (SURVEY §5 failure row).  Both calls are documented as
// safe from a thread other than the one issuing collectives: the host
// watchdog (parallel/watchdog.py) polls async_error() while the training
// thread is blocked on a device synchronize, and abort()s the communicator
// when a peer died or a collective overran its deadline.  Abort makes the
// in-flight RCCL kernels exit, so the stuck synchronize returns.
int RcclComm::async_error() const {
  // never blocks the watchdog: a busy communicator reads as "in progress"
  std::unique_lock<std::timed_mutex> lk(mu_, std::try_to_lock);
  if (!lk.owns_lock()) return (int)ncclInProgress;
  ncclComm_t c = comm_.load();
  if (!c) return aborted_.load() ? (int)ncclRemoteError : (int)ncclSuccess;
  ncclResult_t e = ncclSuccess;
  check(g_api.getAsyncError(c, &e), "CommGetAsyncError");
  return (int)e;
}

void RcclComm::abort() {
  aborted_.store(true);
  // a host call stuck inside RCCL must not keep the watchdog from exiting:
  // after 3 s the process ends without the abort (its exit frees the GPU)
  std::unique_lock<std::timed_mutex> lk(mu_, std::chrono::seconds(3));
  if (!lk.owns_lock()) return;
  ncclComm_t c = comm_.exchange(nullptr);
  if (c) (void)g_api.commAbort(c);
}

int RcclComm::comm_count() const {
  std::lock_guard<std::timed_mutex> lk(mu_);
  ncclComm_t c = comm_.load();
  if (!c) throw std::runtime_error("RCCL communicator was destroyed or aborted");
  int n = 0;
  check(g_api.commCount(c, &n), "CommCount");
  return n;
}

std::string RcclComm::error_string(int code) {
  require_loaded();
  return g_api.getErrorString((ncclResult_t)code);
}

ncclComm_t RcclComm::live() const {
  ncclComm_t c = comm_.load();
  if (!c) throw std::runtime_error("RCCL communicator was destroyed or aborted");
  return c;
}

void RcclComm::all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                          hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  check(g_api.allReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, live(), s),
        "AllReduce");
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root,
                         hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  check(g_api.broadcast(send, recv, count, (ncclDataType_t)dtype, root, live(), s), "Broadcast");
}

void RcclComm::reduce(const void* send, void* recv, size_t count, int dtype, int op, int root,
                      hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  check(g_api.reduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, root, live(), s),
        "Reduce");
}

void RcclComm::all_gather(const void* send, void* recv, size_t send_count, int dtype,
                          hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  check(g_api.allGather(send, recv, send_count, (ncclDataType_t)dtype, live(), s), "AllGather");
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                              hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  check(g_api.reduceScatter(send, recv, recv_count, (ncclDataType_t)dtype, (ncclRedOp_t)op, live(),
                            s),
        "ReduceScatter");
}

void RcclComm::group_start() { check(g_api.groupStart(), "GroupStart"); }
void RcclComm::group_end() { check(g_api.groupEnd(), "GroupEnd"); }
