#include "shm_comm.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

#include <rccl/rccl.h>

#include "kernels/common.h"

namespace {

constexpr uint64_t kMagic = 0x4d5441534843304dULL;
constexpr int kMaxRanks = 64;
constexpr size_t kPage = 4096;

struct Sig {
  uint64_t seq;
  int32_t kind, dtype, op, root;
  uint64_t count;
};

// Shared header.  The counters sit on cache lines of their own.
struct Hdr {
  std::atomic<uint64_t> magic;
  int32_t nranks, pad0;
  uint64_t cap;
  alignas(64) std::atomic<uint32_t> arrive;
  alignas(64) std::atomic<uint32_t> gen;
  alignas(64) std::atomic<uint32_t> abort;
  alignas(64) Sig sig[kMaxRanks];
};
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics");

constexpr size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
constexpr size_t kHdrBytes = round_up(sizeof(Hdr), kPage);

inline Hdr* hdr_of(void* map) { return reinterpret_cast<Hdr*>(map); }

// ---- element-wise reductions over the rank slots, in rank order ----------
inline float bf2f(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f2bf(float f) {  // round to nearest even; NaN stays NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if (std::isnan(f)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

template <class T>
void reduce_typed(T* out, const char* const* src, int n, size_t lo, size_t hi, bool max_op) {
  const T* s0 = reinterpret_cast<const T*>(src[0]);
  for (size_t i = lo; i < hi; ++i) out[i - lo] = s0[i];
  for (int r = 1; r < n; ++r) {
    const T* sr = reinterpret_cast<const T*>(src[r]);
    if (max_op) {
      for (size_t i = lo; i < hi; ++i) out[i - lo] = sr[i] > out[i - lo] ? sr[i] : out[i - lo];
    } else {
      for (size_t i = lo; i < hi; ++i) out[i - lo] += sr[i];
    }
  }
}

void reduce_bf16(uint16_t* out, const char* const* src, int n, size_t lo, size_t hi, bool max_op) {
  constexpr size_t kBlk = 1024;
  float acc[kBlk];
  for (size_t a = lo; a < hi; a += kBlk) {
    const size_t b = a + kBlk < hi ? a + kBlk : hi;
    const uint16_t* s0 = reinterpret_cast<const uint16_t*>(src[0]);
    for (size_t i = a; i < b; ++i) acc[i - a] = bf2f(s0[i]);
    for (int r = 1; r < n; ++r) {
      const uint16_t* sr = reinterpret_cast<const uint16_t*>(src[r]);
      for (size_t i = a; i < b; ++i) {
        const float v = bf2f(sr[i]);
        acc[i - a] = max_op ? (v > acc[i - a] ? v : acc[i - a]) : acc[i - a] + v;
      }
    }
    for (size_t i = a; i < b; ++i) out[i - lo] = f2bf(acc[i - a]);
  }
}

// out[0 .. hi-lo) = reduction of src[r][lo .. hi) (element indices)
void reduce_range(void* out, const char* const* src, int n, size_t lo, size_t hi, int dtype,
                  int op) {
  const bool mx = op == ncclMax;
  switch (dtype) {
    case ncclFloat32: reduce_typed((float*)out, src, n, lo, hi, mx); break;
    case ncclBfloat16: reduce_bf16((uint16_t*)out, src, n, lo, hi, mx); break;
    case ncclInt32: reduce_typed((int32_t*)out, src, n, lo, hi, mx); break;
    case ncclInt64: reduce_typed((int64_t*)out, src, n, lo, hi, mx); break;
    case ncclFloat64: reduce_typed((double*)out, src, n, lo, hi, mx); break;
    default: break;  // rejected at enqueue
  }
}

bool dtype_ok(int dtype) {
  return dtype == ncclFloat32 || dtype == ncclBfloat16 || dtype == ncclInt32 ||
         dtype == ncclInt64 || dtype == ncclFloat64;
}

}  // namespace

ShmComm::ShmComm(const std::string& path, bool create, int nranks, int rank, size_t capacity,
                 double timeout_s, bool pinned)
    : nranks_(nranks), rank_(rank), cap_(round_up(capacity, kPage)), timeout_s_(timeout_s),
      path_(path), pinned_(pinned) {
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || capacity == 0)
    throw std::runtime_error("ShmComm: bad rank layout or capacity");
  map_bytes_ = kHdrBytes + (size_t)(nranks + 1) * cap_;
  fd_ = ::open(path.c_str(), create ? (O_RDWR | O_CREAT | O_EXCL) : O_RDWR, 0600);
  if (fd_ < 0) throw std::runtime_error("ShmComm: cannot open " + path + ": " + strerror(errno));
  if (create) {
    // reserve the blocks now: a full tmpfs fails here with ENOSPC instead of
    // SIGBUS on the first touch of a slot
    int e = posix_fallocate(fd_, 0, (off_t)map_bytes_);
    if (e != 0) {
      ::close(fd_);
      ::unlink(path.c_str());
      throw std::runtime_error("ShmComm: cannot reserve " + std::to_string(map_bytes_) +
                               " bytes in " + path + ": " + strerror(e));
    }
  } else {
    struct stat st;
    if (fstat(fd_, &st) != 0 || (size_t)st.st_size < map_bytes_) {
      ::close(fd_);
      throw std::runtime_error("ShmComm: " + path + " is smaller than this layout needs");
    }
  }
  map_ = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (map_ == MAP_FAILED) {
    map_ = nullptr;
    ::close(fd_);
    throw std::runtime_error("ShmComm: mmap failed: " + std::string(strerror(errno)));
  }
  Hdr* h = hdr_of(map_);
  if (create) {
    h->nranks = nranks;
    h->cap = cap_;
    h->arrive.store(0);
    h->gen.store(0);
    h->abort.store(0);
    std::memset(h->sig, 0, sizeof(h->sig));
    h->magic.store(kMagic, std::memory_order_release);
  } else if (h->magic.load(std::memory_order_acquire) != kMagic || h->nranks != nranks ||
             h->cap != cap_) {
    munmap(map_, map_bytes_);
    ::close(fd_);
    throw std::runtime_error("ShmComm: " + path + " was made for another rank layout");
  }
  if (pinned_) {
    HIP_CHECK(hipHostMalloc(&send_stage_, cap_, hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc(&recv_stage_, (size_t)nranks * cap_, hipHostMallocDefault));
  } else {
    send_stage_ = std::malloc(cap_);
    recv_stage_ = std::malloc((size_t)nranks * cap_);
    if (!send_stage_ || !recv_stage_) throw std::bad_alloc();
  }
}

ShmComm::~ShmComm() {
  if (pinned_) {
    if (send_stage_) (void)hipHostFree(send_stage_);
    if (recv_stage_) (void)hipHostFree(recv_stage_);
  } else {
    std::free(send_stage_);
    std::free(recv_stage_);
  }
  if (map_) munmap(map_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
}

void ShmComm::unlink_path() { (void)::unlink(path_.c_str()); }

char* ShmComm::slot(int r) const { return (char*)map_ + kHdrBytes + (size_t)r * cap_; }
char* ShmComm::result() const { return slot(nranks_); }

std::string ShmComm::error_message() const {
  return msg_set_.load(std::memory_order_acquire) ? std::string(msg_) : std::string();
}

void ShmComm::fail(int code, const std::string& why) {
  int expect = 0;
  if (err_.compare_exchange_strong(expect, code)) {
    std::snprintf(msg_, sizeof(msg_), "%s", why.c_str());
    msg_set_.store(1, std::memory_order_release);
  }
  hdr_of(map_)->abort.store(1, std::memory_order_release);
}

void ShmComm::abort() { fail(ncclRemoteError, "aborted"); }

// Generation barrier over all ranks; false on timeout or abort.
bool ShmComm::barrier() {
  Hdr* h = hdr_of(map_);
  const uint32_t g = h->gen.load(std::memory_order_acquire);
  if (h->arrive.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)nranks_ - 1) {
    h->arrive.store(0, std::memory_order_relaxed);
    h->gen.fetch_add(1, std::memory_order_acq_rel);
    return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned long spin = 0;; ++spin) {
    if (h->gen.load(std::memory_order_acquire) != g) return true;
    if (h->abort.load(std::memory_order_acquire)) {
      fail(ncclRemoteError, "a peer aborted the communicator");
      return false;
    }
    if (spin < 4096) {
      __builtin_ia32_pause();
      continue;
    }
    if ((spin & 255) == 0) {
      const double dt =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (dt > timeout_s_) {
        fail(ncclRemoteError, "peer did not arrive within " + std::to_string(timeout_s_) + " s");
        return false;
      }
    }
    if (spin < 65536) {
      sched_yield();
    } else {
      struct timespec ts {0, 20000};
      nanosleep(&ts, nullptr);
    }
  }
}

void ShmComm::host_fn(void* arg) {
  Op* d = static_cast<Op*>(arg);
  try {
    d->comm->exchange(*d);
  } catch (...) {
    d->comm->fail(ncclInternalError, "exception in the host exchange");
  }
  if (d->owned) delete d;  // an eager launch runs exactly once
}

// Runs on the HIP runtime's host-function thread, in stream order between
// the D2H and H2D copies of this rank.  No HIP calls here.
void ShmComm::exchange(const Op& d) {
  if (err_.load() != 0) return;  // a failed communicator drains without blocking
  Hdr* h = hdr_of(map_);
  const unsigned long long seq = ++seq_;
  const size_t es = dtype_bytes(d.dtype);
  if (d.in_bytes) std::memcpy(slot(rank_), send_stage_, d.in_bytes);
  Sig& me = h->sig[rank_];
  me.seq = seq;
  me.kind = d.kind;
  me.dtype = d.dtype;
  me.op = d.op;
  me.root = d.root;
  me.count = d.count;
  if (!barrier()) return;
  for (int r = 0; r < nranks_; ++r) {
    const Sig& o = h->sig[r];
    if (o.seq != seq || o.kind != d.kind || o.dtype != d.dtype || o.op != d.op ||
        o.root != d.root || o.count != d.count) {
      fail(ncclInvalidUsage, "collective #" + std::to_string(seq) + " differs between rank " +
                                 std::to_string(rank_) + " and rank " + std::to_string(r) +
                                 " (kind " + std::to_string(d.kind) + " vs " +
                                 std::to_string(o.kind) + ", count " + std::to_string(d.count) +
                                 " vs " + std::to_string(o.count) + ")");
      return;
    }
  }
  const char* src[kMaxRanks];
  for (int r = 0; r < nranks_; ++r) src[r] = slot(r);
  char* out = static_cast<char*>(recv_stage_);
  switch (d.kind) {
    case AR:
    case RD: {
      // each rank reduces one chunk into the shared result, then all copy it
      const size_t n = d.count;
      const size_t chunk = round_up((n + nranks_ - 1) / nranks_, 64);
      const size_t lo = std::min(n, chunk * rank_), hi = std::min(n, lo + chunk);
      if (hi > lo) reduce_range(result() + lo * es, src, nranks_, lo, hi, d.dtype, d.op);
      if (!barrier()) return;
      if (d.out_bytes) std::memcpy(out, result(), d.out_bytes);
      break;
    }
    case RS: {
      const size_t lo = d.count * rank_;
      reduce_range(out, src, nranks_, lo, lo + d.count, d.dtype, d.op);
      break;
    }
    case AG:
      for (int r = 0; r < nranks_; ++r) std::memcpy(out + r * d.in_bytes, slot(r), d.in_bytes);
      break;
    case BC:
      if (d.out_bytes) std::memcpy(out, slot(d.root), d.out_bytes);
      break;
    default:
      break;
  }
  if (!barrier()) return;  // slots / result may be rewritten by the next collective
  done_.fetch_add(1);
}

std::unique_ptr<ShmComm::Op> ShmComm::make_op(int kind, const void* send, const void* recv,
                                             size_t count, int dtype, int op, int root) const {
  if (!dtype_ok(dtype)) throw std::runtime_error("ShmComm: unsupported dtype");
  if (op != ncclSum && op != ncclMax) throw std::runtime_error("ShmComm: only sum / max");
  if (root < 0 || root >= nranks_) throw std::runtime_error("ShmComm: bad root");
  const size_t es = dtype_bytes(dtype);
  auto d = std::make_unique<Op>();
  d->comm = const_cast<ShmComm*>(this);
  d->kind = kind;
  d->dtype = dtype;
  d->op = op;
  d->root = (kind == BC || kind == RD) ? root : 0;
  d->count = count;
  switch (kind) {
    case AR: d->in_bytes = d->out_bytes = count * es; break;
    case AG: d->in_bytes = count * es; d->out_bytes = count * es * nranks_; break;
    case RS: d->in_bytes = count * es * nranks_; d->out_bytes = count * es; break;
    case BC:
      d->in_bytes = rank_ == root ? count * es : 0;
      d->out_bytes = (rank_ == root && send == recv) ? 0 : count * es;
      break;
    case RD:
      d->in_bytes = count * es;
      d->out_bytes = rank_ == root ? count * es : 0;
      break;
    default: throw std::runtime_error("ShmComm: bad collective");
  }
  if (d->in_bytes > cap_ || (kind != AG && d->out_bytes > cap_))
    throw std::runtime_error("ShmComm: collective of " + std::to_string(d->in_bytes) +
                             " bytes exceeds the communicator capacity of " +
                             std::to_string(cap_));
  return d;
}

void ShmComm::enqueue(int kind, const void* send, void* recv, size_t count, int dtype, int op,
                      int root, hipStream_t s) {
  if (!pinned_) throw std::runtime_error("ShmComm: a host-only communicator has no stream path");
  auto d = make_op(kind, send, recv, count, dtype, op, root);
  if (count == 0) return;
  // a captured op is replayed by every launch of its graph and lives as long
  // as the communicator; an eager one is freed by its host function
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(s, &cap));
  d->owned = cap == hipStreamCaptureStatusNone;
  const size_t in_bytes = d->in_bytes, out_bytes = d->out_bytes;
  if (in_bytes) HIP_CHECK(hipMemcpyAsync(send_stage_, send, in_bytes, hipMemcpyDeviceToHost, s));
  Op* raw = d.get();
  if (d->owned)
    d.release();  // from here on the host function owns it
  else
    ops_.push_back(std::move(d));
  HIP_CHECK(hipLaunchHostFunc(s, &ShmComm::host_fn, raw));
  if (out_bytes)
    HIP_CHECK(hipMemcpyAsync(recv, recv_stage_, out_bytes, hipMemcpyHostToDevice, s));
}

void ShmComm::run_host(int kind, const void* send, void* recv, size_t count, int dtype, int op,
                       int root) {
  auto d = make_op(kind, send, recv, count, dtype, op, root);
  if (count == 0) return;
  if (d->in_bytes) std::memcpy(send_stage_, send, d->in_bytes);
  exchange(*d);
  if (err_.load() != 0) throw std::runtime_error("ShmComm: " + error_message());
  if (d->out_bytes) std::memcpy(recv, recv_stage_, d->out_bytes);
}

void ShmComm::all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                         hipStream_t s) {
  enqueue(AR, send, recv, count, dtype, op, 0, s);
}

void ShmComm::all_gather(const void* send, void* recv, size_t send_count, int dtype,
                         hipStream_t s) {
  enqueue(AG, send, recv, send_count, dtype, ncclSum, 0, s);
}

void ShmComm::reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                             hipStream_t s) {
  enqueue(RS, send, recv, recv_count, dtype, op, 0, s);
}

void ShmComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root,
                        hipStream_t s) {
  enqueue(BC, send, recv, count, dtype, ncclSum, root, s);
}

void ShmComm::reduce(const void* send, void* recv, size_t count, int dtype, int op, int root,
                     hipStream_t s) {
  enqueue(RD, send, recv, count, dtype, op, root, s);
}
