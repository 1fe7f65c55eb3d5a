// Host-staged, hipGraph-capturable collectives for ranks that share a node
// through a shared-memory segment.
//
// The reference's ranks all run on /GPU:0 and exchange data through host
// memory (mpi4py Gather / Scatter on numpy buffers, /root/reference/mpipy.py:
// 121-127, :236-241; quirk Q13).  RCCL cannot place two ranks on one GPU, so
// this communicator carries that layout (--comm shm: several ranks per GPU)
// and lets every captured sync schedule of the executors run with real
// cross-rank data on ONE GPU.  Each collective is three stream operations,
// all of which a hipGraph captures:
//
//   hipMemcpyAsync D2H  (device send buffer -> this rank's pinned staging)
//   hipLaunchHostFunc   (the exchange: staging -> shared slot, barrier,
//                        reduce / gather in rank order, barrier; the host
//                        function makes NO HIP call)
//   hipMemcpyAsync H2D  (pinned result -> device receive buffer)
//
// Reductions run in fixed rank order (slot 0 + slot 1 + ...), chunked over
// the ranks, so every rank receives bit-identical sums; bf16 is summed in
// fp32 and rounded once (round to nearest even).  A rank whose peer never
// arrives gives up after `timeout_s`, raises the shared abort flag (the
// peers give up too) and reports it through async_error(), which the
// collective watchdog (parallel/watchdog.py) polls as it polls RCCL.  Every
// rank also publishes the signature of each collective (sequence number,
// kind, count, dtype, op, root); a peer issuing a different collective at
// the same position is a collective-order race and fails the communicator
// with ncclInvalidUsage instead of silently mixing buffers.
//
// Host functions of one process may run on ONE runtime thread, so a process
// must reach its blocking exchanges in the same order as its peers:
// host_progress() tells the executors to serialise the collectives of two
// communicators that they would otherwise run concurrently (SCHED_SPLIT).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <deque>
#include <memory>
#include <string>

#include "collective.h"

class ShmComm : public Collective {
 public:
  // path: a file on a tmpfs (/dev/shm/...) or any local filesystem.  The
  // creator (one rank) makes and sizes it; the others open it afterwards
  // (the caller orders creation before opening, e.g. with a gloo barrier).
  // capacity: largest per-rank contribution of one collective, in bytes.
  // pinned = false: plain host staging (no HIP call at all), for run_host()
  // only - host-memory collectives, usable without a GPU.
  ShmComm(const std::string& path, bool create, int nranks, int rank, size_t capacity,
          double timeout_s, bool pinned = true);
  ~ShmComm() override;
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;

  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  bool host_progress() const override { return true; }
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                  hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                  hipStream_t s) override;
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                      hipStream_t s) override;
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s);
  void reduce(const void* send, void* recv, size_t count, int dtype, int op, int root,
              hipStream_t s);

  // The same exchange, synchronously, on HOST buffers (no stream, no copies
  // to the device): kind = Kind value; for AG recv holds nranks x count.
  void run_host(int kind, const void* send, void* recv, size_t count, int dtype, int op, int root);

  // 0 = healthy; 5 (ncclInvalidUsage) = collective-order mismatch between
  // ranks; 6 (ncclRemoteError) = a peer timed out / aborted.
  int async_error() const { return err_.load(); }
  std::string error_message() const;
  void abort();  // raises the shared abort flag: every blocked exchange returns
  size_t capacity() const { return cap_; }
  long long completed() const { return done_.load(); }
  // Unlinks the backing file (call once every rank has opened it: the
  // mappings stay valid, nothing is left behind in /dev/shm).
  void unlink_path();

  enum Kind : int { AR = 1, AG = 2, RS = 3, BC = 4, RD = 5 };
  struct Op {
    ShmComm* comm;
    int kind, dtype, op, root;
    size_t count;     // elements: AR/RD/BC count, AG send count, RS recv count
    size_t in_bytes;  // bytes this rank contributes (0: none)
    size_t out_bytes; // bytes this rank receives (0: none)
    bool owned = false;  // eager launch: the host function frees the op
  };

 private:
  std::unique_ptr<Op> make_op(int kind, const void* send, const void* recv, size_t count,
                              int dtype, int op, int root) const;
  void enqueue(int kind, const void* send, void* recv, size_t count, int dtype, int op, int root,
               hipStream_t s);
  static void host_fn(void* arg);
  void exchange(const Op& d);
  bool barrier();
  void fail(int code, const std::string& why);
  char* slot(int r) const;
  char* result() const;

  int nranks_, rank_;
  size_t cap_;
  double timeout_s_;
  std::string path_;
  int fd_ = -1;
  size_t map_bytes_ = 0;
  void* map_ = nullptr;
  bool pinned_ = true;
  void* send_stage_ = nullptr;  // pinned, cap_ bytes
  void* recv_stage_ = nullptr;  // pinned, nranks_ * cap_ bytes
  std::deque<std::unique_ptr<Op>> ops_;  // ops of captured graphs (replayed later)
  unsigned long long seq_ = 0;           // host-function side sequence number
  std::atomic<int> err_{0};
  std::atomic<long long> done_{0};
  mutable std::atomic<int> msg_set_{0};
  char msg_[256] = {0};
};
