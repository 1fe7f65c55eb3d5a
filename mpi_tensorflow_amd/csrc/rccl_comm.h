// Native RCCL communicator (replaces the reference's mpi4py Scatter/Gather,
// /root/reference/mpipy.py:121-127, :236-241).
//
// RCCL is resolved at run time with dlopen from the librccl that the
// PyTorch-ROCm wheel already loaded (one HIP runtime and one RCCL per
// process), so there is no link-time dependency and no second runtime.
// Collectives are issued on a caller-provided HIP stream and are safe to
// capture into a hipGraph (the training step replays them).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "collective.h"

class RcclComm : public Collective {
 public:
  // Loads RCCL from `lib_path` (e.g. torch/lib/librccl.so).
  static void load(const std::string& lib_path);
  static bool loaded();
  static std::vector<char> unique_id();
  static int version();

  RcclComm(const std::vector<char>& uid, int nranks, int rank);
  ~RcclComm() override;
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const override { return rank_; }
  int size() const override { return nranks_; }

  // dtype: ncclDataType_t value; op: ncclRedOp_t value.
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                  hipStream_t s) override;
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s);
  void reduce(const void* send, void* recv, size_t count, int dtype, int op, int root,
              hipStream_t s);
  void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                  hipStream_t s) override;
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                      hipStream_t s) override;
  void group_start() override;
  void group_end() override;
  void destroy();
  // failure detection: ncclResult_t of the communicator's asynchronous state
  // (0 = ok, 7 = in progress), abort (idempotent, thread safe), rank count as
  // seen by RCCL itself
  int async_error() const;
  void abort();
  int comm_count() const;
  static std::string error_string(int code);

 private:
  ncclComm_t live() const;
  // Serialises every host call on the communicator against abort() /
  // destroy() from the watchdog thread: a collective never runs on a handle
  // that another thread is aborting or freeing.  abort() waits at most a few
  // seconds for it (the watchdog must still reach its exit), async_error()
  // not at all.
  mutable std::timed_mutex mu_;
  std::atomic<ncclComm_t> comm_{nullptr};
  std::atomic<bool> aborted_{false};
  int nranks_ = 0, rank_ = 0;
};
