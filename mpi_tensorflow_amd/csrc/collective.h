// Device-collective interface of the step executors.
//
// The executors issue their gradient / parameter collectives through this
// interface, on a HIP stream, inside the captured step.  Three implementations:
//   RcclComm (rccl_comm.h) - RCCL over xGMI, the production path;
//   ShmComm  (shm_comm.h)  - host-staged exchange through shared memory for
//                            ranks that share a GPU (capturable: D2H copy,
//                            host function, H2D copy);
//   EmuComm  (below)       - a timing stand-in for an N-rank communicator on
//                            ONE GPU, used to measure how a comm schedule
//                            overlaps with the compute stream before the
//                            multi-GPU node is available (bench.py
//                            --comm-emulate).  It moves no data between ranks
//                            (the numerics of an emulated run are NOT those
//                            of N ranks); it only occupies `blocks`
//                            workgroups and the stream for the time a ring
//                            collective of that size would take.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

class Collective {
 public:
  virtual ~Collective() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // dtype: ncclDataType_t value; op: ncclRedOp_t value.  In-place forms are
  // allowed as in RCCL (reduce_scatter: recv == send + rank * recv_count;
  // all_gather: send == recv + rank * send_count).
  virtual void all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                          hipStream_t s) = 0;
  virtual void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                          hipStream_t s) = 0;
  virtual void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                              hipStream_t s) = 0;
  // Collectives issued between group_start() and group_end() form ONE fused
  // operation (ncclGroupStart / ncclGroupEnd): one launch and one latency for
  // several buffers.  Implementations without grouping run them one by one.
  virtual void group_start() {}
  virtual void group_end() {}
  // True when the collectives make progress in blocking host functions
  // (ShmComm): the collectives of two such communicators must then be
  // reached in the same order on every rank, so a schedule that would run
  // them concurrently on two streams orders them instead.
  virtual bool host_progress() const { return false; }
};

// Ring cost model (rccl-tests conventions): an all-reduce of S bytes takes
// lat + 2 (N-1)/N * S / busbw; a reduce-scatter or all-gather whose FULL
// buffer is S bytes takes lat + (N-1)/N * S / busbw.
class EmuComm : public Collective {
 public:
  EmuComm(int nranks, int rank, double lat_us, double busbw_gbps, int blocks);
  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                  hipStream_t s) override;
  void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                  hipStream_t s) override;
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                      hipStream_t s) override;
  // grouped ops pay the latency term once (the first op of the group)
  void group_start() override { grouped_ = 0; in_group_ = true; }
  void group_end() override { in_group_ = false; }
  double all_reduce_us(size_t bytes) const;
  double gather_us(size_t full_bytes) const;  // reduce-scatter / all-gather

 private:
  void occupy(void* buf, size_t bytes, double us, hipStream_t s);
  double lat_once();  // lat_us_, or 0 after the first op of a group
  int nranks_, rank_, blocks_;
  double lat_us_, busbw_;
  bool in_group_ = false;
  int grouped_ = 0;
};

size_t dtype_bytes(int dtype);

namespace commemu {
// `blocks` workgroups touch `bytes` of buf (load + store in place) and stay
// resident until `us` microseconds have passed since they started.
void launch_occupy(void* buf, size_t bytes, double us, int blocks, hipStream_t s);
}  // namespace commemu
