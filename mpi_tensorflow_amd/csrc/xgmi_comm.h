// xGMI peer-to-peer communicator: collectives as kernels on the caller's
// (compute) stream that read the peers' buffers directly over the xGMI mesh.
//
// Why (SURVEY.md §5 "Distributed communication backend"): the
// MNIST step is ~80 us, its 6.65 MB gradient all-reduce is as long as the
// step on an RCCL ring, and every RCCL overlap schedule pays cross-queue graph
// edges (~10 us each, scripts/microbench/edge_lab.hip).  On a fully connected
// 8-GPU node a two-phase direct exchange moves S/N bytes per link per phase on
// all 7 links at once, and it runs IN the compute stream - so the gradient sum
// can be fused with the momentum SGD that consumes it (MnistExecutor
// SCHED_XGMI: one launch reduces this rank's 1/N of the FC gradients from
// every rank, updates those parameters, and gathers everyone else's updated
// segments back).
//
// Buffers a kernel reads remotely are REGISTERED: each rank exports an IPC
// handle of the allocation that holds the buffer (+ offset), the handles are
// exchanged over the gloo bootstrap group (parallel/comm.py XgmiDeviceComm)
// and opened here.  The flag array lives in uncached device memory
// (hipDeviceMallocUncached) so remote flag stores are seen by local polls.
// All ranks must be on ONE node (xGMI); ranks sharing a GPU work too (the IPC
// mapping is then to the same device - the 2-rank GPU tests use that).
//
// Emulation (one GPU): make the communicator with emulate = true; every
// registered buffer gets N - 1 local stand-ins as the "peers", and the
// kernels hold each phase for the time its bytes take on one link
// (link_gbps per direction) plus lat_us per barrier.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "collective.h"
#include "kernels/xgmi.h"

class XgmiComm : public Collective {
 public:
  XgmiComm(int nranks, int rank, bool emulate, double lat_us, double link_gbps, double timeout_s);
  ~XgmiComm() override;
  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  bool emulated() const { return emulate_; }

  // --- set-up (collective through the caller's bootstrap group) ---
  std::string flags_handle() const;               // IPC handle of this rank's flag array
  void open_flags(int r, const std::string& handle);
  // IPC handle of the allocation holding [ptr, ptr + bytes) and ptr's offset in it
  std::pair<std::string, size_t> export_buffer(uintptr_t ptr, size_t bytes) const;
  // maps rank r's counterpart of the local buffer (handle / offset from its export_buffer)
  void open_buffer(uintptr_t local, size_t bytes, int r, const std::string& handle, size_t off);
  // emulation: N - 1 local stand-ins for the local buffer (copies of it)
  void emulate_buffer(uintptr_t local, size_t bytes);
  bool ready() const;  // flags of every rank mapped
  // the ranks share one GPU: the kernels keep their grids small (Sync::lean)
  void set_lean(bool on) { sync_.lean = on ? 1 : 0; }
  // emulation, failure injection: virtual rank r never arrives at a barrier
  void emulate_dead_rank(int r) {
    if (!emulate_) throw std::runtime_error("XgmiComm: dead-rank injection needs emulation");
    sync_.dead_rank = r;
  }
  bool lean() const { return sync_.lean != 0; }

  // --- device views ---
  const xgmi::Sync& sync() const { return sync_; }
  // rank r's counterpart of a local address inside a registered buffer
  void* peer_ptr(const void* local, int r) const;
  bool registered(const void* local, size_t bytes) const;
  // emulated per-phase floor: ticks of the 100 MHz clock per MiB on one link
  long long link_ticks_per_mib() const { return sync_.link_ticks_per_mib; }
  // failure injection (tests): phase-1 reductions leave out rank r (-1: off)
  void inject_skip_peer(int r) {
    if (r >= nranks_) throw std::runtime_error("XgmiComm: skip-peer rank out of range");
    sync_.skip_peer = r < 0 ? -1 : r;
  }
  int skip_peer() const { return sync_.skip_peer; }
  // emulation: writes `bytes` at src (device) into virtual rank r's stand-in of
  // the registered local buffer (the exactness check gives every virtual rank
  // its own contribution)
  void emulate_fill_peer(uintptr_t local, int r, uintptr_t src, size_t bytes);
  unsigned error() const;  // sticky error bits (1: a barrier timed out); synchronizes
  void clear_error();

  // --- Collective: in-place fp32 sum all-reduce of a registered buffer ---
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                  hipStream_t s) override;
  // recv (send_count x N floats) registered; send is copied into this rank's
  // slot first unless it is that slot
  void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                  hipStream_t s) override;
  // in place, fp32: segment r (ceil(count / N) floats, in float4s) of every
  // rank's buffer becomes rank r's (the all-reduce's phase 2 alone)
  void gather_segments(void* buf, size_t count, hipStream_t s);
  // in-place fp32 sum of the registered grads fused with the momentum SGD of
  // the registered params: each rank updates its own segment (the momentum is
  // sharded: gather_segments(mom) makes it whole) and gathers the others'
  // (optim::launch_sgd_momentum's arguments; bit-identical to all_reduce +
  // that SGD with a rank-order sum)
  void all_reduce_sgd(float* grads, float* params, float* mom, size_t count, long long l2_end,
                      float l2, float momentum, float gscale, const float* lr, long long* step,
                      hipStream_t s);
  // small buffers: the one-shot form (kernels/xgmi.h OneShotArgs) - grads2 is
  // the registered double-buffered gradient [2][count] whose slot (*step & 1)
  // the caller wrote this step; one barrier, every rank's slot summed in rank
  // order, the replicated SGD (bit-identical to all_reduce + that SGD with a
  // rank-order sum); *step bumped; done: a zeroed device counter
  void all_reduce_sgd_oneshot(const float* grads2, float* params, float* mom, size_t count,
                              float momentum, float gscale, const float* lr, long long* step,
                              unsigned* done, hipStream_t s);
  // send (recv_count x N floats) registered and left unchanged unless recv is
  // this rank's slot of it (in place: the reduced segment lands there)
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                      hipStream_t s) override;

 private:
  struct Reg {
    uintptr_t local = 0;
    size_t bytes = 0;
    void* peer[xgmi::kMaxRanks] = {};
  };
  const Reg* find(const void* p, size_t bytes) const;
  Reg& reg_for(uintptr_t local, size_t bytes);
  void* open_handle(int r, const std::string& handle);
  void launch(void* buf, size_t count, bool gather_only, hipStream_t s,
              const xgmi::AllReduceArgs* sgd = nullptr, float* out = nullptr);

  int nranks_, rank_;
  bool emulate_;
  xgmi::Sync sync_;
  unsigned* flags_ = nullptr;
  unsigned* epoch_ = nullptr;
  unsigned* error_ = nullptr;
  std::vector<Reg> regs_;
  std::map<std::pair<int, std::string>, void*> opened_;  // (rank, handle) -> mapped base
  std::vector<void*> emu_allocs_;
  std::vector<void*> opened_flags_;
};
