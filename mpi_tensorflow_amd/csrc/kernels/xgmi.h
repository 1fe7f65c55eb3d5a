// Device side of the xGMI peer-to-peer communicator (csrc/xgmi_comm.h).
//
// On an MI355X node every GPU has a direct xGMI link to each of the 7 others,
// so a collective does not need a ring: rank r reads its 1/N segment of a
// buffer straight out of every peer's memory (IPC-mapped), reduces it, and the
// peers read the reduced segment back the same way.  Each link then carries
// S/N bytes per phase in each direction, all links at once, from kernels on
// the COMPUTE stream (no comm stream, no cross-queue graph edge).
//
// Ranks synchronise per workgroup: block b of every rank publishes an epoch
// into slot [stage][me][b] of every rank's flag array (uncached device memory,
// written by remote stores) and waits until slots [stage][r][b] of its own
// array hold that epoch for every r.  All ranks launch the same grids in the
// same order, so per-block epochs agree; blocks are dispatched in increasing
// id order on every GPU, so the lowest waiting block always has its peers
// resident (no deadlock for any grid size).
//
// Memory model (scoped, HIP / LLVM AMDGPU):
//   publish: every storing wave `s_waitcnt vmcnt(0)` -> workgroup barrier ->
//            lane 0 SYSTEM-scope release fence (writes back this XCD's L2) ->
//            `s_waitcnt vmcnt(0)` (MI355X_MICROARCH.md: the compiler may drop
//            the wait after the write-back) -> relaxed system-scope flag stores
//   consume: relaxed system-scope flag polls (bounded) -> SYSTEM-scope
//            acquire fence -> `s_waitcnt vmcnt(0)` -> workgroup barrier ->
//            plain loads of peer memory
// Every spin is bounded: a peer that never arrives sets the error word
// (XgmiComm::error()) and the kernel runs to its end instead of hanging.
//
// Emulation (one GPU, `emulate`): the N - 1 peers are local stand-in buffers,
// a block's flag stores go to its own array for every source slot, and each
// phase lasts at least the time its bytes take on one xGMI link
// (`link_ticks_per_kb`), plus `lat_ticks` per barrier, so schedules can be
// timed before a multi-GPU node is available.  Numerics of an emulated run
// are NOT those of N ranks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xgmi {

constexpr int kMaxRanks = 8;       // one node: 8 GPUs on a full xGMI mesh
constexpr int kMaxBlocks = 2048;   // flag slots per (stage, source rank)
constexpr int kStages = 3;  // arrive / reduced / done

__host__ __device__ constexpr int flag_slot(int stage, int src, int blk) {
  return (stage * kMaxRanks + src) * kMaxBlocks + blk;
}
constexpr size_t kFlagWords = (size_t)kStages * kMaxRanks * kMaxBlocks;

struct Sync {
  int nranks = 1, rank = 0;
  unsigned* flags = nullptr;                  // this rank's flag array (uncached)
  unsigned* peer_flags[kMaxRanks] = {};       // every rank's flag array, mapped here
  unsigned* epoch = nullptr;                  // per-block epoch counters (local)
  unsigned* error = nullptr;                  // bit 0: a barrier timed out
  int emulate = 0;
  long long lat_ticks = 0;                    // emulated hop latency (100 MHz ticks)
  long long link_ticks_per_kb = 0;            // emulated link time per KiB per link
  long long timeout_ticks = 1000000000;       // 10 s
  // the ranks share ONE GPU (tests): launch few spinning blocks, so a rank
  // waiting at a barrier leaves CUs for the other ranks' kernels on the device
  int lean = 0;
};

__device__ __forceinline__ long long now_ticks() {
  return (long long)__builtin_amdgcn_s_memrealtime();  // 100 MHz, shader-clock independent
}

// thread 0 advances this block's epoch; every thread gets the new value
__device__ __forceinline__ unsigned next_epoch(const Sync& s, unsigned* lds) {
  if (threadIdx.x == 0) {
    const unsigned e = s.epoch[blockIdx.x] + 1u;
    s.epoch[blockIdx.x] = e;
    *lds = e;
  }
  __syncthreads();
  return *lds;
}

// Publishes this block's arrival at (stage, e) to every rank and waits for
// every rank's block blockIdx.x to arrive too.  All threads of the block call it.
__device__ __forceinline__ void barrier(const Sync& s, int stage, unsigned e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  if (t < 64) {
    if (t == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t < s.nranks) {
      unsigned* dst = s.emulate ? s.flags + flag_slot(stage, t, b)
                                : s.peer_flags[t] + flag_slot(stage, s.rank, b);
      __hip_atomic_store(dst, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned* src = s.flags + flag_slot(stage, t, b);
      const long long t0 = now_ticks();
      while ((int)(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (now_ticks() - t0 > s.timeout_ticks) {
          __hip_atomic_fetch_or(s.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (s.emulate && s.lat_ticks > 0) {
        const long long t1 = now_ticks();
        while (now_ticks() - t1 < s.lat_ticks) __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// emulation: hold the block until `bytes` (a whole phase's bytes on ONE
// link: every block of the phase shares the links) would have crossed an xGMI
// link since t0 (no-op on real peers)
__device__ __forceinline__ void link_floor(const Sync& s, long long t0, long long bytes) {
  if (!s.emulate || s.link_ticks_per_kb <= 0) return;
  const long long until = t0 + (bytes * s.link_ticks_per_kb) / 1024;
  if (threadIdx.x == 0)
    while (now_ticks() < until) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
}

// In-place fp32 sum all-reduce of a registered buffer (XgmiComm::all_reduce):
// phase 1 - block b of rank r sums float4s [b * per4, (b + 1) * per4) of
// segment r over every rank (rank order 0..N-1, as a host reduction in rank
// order would) and writes them in place; phase 2 - it copies the same slice
// of every other segment from its owner; a third barrier keeps the buffer
// unmodified until every peer has read this rank's segment.
struct AllReduceArgs {
  Sync s;
  float* buf[kMaxRanks] = {};  // every rank's buffer, mapped here ([rank] local)
  long long n4 = 0;            // float4s in the buffer
  long long seg4 = 0;          // float4s per rank segment (last one may be short)
  int per4 = 0;                // float4s per block per segment
  long long link_bytes = 0;    // one phase's bytes on one link (emulation floor)
  int gather_only = 0;         // skip phase 1: every rank's segment is already final
  // momentum SGD fused into phase 1 (all_reduce_sgd): buf = the grads; the
  // reduced segment updates w[rank] / mom there (optim::sgd_momentum_flat's
  // forms; L2 on float4s < l2_end4), and phase 2 gathers w instead of buf
  float* w[kMaxRanks] = {};
  float* mom = nullptr;
  const float* lr = nullptr;
  float momentum = 0.f, gscale = 1.f, l2 = 0.f;
  long long l2_end4 = 0;
  long long* step = nullptr;  // bumped once (optional)
};
void launch_allreduce(const AllReduceArgs& a, int blocks, hipStream_t st);

}  // namespace xgmi
