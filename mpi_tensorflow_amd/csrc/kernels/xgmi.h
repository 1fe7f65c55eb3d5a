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
// same order, so per-block epochs agree.  Each XCD starts its blocks in
// increasing id order (block b goes to XCD (b + o) mod 8, o where the
// dispatcher's round robin stood after the previous launch - it differs
// between ranks), so the lowest unfinished block id is resident on every rank:
// all lower ids have finished everywhere, so nothing is ahead of it in its
// XCD's queue on any rank.  It passes its barriers and finishes, and by
// induction so does every block: no deadlock for any grid size.
// tests/test_xgmi_gpu.py checks that dispatch order on the box
// (dispatch_probe_kernel).
//
// Memory model (scoped, HIP / LLVM AMDGPU).  Every byte a peer reads goes
// through system-scope ("sc0 sc1") 16-byte buffer loads, and every byte a
// kernel publishes to its peers goes through system-scope stores
// (write-through): the same cache treatment the LLVM memory model gives
// system-scope atomics, so no L2-wide fence is needed on either side (an
// acquire fence would invalidate the whole XCD's L2 under the conv blocks that
// share it; measured: the conv2 backward launch 31 -> 45 us with them):
//   publish: every storing wave `s_waitcnt vmcnt(0)` -> workgroup barrier ->
//            relaxed system-scope flag stores (data from EARLIER kernels: a
//            system-scope release fence first, `release`);
//            `s_waitcnt vmcnt(0)` after the fence (MI355X_MICROARCH.md: the
//            compiler may drop the wait after the write-back)
//   consume: relaxed system-scope flag polls (bounded) -> workgroup barrier
//            -> system-scope loads of the peer bytes
// Every spin is bounded: a peer that never arrives sets the error word
// (XgmiComm::error()) and the kernel runs to its end instead of hanging.
//
// Emulation (one GPU, `emulate`): the N - 1 peers are local stand-in buffers,
// a block's flag stores go to its own array for every source slot, and each
// phase lasts at least the time its bytes take on one xGMI link
// (`link_ticks_per_mib`), plus `lat_ticks` per barrier, so schedules can be
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
  // emulated link time per MiB per link, in 100 MHz ticks (a MiB keeps the
  // rounding below 0.1 % at any xGMI rate: 150 GB/s = 699 ticks)
  long long link_ticks_per_mib = 0;
  long long timeout_ticks = 1000000000;       // 10 s
  // the ranks share ONE GPU (tests): launch few spinning blocks, so a rank
  // waiting at a barrier leaves CUs for the other ranks' kernels on the device
  int lean = 0;
  // emulation, failure injection: this virtual rank never arrives (its flag
  // slots stay unwritten), so every barrier times out (-1: none)
  int dead_rank = -1;
  // failure injection (tests, any communicator): the reductions leave out rank
  // skip_peer's contribution (-1: none), on every rank that has it set - rank
  // skip_peer itself included, as if its gradients never arrived anywhere.
  // Every rank then ends with the same wrong sums - identical replicas - which
  // only an exactness check can see (parallel/comm.py xgmi_exactness_check)
  int skip_peer = -1;
};

// rank r's contribution enters a reduction on this rank
__device__ __forceinline__ bool contributes(const Sync& s, int r) {
  return r < s.nranks && r != s.skip_peer;
}

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
// every rank's block blockIdx.x to arrive too.  All threads of the block call
// it.  release: this block's arrival also publishes plain stores of EARLIER
// kernels (a system-scope release fence; the kernels' own peer-visible stores
// are system-scope stores and need none).
__device__ __forceinline__ void barrier(const Sync& s, int stage, unsigned e, bool release) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  if (t < 64) {
    if (release) {
      if (t == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (t < s.nranks) {
      unsigned* dst = s.emulate ? s.flags + flag_slot(stage, t, b)
                                : s.peer_flags[t] + flag_slot(stage, s.rank, b);
      if (!(s.emulate && t == s.dead_rank))
        __hip_atomic_store(dst, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned* src = s.flags + flag_slot(stage, t, b);
      const long long t0 = now_ticks();
      // fail fast: once any barrier of this communicator timed out, later ones
      // do not wait again (the caller sees the sticky error and drops the path)
      const bool failed = __hip_atomic_load(s.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      while (!failed &&
             (int)(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
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
  }
  __syncthreads();
}

// ---- system-scope ("sc0 sc1") 16 / 4-byte accesses of peer-visible memory.
// Buffer descriptors over [base, base + bytes) (< 4 GiB), offsets in bytes.
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kSysCpol = 1 | 16;  // sc0 | sc1: system scope

__device__ __forceinline__ Rsrc rsrc(const void* base, long long bytes) {
  const long long lim = 0xffffffffLL;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < lim ? bytes : lim), 0x00020000);
}
__device__ __forceinline__ float4 ld4_sys(Rsrc r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kSysCpol));
}
__device__ __forceinline__ void st4_sys(Rsrc r, unsigned off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0)), v),
                                         r, (int)off, 0, kSysCpol);
}
__device__ __forceinline__ float ld_sys(Rsrc r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, kSysCpol));
}
__device__ __forceinline__ void st_sys(Rsrc r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, kSysCpol);
}

// a phase-1 operand: rank r's value, or 0 when the skip-peer fault leaves it out
__device__ __forceinline__ float4 ld4_peer(const Sync& s, int r, Rsrc rs, unsigned off) {
  return contributes(s, r) ? ld4_sys(rs, off) : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ float ld_peer(const Sync& s, int r, Rsrc rs, unsigned off) {
  return contributes(s, r) ? ld_sys(rs, off) : 0.f;
}

// emulation: hold the block until `bytes` (a whole phase's bytes on ONE
// link: every block of the phase shares the links) would have crossed an xGMI
// link since t0 (no-op on real peers)
__device__ __forceinline__ void link_floor(const Sync& s, long long t0, long long bytes) {
  if (!s.emulate || s.link_ticks_per_mib <= 0) return;
  const long long until = t0 + (bytes * s.link_ticks_per_mib) / (1LL << 20);
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
  // reduce-scatter: phase 1 only, the reduced segment of this rank goes to
  // `out` (local, seg4 float4s) instead of back into buf (no phase 2)
  float* out = nullptr;
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
// nt: threads per block (64 for small buffers: more blocks, each with one
// float4 a thread in flight per rank; 256 otherwise)
void launch_allreduce(const AllReduceArgs& a, int blocks, int nt, hipStream_t st);
// One-shot all-reduce + momentum SGD for small buffers (LeNet-5's 62 K
// parameters: the two-phase launch's two barriers and two dependent memory
// phases cost ~13 us for 248 KB).  Every rank's gradient lives in slot
// (*step) & 1 of a double-buffered registered buffer g2 [2][n4 float4s]
// (the update launch writes it there); after ONE arrival barrier each block
// loads its float4s of every rank's slot (all in flight), sums them in rank
// order and applies the replicated SGD (optim::sgd_momentum_flat's forms) to
// its params / momentum.  Each link carries the whole buffer once (vs 2 x
// 1/N of it), which is nothing at this size.  No closing barrier: a peer
// rewrites slot p two steps later, after the next launch's arrival barrier,
// which this rank's blocks reach only once this launch has completed.  The
// step is bumped by the last block to finish (a completion ticket on `done`),
// after every block has read it for the parity.
struct OneShotArgs {
  Sync s;
  const float* g[kMaxRanks] = {};  // every rank's g2, mapped here ([rank] local)
  float* w = nullptr;              // this rank's params / momentum
  float* mom = nullptr;
  long long n4 = 0;                // float4s of ONE slot
  const float* lr = nullptr;
  float momentum = 0.f, gscale = 1.f;
  long long* step = nullptr;       // read for the slot parity, bumped once
  unsigned* done = nullptr;        // zeroed completion counter (reset by the last block)
};
void launch_oneshot_sgd(const OneShotArgs& a, hipStream_t st);
// test: per-block XCD and per-XCD start ticket (the dispatch-order assumption)
void launch_dispatch_probe(unsigned* ctr, unsigned long long* out, int blocks,
                           long long spin_ticks, hipStream_t st);

}  // namespace xgmi
