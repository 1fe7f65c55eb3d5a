// Grid-wide barrier for launches whose blocks are all resident at once, and
// the coherent hand-off of data between the phases it separates.
//
// MI355X has one L2 per XCD: a plain store lands in the writer's XCD L2 and a
// plain load on another XCD may hit a stale line of its own L2.  Across a
// kernel boundary the runtime's release / acquire make that coherent; inside
// one launch the data handed from one phase to the next goes through
// system-scope ("sc0 sc1") buffer stores and loads (xgmi.h ld_sys / st_sys:
// write-through, and a read that misses every cache), so no L2-wide fence is
// needed (a device-scope release fence per block writes back the whole XCD
// L2: 4x slower in bn.hip's first fused form).
//
// User: bn.hip's opt-in fused BatchNorm finalize + apply (bn_set_fused).
// Measured (PERF_NOTES round 6): on MI355X a barrier plus the uncached
// hand-offs cost more than the kernel boundary they replace inside a hipGraph
// - the fused BatchNorm and an MNIST FC chain (fc1 forward, loss head, fc1
// backward in one launch: 29.1 us against 21.1 us for the three launches)
// were both slower, so neither is the default.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>

#include "xgmi.h"

namespace gsync {

struct GridBar {
  unsigned* cnt;  // arrivals of the current barrier (reset by the last one)
  unsigned* gen;  // barrier generation
  unsigned* err;  // sticky: a spin timed out (2 s)
};

// Every thread of every block calls it.  Stores this thread published with
// st_sys are complete before its block arrives (s_waitcnt); the last block to
// arrive resets the count and opens the next generation.  The launch must
// keep gridDim.x <= the blocks the CUs hold at once (hipOccupancy... x CUs).
__device__ __forceinline__ void grid_barrier(const GridBar& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned t = __hip_atomic_fetch_add(b.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(b.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(b.gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      // (after one timeout the state is suspect: later barriers do not wait,
      // so a grid that could not be resident ends in ms, flagged, not in hours)
      const long long t0 = xgmi::now_ticks();
      while (__hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (xgmi::now_ticks() - t0 > 200000000LL) {
          __hip_atomic_fetch_or(b.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  __syncthreads();
}

// The barrier state of the including translation unit: a zero-initialised
// device array (three 64-byte lines), so no allocation, memset or device sync
// is needed - the first launch may come while a stream is being captured.
static __device__ unsigned gsync_state_[48];

static inline GridBar tu_bar() {  // internal linkage: one per TU, as gsync_state_
  static GridBar b{nullptr, nullptr, nullptr};
  if (!b.cnt) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(gsync_state_)) != hipSuccess || !p)
      throw std::runtime_error("gsync: barrier state symbol not found");
    unsigned* u = static_cast<unsigned*>(p);
    b = {u, u + 16, u + 32};
  }
  return b;
}

// host: the number of CUs; the sticky timeout word (synchronises the device)
int cu_count();
unsigned bar_error(const GridBar& b);

}  // namespace gsync
