// Device-flag hand-offs between two streams of one process (a producer
// stream signals, a consumer stream waits), for overlap schedules inside
// captured graphs.  scripts/microbench/edge_lab.hip measured what an event
// edge costs in graph replay when the two branches really run at once:
// +15-18 us per step for one fork / join pair, against ~3 us for the same
// concurrency through a device flag with the streams forked once per graph
// (profiles/r5_edge_lab.txt).  parallel/overlap.py uses these for the
// bucketed all-reduce of the generic models.
//
// A flag is a monotonic counter: signal adds 1 after the producer stream's
// earlier kernels (agent-scope release first); wait advances its own expected
// count and polls until the counter reaches it (relaxed polls + an
// agent-scope acquire), so signals and waits pair up one to one in stream
// order, eagerly and in every graph replay.  The poll is bounded: after
// `timeout` it sets the error word and lets the stream go on (a hang-free
// failure the caller can see), e.g. if both branches ever landed on one
// hardware queue.
#include <stdexcept>

#include "common.h"
#include "mnist.h"

namespace optim {

__global__ __launch_bounds__(64) void flag_signal_kernel(unsigned* word) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(64) void flag_wait_kernel(const unsigned* word, unsigned* expect,
                                                       unsigned* error, long long timeout_ticks) {
  if (threadIdx.x == 0) {
    const unsigned e = *expect + 1u;
    *expect = e;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - e) < 0) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_fetch_or(error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

void launch_flag_signal(unsigned* word, hipStream_t s) { flag_signal_kernel<<<1, 64, 0, s>>>(word); }

void launch_flag_wait(const unsigned* word, unsigned* expect, unsigned* error, double timeout_s,
                      hipStream_t s) {
  if (!word || !expect || !error) throw std::runtime_error("flag_wait: null flag words");
  flag_wait_kernel<<<1, 64, 0, s>>>(word, expect, error, (long long)(timeout_s * 1e8));
}

}  // namespace optim
