// Timing kernel of EmuComm (collective.h): stands in for an RCCL collective
// kernel on a single GPU - it holds `blocks` workgroups (RCCL runs one
// workgroup per channel) and the stream for a given wall time, and streams
// the local buffer once (the local HBM traffic of a ring step).
#include "../collective.h"
#include "common.h"

namespace commemu {

__global__ __launch_bounds__(256) void occupy_kernel(float4* __restrict__ buf, long long n4,
                                                     long long ticks) {
  // s_memrealtime: constant 100 MHz clock, independent of the shader clock
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (long long)gridDim.x * 256) {
    const float4 v = buf[i];
    buf[i] = v;
  }
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

void launch_occupy(void* buf, size_t bytes, double us, int blocks, hipStream_t s) {
  const long long ticks = (long long)(us * 100.0);
  occupy_kernel<<<blocks > 0 ? blocks : 1, 256, 0, s>>>(reinterpret_cast<float4*>(buf),
                                                        (long long)(bytes / 16), ticks);
}

}  // namespace commemu
