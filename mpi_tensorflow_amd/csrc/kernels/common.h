// Shared device helpers for the gfx950 (CDNA4) kernel set.
//
// Wave = 64 lanes everywhere (hard-coded, see cdna_hip_programming.md §1).
// MFMA fragment maps used by every GEMM-shaped kernel here
// (v_mfma_f32_32x32x2_f32, f32 in / f32 accumulate, exact fp32):
//   A operand : lane l holds A[i = l & 31][k = l >> 5]
//   B operand : lane l holds B[k = l >> 5][j = l & 31]
//   C / D     : lane l, register r holds C[row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)]
//                                        [col = l & 31]
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define WAVE 64

// row length (elements) of the channel-major zero-padded bf16 activation
// images of the bf16 MNIST engine ([n][C][rows][MNIST16_T_LD])
#define MNIST16_T_LD 24
// ... and of the fp32 engine's channel-major zero-padded dY2 image ([n][64][18][MNIST32_T_LD])
#define MNIST32_T_LD 20

#define HIP_CHECK(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +  \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    }                                                                                \
  } while (0)

// row of accumulator register r for lane l (32x32 MFMA C/D layout)
__device__ __forceinline__ int mfma32_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for
// every outstanding global load (s_waitcnt vmcnt(0)): a prefetch issued before
// it (the next phase's operands) would be drained there instead of landing
// under the phase in between.  Global data exchanged between the waves of a
// block needs __syncthreads().
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ---------------------------------------------------------------- RNG ----
// Counter-based dropout RNG; identical to utils/rng.py (the oracle).
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t dropout_key(uint32_t seed, uint32_t rank,
                                                         uint32_t step, uint32_t salt) {
  uint32_t a = mix32(seed * 0x9E3779B9u + rank);
  return mix32(a ^ (step * 0x85EBCA6Bu + salt));
}

__device__ __forceinline__ bool dropout_keep(uint32_t key, uint32_t idx, float keep_prob) {
  uint32_t h = mix32(idx ^ key);
  float u = (float)(h >> 8) * (1.0f / 16777216.0f);
  return u < keep_prob;
}

// ------------------------------------------------------- reductions -------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Component-wise select of a vector struct.  `ok ? v : zero` on a
// HIP_vector_type (a struct) is lowered by clang to a select between two
// stack slots, i.e. scratch stores + a scratch load per element (it cost the
// bf16 conv loaders 24-48 B of scratch per thread); these stay in VGPRs.
__device__ __forceinline__ uint4 sel(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}
__device__ __forceinline__ uint2 sel(bool ok, uint2 v) {
  return make_uint2(ok ? v.x : 0u, ok ? v.y : 0u);
}
__device__ __forceinline__ float4 sel(bool ok, float4 v) {
  return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): consecutive logical tiles land on the
// same XCD (shared L2) instead of being dealt round-robin over 8 XCDs.  The
// dispatcher deals block b to XCD (b + o) mod 8 with o carried over from the
// previous launch (measured, tests/test_xgmi_gpu.py), so the ids of one XCD
// are those of one residue b mod 8 - the grouping below - whatever o is.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int NX = 8;
  if (nwg < NX) return bid;
  int q = nwg / NX, r = nwg % NX;
  int xcd = bid % NX, idx = bid / NX;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
