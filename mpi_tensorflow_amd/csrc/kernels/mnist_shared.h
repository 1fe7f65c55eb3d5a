// Device helpers and constants shared by the fp32 (mnist.hip) and bf16
// (mnist_bf16.hip) MNIST kernel sets.
#pragma once
#include "common.h"

namespace mnist {

constexpr int FC1_IN = 3136, FC1_OUT = 512, NCLS = 10;
constexpr int FC1_SPLITS = 14;  // train fc1 split-K slabs
constexpr int SMALL_BLOCKS = 8;  // blocks of the fc2 / bias grads role in fc1 backward

// reference batch offset (step * B) % (N_local - B) (/root/reference/mpipy.py:80)
__device__ __forceinline__ long long batch_offset_dev(const long long* step_ptr, int n_local,
                                                      int batch) {
  if (step_ptr == nullptr) return 0;
  long long s = *step_ptr;
  return (s * batch) % (long long)(n_local - batch);
}

// fc2 weight / bias and fc1 bias grads (B1, B2): dW4 = hd^T dlog, db4 = sum
// dlog, db3 = sum dh.  Block blk owns hidden units [64 blk, 64 blk + 64).
__device__ inline void fc1_small_grads(int blk, const float* hd, const float* dh, const float* dlog,
                                int batch, float* g_w4, float* g_b4, float* g_b3, float* smem) {
  // block blk handles hidden units j in [64 blk, 64 blk + 64); 4 row groups
  const int tid = threadIdx.x, jl = tid & 63, rg = tid >> 6;
  const int j = blk * 64 + jl;
  float acc[NCLS + 1];
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) acc[c] = 0.f;
  for (int n0 = rg; n0 < batch; n0 += 32) {  // 8 rows per round, loads issued together
    float hv[8], dv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int n = min(n0 + 4 * u, batch - 1);
      hv[u] = hd[n * FC1_OUT + j];
      dv[u] = dh[n * FC1_OUT + j];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int n = n0 + 4 * u;
      if (n < batch) {
#pragma unroll
        for (int c = 0; c < NCLS; ++c) acc[c] += hv[u] * dlog[n * NCLS + c];
        acc[NCLS] += dv[u];
      }
    }
  }
  float* s = smem;  // [4][11][64]
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) s[(rg * (NCLS + 1) + c) * 64 + jl] = acc[c];
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int c = 0; c <= NCLS; ++c) {
      const float v = s[c * 64 + jl] + s[((NCLS + 1) + c) * 64 + jl] +
                      s[(2 * (NCLS + 1) + c) * 64 + jl] + s[(3 * (NCLS + 1) + c) * 64 + jl];
      if (c < NCLS)
        g_w4[j * NCLS + c] = v;
      else
        g_b3[j] = v;
    }
  }
  if (blk == 0 && tid < NCLS) {
    float v = 0.f;
    for (int n = 0; n < batch; ++n) v += dlog[n * NCLS + tid];
    g_b4[tid] = v;
  }
}


}  // namespace mnist
