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


// ------------------------------------------------------- bf16 shadows ----
// bf16 engine: the MFMA operand copies of the fp32 master weights (layouts in
// mnist_bf16.h), re-derived at the start of every step.  Blocks [0, 392): one
// 64x64 tile of W1 (fp32 [3136][512], rows i0.., cols j0..) -> w1b
// [j/16][i][16] and, through the LDS tile, w1t [i/16][j][16]; blocks
// [392, 442): 1024 conv2 weights each -> w2t [t][ci/16][co][16] and w2b
// [t][co/16][ci][16].  256 threads, `tile` = 64 x 65 floats of LDS.
struct ShadowPtrs {
  const float* w1;
  const float* w2;
  __bf16* w1b;
  __bf16* w1t;
  __bf16* w2t;
  __bf16* w2b;
};
constexpr int SHADOW_W1_BLOCKS = (FC1_IN / 64) * (FC1_OUT / 64), SHADOW_W2_BLOCKS = 51200 / 1024;
constexpr int SHADOW_BLOCKS = SHADOW_W1_BLOCKS + SHADOW_W2_BLOCKS;
constexpr int SHADOW_SMEM_FLOATS = 64 * 65;

__device__ __forceinline__ void shadow_store16(__bf16* dst, const float* v) {  // 16 floats -> 32 B
  __bf16 t[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) t[e] = (__bf16)v[e];
  const uint4* s4 = reinterpret_cast<const uint4*>(t);
  reinterpret_cast<uint4*>(dst)[0] = s4[0];
  reinterpret_cast<uint4*>(dst)[1] = s4[1];
}

__device__ inline void shadow_block(int L, const ShadowPtrs sp, float* tile) {
  const int tid = threadIdx.x;
  if (L < SHADOW_W1_BLOCKS) {
    const int i0 = (L % (FC1_IN / 64)) * 64, j0 = (L / (FC1_IN / 64)) * 64;
    {  // thread = (row i, 16-col chunk): 4 float4 loads, one 32 B store into w1b
      const int row = tid >> 2, ck = tid & 3;
      float v[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 f = *reinterpret_cast<const float4*>(sp.w1 + (size_t)(i0 + row) * FC1_OUT +
                                                           j0 + 16 * ck + 4 * u);
        v[4 * u] = f.x;
        v[4 * u + 1] = f.y;
        v[4 * u + 2] = f.z;
        v[4 * u + 3] = f.w;
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) tile[row * 65 + 16 * ck + e] = v[e];
      shadow_store16(sp.w1b + ((size_t)((j0 >> 4) + ck) * FC1_IN + i0 + row) * 16, v);
    }
    __syncthreads();
    {  // thread = (col j, 16-row chunk) -> w1t
      const int col = tid >> 2, ck = tid & 3;
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = tile[(16 * ck + e) * 65 + col];
      shadow_store16(sp.w1t + ((size_t)((i0 >> 4) + ck) * FC1_OUT + j0 + col) * 16, v);
    }
    return;
  }
  const int base = (L - SHADOW_W1_BLOCKS) * 1024;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = base + tid + 256 * e;  // HWIO: (t * 32 + ci) * 64 + co
    const __bf16 v = (__bf16)sp.w2[idx];
    const int t = idx >> 11, ci = (idx >> 6) & 31, co = idx & 63;
    sp.w2t[((t * 2 + (ci >> 4)) * 64 + co) * 16 + (ci & 15)] = v;
    sp.w2b[((t * 4 + (co >> 4)) * 32 + ci) * 16 + (co & 15)] = v;
  }
}

}  // namespace mnist
