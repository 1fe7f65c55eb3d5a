// Winograd F(2x2, 5x5) transforms for the fp32 MNIST conv2 (5x5, SAME, s1).
//
// Each 2x2 block of conv2 outputs is exactly one 2x2 max-pooling window of the
// reference model (/root/reference/mpipy.py:159-161), so the Winograd output
// tile IS the pool window: the output transform ends in the pool + argmax
// epilogue.  Per tile the 5x5 correlation over 32 input channels becomes 36
// independent channel products (a batched [tiles x 32] x [32 x 64] GEMM on
// the matrix cores) instead of 25 taps x 4 outputs: 2.78x fewer MFMAs.
//
// Toom-Cook points {0, 1, -1, 2, -1/2, inf} (Lavin & Gray 2016):
//   Y = AT [ (G g G^T) .* (BT d BT^T) ] AT^T
// d: 6x6 input window at (2 py - 2, 2 px - 2), g: 5x5 filter (HWIO slice),
// correlation convention (TF Conv2D).  Measured fp32 error on random data vs
// an fp64 reference: ~1.4e-6 relative (mean), 6e-6 (max) over 32 channels;
// direct fp32 summation: 1.5e-7 / 4e-7 (scripts/wino_check.py).  Every step
// is fp32 arithmetic; only the algorithm differs from the 25-tap sum, as with
// cuDNN's Winograd convolutions.
//
// All coefficients are compile-time constants: with the loops fully unrolled
// the zero terms fold away and products by +-1 become adds.
#pragma once

namespace wino {

constexpr int A = 6;  // transform size m + r - 1
constexpr float kBT[6][6] = {
    {1.f, 1.5f, -2.f, -1.5f, 1.f, 0.f},  {0.f, -1.f, -2.5f, -0.5f, 1.f, 0.f},
    {0.f, 1.f, 0.5f, -2.5f, 1.f, 0.f},   {0.f, -0.5f, -1.f, 0.5f, 1.f, 0.f},
    {0.f, 2.f, -1.f, -2.f, 1.f, 0.f},    {0.f, 1.f, 1.5f, -2.f, -1.5f, 1.f}};
constexpr float kG[6][5] = {{1.f, 0.f, 0.f, 0.f, 0.f},
                            {-1.f / 3, -1.f / 3, -1.f / 3, -1.f / 3, -1.f / 3},
                            {1.f / 3, -1.f / 3, 1.f / 3, -1.f / 3, 1.f / 3},
                            {1.f / 15, 2.f / 15, 4.f / 15, 8.f / 15, 16.f / 15},
                            {-16.f / 15, 8.f / 15, -4.f / 15, 2.f / 15, -1.f / 15},
                            {0.f, 0.f, 0.f, 0.f, 1.f}};
constexpr float kAT[2][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f}, {0.f, 1.f, -1.f, 2.f, -0.5f, 1.f}};

// out[a] = sum_i kBT[a][i] in[i*stride]  (input side, 1-D)
template <int S_IN, int S_OUT>
__host__ __device__ __forceinline__ void bt6(const float* in, float* out) {
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i)
      if (kBT[a][i] != 0.f) s += kBT[a][i] * in[i * S_IN];
    out[a * S_OUT] = s;
  }
}

// out[a] = sum_k kG[a][k] in[k*stride]  (filter side, 1-D)
template <int S_IN, int S_OUT>
__host__ __device__ __forceinline__ void g6(const float* in, float* out) {
  // no FMA contraction: the filter transform is computed by several kernels
  // (the per-step transform and the fused SGD) and must round identically
#pragma clang fp contract(off)
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (kG[a][k] != 0.f) s += kG[a][k] * in[k * S_IN];
    out[a * S_OUT] = s;
  }
}

// 2-D input transform of a 6x6 window (row-major, ld 6) -> 6x6
__host__ __device__ __forceinline__ void input_tile(const float* d, float* v) {
  float t[36];
#pragma unroll
  for (int j = 0; j < 6; ++j) bt6<6, 6>(d + j, t + j);  // columns: t = BT d
#pragma unroll
  for (int a = 0; a < 6; ++a) bt6<1, 1>(t + 6 * a, v + 6 * a);  // rows: v = t BT^T
}

// 2-D filter transform of a 5x5 filter (row-major, ld 5) -> 6x6
__host__ __device__ __forceinline__ void filter_tile(const float* g, float* u) {
  float t[30];
#pragma unroll
  for (int kw = 0; kw < 5; ++kw) g6<5, 5>(g + kw, t + kw);  // t[a][kw] = sum_kh G[a][kh] g[kh][kw]
#pragma unroll
  for (int a = 0; a < 6; ++a) g6<1, 1>(t + 5 * a, u + 6 * a);  // u[a][b] = sum_kw G[b][kw] t[a][kw]
}

// Output-transform weight of point (a, b) for output (i, j) of the 2x2 tile.
__host__ __device__ constexpr float out_coef(int a, int b, int i, int j) {
  return kAT[i][a] * kAT[j][b];
}

}  // namespace wino
