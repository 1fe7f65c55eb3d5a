// Generic NHWC layer kernels for the LeNet-5 / ResNet-18 configs (BASELINE.json
// configs 4-5) on gfx950: the per-element gather implicit-GEMM convolution
// (forward with fused bias + ReLU, backward-data, backward-filter with
// split-K slabs) for shapes the LDS-tiled family (conv_tiled.hip) does not
// take, max / global average pooling, fused softmax cross-entropy, batch
// gather and slab reduction.  BatchNorm lives in bn.hip.  Linear layers are
// 1x1 convolutions over a 1x1 image.
//
// Every GEMM-shaped op runs on v_mfma_f32_32x32x2_f32 through gemm_core.h;
// shapes are runtime values (one code object serves every layer), with the
// per-slot address decode hoisted out of the K loop by the gather contexts.
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "gemm_core.h"
#include "ops_generic.h"

namespace gops {

// ---------------------------------------------------------------- conv ----
struct ConvFwdProb {
  static constexpr bool A_KC = true, B_NC = true;
  struct ACtx {
    const float* img;  // x + n*H*W*C + ci0 (slot's channel inside the tile)
    int iy0, ix0, kl;
    bool v;
  };
  struct BCtx {
    const float* p;
    int kl;
    bool v;
  };
  ConvShape s;
  const float* x;
  const float* w;
  int Ktot, M;
  __device__ __forceinline__ ACtx a_ctx(int m, int kl) const {
    const bool v = m < M;
    const int mm = v ? m : 0;
    const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
    return {x + (size_t)n * s.H * s.W * s.C, oy * s.stride - s.pad, ox * s.stride - s.pad, kl, v};
  }
  __device__ __forceinline__ float a_get(const ACtx& c, int k0) const {
    const int k = k0 + c.kl;
    const int ci = k % s.C, t = k / s.C;
    const int kh = t / s.S, kw = t % s.S;
    const int iy = c.iy0 + kh, ix = c.ix0 + kw;
    const bool ok = c.v && k < Ktot && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
    const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
    const float val = c.img[(iyc * s.W + ixc) * s.C + ci];
    return ok ? val : 0.f;
  }
  __device__ __forceinline__ BCtx b_ctx(int kl, int n) const {
    const bool v = n < s.K;
    return {w + (v ? n : 0), kl, v};
  }
  __device__ __forceinline__ float b_get(const BCtx& c, int k0) const {
    const int k = k0 + c.kl;
    const float val = c.p[(size_t)min(k, Ktot - 1) * s.K];
    return (c.v && k < Ktot) ? val : 0.f;
  }
};

// dX[n,iy,ix,ci] = sum_{kh,kw,co} dY[n,oy,ox,co] W[kh,kw,ci,co], iy = oy*s - p + kh
struct ConvDataProb {
  static constexpr bool A_KC = true, B_NC = false;
  struct ACtx {
    const float* img;  // dy + n*OH*OW*K
    int iyp, ixp, kl;  // iy + pad, ix + pad
    bool v;
  };
  struct BCtx {
    const float* p;  // w + ci*K
    int kl;
    bool v;
  };
  ConvShape s;
  const float* dy;
  const float* w;
  int Ktot, M;  // Ktot = R*S*K (co fastest)
  __device__ __forceinline__ ACtx a_ctx(int m, int kl) const {
    const bool v = m < M;
    const int mm = v ? m : 0;
    const int ix = mm % s.W, t = mm / s.W, iy = t % s.H, n = t / s.H;
    return {dy + (size_t)n * s.OH * s.OW * s.K, iy + s.pad, ix + s.pad, kl, v};
  }
  __device__ __forceinline__ float a_get(const ACtx& c, int k0) const {
    const int k = k0 + c.kl;
    const int co = k % s.K, t = k / s.K;
    const int kh = t / s.S, kw = t % s.S;
    const int ny = c.iyp - kh, nx = c.ixp - kw;
    const int oy = ny / s.stride, ox = nx / s.stride;
    const bool ok = c.v && k < Ktot && ny >= 0 && nx >= 0 && oy * s.stride == ny &&
                    ox * s.stride == nx && oy < s.OH && ox < s.OW;
    const int oyc = min(max(oy, 0), s.OH - 1), oxc = min(max(ox, 0), s.OW - 1);
    const float val = c.img[(oyc * s.OW + oxc) * s.K + co];
    return ok ? val : 0.f;
  }
  __device__ __forceinline__ BCtx b_ctx(int kl, int n) const {
    const bool v = n < s.C;
    return {w + (size_t)(v ? n : 0) * s.K, kl, v};
  }
  __device__ __forceinline__ float b_get(const BCtx& c, int k0) const {
    const int k = min(k0 + c.kl, Ktot - 1);
    const int co = k % s.K, t = k / s.K;
    const float val = c.p[(size_t)t * s.C * s.K + co];
    return (c.v && k0 + c.kl < Ktot) ? val : 0.f;
  }
};

// dW[(kh,kw,ci)][co] = sum_pix X[n, oy*s+kh-p, ox*s+kw-p, ci] dY[pix][co]
struct ConvFilterProb {
  static constexpr bool A_KC = false, B_NC = true;
  struct ACtx {
    int kh, kw, ci, kl;
    bool v;
  };
  struct BCtx {
    const float* p;
    int kl;
    bool v;
  };
  ConvShape s;
  const float* x;
  const float* dy;
  int Mw, npix;  // Mw = R*S*C
  __device__ __forceinline__ ACtx a_ctx(int m, int kl) const {
    const bool v = m < Mw;
    const int mm = v ? m : 0;
    const int ci = mm % s.C, t = mm / s.C;
    return {t / s.S, t % s.S, ci, kl, v};
  }
  __device__ __forceinline__ float a_get(const ACtx& c, int k0) const {
    const int pix = k0 + c.kl;
    const int pc = min(pix, npix - 1);
    const int ox = pc % s.OW, t = pc / s.OW, oy = t % s.OH, n = t / s.OH;
    const int iy = oy * s.stride + c.kh - s.pad, ix = ox * s.stride + c.kw - s.pad;
    const bool ok = c.v && pix < npix && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
    const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
    const float val = x[(((size_t)n * s.H + iyc) * s.W + ixc) * s.C + c.ci];
    return ok ? val : 0.f;
  }
  __device__ __forceinline__ BCtx b_ctx(int kl, int n) const {
    const bool v = n < s.K;
    return {dy + (size_t)kl * s.K + (v ? n : 0), kl, v};
  }
  __device__ __forceinline__ float b_get(const BCtx& c, int k0) const {
    const int pix = k0 + c.kl;
    const float val = c.p[(size_t)(min(pix, npix - 1) - c.kl) * s.K];
    return (c.v && pix < npix) ? val : 0.f;
  }
};

constexpr int WM = 2, WN = 2, BK = 32;
using CFG_F = gemm::Cfg<WM, WN, 1, BK, true, true>;

__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvShape s, const float* __restrict__ x,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ y, int relu) {
  __shared__ float smem[CFG_F::SMEM_FLOATS];
  const int M = s.N * s.OH * s.OW, Ktot = s.R * s.S * s.C;
  ConvFwdProb p{s, x, w, Ktot, M};
  const int mt = (M + CFG_F::BM - 1) / CFG_F::BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * CFG_F::BM, n0 = (bid / mt) * CFG_F::BN;
  const int kend = (Ktot + BK - 1) / BK * BK;
  f32x16 acc;
  int wm, wn;
  gemm::run_tile<WM, WN, 1, BK>(p, smem, m0, n0, 0, kend, acc, wm, wn);
  const int lane = threadIdx.x & 63;
  const int co = n0 + 32 * wn + (lane & 31);
  if (co >= s.K) return;
  const float b = bias ? bias[co] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + 32 * wm + mfma32_row(r, lane);
    if (m >= M) continue;
    float v = acc[r] + b;
    if (relu) v = fmaxf(v, 0.f);
    y[(size_t)m * s.K + co] = v;
  }
}

using CFG_D = gemm::Cfg<WM, WN, 1, BK, true, false>;
__global__ __launch_bounds__(256) void conv_bwd_data_kernel(ConvShape s,
                                                            const float* __restrict__ dy,
                                                            const float* __restrict__ w,
                                                            float* __restrict__ dx, int kchunk) {
  // split-K over gridDim.y (kchunk K per slice): slice y writes the raw slab
  // dx + y * M * C, summed by slab_sum_kernel
  __shared__ float smem[CFG_D::SMEM_FLOATS];
  const int M = s.N * s.H * s.W, Ktot = s.R * s.S * s.K;
  ConvDataProb p{s, dy, w, Ktot, M};
  const int mt = (M + CFG_D::BM - 1) / CFG_D::BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * CFG_D::BM, n0 = (bid / mt) * CFG_D::BN;
  const int kend = (Ktot + BK - 1) / BK * BK;
  const int kb = blockIdx.y * kchunk, ke = min(kend, kb + kchunk);
  dx += (size_t)blockIdx.y * M * s.C;
  f32x16 acc;
  int wm, wn;
  gemm::run_tile<WM, WN, 1, BK>(p, smem, m0, n0, kb, ke, acc, wm, wn);
  const int lane = threadIdx.x & 63;
  const int ci = n0 + 32 * wn + (lane & 31);
  if (ci >= s.C) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + 32 * wm + mfma32_row(r, lane);
    if (m < M) dx[(size_t)m * s.C + ci] = acc[r];
  }
}

using CFG_W = gemm::Cfg<WM, WN, 1, BK, false, true>;
__global__ __launch_bounds__(256) void conv_bwd_filter_kernel(ConvShape s,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ dy,
                                                              float* __restrict__ part,
                                                              int kchunk) {
  __shared__ float smem[CFG_W::SMEM_FLOATS];
  const int Mw = s.R * s.S * s.C, npix = s.N * s.OH * s.OW;
  ConvFilterProb p{s, x, dy, Mw, npix};
  const int mt = (Mw + CFG_W::BM - 1) / CFG_W::BM, nt = (s.K + CFG_W::BN - 1) / CFG_W::BN;
  const int bid = blockIdx.x;
  const int tile = bid % (mt * nt), z = bid / (mt * nt);
  const int m0 = (tile % mt) * CFG_W::BM, n0 = (tile / mt) * CFG_W::BN;
  const int kb = z * kchunk, ke = min(kb + kchunk, (npix + BK - 1) / BK * BK);
  f32x16 acc;
  int wm, wn;
  gemm::run_tile<WM, WN, 1, BK>(p, smem, m0, n0, kb, ke, acc, wm, wn);
  const int lane = threadIdx.x & 63;
  const int co = n0 + 32 * wn + (lane & 31);
  if (co >= s.K) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + 32 * wm + mfma32_row(r, lane);
    if (m < Mw) part[((size_t)z * Mw + m) * s.K + co] = acc[r];
  }
}

// out[i] = sum_z part[z][i]  (+ optional per-column bias-grad: colsum of dY)
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ part, int nz,
                                                       long long n, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += part[z * n + i];
    out[i] = s;
  }
}

// Many slabs over few elements (thin-layer filter grads: 512 slabs x 450
// floats): block = 16 consecutive elements x 16 slab lanes; lane j sums slabs
// j, j + 16, ... (independent loads, 8 in flight), then a fixed-order LDS fold
// over the 16 lanes - deterministic, and no 512-long serial chain per thread.
__global__ __launch_bounds__(256) void slab_sum_wide_kernel(const float* __restrict__ part, int nz,
                                                            long long n, float* __restrict__ out) {
  __shared__ float red[16][17];
  const int e = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const long long i = (long long)blockIdx.x * 16 + e;
  float acc = 0.f;
  if (i < n) {
#pragma unroll 8
    for (int z = zl; z < nz; z += 16) acc += part[(long long)z * n + i];
  }
  red[zl][e] = acc;
  __syncthreads();
  if (zl == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][e];
    out[i] = t;
  }
}

// ------------------------------------------------- per-channel reductions ----
// sums[c] = sum_rows a[r][c], sums2[c] = sum_rows a[r][c]*b[r][c] (b optional).
// Block = 256 threads = (64 channels) x (4 row groups); grid-y splits rows;
// partials reduced by atomics into zeroed outputs (two scalars per channel).
__global__ __launch_bounds__(256) void colsum2_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ b, int rows,
                                                      int C, int rows_per_block,
                                                      float* __restrict__ s1,
                                                      float* __restrict__ s2, int mode) {
  // mode 0: s1 = sum a, s2 = sum a^2 ; mode 1: s1 = sum a, s2 = sum a*b
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float x1 = 0.f, x2 = 0.f;
  if (c < C) {
    for (int r = r0 + rg; r < r1; r += 4) {
      const float v = a[(size_t)r * C + c];
      x1 += v;
      x2 += mode == 0 ? v * v : v * b[(size_t)r * C + c];
    }
  }
  __shared__ float red[2][4][64];
  red[0][rg][threadIdx.x & 63] = x1;
  red[1][rg][threadIdx.x & 63] = x2;
  __syncthreads();
  if (rg == 0 && c < C) {
    const int l = threadIdx.x & 63;
    const float t1 = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
    const float t2 = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
    atomicAdd(&s1[c], t1);
    atomicAdd(&s2[c], t2);
  }
}

// ------------------------------------------------------------- pooling ----
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(PoolShape p, const float* __restrict__ x,
                                                          float* __restrict__ y,
                                                          int* __restrict__ arg) {
  const long long n = (long long)p.N * p.OH * p.OW * p.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % p.C);
    long long t = i / p.C;
    const int ox = (int)(t % p.OW);
    t /= p.OW;
    const int oy = (int)(t % p.OH);
    const int nn = (int)(t / p.OH);
    float best = -INFINITY;
    int bi = -1;
    for (int kh = 0; kh < p.k; ++kh)
      for (int kw = 0; kw < p.k; ++kw) {
        const int iy = oy * p.stride - p.pad + kh, ix = ox * p.stride - p.pad + kw;
        if (iy < 0 || iy >= p.H || ix < 0 || ix >= p.W) continue;
        const int idx = (nn * p.H + iy) * p.W + ix;
        const float v = x[(size_t)idx * p.C + c];
        if (v > best) {
          best = v;
          bi = idx;
        }
      }
    y[i] = best;
    arg[i] = bi;
  }
}

// gather form (deterministic): each input element sums the outputs whose argmax it is
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(PoolShape p, const float* __restrict__ dy,
                                                          const int* __restrict__ arg,
                                                          float* __restrict__ dx) {
  const long long n = (long long)p.N * p.H * p.W * p.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % p.C);
    const long long pix = i / p.C;
    const int ix = (int)(pix % p.W);
    const int iy = (int)((pix / p.W) % p.H);
    const int nn = (int)(pix / ((long long)p.W * p.H));
    float g = 0.f;
    const int oy0 = max(0, (iy + p.pad - p.k + p.stride) / p.stride);
    const int oy1 = min(p.OH - 1, (iy + p.pad) / p.stride);
    const int ox0 = max(0, (ix + p.pad - p.k + p.stride) / p.stride);
    const int ox1 = min(p.OW - 1, (ix + p.pad) / p.stride);
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const size_t o = (((size_t)nn * p.OH + oy) * p.OW + ox) * p.C + c;
        if (arg[o] == (int)pix) g += dy[o];
      }
    dx[i] = g;
  }
}

// C % 4 == 0 forms of the two kernels above: a thread owns 4 channels of one
// pixel (float4 / int4 loads and stores) and all index math is 32-bit (the
// host checks N H W C < 2^31).  ResNet-18 stem pool at B=32: the scalar forms
// spent 59 + 151 us per step on 64-bit divides and scalar loads.
__global__ __launch_bounds__(256) void maxpool_fwd4_kernel(PoolShape p, const float4* __restrict__ x,
                                                           float4* __restrict__ y,
                                                           int4* __restrict__ arg) {
  const int C4 = p.C / 4;
  const int n = p.N * p.OH * p.OW * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    int t = i / C4;
    const int ox = t % p.OW;
    t /= p.OW;
    const int oy = t % p.OH, nn = t / p.OH;
    float4 b = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    int4 bi = make_int4(-1, -1, -1, -1);
    for (int kh = 0; kh < p.k; ++kh) {
      const int iy = oy * p.stride - p.pad + kh;
      if (iy < 0 || iy >= p.H) continue;
      for (int kw = 0; kw < p.k; ++kw) {
        const int ix = ox * p.stride - p.pad + kw;
        if (ix < 0 || ix >= p.W) continue;
        const int idx = (nn * p.H + iy) * p.W + ix;
        const float4 v = x[idx * C4 + c4];
        if (v.x > b.x) { b.x = v.x; bi.x = idx; }
        if (v.y > b.y) { b.y = v.y; bi.y = idx; }
        if (v.z > b.z) { b.z = v.z; bi.z = idx; }
        if (v.w > b.w) { b.w = v.w; bi.w = idx; }
      }
    }
    y[i] = b;
    arg[i] = bi;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd4_kernel(PoolShape p, const float4* __restrict__ dy,
                                                           const int4* __restrict__ arg,
                                                           float4* __restrict__ dx) {
  const int C4 = p.C / 4;
  const int n = p.N * p.H * p.W * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    const int pix = i / C4;
    const int ix = pix % p.W, t = pix / p.W;
    const int iy = t % p.H, nn = t / p.H;
    const int oy0 = max(0, (iy + p.pad - p.k + p.stride) / p.stride);
    const int oy1 = min(p.OH - 1, (iy + p.pad) / p.stride);
    const int ox0 = max(0, (ix + p.pad - p.k + p.stride) / p.stride);
    const int ox1 = min(p.OW - 1, (ix + p.pad) / p.stride);
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int o = ((nn * p.OH + oy) * p.OW + ox) * C4 + c4;
        const int4 a = arg[o];
        if (a.x == pix || a.y == pix || a.z == pix || a.w == pix) {
          const float4 d = dy[o];
          if (a.x == pix) g.x += d.x;
          if (a.y == pix) g.y += d.y;
          if (a.z == pix) g.z += d.z;
          if (a.w == pix) g.w += d.w;
        }
      }
    dx[i] = g;
  }
}

// bf16-twin form (ResNet stem in bf16 conv mode): x is the bf16 twin of the
// BatchNorm output (whose fp32 storage is then never written), the argmax is
// the window-relative tap (uint8: kh * k + kw, 255 = empty window) instead of
// an int32 pixel index, and the output gets its own bf16 twin for the next
// conv.  Per step at B=32 this drops the BN's 102 MB fp32 store, half of the
// pool's input bytes, 3/4 of its argmax bytes and a to_bf16 pass.
__device__ __forceinline__ float4 bf4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

// KK / SS / PP / CC4: compile-time window, stride, pad and C/4 (the ResNet
// stem's 3 / 2 / 1 / 16; 0 = read from p): the index math is then multiplies
// and shifts instead of integer divides
__device__ __forceinline__ float4 pool_ld4(const uint2* x, int i) { return bf4(x[i]); }
__device__ __forceinline__ float4 pool_ld4(const float4* x, int i) { return x[i]; }

// XT: uint2 = 4 bf16 (the bf16 twin of the input), float4 = fp32 input
template <int KK, int SS, int PP, int CC4, class XT = uint2>
__global__ __launch_bounds__(256) void maxpool_fwd4b_kernel(PoolShape p, const XT* __restrict__ x,
                                                            float4* __restrict__ y,
                                                            uint2* __restrict__ yb,
                                                            uchar4* __restrict__ arg) {
  if constexpr (KK > 0) {
    p.k = KK;
    p.stride = SS;
    p.pad = PP;
  }
  const int C4 = CC4 > 0 ? CC4 : p.C / 4;
  const int n = p.N * p.OH * p.OW * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    int t = i / C4;
    const int ox = t % p.OW;
    t /= p.OW;
    const int oy = t % p.OH, nn = t / p.OH;
    float4 b = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    uchar4 bi = make_uchar4(255, 255, 255, 255);
    for (int kh = 0; kh < p.k; ++kh) {
      const int iy = oy * p.stride - p.pad + kh;
      if (iy < 0 || iy >= p.H) continue;
      for (int kw = 0; kw < p.k; ++kw) {
        const int ix = ox * p.stride - p.pad + kw;
        if (ix < 0 || ix >= p.W) continue;
        const float4 v = pool_ld4(x, ((nn * p.H + iy) * p.W + ix) * C4 + c4);
        const unsigned char r = (unsigned char)(kh * p.k + kw);
        if (v.x > b.x) { b.x = v.x; bi.x = r; }
        if (v.y > b.y) { b.y = v.y; bi.y = r; }
        if (v.z > b.z) { b.z = v.z; bi.z = r; }
        if (v.w > b.w) { b.w = v.w; bi.w = r; }
      }
    }
    if (y) y[i] = b;
    if (yb) {  // the maxima are bf16 values already: exact
      __bf16 h[4] = {(__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
      yb[i] = __builtin_bit_cast(uint2, h);
    }
    arg[i] = bi;
  }
}

template <int KK, int SS, int PP, int CC4>
__global__ __launch_bounds__(256) void maxpool_bwd4b_kernel(PoolShape p, const float4* __restrict__ dy,
                                                            const uchar4* __restrict__ arg,
                                                            float4* __restrict__ dx) {
  if constexpr (KK > 0) {
    p.k = KK;
    p.stride = SS;
    p.pad = PP;
  }
  const int C4 = CC4 > 0 ? CC4 : p.C / 4;
  const int n = p.N * p.H * p.W * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    const int pix = i / C4;
    const int ix = pix % p.W, t = pix / p.W;
    const int iy = t % p.H, nn = t / p.H;
    const int oy0 = max(0, (iy + p.pad - p.k + p.stride) / p.stride);
    const int oy1 = min(p.OH - 1, (iy + p.pad) / p.stride);
    const int ox0 = max(0, (ix + p.pad - p.k + p.stride) / p.stride);
    const int ox1 = min(p.OW - 1, (ix + p.pad) / p.stride);
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int o = ((nn * p.OH + oy) * p.OW + ox) * C4 + c4;
        // this pixel's tap index inside window (oy, ox)
        const unsigned char r =
            (unsigned char)((iy - (oy * p.stride - p.pad)) * p.k + (ix - (ox * p.stride - p.pad)));
        const uchar4 a = arg[o];
        if (a.x == r || a.y == r || a.z == r || a.w == r) {
          const float4 d = dy[o];
          if (a.x == r) g.x += d.x;
          if (a.y == r) g.y += d.y;
          if (a.z == r) g.z += d.z;
          if (a.w == r) g.w += d.w;
        }
      }
    dx[i] = g;
  }
}

// The ResNet stem pool's backward (3x3, stride 2, pad 1, uint8 window taps):
// a thread owns 8 channels (two float4) of one input pixel.  Its windows are
// rows iy >> 1 and (odd iy) (iy + 1) >> 1, columns likewise; every candidate
// window's taps and gradients are loaded up front, unconditionally from
// clamped addresses (one latency round instead of a tap load -> gradient load
// chain per window), and summed in the (oy, ox) order of maxpool_bwd4b_kernel
// (bit-identical dX).
template <int C4>
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2_kernel(PoolShape p,
                                                               const float4* __restrict__ dy,
                                                               const uint2* __restrict__ arg,
                                                               float4* __restrict__ dx) {
  static_assert(C4 % 2 == 0, "two float4 per thread");
  constexpr int C8 = C4 / 2;
  const int n = p.N * p.H * p.W * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    const int pix = i / C8;
    const int ix = pix % p.W, t = pix / p.W;
    const int iy = t % p.H, nn = t / p.H;
    const int oy0 = iy >> 1, ox0 = ix >> 1;
    const bool y2 = (iy & 1) && oy0 + 1 < p.OH, x2 = (ix & 1) && ox0 + 1 < p.OW;
    uint2 a[4];
    float4 d[4][2];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int oy = oy0 + ((w >> 1) & (int)y2), ox = ox0 + ((w & 1) & (int)x2);
      const int o = ((nn * p.OH + oy) * p.OW + ox) * C8 + c8;
      a[w] = arg[o];
      d[w][0] = dy[2 * o];
      d[w][1] = dy[2 * o + 1];
    }
    float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const bool live = ((w >> 1) == 0 || y2) && ((w & 1) == 0 || x2);
      const int oy = oy0 + (w >> 1), ox = ox0 + (w & 1);
      const unsigned r = live ? (unsigned)((iy - 2 * oy + 1) * 3 + (ix - 2 * ox + 1)) : 255u;
      const uchar4 q0 = __builtin_bit_cast(uchar4, a[w].x), q1 = __builtin_bit_cast(uchar4, a[w].y);
      if (q0.x == r) g0.x += d[w][0].x;
      if (q0.y == r) g0.y += d[w][0].y;
      if (q0.z == r) g0.z += d[w][0].z;
      if (q0.w == r) g0.w += d[w][0].w;
      if (q1.x == r) g1.x += d[w][1].x;
      if (q1.y == r) g1.y += d[w][1].y;
      if (q1.z == r) g1.z += d[w][1].z;
      if (q1.w == r) g1.w += d[w][1].w;
    }
    dx[2 * i] = g0;
    dx[2 * i + 1] = g1;
  }
}

// The same over 2 x 2 input pixels per thread (even H, W): the block's four
// pixels draw on the same <= 4 windows (rows H / 2 ... (iy + 1) / 2, columns
// likewise), so each window's taps and gradients are loaded once for four
// pixels instead of once per pixel (4x fewer L2 reads); each pixel sums its
// live windows in the (oy, ox) order of maxpool_bwd4b_kernel (bit-identical).
template <int C4>
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2_quad_kernel(PoolShape p,
                                                                    const float4* __restrict__ dy,
                                                                    const uint2* __restrict__ arg,
                                                                    float4* __restrict__ dx) {
  static_assert(C4 % 2 == 0, "two float4 per thread");
  constexpr int C8 = C4 / 2;
  const int HB = p.H / 2, WB = p.W / 2;
  const int n = p.N * HB * WB * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    const int blk = i / C8;
    const int b = blk % WB, t = blk / WB;
    const int a = t % HB, nn = t / HB;
    const bool y1 = a + 1 < p.OH, x1 = b + 1 < p.OW;
    uint2 ar[4];
    float4 d[4][2];
#pragma unroll
    for (int w = 0; w < 4; ++w) {  // windows (a + (w >> 1), b + (w & 1)), clamped
      const int oy = a + ((w >> 1) & (int)y1), ox = b + ((w & 1) & (int)x1);
      const int o = ((nn * p.OH + oy) * p.OW + ox) * C8 + c8;
      ar[w] = arg[o];
      d[w][0] = dy[2 * o];
      d[w][1] = dy[2 * o + 1];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // pixel (2a + (q >> 1), 2b + (q & 1))
      const int py = q >> 1, px = q & 1;
      float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int wy = w >> 1, wx = w & 1;
        // window row a + 1 reaches only the odd pixel row, and only inside the map
        const bool live = (wy == 0 || (py == 1 && y1)) && (wx == 0 || (px == 1 && x1));
        const unsigned r = live ? (unsigned)((py - 2 * wy + 1) * 3 + (px - 2 * wx + 1)) : 255u;
        const uchar4 q0 = __builtin_bit_cast(uchar4, ar[w].x), q1 = __builtin_bit_cast(uchar4, ar[w].y);
        if (q0.x == r) g0.x += d[w][0].x;
        if (q0.y == r) g0.y += d[w][0].y;
        if (q0.z == r) g0.z += d[w][0].z;
        if (q0.w == r) g0.w += d[w][0].w;
        if (q1.x == r) g1.x += d[w][1].x;
        if (q1.y == r) g1.y += d[w][1].y;
        if (q1.z == r) g1.z += d[w][1].z;
        if (q1.w == r) g1.w += d[w][1].w;
      }
      const int pix = (nn * p.H + 2 * a + py) * p.W + 2 * b + px;
      dx[2 * (pix * C8 + c8)] = g0;
      dx[2 * (pix * C8 + c8) + 1] = g1;
    }
  }
}

// block = (image n, 32 channels) x 8 pixel groups; the group partials are
// summed through LDS in a fixed order (ResNet-18 head: 512 blocks instead of
// 64 threads-per-channel blocks walking 49 dependent loads, 13 -> ~3 us)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const float* __restrict__ x,
                                                          float* __restrict__ y, int N, int HW,
                                                          int C) {
  __shared__ float red[8][33];
  const int cb = C / 32, n = blockIdx.x / cb, c0 = (blockIdx.x % cb) * 32;
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5, c = c0 + cl;
  float s0 = 0.f, s1 = 0.f;
  const float* xp = x + (size_t)n * HW * C + c;
  int p = g;
  for (; p + 8 < HW; p += 16) {
    s0 += xp[(size_t)p * C];
    s1 += xp[(size_t)(p + 8) * C];
  }
  if (p < HW) s0 += xp[(size_t)p * C];
  red[g][cl] = s0 + s1;
  __syncthreads();
  if (g == 0) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += red[j][cl];
    y[(size_t)n * C + c] = t / (float)HW;
  }
}

// C % 32 != 0 fallback: thread per (n, c)
__global__ __launch_bounds__(256) void avgpool_fwd1_kernel(const float* __restrict__ x,
                                                           float* __restrict__ y, int N, int HW,
                                                           int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += x[((size_t)n * HW + p) * C + c];
  y[i] = s / (float)HW;
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dy,
                                                          float* __restrict__ dx, int N, int HW,
                                                          int C) {
  const int n = N * HW * C;  // host checks < 2^31: 32-bit index math
  const int stride = gridDim.x * blockDim.x, hwc = HW * C;
  const float inv = 1.f / (float)HW;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = dy[(i / hwc) * C + i % C] * inv;
}

// ----------------------------------------------------- softmax xent ----
// one wave per row: loss_row = lse - logit[label]; dlogits = (p - onehot)/B
__global__ __launch_bounds__(256) void xent_kernel(const float* __restrict__ logits,
                                                   const int* __restrict__ labels, int B, int C,
                                                   float* __restrict__ loss_rows,
                                                   float* __restrict__ dlogits,
                                                   int* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const int lab = labels[row];
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, logits[(size_t)row * C + c]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(logits[(size_t)row * C + c] - mx);
  se = wave_sum(se);
  int am = C;
  for (int c = lane; c < C; c += 64)
    if (logits[(size_t)row * C + c] == mx) am = min(am, c);
  for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o, 64));
  for (int c = lane; c < C; c += 64) {
    const float p = __expf(logits[(size_t)row * C + c] - mx) / se;
    if (dlogits) dlogits[(size_t)row * C + c] = (p - (c == lab ? 1.f : 0.f)) / (float)B;
  }
  if (lane == 0) {
    loss_rows[row] = logf(se) + mx - logits[(size_t)row * C + lab];
    if (correct) atomicAdd(correct, am == lab ? 1 : 0);
  }
}

// mean softmax cross-entropy of B rows in ONE workgroup (B <= a few
// thousand): wave w takes rows w, w + 4, ...; writes loss_rows, dlogits =
// (p - onehot) / B, the mean loss (fixed summation order) and optionally the
// argmax hit count.  Replaces xent + torch's mean + the copy into the
// engine's loss scalar (3 launches, two of them ATen).
__global__ __launch_bounds__(256) void xent_mean_kernel(const float* __restrict__ logits,
                                                        const int* __restrict__ labels, int B,
                                                        int C, float* __restrict__ loss_rows,
                                                        float* __restrict__ dlogits,
                                                        float* __restrict__ mean_out,
                                                        int* __restrict__ correct) {
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (int row = w; row < B; row += 4) {
    const int lab = labels[row];
    const float* lg = logits + (size_t)row * C;
    float mx = -INFINITY;
    for (int c = lane; c < C; c += 64) mx = fmaxf(mx, lg[c]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(lg[c] - mx);
    se = wave_sum(se);
    int am = C;
    for (int c = lane; c < C; c += 64)
      if (lg[c] == mx) am = min(am, c);
    for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o, 64));
    for (int c = lane; c < C; c += 64)
      dlogits[(size_t)row * C + c] = (__expf(lg[c] - mx) / se - (c == lab ? 1.f : 0.f)) / (float)B;
    const float l = logf(se) + mx - lg[lab];
    if (lane == 0) {
      loss_rows[row] = l;
      if (correct && am == lab) atomicAdd(correct, 1);
    }
    acc += l;
  }
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) mean_out[0] = (part[0] + part[1] + part[2] + part[3]) / (float)B;
}

// Small fully connected layers (LeNet-5's 400-120-84-10 at batch 64, the
// ResNet-18 512 -> 10 head at batch 32-128): far below MFMA tile sizes, so
// plain VALU dot products with one output per thread; deterministic.
// forward: y[m][n] = b[n] + sum_k x[m][k] W[k][n] (+ ReLU)
// y[m][n] = x[m] . W[:, n] (+ b) (+ ReLU).  A workgroup owns LIN_MT rows and
// an NT-wide column tile (NT = pow2 >= N, at most 64); its 256 threads split K
// into 256 / NT interleaved groups (W row reads coalesce over n, one W load
// feeds LIN_MT rows), and the partial sums meet in LDS.  A thread-per-output
// loop over K was latency bound (ResNet-18 head 512 -> 10: 51 us).
constexpr int LIN_MT = 4;

__global__ __launch_bounds__(256) void linear_fwd_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b,
                                                         float* __restrict__ y, int M, int K,
                                                         int N, int relu, int nt_log2) {
  __shared__ float red[256 * LIN_MT];
  const int NT = 1 << nt_log2, KG = 256 >> nt_log2;
  const int t = threadIdx.x, j = t & (NT - 1), kg = t >> nt_log2;
  const int m0 = blockIdx.x * LIN_MT, n = blockIdx.y * NT + j;
  const bool nok = n < N;
  float acc[LIN_MT];
#pragma unroll
  for (int r = 0; r < LIN_MT; ++r) acc[r] = 0.f;
  for (int k = kg; k < K; k += KG) {
    const float wv = nok ? w[(size_t)k * N + n] : 0.f;
#pragma unroll
    for (int r = 0; r < LIN_MT; ++r) {
      const int m = min(m0 + r, M - 1);
      acc[r] = fmaf(x[(size_t)m * K + k], wv, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < LIN_MT; ++r) red[(r * KG + kg) * NT + j] = acc[r];
  __syncthreads();
  if (t < LIN_MT * NT) {
    const int r = t >> nt_log2, m = m0 + r;
    float v = 0.f;
    for (int g = 0; g < KG; ++g) v += red[(r * KG + g) * NT + j];
    if (m < M && nok) {
      v += b ? b[n] : 0.f;
      y[(size_t)m * N + n] = relu ? fmaxf(v, 0.f) : v;
    }
  }
}

// backward, three block roles in one launch: dW[k][n] = sum_m x[m][k] dy'[m][n],
// db[n] = sum_m dy'[m][n], dX[m][k] = sum_n dy'[m][n] W[k][n], with dy' = dy
// masked by ReLU (y > 0) when the forward fused it
__global__ __launch_bounds__(256) void linear_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ y,
    const float* __restrict__ dy, float* __restrict__ dw, float* __restrict__ db,
    float* __restrict__ dx, int M, int K, int N, int relu, int bw, int bb) {
  const int blk = blockIdx.x;
  auto g = [&](int m, int n) {
    const float d = dy[(size_t)m * N + n];
    return (relu && y[(size_t)m * N + n] <= 0.f) ? 0.f : d;
  };
  if (blk < bw) {  // dW
    const int i = blk * 256 + threadIdx.x;
    if (i >= K * N) return;
    const int k = i / N, n = i - k * N;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s = fmaf(x[(size_t)m * K + k], g(m, n), s);
    dw[i] = s;
    return;
  }
  if (blk < bw + bb) {  // db
    const int n = (blk - bw) * 256 + threadIdx.x;
    if (n >= N || !db) return;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += g(m, n);
    db[n] = s;
    return;
  }
  if (!dx) return;  // dX
  const int i = (blk - bw - bb) * 256 + threadIdx.x;
  if (i >= M * K) return;
  const int m = i / K, k = i - m * K;
  float s = 0.f;
  for (int n = 0; n < N; ++n) s = fmaf(g(m, n), w[(size_t)k * N + n], s);
  dx[i] = s;
}

// batch gather from a device-resident dataset at the device-step offset
// lr_out (optional): also the step's learning rate of the reference schedule
// (mpipy.py:59-64), so the SGD that follows needs no LR launch of its own
__global__ __launch_bounds__(256) void gather_batch_kernel(const float* __restrict__ data,
                                                           const int* __restrict__ labels,
                                                           const long long* step, int n_local,
                                                           int batch, long long row_elems,
                                                           float* __restrict__ xb,
                                                           int* __restrict__ yb, float lr_base,
                                                           float lr_decay, float* lr_out) {
  const long long s = step ? *step : 0;
  if (lr_out && blockIdx.x == 0 && threadIdx.x == 0)
    lr_out[0] = lr_base * powf(lr_decay, (float)((s * batch) / n_local));
  const long long off = (s * batch) % (long long)(n_local - batch);
  const long long n = (long long)batch * row_elems;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float4* src = reinterpret_cast<const float4*>(data + off * row_elems);
  float4* dst = reinterpret_cast<float4*>(xb);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += stride)
    dst[i] = src[i];
  if (blockIdx.x == 0 && threadIdx.x < batch) yb[threadIdx.x] = labels[off + threadIdx.x];
}

// dx = dy * [y > 0]
__global__ __launch_bounds__(256) void relu_bwd_kernel(const float* __restrict__ dy,
                                                       const float* __restrict__ y,
                                                       float* __restrict__ dx, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

// device-side learning rate of the reference schedule (mpipy.py:59-64)
__global__ void lr_kernel(const long long* step, int n_local, int batch, float base, float decay,
                          float* lr) {
  const long long s = *step;
  lr[0] = base * powf(decay, (float)((s * batch) / n_local));
}

// one element per thread up to 2^16 blocks (16M elements), grid-stride beyond
static inline int grid1d(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

// Direct VALU forward conv for thin layers (LeNet-5: 3 / 6 input channels,
// 6 / 16 outputs; reduction length R S C <= 512).  The gather engine's
// 64-wide output tiles leave 90 % of the MFMA lanes idle on K = 6 / 16 and
// run the short reduction as a serial K-tile chain (24 us per LeNet conv);
// here the whole HWIO filter sits in LDS, one thread computes one (pixel,
// output channel) with bias + ReLU fused, consecutive threads take
// consecutive channels (coalesced stores, conflict-free LDS reads, the
// input pixel is a wave-wide broadcast).
constexpr int DIRECT_W_MAX = 8192;  // filter floats staged in LDS (32 KB)

// CT: compile-time input channel count (0 = runtime s.C); with it the
// channel and filter-column loops unroll, so a thread issues its input loads
// back to back instead of one dependent load -> FMA round trip at a time.
template <int CT>
__global__ __launch_bounds__(256) void conv_fwd_direct_kernel(ConvShape s,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ y, int relu) {
  __shared__ float wl[DIRECT_W_MAX];
  const int nw = s.R * s.S * s.C * s.K;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) wl[i] = w[i];
  __syncthreads();
  const long long total = (long long)s.N * s.OH * s.OW * s.K;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int C = CT > 0 ? CT : s.C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int co = (int)(i % s.K);
    const long long m = i / s.K;
    const int ox = (int)(m % s.OW);
    const long long t = m / s.OW;
    const int oy = (int)(t % s.OH), n = (int)(t / s.OH);
    float acc = bias ? bias[co] : 0.f;
    for (int r = 0; r < s.R; ++r) {
      const int iy = oy * s.stride - s.pad + r;
      if (iy < 0 || iy >= s.H) continue;
#pragma unroll 5
      for (int q = 0; q < s.S; ++q) {
        const int ix = ox * s.stride - s.pad + q;
        if (ix < 0 || ix >= s.W) continue;
        const float* xp = x + (((long long)n * s.H + iy) * s.W + ix) * C;
        const float* wp = wl + (r * s.S + q) * C * s.K + co;
#pragma unroll
        for (int ci = 0; ci < C; ++ci) acc = fmaf(xp[ci], wp[ci * s.K], acc);
      }
    }
    y[i] = relu ? fmaxf(acc, 0.f) : acc;
  }
}

// Direct VALU backward-data conv for thin layers (LeNet-5 conv2: 6 input,
// 16 output channels), the transpose of the kernel above: one thread per
// (input pixel, input channel) sums dY[n, oy, ox, :] W[r][q][ci][:] over the
// taps that reach it (oy = (iy + pad - r) / stride when divisible).  KT:
// compile-time output channel count, so the dY row (KT contiguous floats)
// loads as float4s back to back.
template <int KT>
__global__ __launch_bounds__(256) void conv_bwd_data_direct_kernel(ConvShape s,
                                                                   const float* __restrict__ dy,
                                                                   const float* __restrict__ w,
                                                                   float* __restrict__ dx) {
  __shared__ float wl[DIRECT_W_MAX];
  const int nw = s.R * s.S * s.C * KT;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) wl[i] = w[i];
  __syncthreads();
  const long long total = (long long)s.N * s.H * s.W * s.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ci = (int)(i % s.C);
    const long long m = i / s.C;
    const int ix = (int)(m % s.W);
    const long long t = m / s.W;
    const int iy = (int)(t % s.H), n = (int)(t / s.H);
    float acc = 0.f;
    for (int r = 0; r < s.R; ++r) {
      const int ty = iy + s.pad - r;
      if (ty < 0 || ty % s.stride != 0) continue;
      const int oy = ty / s.stride;
      if (oy >= s.OH) continue;
#pragma unroll 5
      for (int q = 0; q < s.S; ++q) {
        const int tx = ix + s.pad - q;
        if (tx < 0 || tx % s.stride != 0) continue;
        const int ox = tx / s.stride;
        if (ox >= s.OW) continue;
        const float4* dp =
            reinterpret_cast<const float4*>(dy + (((long long)n * s.OH + oy) * s.OW + ox) * KT);
        const float* wp = wl + ((r * s.S + q) * s.C + ci) * KT;
#pragma unroll
        for (int k = 0; k < KT / 4; ++k) {
          const float4 d = dp[k];
          acc = fmaf(d.x, wp[4 * k], acc);
          acc = fmaf(d.y, wp[4 * k + 1], acc);
          acc = fmaf(d.z, wp[4 * k + 2], acc);
          acc = fmaf(d.w, wp[4 * k + 3], acc);
        }
      }
    }
    dx[i] = acc;
  }
}

static inline bool conv_fwd_direct_ok(const ConvShape& s) {
  return s.C < 32 && s.K <= 64 && s.R * s.S * s.C <= 512 &&
         (long long)s.R * s.S * s.C * s.K <= DIRECT_W_MAX;
}

// ------------------------------------------------------------ launchers ----
// The LDS-tiled conv family (conv_tiled.hip) takes every shape it supports
// (channel counts that are multiples of 32 / 4: all of ResNet-18 but its
// 3-channel stem); the per-element gather engine above covers the rest
// (LeNet-5's 3- and 6-channel layers, thin FC layers).
void conv_fwd(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
              bool relu, float* ws, hipStream_t st, bool bf16, const void* xb, const void* wtb,
              void* yb, const ConvStats* stats) {
  if (bf16 && conv_fwd_bf16_ok(s))
    return conv_fwd_bf16(s, x, w, bias, y, relu, ws, st, xb, wtb, yb, stats);
  if (yb) throw std::runtime_error("conv_fwd: bf16 output needs the bf16 conv family");
  if (stats && stats->part) {  // fp32 route: the tiled forward's epilogue / slab reduction
    if (bf16 || !(conv_fwd_tiled_ok(s) || conv_fwd_tiled_gather_ok(s)))
      throw std::runtime_error("conv_fwd: BatchNorm statistics need the bf16 or fp32 tiled family");
    return conv_fwd_tiled(s, x, w, bias, y, relu, ws, st, false, stats);
  }
  // fp32 with the stride-1 dgrad weight copy (wtb, ConvWeightCopies f32flip):
  // the 3x3 stride-1 layers on the halo kernel
  if (!bf16 && wtb && !bias && !relu && conv3f_ok(s))
    return conv3f(s, x, static_cast<const float*>(wtb), y, ws, st, nullptr);
  if (conv_fwd_tiled_ok(s)) return conv_fwd_tiled(s, x, w, bias, y, relu, ws, st, bf16);
  if (conv_fwd_direct_ok(s)) {
    const long long total = (long long)s.N * s.OH * s.OW * s.K;
    const int b = grid1d(total), rl = relu ? 1 : 0;
    switch (s.C) {
      case 1: conv_fwd_direct_kernel<1><<<b, 256, 0, st>>>(s, x, w, bias, y, rl); break;
      case 3: conv_fwd_direct_kernel<3><<<b, 256, 0, st>>>(s, x, w, bias, y, rl); break;
      case 6: conv_fwd_direct_kernel<6><<<b, 256, 0, st>>>(s, x, w, bias, y, rl); break;
      case 8: conv_fwd_direct_kernel<8><<<b, 256, 0, st>>>(s, x, w, bias, y, rl); break;
      default: conv_fwd_direct_kernel<0><<<b, 256, 0, st>>>(s, x, w, bias, y, rl);
    }
    return;
  }
  // thin-input convs too big for the direct kernel (the ResNet stem): fp32
  // MFMA tiles over the flattened (kh, kw, ci) axis
  if (!bf16 && conv_fwd_tiled_gather_ok(s))
    return conv_fwd_tiled(s, x, w, bias, y, relu, ws, st, false);
  const int M = s.N * s.OH * s.OW;
  const int blocks = ((M + CFG_F::BM - 1) / CFG_F::BM) * ((s.K + CFG_F::BN - 1) / CFG_F::BN);
  conv_fwd_kernel<<<blocks, 256, 0, st>>>(s, x, w, bias, y, relu ? 1 : 0);
}

// gather-engine backward-data split-K: a block's K tiles are a serial chain,
// so with few output tiles (LeNet conv2: 196 blocks x 13 K tiles) slice K to
// reach ~1024 blocks of >= 3 K tiles
static void gather_data_plan(const ConvShape& s, int& z, int& kchunk) {
  const int M = s.N * s.H * s.W;
  const int blocks = ((M + CFG_D::BM - 1) / CFG_D::BM) * ((s.C + CFG_D::BN - 1) / CFG_D::BN);
  const int ktiles = (s.R * s.S * s.K + BK - 1) / BK;
  z = (1024 + blocks - 1) / blocks;
  if (z > ktiles / 3) z = ktiles / 3;
  if (z < 1) z = 1;
  kchunk = ((ktiles + z - 1) / z) * BK;
  z = (ktiles * BK + kchunk - 1) / kchunk;
}

bool conv_bwd_data_join_ok(const ConvShape& s, bool bf16) {
  return (bf16 && conv_bwd_data_bf16_ok(s)) || conv_bwd_data_tiled_ok(s);
}

void conv_bwd_data(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                   hipStream_t st, bool bf16, const void* dyb, const float* addend,
                   const void* wtb, const BnBwdStats* bstats) {
  if (bf16 && conv_bwd_data_bf16_ok(s))
    return conv_bwd_data_bf16(s, dy, w, dx, ws, st, dyb, addend, wtb, bstats);
  if (bstats && bstats->part)
    throw std::runtime_error("conv_bwd_data: BatchNorm backward statistics need the bf16 family");
  if (conv_bwd_data_tiled_ok(s))  // fp32: wtb = the pre-flipped fp32 weights, when given
    return conv_bwd_data_tiled(s, dy, w, dx, ws, st, bf16, addend, dyb,
                               bf16 ? nullptr : static_cast<const float*>(wtb));
  if (!dy) throw std::runtime_error("conv_bwd_data: this shape needs the fp32 dY");
  if (addend) throw std::runtime_error("conv_bwd_data: no gradient-join epilogue for this shape");
  if (s.C < 32 && (long long)s.R * s.S * s.C * s.K <= DIRECT_W_MAX && (s.K == 8 || s.K == 16)) {
    const int b = grid1d((long long)s.N * s.H * s.W * s.C);
    if (s.K == 8)
      conv_bwd_data_direct_kernel<8><<<b, 256, 0, st>>>(s, dy, w, dx);
    else
      conv_bwd_data_direct_kernel<16><<<b, 256, 0, st>>>(s, dy, w, dx);
    return;
  }
  const int M = s.N * s.H * s.W;
  const int blocks = ((M + CFG_D::BM - 1) / CFG_D::BM) * ((s.C + CFG_D::BN - 1) / CFG_D::BN);
  int z, kchunk;
  gather_data_plan(s, z, kchunk);
  if (z > 1 && !ws) z = 1, kchunk = (s.R * s.S * s.K + BK - 1) / BK * BK;
  conv_bwd_data_kernel<<<dim3(blocks, z), 256, 0, st>>>(s, dy, w, z > 1 ? ws : dx, kchunk);
  if (z > 1) {
    const long long n = (long long)M * s.C;
    slab_sum_kernel<<<grid1d(n), 256, 0, st>>>(ws, z, n, dx);
  }
}

int conv_filter_splits(const ConvShape& s) {
  if (conv_bwd_filter_tiled_ok(s)) return conv_filter_tiled_splits(s);
  const int Mw = s.R * s.S * s.C;
  const int tiles = ((Mw + CFG_W::BM - 1) / CFG_W::BM) * ((s.K + CFG_W::BN - 1) / CFG_W::BN);
  const int ktiles = (s.N * s.OH * s.OW + BK - 1) / BK;
  // aim for ~1024 blocks of >= 2 K tiles: a block's K tiles form a serial
  // latency chain (~4 us each on this engine), so thin layers with few output
  // tiles (LeNet conv1: 2 tiles, 1568 K tiles) need many slices (measured:
  // a 64-slice cap left that layer at 101 us per step)
  int z = (1024 + tiles - 1) / tiles;
  z = z < 1 ? 1 : z;
  z = z > ktiles / 2 ? ktiles / 2 : z;
  z = z > 512 ? 512 : z;
  return z < 1 ? 1 : z;
}

long long conv_ws_floats(const ConvShape& s, bool fwd_epilogue) {
  long long n = (long long)conv_filter_splits(s) * s.R * s.S * s.C * s.K;
  if (!conv_bwd_data_tiled_ok(s)) {
    int z, kchunk;
    gather_data_plan(s, z, kchunk);
    if (z > 1) n = std::max(n, (long long)z * s.N * s.H * s.W * s.C);
  }
  if (conv_fwd_tiled_ok(s) || conv_fwd_tiled_gather_ok(s))
    n = std::max(n, conv_fwd_tiled_ws_floats(s, fwd_epilogue));
  if (conv_bwd_data_tiled_ok(s)) n = std::max(n, conv_bwd_data_tiled_ws_floats(s));
  return std::max(n, conv_bf16_ws_floats(s, fwd_epilogue));
}

void conv_bwd_filter(const ConvShape& s, const float* x, const float* dy, float* part, float* dw,
                     hipStream_t st, bool bf16, const void* xb,
                     const void* dyb) {
  if (bf16 && conv_bwd_filter_bf16_ok(s))
    return conv_bwd_filter_bf16(s, x, dy, part, dw, st, xb, dyb);
  if (conv_bwd_filter_tiled_ok(s)) return conv_bwd_filter_tiled(s, x, dy, part, dw, st, bf16);
  const int Mw = s.R * s.S * s.C;
  const int tiles = ((Mw + CFG_W::BM - 1) / CFG_W::BM) * ((s.K + CFG_W::BN - 1) / CFG_W::BN);
  const int ktiles = (s.N * s.OH * s.OW + BK - 1) / BK;
  const int z = conv_filter_splits(s);
  const int kchunk = ((ktiles + z - 1) / z) * BK;
  const int zz = (ktiles * BK + kchunk - 1) / kchunk;
  conv_bwd_filter_kernel<<<tiles * zz, 256, 0, st>>>(s, x, dy, part, kchunk);
  const long long n = (long long)Mw * s.K;
  if (zz >= 32)
    slab_sum_wide_kernel<<<(int)((n + 15) / 16), 256, 0, st>>>(part, zz, n, dw);
  else
    slab_sum_kernel<<<grid1d(n), 256, 0, st>>>(part, zz, n, dw);
}

void colsum2(const float* a, const float* b, long long rows, int C, float* s1, float* s2, int mode,
             float* ws, hipStream_t st) {
  // deterministic two-pass reduction (bn.hip); the memset + atomic kernel
  // above is only a fallback for callers without a workspace (memset nodes +
  // atomics inside captured graphs were the source of a replay divergence)
  if (ws && chan_reduce_ok(C)) return chan_reduce(a, b, rows, C, s1, s2, mode, ws, st);
  (void)hipMemsetAsync(s1, 0, C * sizeof(float), st);
  (void)hipMemsetAsync(s2, 0, C * sizeof(float), st);
  int gy = (int)((rows + 511) / 512);
  if (gy > 1024) gy = 1024;
  const int rpb = (int)((rows + gy - 1) / gy);
  dim3 grid((C + 63) / 64, gy);
  colsum2_kernel<<<grid, 256, 0, st>>>(a, b, (int)rows, C, rpb, s1, s2, mode);
}

static inline bool pool_vec4(const PoolShape& p) {
  return p.C % 4 == 0 && (long long)p.N * p.H * p.W * p.C < (1LL << 31) &&
         (long long)p.N * p.OH * p.OW * p.C < (1LL << 31);
}

void maxpool_fwd(const PoolShape& p, const float* x, float* y, int* arg, hipStream_t st) {
  const long long n = (long long)p.N * p.OH * p.OW * p.C;
  if (pool_vec4(p))
    maxpool_fwd4_kernel<<<grid1d(n / 4), 256, 0, st>>>(p, reinterpret_cast<const float4*>(x),
                                                       reinterpret_cast<float4*>(y),
                                                       reinterpret_cast<int4*>(arg));
  else
    maxpool_fwd_kernel<<<grid1d(n), 256, 0, st>>>(p, x, y, arg);
}

void maxpool_bwd(const PoolShape& p, const float* dy, const int* arg, float* dx, hipStream_t st) {
  const long long n = (long long)p.N * p.H * p.W * p.C;
  if (pool_vec4(p))
    maxpool_bwd4_kernel<<<grid1d(n / 4), 256, 0, st>>>(p, reinterpret_cast<const float4*>(dy),
                                                       reinterpret_cast<const int4*>(arg),
                                                       reinterpret_cast<float4*>(dx));
  else
    maxpool_bwd_kernel<<<grid1d(n), 256, 0, st>>>(p, dy, arg, dx);
}

bool maxpool_b16_ok(const PoolShape& p) { return pool_vec4(p) && p.k * p.k < 255; }

void maxpool_fwd_b16(const PoolShape& p, const void* xb, float* y, void* yb, uint8_t* arg,
                     hipStream_t st) {
  if (!maxpool_b16_ok(p)) throw std::runtime_error("maxpool_fwd_b16: unsupported shape");
  const long long n = (long long)p.N * p.OH * p.OW * p.C;
  const auto X = reinterpret_cast<const uint2*>(xb);
  const auto Y = reinterpret_cast<float4*>(y);
  const auto YB = reinterpret_cast<uint2*>(yb);
  const auto A = reinterpret_cast<uchar4*>(arg);
  if (p.k == 3 && p.stride == 2 && p.pad == 1 && p.C == 64)  // the ResNet stem pool
    maxpool_fwd4b_kernel<3, 2, 1, 16><<<grid1d(n / 4), 256, 0, st>>>(p, X, Y, YB, A);
  else
    maxpool_fwd4b_kernel<0, 0, 0, 0><<<grid1d(n / 4), 256, 0, st>>>(p, X, Y, YB, A);
}

void maxpool_fwd_u8(const PoolShape& p, const float* x, float* y, uint8_t* arg, hipStream_t st) {
  if (!maxpool_b16_ok(p)) throw std::runtime_error("maxpool_fwd_u8: unsupported shape");
  const long long n = (long long)p.N * p.OH * p.OW * p.C;
  const auto X = reinterpret_cast<const float4*>(x);
  const auto Y = reinterpret_cast<float4*>(y);
  const auto A = reinterpret_cast<uchar4*>(arg);
  if (p.k == 3 && p.stride == 2 && p.pad == 1 && p.C == 64)  // the ResNet stem pool
    maxpool_fwd4b_kernel<3, 2, 1, 16, float4><<<grid1d(n / 4), 256, 0, st>>>(p, X, Y, nullptr, A);
  else
    maxpool_fwd4b_kernel<0, 0, 0, 0, float4><<<grid1d(n / 4), 256, 0, st>>>(p, X, Y, nullptr, A);
}

void maxpool_bwd_b8(const PoolShape& p, const float* dy, const uint8_t* arg, float* dx,
                    hipStream_t st) {
  if (!maxpool_b16_ok(p)) throw std::runtime_error("maxpool_bwd_b8: unsupported shape");
  const long long n = (long long)p.N * p.H * p.W * p.C;
  const auto D = reinterpret_cast<const float4*>(dy);
  const auto A = reinterpret_cast<const uchar4*>(arg);
  const auto DX = reinterpret_cast<float4*>(dx);
  if (p.k == 3 && p.stride == 2 && p.pad == 1 && p.C == 64 && p.H % 2 == 0 && p.W % 2 == 0 &&
      p.OH == p.H / 2 && p.OW == p.W / 2)  // the ResNet stem pool
    maxpool_bwd_k3s2_quad_kernel<16><<<grid1d(n / 32), 256, 0, st>>>(
        p, D, reinterpret_cast<const uint2*>(arg), DX);
  else if (p.k == 3 && p.stride == 2 && p.pad == 1 && p.C == 64)
    maxpool_bwd_k3s2_kernel<16><<<grid1d(n / 8), 256, 0, st>>>(
        p, D, reinterpret_cast<const uint2*>(arg), DX);
  else
    maxpool_bwd4b_kernel<0, 0, 0, 0><<<grid1d(n / 4), 256, 0, st>>>(p, D, A, DX);
}

void avgpool_fwd(const float* x, float* y, int N, int HW, int C, hipStream_t st) {
  if (C % 32 == 0)
    avgpool_fwd_kernel<<<N * (C / 32), 256, 0, st>>>(x, y, N, HW, C);
  else
    avgpool_fwd1_kernel<<<(N * C + 255) / 256, 256, 0, st>>>(x, y, N, HW, C);
}

void avgpool_bwd(const float* dy, float* dx, int N, int HW, int C, hipStream_t st) {
  if ((long long)N * HW * C >= (1LL << 31)) throw std::runtime_error("avgpool_bwd: too large");
  avgpool_bwd_kernel<<<grid1d((long long)N * HW * C), 256, 0, st>>>(dy, dx, N, HW, C);
}

void xent(const float* logits, const int* labels, int B, int C, float* loss_rows, float* dlogits,
          int* correct, hipStream_t st) {
  xent_kernel<<<(B + 3) / 4, 256, 0, st>>>(logits, labels, B, C, loss_rows, dlogits, correct);
}

void xent_mean(const float* logits, const int* labels, int B, int C, float* loss_rows,
               float* dlogits, float* mean, int* correct, hipStream_t st) {
  xent_mean_kernel<<<1, 256, 0, st>>>(logits, labels, B, C, loss_rows, dlogits, mean, correct);
}

void linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int K, int N,
                bool relu, hipStream_t st) {
  int lg = 0;
  while ((1 << lg) < N && lg < 6) ++lg;
  const dim3 grid((M + LIN_MT - 1) / LIN_MT, (N + (1 << lg) - 1) >> lg);
  linear_fwd_kernel<<<grid, 256, 0, st>>>(x, w, b, y, M, K, N, relu ? 1 : 0, lg);
}

void linear_bwd(const float* x, const float* w, const float* y, const float* dy, float* dw,
                float* db, float* dx, int M, int K, int N, bool relu, hipStream_t st) {
  const int bw = (K * N + 255) / 256, bb = (N + 255) / 256, bx = dx ? (M * K + 255) / 256 : 0;
  linear_bwd_kernel<<<bw + bb + bx, 256, 0, st>>>(x, w, y, dy, dw, db, dx, M, K, N, relu ? 1 : 0,
                                                  bw, bb);
}

// Stem (im2col route, ops/functional.py _ConvIm2colFn): HWIO fp32
// [R][S][C][K] -> the 1x1 conv's pre-laid-out bf16 forward weight [K][kp] in
// the im2col's k order (k = kh * seg + kw * C + ci, zero-padded to seg per tap
// row and to kp overall), and the 1x1 conv's filter gradient [kp][K] back to
// HWIO.  (They were a torch.zeros + strided copy_ each way: ATen kernels.)
__global__ __launch_bounds__(256) void stem_wt_kernel(const float* __restrict__ w, int R, int sc,
                                                      int seg, int kp, int K,
                                                      __bf16* __restrict__ out) {
  const int n = K * kp;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int co = i / kp, k = i - co * kp, kh = k / seg, j = k - kh * seg;
    out[i] = (__bf16)((kh < R && j < sc) ? w[((size_t)kh * sc + j) * K + co] : 0.f);
  }
}

__global__ __launch_bounds__(256) void stem_wgrad_kernel(const float* __restrict__ gpad, int R,
                                                         int sc, int seg, int K,
                                                         float* __restrict__ gw) {
  const int n = R * sc * K;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int co = i % K, t = i / K, kh = t / sc, j = t - kh * sc;
    gw[i] = gpad[((size_t)kh * seg + j) * K + co];
  }
}

void stem_weight_bf16(const float* w, int R, int sc, int seg, int kp, int K, void* out,
                      hipStream_t st) {
  stem_wt_kernel<<<grid1d((long long)K * kp), 256, 0, st>>>(w, R, sc, seg, kp, K,
                                                            reinterpret_cast<__bf16*>(out));
}

void stem_wgrad(const float* gpad, int R, int sc, int seg, int K, float* gw, hipStream_t st) {
  stem_wgrad_kernel<<<grid1d((long long)R * sc * K), 256, 0, st>>>(gpad, R, sc, seg, K, gw);
}

// Space-to-depth stem (conv_bf16.hip conv_fwd_s2d_stem_bf16): one thread per
// s2d pixel (n, Y, X) of [N][OH + 3][OW + 3]: channels (p * 2 + q) * 3 + ci
// = x[n][2 (Y - 2) + p][2 (X - 2) + q][ci] (zero outside the image), 4 zero
// channels; two 16-byte stores.
__global__ __launch_bounds__(256) void s2d_stem_input_kernel(const float* __restrict__ x, int N,
                                                             int H, int W, int Hs, int Ws,
                                                             uint4* __restrict__ xs) {
  const long long n_pix = (long long)N * Hs * Ws;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n_pix;
       i += (long long)gridDim.x * 256) {
    const int X = (int)(i % Ws);
    const long long t = i / Ws;
    const int Y = (int)(t % Hs), n = (int)(t / Hs);
    __bf16 v[16];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int iy = 2 * (Y - 2) + p;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ix = 2 * (X - 2) + q;
        const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
        const float* src = x + (((size_t)n * H + (ok ? iy : 0)) * W + (ok ? ix : 0)) * 3;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) v[(p * 2 + q) * 3 + ci] = (__bf16)(ok ? src[ci] : 0.f);
      }
    }
#pragma unroll
    for (int c = 12; c < 16; ++c) v[c] = (__bf16)0.f;
    const uint4* pv = reinterpret_cast<const uint4*>(v);
    xs[2 * i] = pv[0];
    xs[2 * i + 1] = pv[1];
  }
}

// wt8 [co][k], k = (a * 4 + b) * 16 + (p * 2 + q) * 3 + ci  <-  w[2a + p - 1][2b + q - 1][ci][co]
// (zero off the 7x7 kernel and on the 4 padding channels)
__global__ __launch_bounds__(256) void s2d_stem_weight_kernel(const float* __restrict__ w, int K,
                                                              __bf16* __restrict__ wt8) {
  const int n = K * 256;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int co = i >> 8, k = i & 255, tap = k >> 4, ch = k & 15;
    const int a = tap >> 2, b = tap & 3, pq = ch / 3, ci = ch - 3 * pq;
    const int ky = 2 * a + (pq >> 1) - 1, kx = 2 * b + (pq & 1) - 1;
    const bool ok = ch < 12 && ky >= 0 && ky < 7 && kx >= 0 && kx < 7;
    wt8[i] = (__bf16)(ok ? w[((size_t)(ky * 7 + kx) * 3 + ci) * K + co] : 0.f);
  }
}

// gw HWIO [7][7][3][K]  <-  dw8 [k][K] at the k of each real (ky, kx, ci)
__global__ __launch_bounds__(256) void s2d_stem_wgrad_kernel(const float* __restrict__ dw8, int K,
                                                             float* __restrict__ gw) {
  const int n = 147 * K;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int co = i % K, t = i / K, ci = t % 3, kk = t / 3, ky = kk / 7, kx = kk % 7;
    const int a = (ky + 1) >> 1, p = (ky + 1) & 1, b = (kx + 1) >> 1, q = (kx + 1) & 1;
    gw[i] = dw8[(size_t)((a * 4 + b) * 16 + (p * 2 + q) * 3 + ci) * K + co];
  }
}

void s2d_stem_input(const float* x, int N, int H, int W, int OH, int OW, void* xs,
                    hipStream_t st) {
  const long long n = (long long)N * (OH + 3) * (OW + 3);
  s2d_stem_input_kernel<<<grid1d(n), 256, 0, st>>>(x, N, H, W, OH + 3, OW + 3,
                                                   reinterpret_cast<uint4*>(xs));
}

void s2d_stem_weight(const float* w, int K, void* wt8, hipStream_t st) {
  s2d_stem_weight_kernel<<<grid1d((long long)K * 256), 256, 0, st>>>(w, K,
                                                                    reinterpret_cast<__bf16*>(wt8));
}

void s2d_stem_wgrad(const float* dw8, int K, float* gw, hipStream_t st) {
  s2d_stem_wgrad_kernel<<<grid1d(147LL * K), 256, 0, st>>>(dw8, K, gw);
}

// Row softmax (the reference's train_prediction / eval_prediction heads,
// /root/reference/mpipy.py:67-68): one wave per row, max-subtracted.
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ x,
                                                          float* __restrict__ y, int M, int N) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (size_t)row * N;
  float mx = -INFINITY;
  for (int j = lane; j < N; j += 64) mx = fmaxf(mx, xr[j]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int j = lane; j < N; j += 64) s += __expf(xr[j] - mx);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < N; j += 64) y[(size_t)row * N + j] = __expf(xr[j] - mx) * inv;
}

void softmax_rows(const float* x, float* y, int M, int N, hipStream_t st) {
  if (M > 0) softmax_rows_kernel<<<(M + 3) / 4, 256, 0, st>>>(x, y, M, N);
}

void relu_bwd(const float* dy, const float* y, float* dx, long long n, hipStream_t st) {
  relu_bwd_kernel<<<grid1d(n), 256, 0, st>>>(dy, y, dx, n);
}

void lr_from_step(const long long* step, int n_local, int batch, float base, float decay,
                  float* lr, hipStream_t st) {
  lr_kernel<<<1, 1, 0, st>>>(step, n_local, batch, base, decay, lr);
}

void gather_batch(const float* data, const int* labels, const long long* step, int n_local,
                  int batch, long long row_elems, float* xb, int* yb, hipStream_t st,
                  float lr_base, float lr_decay, float* lr_out) {
  if (row_elems % 4 != 0 || batch > 256) throw std::runtime_error("gather_batch: unsupported shape");
  gather_batch_kernel<<<grid1d((long long)batch * row_elems / 4), 256, 0, st>>>(
      data, labels, step, n_local, batch, row_elems, xb, yb, lr_base, lr_decay, lr_out);
}

}  // namespace gops
