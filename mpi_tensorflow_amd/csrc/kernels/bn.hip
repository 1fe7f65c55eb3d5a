// Per-channel reductions and BatchNorm for NHWC tensors (ResNet-18 config).
//
// The statistics are a deterministic two-pass column reduction: pass 1 has
// each 1024-thread block reduce a slab of rows into per-channel partials
// (thread = one float4 of channels x a row stride, so every global load is a
// coalesced 16-byte access; 16 waves per block keep enough loads in flight
// with ~one block per CU, so there are at most 256 partial rows), stored
// channel-major; pass 2 has one wave per channel sum its contiguous partials
// (<= 4 coalesced loads a lane) and apply the per-channel epilogue (sums, or
// mean / rstd / running statistics).  No atomics, no memsets: the result
// (and a graph replay of it) is bitwise reproducible.
// (Measured alternative: fusing pass 2 into pass 1 with a last-block ticket
// was SLOWER - the write-through partial stores, the ticket round trip and the
// single block's serial reads cost ~10 us of tail, against ~3 us for the
// separate launch; a device-scope release fence per block, the textbook
// version, writes back the XCD's L2 and made the kernel 4x slower.)
//
// BN backward needs sum(dy') and sum(dy' * xhat) with dy' = dy [y > 0] when a
// ReLU is fused; the pass-1 kernel computes both straight from (x, dy, y,
// mean, rstd), so neither dy' nor xhat is ever materialised.  The BN forward
// epilogue also updates the running statistics (momentum, unbiased variance),
// so a BN layer is two kernels per direction with no host-side tensor ops.
//
// bf16 conv mode: the apply kernels can also write a bf16 copy of their
// output (y forward, dx backward), which the next conv reads as its bf16
// operand (forward input / dY of the filter and data gradients) instead of
// a separate to_bf16 pass over the fp32 tensor.
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "ops_generic.h"
#include "grid_sync.h"  // grid barrier + system-scope hand-off (fused finalize)

namespace gops {
namespace bn {

enum Mode { SUM_SQ = 0, SUM_PROD = 1, BN_BWD = 2 };

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// 4 consecutive elements of x at element offset i: fp32, or (XB) bf16 - the
// bf16 conv outputs of the ResNet bf16 path, half the bytes of every x read
template <bool XB>
__device__ __forceinline__ float4 ldx(const void* p, size_t i) {
  if constexpr (XB) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const __bf16*>(p) + i);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  } else {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
  }
}
// 4 floats -> 4 bf16 (round to nearest even, as to_bf16_kernel)
__device__ __forceinline__ uint2 pack4(float4 a) {
  __bf16 v[4] = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w};
  return __builtin_bit_cast(uint2, v);
}

// Epilogue of the reduction (run by the last block): s1 / s2 = the column
// sums, or (bn_fwd) mean / rstd and the running statistics from shifted sums.
struct Fin {
  float* s1;
  float* s2;
  int bn_fwd;
  float eps, momentum;
  float* mean;
  float* rstd;
  float* rmean;
  float* rvar;
  const void* shift;  // row 0 of x (fp32, or bf16 when shift_b16)
  int shift_b16;
};

__device__ __forceinline__ void fin_channel(const Fin& f, int c, float a, float b, long long rows) {
  if (f.s1) f.s1[c] = a;
  if (f.s2) f.s2[c] = b;
  if (f.bn_fwd) {
    // The BN forward partials are SHIFTED sums, of (x - K) and (x - K)^2 with
    // K = the channel's value in row 0 (`shift`): var = E[(x-K)^2] - E[x-K]^2
    // cancels only (mean - K)^2 / var, a few units for a sample of the
    // channel, instead of mean^2 / var for the plain E[x^2] - mean^2 (a
    // channel with mean 1e3 and std 1 loses every digit of its variance in
    // fp32 that way).
    const float inv = 1.f / (float)rows;
    const float ms = a * inv;  // mean of the shifted data
    const float var = fmaxf(b * inv - ms * ms, 0.f);
    float k = 0.f;
    if (f.shift)
      k = f.shift_b16 ? (float)reinterpret_cast<const __bf16*>(f.shift)[c]
                      : reinterpret_cast<const float*>(f.shift)[c];
    const float m = ms + k;
    f.mean[c] = m;
    f.rstd[c] = rsqrtf(var + f.eps);
    if (f.rmean) {  // torch semantics: unbiased variance in the running estimate
      const float unb = rows > 1 ? var * (float)rows / (float)(rows - 1) : var;
      f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * m;
      f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * unb;
    }
  }
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// Tree fold of the row lanes of red[2][PT] (lane rl of quad q at rl * cq +
// q) into lane 0; fixed order.
template <int PT>
__device__ __forceinline__ void fold_rows(float4 (*red)[PT], int cq, int RP, int tid, int rl) {
  for (int h = RP >> 1; h >= 1; h >>= 1) {
    if (rl < h) {
      add4(red[0][tid], red[0][tid + h * cq]);
      add4(red[1][tid], red[1][tid + h * cq]);
    }
    __syncthreads();
  }
}

// Vector path (C % 4 == 0): PT = 1024 threads = cq channel quads x RP row
// lanes (RP = the largest power of two <= PT / cq).  16 waves per block keep
// enough loads in flight with ~one block per CU, so the partial rows are few
// (<= 256) and the last block's sum of them is short.
constexpr int PT = 1024;

// XB: x is bf16; YB: the ReLU-mask tensor y is the bf16 twin of the output
template <int MODE, bool XB, bool YB>
__global__ __launch_bounds__(PT) void partial_kernel(const void* __restrict__ a,
                                                     const float* __restrict__ b,
                                                     const void* __restrict__ yv,
                                                     const void* __restrict__ mean,
                                                     const float* __restrict__ rstd, int relu,
                                                     long long rows, int C, int rows_per_block,
                                                     float* __restrict__ part) {
  __shared__ float4 red[2][PT];
  const int cq = C >> 2;
  int RP = 1;
  while (RP * 2 * cq <= PT) RP *= 2;
  const int tid = threadIdx.x, q = tid % cq, rl = tid / cq;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(rows, r0 + rows_per_block);
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  float4 mu = s1, rs = s1;
  if (rl < RP) {
    if (MODE == BN_BWD) {
      mu = ld4(reinterpret_cast<const float*>(mean) + 4 * q);
      rs = ld4(rstd + 4 * q);
    } else if (MODE == SUM_SQ && mean) {
      mu = ldx<XB>(mean, 4 * q);  // shifted data: sums of (x - K), K = a sample of the channel
    }
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += RP) {
      const size_t o = (size_t)r * C + 4 * q;
      const float4 v = ldx<XB>(a, o);
      if (MODE == SUM_SQ) {
        const float4 w = make_float4(v.x - mu.x, v.y - mu.y, v.z - mu.z, v.w - mu.w);
        s1.x += w.x; s1.y += w.y; s1.z += w.z; s1.w += w.w;
        s2.x += w.x * w.x; s2.y += w.y * w.y; s2.z += w.z * w.z; s2.w += w.w * w.w;
      } else if (MODE == SUM_PROD) {
        const float4 u = ld4(b + o);
        s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
        s2.x += v.x * u.x; s2.y += v.y * u.y; s2.z += v.z * u.z; s2.w += v.w * u.w;
      } else {  // a = x, b = dy, yv = y (relu mask)
        float4 d = ld4(b + o);
        if (relu) {
          const float4 yy = ldx<YB>(yv, o);
          d.x = yy.x > 0.f ? d.x : 0.f;
          d.y = yy.y > 0.f ? d.y : 0.f;
          d.z = yy.z > 0.f ? d.z : 0.f;
          d.w = yy.w > 0.f ? d.w : 0.f;
        }
        s1.x += d.x; s1.y += d.y; s1.z += d.z; s1.w += d.w;
        s2.x += d.x * (v.x - mu.x) * rs.x;
        s2.y += d.y * (v.y - mu.y) * rs.y;
        s2.z += d.z * (v.z - mu.z) * rs.z;
        s2.w += d.w * (v.w - mu.w) * rs.w;
      }
    }
  }
  red[0][tid] = s1;
  red[1][tid] = s2;
  __syncthreads();
  fold_rows<PT>(red, cq, RP, tid, rl);
  if (tid < cq) {  // channel-major partial table [2][C][nb]
    const int nb = gridDim.x, k = blockIdx.x;
    const float4 t1 = red[0][tid], t2 = red[1][tid];
    float* p = part + (size_t)(4 * tid) * nb + k;
    p[0] = t1.x; p[nb] = t1.y; p[2 * nb] = t1.z; p[3 * nb] = t1.w;
    p += (size_t)C * nb;
    p[0] = t2.x; p[nb] = t2.y; p[2 * nb] = t2.z; p[3 * nb] = t2.w;
  }
}

// Scalar variant of pass 1 for channel counts that are not a multiple of 4
// (thin layers: LeNet's 6 / 10 channel convs and FCs): thread = one channel
// x a row stride.  Modes SUM_SQ / SUM_PROD only.
__global__ __launch_bounds__(256) void partial1_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ b, int mode,
                                                       long long rows, int C, int rows_per_block,
                                                       float* __restrict__ part) {
  __shared__ float red[2][256];
  const int RP = 256 / C;
  const int tid = threadIdx.x, c = tid % C, rl = tid / C;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(rows, r0 + rows_per_block);
  float s1 = 0.f, s2 = 0.f;
  if (rl < RP) {
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += RP) {
      const float v = a[(size_t)r * C + c];
      s1 += v;
      s2 += mode == SUM_SQ ? v * v : v * b[(size_t)r * C + c];
    }
  }
  red[0][tid] = s1;
  red[1][tid] = s2;
  __syncthreads();
  if (tid < C) {
    float t1 = 0.f, t2 = 0.f;
    for (int j = 0; j < RP; ++j) {
      t1 += red[0][tid + j * C];
      t2 += red[1][tid + j * C];
    }
    part[(size_t)tid * gridDim.x + blockIdx.x] = t1;
    part[(size_t)(C + tid) * gridDim.x + blockIdx.x] = t2;
  }
}

// Pass 2: one block per channel sums its nb contiguous partials (fixed
// order: thread strides, then the waves in order), thread 0 applies the
// epilogue.  (One wave per channel ran 6.2 us on the ~1.5 K partial rows a
// conv epilogue writes for ResNet-18 layer 1; one block per channel keeps
// every load of a thread independent and 4x as many in flight.)
// grp64: the conv-epilogue layout [2][C / 64][nb][64] (a row of 64 channels
// per producing wave: coalesced writes), else channel-major [2][C][nb]
__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ part, int nb,
                                                       int C, long long rows, Fin fin,
                                                       int grp64) {
  __shared__ float red[2][4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = grp64 ? (size_t)(c >> 6) * nb * 64 + (c & 63) : (size_t)c * nb;
  const size_t step = grp64 ? 64 : 1, half = (size_t)C * nb;
  const float* pa = part + base;
  const float* pb = part + half + base;
  float a = 0.f, b = 0.f;
#pragma unroll 4
  for (int k = tid; k < nb; k += 256) {
    a += pa[k * step];
    b += pb[k * step];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    red[0][wave] = a;
    red[1][wave] = b;
  }
  __syncthreads();
  if (tid == 0)
    fin_channel(fin, c, (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]),
                (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]), rows);
}

// Pass 2 for the conv-epilogue layout with few partial rows (P <= 128: the
// deep layers): one block per 64-channel group, lane = channel, so every load
// is a coalesced 256-byte row, and wave w sums rows w, w + 4, ... (all of a
// lane's <= 32 loads in flight at once); the 4 wave sums are added in order.
// (finalize_kernel's block per channel reads each row 64 times over, strided,
// and launches C blocks for a few dozen partials: ~5.5 us a call.)
constexpr int FIN64_MAXP = 128;
__global__ __launch_bounds__(256) void finalize64_kernel(const float* __restrict__ part, int nb,
                                                         int C, long long rows, Fin fin) {
  __shared__ float red[2][4][64];
  const int grp = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)grp * nb * 64 + lane, half = (size_t)C * nb;
  constexpr int PER = FIN64_MAXP / 4;
  float va[PER], vb[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int r = wave + 4 * k;
    va[k] = r < nb ? part[base + (size_t)r * 64] : 0.f;
    vb[k] = r < nb ? part[half + base + (size_t)r * 64] : 0.f;
  }
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    a += va[k];
    b += vb[k];
  }
  red[0][wave][lane] = a;
  red[1][wave][lane] = b;
  __syncthreads();
  if (tid < 64)
    fin_channel(fin, grp * 64 + tid, (red[0][0][tid] + red[0][1][tid]) + (red[0][2][tid] + red[0][3][tid]),
                (red[1][0][tid] + red[1][1][tid]) + (red[1][2][tid] + red[1][3][tid]), rows);
}

// the conv-epilogue layout [2][C / 64][P][64] -> fin
static void finalize_grp64(const float* part, int P, int C, long long rows, const Fin& fin,
                           hipStream_t st) {
  if (P <= FIN64_MAXP)
    finalize64_kernel<<<C / 64, 256, 0, st>>>(part, P, C, rows, fin);
  else
    finalize_kernel<<<C, 256, 0, st>>>(part, P, C, rows, fin, 1);
}

// y = (x - mean) rstd g + b (+ res) (relu); eval: mean / var from running stats
template <bool XB>
__global__ __launch_bounds__(256) void apply_kernel(const void* __restrict__ x,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ rstd,
                                                    const float* __restrict__ g,
                                                    const float* __restrict__ bb,
                                                    const float* __restrict__ res,
                                                    float* __restrict__ y, long long n4, int C,
                                                    int relu, int eval, float eps,
                                                    uint2* __restrict__ yb) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int cq = C >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int c = (int)(i % cq) * 4;
    const float4 v = ldx<XB>(x, 4 * i);
    float4 m = ld4(mean + c), r = ld4(rstd + c);
    if (eval) {
      r.x = rsqrtf(r.x + eps); r.y = rsqrtf(r.y + eps); r.z = rsqrtf(r.z + eps); r.w = rsqrtf(r.w + eps);
    }
    const float4 gg = ld4(g + c), b4 = ld4(bb + c);
    float4 o;
    o.x = (v.x - m.x) * r.x * gg.x + b4.x;
    o.y = (v.y - m.y) * r.y * gg.y + b4.y;
    o.z = (v.z - m.z) * r.z * gg.z + b4.z;
    o.w = (v.w - m.w) * r.w * gg.w + b4.w;
    if (res) {
      const float4 q = ld4(res + 4 * i);
      o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
    }
    if (relu) {
      o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
    }
    if (y) *reinterpret_cast<float4*>(y + 4 * i) = o;  // null: the bf16 twin only
    if (yb) yb[i] = pack4(o);
  }
}

// dx = g rstd (dy' - s1/rows - xhat s2/rows); dres = dy' (residual branch).
// dx (fp32) and dxb (bf16) are each optional.
template <bool XB, bool YB>
__global__ __launch_bounds__(256) void bwd_apply_kernel(
    const void* __restrict__ x, const float* __restrict__ dy, const void* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ g,
    const float* __restrict__ s1, const float* __restrict__ s2, float* __restrict__ dx,
    float* __restrict__ dres, long long n4, int C, long long rows, int relu,
    uint2* __restrict__ dxb) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int cq = C >> 2;
  const float inv = 1.f / (float)rows;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int c = (int)(i % cq) * 4;
    float4 d = ld4(dy + 4 * i);
    if (relu) {
      const float4 yy = ldx<YB>(y, 4 * i);
      d.x = yy.x > 0.f ? d.x : 0.f;
      d.y = yy.y > 0.f ? d.y : 0.f;
      d.z = yy.z > 0.f ? d.z : 0.f;
      d.w = yy.w > 0.f ? d.w : 0.f;
    }
    if (dres) *reinterpret_cast<float4*>(dres + 4 * i) = d;
    const float4 v = ldx<XB>(x, 4 * i), m = ld4(mean + c), r = ld4(rstd + c), gg = ld4(g + c);
    const float4 a = ld4(s1 + c), b = ld4(s2 + c);
    float4 o;
    o.x = gg.x * r.x * (d.x - a.x * inv - (v.x - m.x) * r.x * b.x * inv);
    o.y = gg.y * r.y * (d.y - a.y * inv - (v.y - m.y) * r.y * b.y * inv);
    o.z = gg.z * r.z * (d.z - a.z * inv - (v.z - m.z) * r.z * b.z * inv);
    o.w = gg.w * r.w * (d.w - a.w * inv - (v.w - m.w) * r.w * b.w * inv);
    if (dx) *reinterpret_cast<float4*>(dx + 4 * i) = o;
    if (dxb) dxb[i] = pack4(o);
  }
}

// ---- finalize fused into the apply launch (bn_fwd_partials /
// bn_bwd_partials): phase A - block b reduces the partial rows of channels
// b, b + G, ... (finalize_kernel's order) and publishes the statistics with
// system-scope stores; a grid-wide barrier; phase B - every block stages the
// C channels' statistics in LDS (system-scope loads: another XCD's L2 may hold
// the writer's line) and runs the apply loop.  One launch and one dispatch
// instead of two per BatchNorm and direction (ResNet-18: 40 finalize launches
// a step).  The grid is capped at FUSED_BLOCKS_PER_CU blocks a CU, well under
// what the CUs hold next to a concurrent collective, so every block is
// resident before any waits; the spin is bounded (a timeout sets *err).
constexpr int FUSED_BLOCKS_PER_CU = 2;  // default; bn_set_fused_blocks_per_cu
constexpr int FU = 4;

using gsync::GridBar;
using gsync::grid_barrier;

// phase A: channels blockIdx.x, + gridDim.x, ... of the partial table - the
// conv-epilogue layout [2][C / 64][P][64] (grp64), or partial_kernel's
// channel-major [2][C][P]; stat 0 / 1 of channel c published at pub0 / pub1
// (system scope): mean / rstd (forward) or the sums db / dg (backward)
__device__ __forceinline__ void fused_finalize(const float* __restrict__ part, int P, int C,
                                               long long rows, const Fin& fin, float* pub0,
                                               float* pub1, int grp64) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t half = (size_t)C * P, step = grp64 ? 64 : 1;
  const xgmi::Rsrc r0 = xgmi::rsrc(pub0, 4LL * C), r1 = xgmi::rsrc(pub1, 4LL * C);
  for (int c = blockIdx.x; c < C; c += gridDim.x) {
    const float* pa = part + (grp64 ? (size_t)(c >> 6) * P * 64 + (c & 63) : (size_t)c * P);
    const float* pb = pa + half;
    float a = 0.f, b = 0.f;
#pragma unroll 4
    for (int k = tid; k < P; k += 256) {
      a += pa[(size_t)k * step];
      b += pb[(size_t)k * step];
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      red[0][wave] = a;
      red[1][wave] = b;
    }
    __syncthreads();
    if (tid == 0) {
      const float sa = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
      const float sb = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
      fin_channel(fin, c, sa, sb, rows);
      xgmi::st_sys(r0, 4u * c, fin.bn_fwd ? fin.mean[c] : sa);
      xgmi::st_sys(r1, 4u * c, fin.bn_fwd ? fin.rstd[c] : sb);
    }
    __syncthreads();
  }
}

// phase B's statistics: C floats of each of the n arrays into LDS
__device__ __forceinline__ void stage_stats(float* lds, const float* const* src, int n, int C) {
  for (int j = 0; j < n; ++j) {
    const xgmi::Rsrc r = xgmi::rsrc(src[j], 4LL * C);
    for (int c = threadIdx.x; c < C; c += blockDim.x) lds[j * C + c] = xgmi::ld_sys(r, 4u * c);
  }
  __syncthreads();
}

constexpr int FUSED_MAXC = 1024;

template <bool XB>
__global__ __launch_bounds__(256) void finalize_apply_kernel(
    const float* __restrict__ part, int P, int grp64, long long rows, Fin fin, GridBar bar,
    const void* __restrict__ x, const float* __restrict__ g, const float* __restrict__ bb,
    const float* __restrict__ res, float* __restrict__ y, long long n4, int C, int relu,
    uint2* __restrict__ yb) {
  __shared__ float st[2 * FUSED_MAXC];
  fused_finalize(part, P, C, rows, fin, fin.mean, fin.rstd, grp64);
  grid_barrier(bar);
  const float* srcs[2] = {fin.mean, fin.rstd};
  stage_stats(st, srcs, 2, C);
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int cq = C >> 2;
  // FU elements a thread in flight: the grid is a few blocks a CU, so each
  // thread's loads are batched ahead of its math (one load at a time left
  // HBM latency exposed: 28.5 us against apply_kernel's 7.6)
  for (long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4;
       i0 += FU * stride) {
    float4 v[FU], q[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const long long i = i0 + u * stride;
      if (i < n4) {
        v[u] = ldx<XB>(x, 4 * i);
        if (res) q[u] = ld4(res + 4 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n4) break;
      const int c = (int)(i % cq) * 4;
      const float4 m = *reinterpret_cast<const float4*>(st + c);
      const float4 r = *reinterpret_cast<const float4*>(st + C + c);
      const float4 gg = ld4(g + c), b4 = ld4(bb + c);
      float4 o;  // apply_kernel's expression forms
      o.x = (v[u].x - m.x) * r.x * gg.x + b4.x;
      o.y = (v[u].y - m.y) * r.y * gg.y + b4.y;
      o.z = (v[u].z - m.z) * r.z * gg.z + b4.z;
      o.w = (v[u].w - m.w) * r.w * gg.w + b4.w;
      if (res) {
        o.x += q[u].x; o.y += q[u].y; o.z += q[u].z; o.w += q[u].w;
      }
      if (relu) {
        o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
      }
      if (y) *reinterpret_cast<float4*>(y + 4 * i) = o;
      if (yb) yb[i] = pack4(o);
    }
  }
}

// backward: phase A forms db = sum dy', dg = sum dy' xhat (fin.s1 / fin.s2)
template <bool XB, bool YB>
__global__ __launch_bounds__(256) void finalize_bwd_apply_kernel(
    const float* __restrict__ part, int P, int grp64, Fin fin, GridBar bar,
    const void* __restrict__ x, const float* __restrict__ dy, const void* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ g,
    float* __restrict__ dx, float* __restrict__ dres, long long n4, int C, long long rows,
    int relu, uint2* __restrict__ dxb) {
  __shared__ float st[2 * FUSED_MAXC];
  fused_finalize(part, P, C, rows, fin, fin.s1, fin.s2, grp64);
  grid_barrier(bar);
  const float* srcs[2] = {fin.s1, fin.s2};
  stage_stats(st, srcs, 2, C);
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int cq = C >> 2;
  const float inv = 1.f / (float)rows;
  for (long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4;
       i0 += FU * stride) {  // FU elements in flight (finalize_apply_kernel)
    float4 dd[FU], yv[FU], xv[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const long long i = i0 + u * stride;
      if (i < n4) {
        dd[u] = ld4(dy + 4 * i);
        if (relu) yv[u] = ldx<YB>(y, 4 * i);
        xv[u] = ldx<XB>(x, 4 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n4) break;
      const int c = (int)(i % cq) * 4;
      float4 d = dd[u];
      if (relu) {
        d.x = yv[u].x > 0.f ? d.x : 0.f;
        d.y = yv[u].y > 0.f ? d.y : 0.f;
        d.z = yv[u].z > 0.f ? d.z : 0.f;
        d.w = yv[u].w > 0.f ? d.w : 0.f;
      }
      if (dres) *reinterpret_cast<float4*>(dres + 4 * i) = d;
      const float4 v = xv[u], m = ld4(mean + c), r = ld4(rstd + c), gg = ld4(g + c);
      const float4 a = *reinterpret_cast<const float4*>(st + c);
      const float4 b = *reinterpret_cast<const float4*>(st + C + c);
      float4 o;  // bwd_apply_kernel's expression forms
      o.x = gg.x * r.x * (d.x - a.x * inv - (v.x - m.x) * r.x * b.x * inv);
      o.y = gg.y * r.y * (d.y - a.y * inv - (v.y - m.y) * r.y * b.y * inv);
      o.z = gg.z * r.z * (d.z - a.z * inv - (v.z - m.z) * r.z * b.z * inv);
      o.w = gg.w * r.w * (d.w - a.w * inv - (v.w - m.w) * r.w * b.w * inv);
      if (dx) *reinterpret_cast<float4*>(dx + 4 * i) = o;
      if (dxb) dxb[i] = pack4(o);
    }
  }
}

// a grid of back-to-back barriers (gsync_barrier_us: the cost of one)
__global__ __launch_bounds__(256) void barrier_lab_kernel(GridBar bar, int iters) {
  for (int k = 0; k < iters; ++k) grid_barrier(bar);
}

static inline int grid_elems(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

static inline int nblocks(long long rows, int C) {
  long long nb;
  if (C % 4 == 0) {  // vector path: PT threads, >= 8 row passes, <= 256 blocks
    int RP = 1;
    while (RP * 2 * (C / 4) <= PT) RP *= 2;
    nb = (rows + RP * 8 - 1) / (RP * 8);
    if (nb > 256) nb = 256;
  } else {
    const int RP = 256 / C;
    nb = (rows + RP * 16 - 1) / (RP * 16);  // >= 16 row passes per block
    if (nb > 1024) nb = 1024;
  }
  return (int)(nb < 1 ? 1 : nb);
}

}  // namespace bn

// vector path: C % 4 == 0, C <= 1024; scalar path (column sums only): C <= 256
bool chan_reduce_ok(int C) { return (C % 4 == 0 && C >= 4 && C <= 1024) || (C >= 1 && C <= 256); }

long long chan_reduce_ws_floats(long long rows, int C) {
  return chan_reduce_ok(C) ? (long long)bn::nblocks(rows, C) * 2 * C : 0;
}

template <bool XB, bool YB>
static void run_partials_t(int mode, const void* a, const float* b, const void* y,
                           const void* mean, const float* rstd, int relu, long long rows, int C,
                           float* ws, int nb, const bn::Fin& fin, hipStream_t st, bool finalize) {
  const int rpb = (int)((rows + nb - 1) / nb);
  switch (mode) {
    case bn::SUM_SQ:
      bn::partial_kernel<bn::SUM_SQ, XB, YB><<<nb, bn::PT, 0, st>>>(a, b, y, mean, rstd, relu, rows, C, rpb, ws);
      break;
    case bn::SUM_PROD:
      bn::partial_kernel<bn::SUM_PROD, XB, YB><<<nb, bn::PT, 0, st>>>(a, b, y, mean, rstd, relu, rows, C, rpb, ws);
      break;
    default:
      bn::partial_kernel<bn::BN_BWD, XB, YB><<<nb, bn::PT, 0, st>>>(a, b, y, mean, rstd, relu, rows, C, rpb, ws);
  }
  if (finalize) bn::finalize_kernel<<<C, 256, 0, st>>>(ws, nb, C, rows, fin, 0);
}

// finalize = false: only the partial rows (the caller's fused launch finalizes)
static void run_partials(int mode, const void* a, bool ab16, const float* b, const void* y,
                         bool yb16, const void* mean, const float* rstd, int relu, long long rows,
                         int C, float* ws, int nb, const bn::Fin& fin, hipStream_t st,
                         bool finalize = true) {
  if (ab16 && yb16)
    run_partials_t<true, true>(mode, a, b, y, mean, rstd, relu, rows, C, ws, nb, fin, st, finalize);
  else if (ab16)
    run_partials_t<true, false>(mode, a, b, y, mean, rstd, relu, rows, C, ws, nb, fin, st, finalize);
  else if (yb16)
    run_partials_t<false, true>(mode, a, b, y, mean, rstd, relu, rows, C, ws, nb, fin, st, finalize);
  else
    run_partials_t<false, false>(mode, a, b, y, mean, rstd, relu, rows, C, ws, nb, fin, st, finalize);
}

static bn::Fin sums(float* s1, float* s2) {
  return {s1, s2, 0, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
}

void chan_reduce(const float* a, const float* b, long long rows, int C, float* s1, float* s2,
                 int mode, float* ws, hipStream_t st) {
  if (!chan_reduce_ok(C)) throw std::runtime_error("chan_reduce: unsupported channel count");
  const int nb = bn::nblocks(rows, C);
  if (C % 4 == 0 && C <= 1024) {
    run_partials(mode, a, false, b, nullptr, false, nullptr, nullptr, 0, rows, C, ws, nb,
                 sums(s1, s2), st);
  } else {
    const int rpb = (int)((rows + nb - 1) / nb);
    bn::partial1_kernel<<<nb, 256, 0, st>>>(a, b, mode, rows, C, rpb, ws);
    bn::finalize_kernel<<<C, 256, 0, st>>>(ws, nb, C, rows, sums(s1, s2), 0);
  }
}

// the fused launches' barrier state and grid cap (one device per process)
static bn::GridBar g_bar{nullptr, nullptr, nullptr};
static int g_fused_cap = 0;
static bool g_fused_on = false;  // opt-in: PERF_NOTES round 6

static int g_bpc = bn::FUSED_BLOCKS_PER_CU;

// blocks a CU holds of every fused kernel (VGPRs: the backward ones hold 3)
static int fused_occupancy() {
  int lo = 8;
  auto occ = [&](const void* f) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) n = 0;
    lo = std::min(lo, n);
  };
  occ(reinterpret_cast<const void*>(&bn::finalize_apply_kernel<true>));
  occ(reinterpret_cast<const void*>(&bn::finalize_apply_kernel<false>));
  occ(reinterpret_cast<const void*>(&bn::finalize_bwd_apply_kernel<true, true>));
  occ(reinterpret_cast<const void*>(&bn::finalize_bwd_apply_kernel<true, false>));
  occ(reinterpret_cast<const void*>(&bn::finalize_bwd_apply_kernel<false, true>));
  occ(reinterpret_cast<const void*>(&bn::finalize_bwd_apply_kernel<false, false>));
  return lo;
}

static bool fused_ready() {
  if (!g_fused_on) return false;
  if (!g_bar.cnt) {
    g_bar = gsync::tu_bar();
    g_fused_cap = gsync::cu_count() * std::min(g_bpc, fused_occupancy());
  }
  return g_fused_cap > 0;
}

void bn_set_fused(bool on) { g_fused_on = on; }
void bn_set_fused_blocks_per_cu(int bpc) {
  if (bpc < 1 || bpc > 8) throw std::runtime_error("bn_set_fused_blocks_per_cu: 1..8");
  g_bpc = bpc;
  g_fused_cap = g_bar.cnt ? gsync::cu_count() * std::min(g_bpc, fused_occupancy()) : 0;
}
int bn_fused_grid_cap() { fused_ready(); return g_fused_cap; }

float gsync_barrier_us(int blocks, int iters) {
  int occ = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &occ, reinterpret_cast<const void*>(&bn::barrier_lab_kernel), 256, 0));
  if (blocks < 1 || blocks > gsync::cu_count() * occ || iters < 1)
    throw std::runtime_error("gsync_barrier_us: 1 <= blocks <= resident capacity");
  const bn::GridBar bar = gsync::tu_bar();
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  bn::barrier_lab_kernel<<<blocks, 256>>>(bar, 1);  // warm
  HIP_CHECK(hipEventRecord(e0, nullptr));
  bn::barrier_lab_kernel<<<blocks, 256>>>(bar, iters);
  HIP_CHECK(hipEventRecord(e1, nullptr));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  return 1000.f * ms / (float)iters;
}
unsigned bn_fused_error() { return g_bar.cnt ? gsync::bar_error(g_bar) : 0u; }

void bn_fwd(const void* x, long long rows, int C, const float* g, const float* b,
            const float* res, float* y, float* mean, float* rstd, float* ws, float eps,
            float momentum, bool relu, bool training, float* rmean, float* rvar, hipStream_t st,
            void* yb, bool xb16) {
  if (C % 4 != 0 || C > 1024) throw std::runtime_error("bn_fwd: needs C % 4 == 0, C <= 1024");
  const long long n4 = rows * C / 4;
  uint2* ybv = reinterpret_cast<uint2*>(yb);
  if (training) {
    const int nb = bn::nblocks(rows, C);
    // shift K = row 0 of x (passed as the partials' `mean`)
    const bn::Fin fin{nullptr, nullptr, 1, eps, momentum, mean, rstd, rmean, rvar, x, xb16 ? 1 : 0};
    if (fused_ready()) {  // statistics pass, then finalize + apply in one launch
      run_partials(bn::SUM_SQ, x, xb16, nullptr, nullptr, false, x, nullptr, 0, rows, C, ws, nb,
                   fin, st, /*finalize=*/false);
      const int grid = std::min(bn::grid_elems(n4), g_fused_cap);
      if (xb16)
        bn::finalize_apply_kernel<true><<<grid, 256, 0, st>>>(ws, nb, 0, rows, fin, g_bar, x, g, b,
                                                              res, y, n4, C, relu ? 1 : 0, ybv);
      else
        bn::finalize_apply_kernel<false><<<grid, 256, 0, st>>>(ws, nb, 0, rows, fin, g_bar, x, g, b,
                                                               res, y, n4, C, relu ? 1 : 0, ybv);
      return;
    }
    run_partials(bn::SUM_SQ, x, xb16, nullptr, nullptr, false, x, nullptr, 0, rows, C, ws, nb, fin,
                 st);
    if (xb16)
      bn::apply_kernel<true><<<bn::grid_elems(n4), 256, 0, st>>>(x, mean, rstd, g, b, res, y, n4, C,
                                                                 relu ? 1 : 0, 0, eps, ybv);
    else
      bn::apply_kernel<false><<<bn::grid_elems(n4), 256, 0, st>>>(x, mean, rstd, g, b, res, y, n4,
                                                                  C, relu ? 1 : 0, 0, eps, ybv);
  } else {
    if (xb16)
      bn::apply_kernel<true><<<bn::grid_elems(n4), 256, 0, st>>>(x, rmean, rvar, g, b, res, y, n4,
                                                                 C, relu ? 1 : 0, 1, eps, ybv);
    else
      bn::apply_kernel<false><<<bn::grid_elems(n4), 256, 0, st>>>(x, rmean, rvar, g, b, res, y, n4,
                                                                  C, relu ? 1 : 0, 1, eps, ybv);
  }
}

void bn_fwd_partials(const float* part, int P, const float* shift, const void* x, long long rows,
                     int C, const float* g, const float* b, const float* res, float* y, float* mean,
                     float* rstd, float eps, float momentum, bool relu, float* rmean, float* rvar,
                     hipStream_t st, void* yb, bool xb16) {
  if (C % 64 != 0 || C > 1024 || P < 1 || !part || !shift || shift != rmean)
    throw std::runtime_error("bn_fwd_partials: needs C % 64 == 0, C <= 1024, shift == rmean");
  const long long n4 = rows * C / 4;
  uint2* ybv = reinterpret_cast<uint2*>(yb);
  // fp32 shift (the running mean, read by fin_channel before its update)
  const bn::Fin fin{nullptr, nullptr, 1, eps, momentum, mean, rstd, rmean, rvar, shift, 0};
  if (fused_ready()) {  // finalize + apply in one launch
    const int grid = std::min(bn::grid_elems(n4), g_fused_cap);
    if (xb16)
      bn::finalize_apply_kernel<true><<<grid, 256, 0, st>>>(part, P, 1, rows, fin, g_bar, x, g, b,
                                                            res, y, n4, C, relu ? 1 : 0, ybv);
    else
      bn::finalize_apply_kernel<false><<<grid, 256, 0, st>>>(part, P, 1, rows, fin, g_bar, x, g, b,
                                                             res, y, n4, C, relu ? 1 : 0, ybv);
    return;
  }
  bn::finalize_grp64(part, P, C, rows, fin, st);
  if (xb16)
    bn::apply_kernel<true><<<bn::grid_elems(n4), 256, 0, st>>>(x, mean, rstd, g, b, res, y, n4, C,
                                                               relu ? 1 : 0, 0, eps, ybv);
  else
    bn::apply_kernel<false><<<bn::grid_elems(n4), 256, 0, st>>>(x, mean, rstd, g, b, res, y, n4, C,
                                                                relu ? 1 : 0, 0, eps, ybv);
}

void bn_bwd(const void* x, const float* dy, const void* y, const float* mean, const float* rstd,
            const float* g, long long rows, int C, bool relu, float* ws, float* dg, float* db,
            float* dx, float* dres, hipStream_t st, void* dxb, bool xb16, bool yb16) {
  if (C % 4 != 0 || C > 1024) throw std::runtime_error("bn_bwd: needs C % 4 == 0, C <= 1024");
  if (!dx && !dxb) throw std::runtime_error("bn_bwd: no dx output");
  const int nb = bn::nblocks(rows, C);
  const long long n4 = rows * C / 4;
  uint2* dxbv = reinterpret_cast<uint2*>(dxb);
  const int rl = relu ? 1 : 0;
  // db = sum dy', dg = sum dy' xhat
  const bool fused = fused_ready() && db && dg;
  run_partials(bn::BN_BWD, x, xb16, dy, y, yb16, mean, rstd, relu ? 1 : 0, rows, C, ws, nb,
               sums(db, dg), st, /*finalize=*/!fused);
  if (fused) {  // finalize + apply in one launch
    const int grid = std::min(bn::grid_elems(n4), g_fused_cap);
#define FBWD(XB_, YB_)                                                                          \
  bn::finalize_bwd_apply_kernel<XB_, YB_><<<grid, 256, 0, st>>>(ws, nb, 0, sums(db, dg), g_bar, x, \
                                                                dy, y, mean, rstd, g, dx, dres, n4, \
                                                                C, rows, rl, dxbv)
    if (xb16 && yb16)
      FBWD(true, true);
    else if (xb16)
      FBWD(true, false);
    else if (yb16)
      FBWD(false, true);
    else
      FBWD(false, false);
#undef FBWD
    return;
  }
  const int gr = bn::grid_elems(n4);
#define BWD_APPLY(XB_, YB_)                                                               \
  bn::bwd_apply_kernel<XB_, YB_><<<gr, 256, 0, st>>>(x, dy, y, mean, rstd, g, db, dg, dx, dres, \
                                                     n4, C, rows, rl, dxbv)
  if (xb16 && yb16)
    BWD_APPLY(true, true);
  else if (xb16)
    BWD_APPLY(true, false);
  else if (yb16)
    BWD_APPLY(false, true);
  else
    BWD_APPLY(false, false);
#undef BWD_APPLY
}

void bn_bwd_partials(const float* part, int P, const void* x, const float* dy, const void* y,
                     const float* mean, const float* rstd, const float* g, long long rows, int C,
                     bool relu, float* dg, float* db, float* dx, float* dres, hipStream_t st,
                     void* dxb) {
  if (C % 64 != 0 || C > 1024 || P < 1 || !part || (!dx && !dxb) || (relu && !y))
    throw std::runtime_error("bn_bwd_partials: needs C % 64 == 0, C <= 1024, a dx output");
  // the dgrad epilogue's rows [2][C / 64][P][64] -> db, dg
  const long long n4 = rows * C / 4;
  if (fused_ready() && db && dg) {  // finalize + apply in one launch
    const int grid = std::min(bn::grid_elems(n4), g_fused_cap);
    bn::finalize_bwd_apply_kernel<true, true><<<grid, 256, 0, st>>>(
        part, P, 1, sums(db, dg), g_bar, x, dy, y, mean, rstd, g, dx, dres, n4, C, rows,
        relu ? 1 : 0, reinterpret_cast<uint2*>(dxb));
    return;
  }
  bn::finalize_grp64(part, P, C, rows, sums(db, dg), st);
  bn::bwd_apply_kernel<true, true><<<bn::grid_elems(n4), 256, 0, st>>>(
      x, dy, y, mean, rstd, g, db, dg, dx, dres, n4, C, rows, relu ? 1 : 0,
      reinterpret_cast<uint2*>(dxb));
}

}  // namespace gops

namespace gsync {
int cu_count() {
  int dev = 0, cus = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus;
}
unsigned bar_error(const GridBar& b) {
  unsigned v = 0;
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(&v, b.err, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}
}  // namespace gsync
