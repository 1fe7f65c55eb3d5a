// bf16 MFMA kernel set for the reference MNIST CNN on gfx950 (BASELINE config
// 2).  Same graph and fusion boundaries as the fp32 set (mnist.hip; reference
// /root/reference/mpipy.py:155-167, loss :54-58), but every GEMM-shaped op
// runs on v_mfma_f32_32x32x16_bf16 (16x the fp32-MFMA rate) with fp32
// accumulation, and activations travel in bf16 (layouts: mnist_bf16.h).
//
// Operand fetch: every wave owns a 32x32 output tile and streams its K range
// as 16-byte fragments (8 bf16 per lane: lane l holds A[l&31][8(l>>5)+j] and
// B[8(l>>5)+j][l&31]) straight from L2 into a D-deep register ring.  The
// producers of each operand write it K-packed ([K/16][rows][16], mnist_bf16.h)
// in exactly the form its consumer reads, so each fragment load is one
// contiguous 1 KB wave access, and no kernel here needs LDS staging, bounds
// checks or a transpose - only the split-K reductions touch LDS.  The filter
// grad reads its shifted operand at 2-byte alignment, which runs at full
// speed on gfx950 (scripts/microbench/unaligned_b128.hip).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "mnist_bf16.h"
#include "mnist_shared.h"

namespace mnist16 {

using bf = __bf16;
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
using mnist::FC1_IN;
using mnist::FC1_OUT;
using mnist::FC1_SPLITS;
using mnist::NCLS;

constexpr int TLD = MNIST16_T_LD;  // row length of the channel-major padded images

__device__ __forceinline__ bfx8 ld8(const bf* p) {
  return __builtin_bit_cast(bfx8, *reinterpret_cast<const uint4*>(p));
}

__device__ __forceinline__ f32x16 mma(bfx8 a, bfx8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sum8(bfx8 v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)v[j];
  return s;
}

// K loop over nks K-steps (nks % D == 0) with a D-deep register ring:
// frag(ks, a, b) issues the two 16-byte fragment loads of K-step ks and
// use(a, b) (optional) sees each fragment pair as it is consumed.  The
// sched_barriers pin each refill ahead of the MFMA that frees its slot (the
// scheduler would otherwise sink it next to its use); two accumulator chains
// keep consecutive MFMAs independent.
struct NoUse {
  __device__ __forceinline__ void operator()(const bfx8&, const bfx8&) const {}
};

template <int D, class F, class U = NoUse>
__device__ __forceinline__ void kloop(int nks, F&& frag, f32x16& c0, f32x16& c1, U use = U()) {
  bfx8 ra[D], rb[D];
#pragma unroll
  for (int d = 0; d < D; ++d) frag(d, ra[d], rb[d]);
#pragma unroll
  for (int ks = 0; ks < nks; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const bfx8 a = ra[d], b = rb[d];
      if (ks + D < nks) frag(ks + D + d, ra[d], rb[d]);
      __builtin_amdgcn_sched_barrier(0);
      if (d & 1)
        c1 = mma(a, b, c1);
      else
        c0 = mma(a, b, c0);
      use(a, b);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ---------------------------------------------------------- shadows ----
// The shadow conversion lives in mnist_shared.h (shadow_block); the train step
// runs it as a block role of the conv1 forward launch, the standalone kernel
// below serves callers that only need the shadows.
__global__ __launch_bounds__(256) void shadow_kernel(const float* __restrict__ w1,
                                                     const float* __restrict__ w2,
                                                     bf* __restrict__ w1b, bf* __restrict__ w1t,
                                                     bf* __restrict__ w2t, bf* __restrict__ w2b) {
  __shared__ float tile[64 * 65];
  mnist::shadow_block((int)blockIdx.x, {w1, w2, w1b, w1t, w2t, w2b}, tile);
}

// ------------------------------------------------------------ conv2 fwd ----
// M = pre-pool pixels of the whole batch in (n, py, px, quadrant) order (the 4
// pixels of a pooling window = 4 accumulator registers of one lane, see
// mnist.hip), N = 64 output channels, K = 25 taps x 2 channel halves.  One
// 32x32 tile per wave, 4 waves per block, no LDS.
constexpr int IMG = 18 * 18 * 16;  // one padded 16-channel image plane

__global__ __launch_bounds__(256) void conv2_fwd_kernel(const bf* __restrict__ a1p, int batch,
                                                        const bf* __restrict__ w2t,
                                                        const float* __restrict__ b2,
                                                        bf* __restrict__ a2p, bf* __restrict__ a2t,
                                                        uint8_t* __restrict__ idx2) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int mtiles = batch * 49 / 8;
  const int gw = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  if (gw >= 2 * mtiles) return;
  const int mt = gw >> 1, nt = gw & 1;
  const int m = mt * 32 + r, q = m & 3, win = m >> 2;
  const int n = win / 49, pp = win % 49, py = pp / 7, px = pp % 7;
  const int y = 2 * py + (q >> 1), x = 2 * px + (q & 1);
  const bf* ap = a1p + (size_t)n * IMG + (y * 18 + x) * 16 + 8 * h;
  const size_t splane = (size_t)batch * IMG;
  const bf* bp = w2t + (nt * 32 + r) * 16 + 8 * h;
  f32x16 c0 = zero16(), c1 = zero16();
  kloop<5>(
      50,
      [&](int ks, bfx8& a, bfx8& b) {
        const int t = ks >> 1, s = ks & 1, kh = t / 5, kw = t % 5;
        a = ld8(ap + s * splane + (kh * 18 + kw) * 16);
        b = ld8(bp + (t * 2 + s) * 1024);
      },
      c0, c1);
  const int co = nt * 32 + r;
  const float bias = b2[co];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float v = c0[4 * g] + c1[4 * g];
    int qq = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float u = c0[4 * g + j] + c1[4 * g + j];
      if (u > v) {  // strict: first max wins (TF MaxPool order)
        v = u;
        qq = j;
      }
    }
    const int w2_ = mt * 8 + 2 * g + h;  // pooling window of registers 4g..4g+3
    const int n2 = w2_ / 49, p2 = w2_ % 49;
    const int i = p2 * 64 + co;
    const bf out = (bf)fmaxf(v + bias, 0.f);
    a2p[((size_t)(i >> 4) * batch + n2) * 16 + (i & 15)] = out;
    if (idx2) idx2[(size_t)n2 * FC1_IN + i] = (uint8_t)qq;
    if (a2t) a2t[((size_t)(n2 >> 4) * FC1_IN + i) * 16 + (n2 & 15)] = out;
  }
}

// -------------------------------------------------------------- fc1 fwd ----
// M = rows, N = 512 hidden units, K = 3136.  Train: split-K slabs (z) of
// 14 K-steps; eval: the full K with bias + ReLU (+dropout) epilogue.  a2p
// holds `ld` rows per K-step.
template <bool EVAL, int D>
__global__ __launch_bounds__(256) void fc1_fwd_kernel(const bf* __restrict__ a2p, int ld,
                                                      const bf* __restrict__ w1t,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ out, int M, int nz,
                                                      uint32_t key, float keep_prob) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int mtiles = (M + 31) / 32;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= mtiles * (FC1_OUT / 32) * nz) return;
  const int mt = gw % mtiles, rest = gw / mtiles, nt = rest % (FC1_OUT / 32), z = rest / (FC1_OUT / 32);
  const int nks = FC1_IN / 16 / nz, k0 = z * nks;
  const int row = min(mt * 32 + r, M - 1);
  const bf* ap = a2p + ((size_t)k0 * ld + row) * 16 + 8 * h;
  const bf* bp = w1t + ((size_t)k0 * FC1_OUT + nt * 32 + r) * 16 + 8 * h;
  f32x16 c0 = zero16(), c1 = zero16();
  kloop<D>(
      nks,
      [&](int ks, bfx8& a, bfx8& b) {
        a = ld8(ap + (size_t)ks * ld * 16);
        b = ld8(bp + ks * FC1_OUT * 16);
      },
      c0, c1);
  const int n = nt * 32 + r;
  const float bn = EVAL ? bias[n] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = mt * 32 + mfma32_row(i, lane);
    if (m >= M) continue;
    const float acc = c0[i] + c1[i];
    if (EVAL) {
      float hv = fmaxf(acc + bn, 0.f);
      if (keep_prob < 1.f)
        hv = dropout_keep(key, (uint32_t)(m * FC1_OUT + n), keep_prob) ? hv / keep_prob : 0.f;
      out[(size_t)m * FC1_OUT + n] = hv;
    } else {
      out[((size_t)z * M + m) * FC1_OUT + n] = acc;
    }
  }
}

// -------------------------------------------------------------- fc1 bwd ----
// One launch, block roles: [0, n_dx) dX = dh W1^T (M = rows, N = 3136, K =
// 512) with the pool2 / ReLU2 backward scatter into dy2p and dy2t; then dW1 =
// a2^T dh (M = 3136, N = 512, K = rows) tiles; then the small fc2 / bias grads.
__global__ __launch_bounds__(256) void fc1_bwd_kernel(
    const bf* __restrict__ a2p, const bf* __restrict__ a2t, const uint8_t* __restrict__ idx2,
    const bf* __restrict__ dh16, const bf* __restrict__ dht16, const float* __restrict__ hd,
    const float* __restrict__ dh, const float* __restrict__ dlog, const bf* __restrict__ w1b,
    int batch, float* __restrict__ g_w3, float* __restrict__ g_b3, float* __restrict__ g_w4,
    float* __restrict__ g_b4, bf* __restrict__ dy2p, bf* __restrict__ dy2t) {
  __shared__ float smem[mnist::FC1_SMALL_SMEM];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int bm = batch / 32;
  const int n_dx = (bm * (FC1_IN / 32) + 3) / 4;
  constexpr int n_dw = (FC1_IN / 32) * (FC1_OUT / 32) / 4;
  int bid = blockIdx.x;
  f32x16 c0 = zero16(), c1 = zero16();
  if (bid < n_dx) {
    const int gw = bid * 4 + wave;
    if (gw >= bm * (FC1_IN / 32)) return;
    const int mt = gw % bm, nt = gw / bm;
    const bf* ap = dh16 + (size_t)(mt * 32 + r) * 16 + 8 * h;
    const bf* bp = w1b + (size_t)(nt * 32 + r) * 16 + 8 * h;
    kloop<8>(
        FC1_OUT / 16,
        [&](int ks, bfx8& a, bfx8& b) {
          a = ld8(ap + (size_t)ks * batch * 16);
          b = ld8(bp + (size_t)ks * FC1_IN * 16);
        },
        c0, c1);
    const int i = nt * 32 + r;  // (py, px, co) flat
    const int co = i & 63, pp = i >> 6, py = pp / 7, px = pp % 7;
    const size_t cplane = (size_t)(co >> 4) * batch * IMG + (co & 15);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int n = mt * 32 + mfma32_row(k, lane);
      float g = c0[k] + c1[k];
      const float a = (float)a2p[((size_t)(i >> 4) * batch + n) * 16 + (i & 15)];
      if (!(a > 0.f)) g = 0.f;  // ReLU2 inactive at the argmax
      const int q = idx2[(size_t)n * FC1_IN + i];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int y = 2 * py + (d >> 1), x = 2 * px + (d & 1);
        const bf v = (bf)(d == q ? g : 0.f);
        dy2p[cplane + (size_t)n * IMG + ((y + 2) * 18 + x + 2) * 16] = v;
        dy2t[((size_t)(n * 14 + y) * 64 + co) * 16 + x] = v;
      }
    }
    return;
  }
  bid -= n_dx;
  if (bid < n_dw) {
    const int gw = bid * 4 + wave;
    const int mi = gw % (FC1_IN / 32), nj = gw / (FC1_IN / 32);
    const bf* ap = a2t + (size_t)(mi * 32 + r) * 16 + 8 * h;
    const bf* bp = dht16 + (size_t)(nj * 32 + r) * 16 + 8 * h;
    kloop<2>(
        batch / 16,
        [&](int ks, bfx8& a, bfx8& b) {
          a = ld8(ap + (size_t)ks * FC1_IN * 16);
          b = ld8(bp + (size_t)ks * FC1_OUT * 16);
        },
        c0, c1);
    const int n = nj * 32 + r;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int m = mi * 32 + mfma32_row(k, lane);
      g_w3[(size_t)m * FC1_OUT + n] = c0[k] + c1[k];
    }
    return;
  }
  bid -= n_dw;
  mnist::fc1_small_grads(bid, hd, dh, dlog, batch, g_w4, g_b4, g_b3, smem);
}

// ------------------------------------------------------ conv2 bwd-data ----
// dA1[n,y,x,ci] = [a1 > 0] sum_{kh,kw,co} dY2[n, y+2-kh, x+2-kw, co] W2[kh,kw,ci,co]:
// M = pixels (n, y, x), N = 32 input channels, K = 25 taps x 4 channel
// chunks.  Block = 2 M tiles x 2 K halves (chunks 0-1 / 2-3), summed in LDS.
__global__ __launch_bounds__(256) void conv2_bwd_data_kernel(const bf* __restrict__ dy2p,
                                                             const bf* __restrict__ w2b,
                                                             const bf* __restrict__ a1p, int batch,
                                                             float* __restrict__ da1m,
                                                             const mnist::FcSgd sgd) {
  constexpr int SM = mnist::SHADOW_SMEM_FLOATS > 2 * 16 * 64 ? mnist::SHADOW_SMEM_FLOATS : 2 * 16 * 64;
  __shared__ float smem[SM];
  if ((int)blockIdx.x >= (int)gridDim.x - sgd.nblk) {  // world-1 FC SGD role (mnist_shared.h)
    mnist::fc_sgd_role(sgd, blockIdx.x - (gridDim.x - sgd.nblk), smem);
    return;
  }
  auto red = reinterpret_cast<float(*)[16][64]>(smem);
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int mtiles = batch * 196 / 32;
  const int mt_raw = blockIdx.x * 2 + (wave & 1), kk = wave >> 1;
  const int mt = min(mt_raw, mtiles - 1);
  const int m = mt * 32 + r, n = m / 196, p = m % 196, y = p / 14, x = p % 14;
  const size_t cplane = (size_t)batch * IMG;
  const bf* ap = dy2p + 2 * kk * cplane + (size_t)n * IMG + ((y + 4) * 18 + x + 4) * 16 + 8 * h;
  const bf* bp = w2b + (2 * kk * 32 + r) * 16 + 8 * h;
  f32x16 c0 = zero16(), c1 = zero16();
  kloop<5>(
      50,
      [&](int ks, bfx8& a, bfx8& b) {
        const int t = ks >> 1, s = ks & 1, kh = t / 5, kw = t % 5;
        a = ld8(ap + s * cplane - (kh * 18 + kw) * 16);
        b = ld8(bp + (t * 4 + s) * 512);
      },
      c0, c1);
  if (kk == 1) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[wave & 1][k][lane] = c0[k] + c1[k];
  }
  __syncthreads();
  if (kk == 1 || mt_raw >= mtiles) return;
  const bf* a1c = a1p + (size_t)(r >> 4) * cplane + (r & 15);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int mm = mt * 32 + mfma32_row(k, lane);
    const int nn = mm / 196, pq = mm % 196, yy = pq / 14, xx = pq % 14;
    const float g = c0[k] + c1[k] + red[wave & 1][k][lane];
    const float a = (float)a1c[(size_t)nn * IMG + ((yy + 2) * 18 + xx + 2) * 16];
    da1m[(size_t)mm * 32 + r] = a > 0.f ? g : 0.f;
  }
}

// ---------------------------------------------------- conv2 bwd-filter ----
// dW2[t][ci][co] = sum_{n,y,x} a1[n, y+kh-2, x+kw-2, ci] dY2[n, y, x, co]:
// M = 32 input channels, N = 64 output channels (2 tiles), K = pixels, one
// K-step = one image row (x = 0..15; dy2t columns 14/15 are zero).  Block =
// (tap, group of 8 images); 8 waves = 2 (co half) x 4 (image pairs), the
// image pairs summed through LDS into one slab per group.  The centre tap
// (which visits every pixel once) also sums dY2 per channel (db2).
constexpr int C2F_IMG = 8;

// filter-grad block bid (< 25 x groups) of 512 threads; smem >= 3 x 2 x 16 x 64
__device__ __forceinline__ void conv2_bwd_filter_body(int bid, const bf* __restrict__ a1t,
                                                      const bf* __restrict__ dy2t, int batch,
                                                      float* __restrict__ part2,
                                                      float* __restrict__ part_db2, float* smem) {
  auto red = reinterpret_cast<float(*)[2][16][64]>(smem);
  const int ngroups = (batch + C2F_IMG - 1) / C2F_IMG;
  int t, g;
  if (ngroups % 8 == 0) {  // all taps of an image group on one XCD (shared L2)
    const int xx = bid & 7, idx = bid >> 3;
    t = idx % 25;
    g = xx + 8 * (idx / 25);
  } else {
    t = bid % 25;
    g = bid / 25;
  }
  const int kh = t / 5, kw = t % 5;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int nt = wave & 1, ip = wave >> 1;
  const int co = nt * 32 + r;
  f32x16 c0 = zero16(), c1 = zero16();
  float dbs = 0.f;
#pragma unroll
  for (int im = 0; im < 2; ++im) {
    const int n = g * C2F_IMG + 2 * ip + im;
    if (n < batch) {
      const bf* ap = a1t + ((size_t)(n * 18 + kh) * 32 + r) * TLD + kw + 8 * h;
      const bf* bp = dy2t + ((size_t)n * 14 * 64 + co) * 16 + 8 * h;
      kloop<7>(
          14,
          [&](int y, bfx8& a, bfx8& b) {
            a = ld8(ap + y * 32 * TLD);
            b = ld8(bp + y * 64 * 16);
          },
          c0, c1, [&](const bfx8&, const bfx8& b) {
            if (t == 12) dbs += sum8(b);
          });
    }
  }
  f32x16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = c0[k] + c1[k];
  if (ip > 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[ip - 1][nt][k][lane] = acc[k];
  }
  __syncthreads();
  if (ip == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float s = acc[k] + red[0][nt][k][lane] + red[1][nt][k][lane] + red[2][nt][k][lane];
      const int ci = mfma32_row(k, lane);
      part2[((size_t)g * 800 + t * 32 + ci) * 64 + co] = s;
    }
  }
  if (t == 12) {
    dbs += __shfl_xor(dbs, 32, 64);
    if (h == 0) part_db2[(g * 4 + ip) * 64 + co] = dbs;
  }
}

__global__ __launch_bounds__(512) void conv2_bwd_filter_kernel(const bf* __restrict__ a1t,
                                                               const bf* __restrict__ dy2t,
                                                               int batch, float* __restrict__ part2,
                                                               float* __restrict__ part_db2,
                                                               int nc2, const mnist::C1Filter c1f) {
  constexpr int SM = 3 * 2 * 16 * 64 > mnist::C1F_SMEM ? 3 * 2 * 16 * 64 : mnist::C1F_SMEM;
  __shared__ float smem[SM];
  if ((int)blockIdx.x >= nc2) {  // conv1 filter-grad role (mnist_shared.h)
    mnist::conv1_filter_unit<512>(blockIdx.x - nc2, batch, c1f, smem);
    return;
  }
  conv2_bwd_filter_body(blockIdx.x, a1t, dy2t, batch, part2, part_db2, smem);
}

// ------------------------------------------------ conv2 backward, merged ----
// The whole conv2 backward in ONE launch of 512-thread blocks (the fp32 set's
// merged Winograd launch is the model).  Standalone, bwd-data (196 blocks) and
// bwd-filter (200) each left CUs idle with their operand latency exposed: the
// two launches ran 25.3 us, this one ~17 (step 64.8 -> 57.2 us).  Roles:
//   [0, nd)             bwd-data: 64 pooled pixels (2 M tiles) a block, 8 waves
//                       = 2 tiles x 4 K quarters (one 16-channel dY2 chunk
//                       each, 25 taps), summed in LDS; then the conv1
//                       filter-grad partial of those pixels from the masked dA1
//                       they just produced, kept in LDS (one part1 row per
//                       block: no second pass over da1m and no role that has to
//                       wait for it);
//   [nd, nd + nc2)      filter grad: the conv2_bwd_filter_kernel body;
//   [nd + nc2, ...)     the single-rank FC SGD (two fc_sgd_role units a round).
// Every global operand of the data role is requested up front (all its blocks
// load at the launch start, where a round trip costs several us - per-phase
// stamps, scripts/c2b_stamps.py): the dY2 rows of its pixels (staged into LDS,
// no per-K-step L2 latency), a1 for the ReLU1 mask, the input images and pool1
// argmax bytes for conv1, all coalesced.
// The conv1 filter grad of a block is one fp32-MFMA GEMM: dW1[tap][co] = sum
// over k = (pixel, pool1 quadrant q) of X[tap][k] S[k][co], X = the input
// window of the pixel at quadrant q (row 25: 1, the bias), S = the masked dA1
// where the channel's argmax IS q, else 0: K = 64 x 4, 16 products of
// v_mfma_f32_32x32x2f32 a wave.  (Per-thread FMA loops over the 25 taps, the
// conv1_filter_unit form, cost ~2x: 2-way conflicted LDS reads.)  The images
// sit in LDS with a 37-float row pitch: one window's 25 taps, 25 banks.
constexpr int C2B_PIX = 64;                  // pooled pixels per data block
constexpr int C2B_RED = 2 * 3 * 16 * 64;     // K quarters 1..3 of the 2 tiles
constexpr int C2B_DA = C2B_PIX * 32;         // masked dA1 of the block's pixels
constexpr int C2B_XLD = 37, C2B_XIMG = 32 * C2B_XLD;
constexpr int C2B_XS = 2 * C2B_XIMG;         // <= 2 input images, zero-padded by 2
constexpr int C2B_QS = C2B_PIX * 32 / 4;     // pool1 argmax bytes
constexpr int C2B_CRED = 8 * 832;            // per-wave conv1 partials
constexpr int C2B_A1S = C2B_PIX * 32 / 2;    // a1 (the ReLU1 mask source), bf16
constexpr int C2B_DATA_SM = C2B_RED + C2B_DA + C2B_XS + C2B_QS + C2B_CRED + C2B_A1S;
// the staged dY2 rows alias dA .. cred (used only after the K loop)
constexpr int C2B_ROWS = 16;
static_assert(4 * 2 * C2B_ROWS * 18 * 4 <= C2B_DA + C2B_XS + C2B_QS + C2B_CRED, "dY2 stage");
constexpr int C2B_FILT_SM = 3 * 2 * 16 * 64;
constexpr int C2B_SM = C2B_DATA_SM > C2B_FILT_SM ? C2B_DATA_SM : C2B_FILT_SM;
static_assert(C2B_SM >= 2 * 64 * 65, "FC SGD tiles of two units");

__device__ __forceinline__ void c2b_data_block(int db, const bf* __restrict__ dy2p,
                                               const bf* __restrict__ w2b,
                                               const bf* __restrict__ a1p, int batch,
                                               float* __restrict__ da1m,
                                               const mnist::C1Filter& c1, float* smem,
                                               unsigned long long* __restrict__ stamps) {
  // stamps (labs): wave 0's clock after each phase -> stamps[0..4]
  auto stamp = [&](int i) {
    if (stamps && threadIdx.x == 0) stamps[i] = __builtin_amdgcn_s_memrealtime();
  };
  auto red = reinterpret_cast<float(*)[3][16][64]>(smem);  // [tile][K quarter - 1][k][lane]
  float* dA = smem + C2B_RED;
  float* xs = dA + C2B_DA;
  uint8_t* qs = reinterpret_cast<uint8_t*>(xs + C2B_XS);
  float* cred = xs + C2B_XS + C2B_QS;
  uint16_t* a1s = reinterpret_cast<uint16_t*>(cred + C2B_CRED);  // own region
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5, wave = tid >> 6;
  const int tl = wave & 1, kq = wave >> 1;
  const int M = batch * 196, mtiles = M / 32, pbase = db * C2B_PIX;
  const int mt_raw = db * 2 + tl;
  const int mt = min(mt_raw, mtiles - 1);
  const bool conv1 = c1.part1 != nullptr;
  const int n_first = pbase / 196;
  // dY2 rows: image n0's padded rows ya0 .. ya1 + 4, then (pixels past that
  // image) image n0 + 1's rows 0 .. yb1 + 4, all 18 columns, as [chunk 4]
  // [half 2][row][18][8 bf16] - a 16-lane group of a fragment read covers 256
  // contiguous bytes
  const size_t cplane = (size_t)batch * IMG;
  const int pend = min(pbase + C2B_PIX, M), pa_end = min(pend, (n_first + 1) * 196);
  const int ya0 = (pbase - n_first * 196) / 14, ya1 = (pa_end - 1 - n_first * 196) / 14;
  const int Ra = ya1 - ya0 + 5;
  const int Rb = pend > pa_end ? (pend - 1 - (n_first + 1) * 196) / 14 + 5 : 0;
  const int R = Ra + Rb;  // <= C2B_ROWS
  uint4* stg = reinterpret_cast<uint4*>(dA);
  constexpr int SJ = (4 * C2B_ROWS * 18 * 2 + 511) / 512;
  uint4 sv[SJ];
  const int npc = 4 * R * 18 * 2;
#pragma unroll
  for (int j = 0; j < SJ; ++j) {
    const int i = min(tid + 512 * j, npc - 1);
    const int hh = i & 1, col = (i >> 1) % 18, rw = (i >> 1) / 18, row = rw % R, c = rw / R;
    const int nn = row < Ra ? n_first : n_first + 1, Y = row < Ra ? ya0 + row : row - Ra;
    sv[j] = *reinterpret_cast<const uint4*>(dy2p + c * cplane + (size_t)nn * IMG +
                                            (Y * 18 + col) * 16 + 8 * hh);
  }
  // a1 of the block's pixels x 32 channels, a 16-byte piece a thread (< 256)
  uint4 a1v = make_uint4(0u, 0u, 0u, 0u);
  {
    const int pl = tid >> 2, pg = pbase + pl, pc = (tid >> 1) & 1, hh = tid & 1;
    if (pl < C2B_PIX && pg < M) {
      const int nn = pg / 196, pp = pg % 196, yy = pp / 14, xx = pp % 14;
      a1v = *reinterpret_cast<const uint4*>(a1p + pc * cplane + (size_t)nn * IMG +
                                            ((yy + 2) * 18 + xx + 2) * 16 + 8 * hh);
    }
  }
  // conv1 operands: the input images (the block's pixels span <= 2) and the
  // pool1 argmax bytes (contiguous: 8 a thread, < 256)
  constexpr int XJ = (C2B_XS + 511) / 512;
  float xv[XJ];
  uint2 qv = make_uint2(0u, 0u);
  if (conv1) {
    if (tid < C2B_PIX * 4 && pbase + (tid >> 2) < M)
      qv = *reinterpret_cast<const uint2*>(c1.idx1 + (size_t)pbase * 32 + 8 * tid);
    const long long off = mnist::batch_offset_dev(c1.step, c1.n_local, batch);
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int i = tid + 512 * j;
      const int im = i / C2B_XIMG, rc = i - im * C2B_XIMG, row = rc / C2B_XLD;
      const int nn = n_first + im, yy = row - 2, xx = rc - row * C2B_XLD - 2;
      const bool ok = i < C2B_XS && nn < batch && yy >= 0 && yy < 28 && xx >= 0 && xx < 28;
      xv[j] = c1.data[ok ? (off + nn) * 784 + yy * 28 + xx : off * 784];
      if (!ok) xv[j] = 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < SJ; ++j) {
    const int i = tid + 512 * j;
    if (i < npc) {
      const int hh = i & 1, col = (i >> 1) % 18, rw = (i >> 1) / 18, row = rw % R, c = rw / R;
      stg[((c * 2 + hh) * R + row) * 18 + col] = sv[j];
    }
  }
  if (tid < C2B_PIX * 4) reinterpret_cast<uint4*>(a1s)[tid] = a1v;  // a1s[pixel][channel]
  __syncthreads();
  stamp(0);
  // this lane's pixel (a dead tile - M % 32 == 0 - takes the block's first)
  const int m = mt_raw < mtiles ? mt_raw * 32 + r : pbase, n = m / 196, p = m % 196,
            y = p / 14, x = p % 14;
  const int row0 = (n == n_first ? y - ya0 : Ra + y) + 4;  // LDS row of tap kh = 0
  const uint4* sa = stg + ((kq * 2 + h) * R + row0) * 18 + x + 4;
  const bf* bp = w2b + (kq * 32 + r) * 16 + 8 * h;
  f32x16 c0 = zero16(), c1a = zero16();
  kloop<5>(
      25,
      [&](int t, bfx8& a, bfx8& b) {
        const int kh = t / 5, kw = t % 5;
        a = __builtin_bit_cast(bfx8, sa[-kh * 18 - kw]);
        b = ld8(bp + t * 4 * 512);
      },
      c0, c1a);
  stamp(1);
  if (kq > 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[tl][kq - 1][k][lane] = c0[k] + c1a[k];
  }
  __syncthreads();
  if (kq == 0) {
    const bool live = mt_raw < mtiles;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int mm = mt * 32 + mfma32_row(k, lane);
      const float g = ((c0[k] + c1a[k]) + red[tl][0][k][lane]) + (red[tl][1][k][lane] +
                                                                  red[tl][2][k][lane]);
      const float a = __uint_as_float(
          (uint32_t)a1s[(tl * 32 + mfma32_row(k, lane)) * 32 + r] << 16);
      const float v = a > 0.f ? g : 0.f;
      if (live) da1m[(size_t)mm * 32 + r] = v;
      dA[(tl * 32 + mfma32_row(k, lane)) * 32 + r] = live ? v : 0.f;
    }
  }
  stamp(2);
  if (!conv1) return;  // block-uniform
#pragma unroll
  for (int j = 0; j < XJ; ++j)
    if (tid + 512 * j < C2B_XS) xs[tid + 512 * j] = xv[j];
  if (tid < C2B_PIX * 4) reinterpret_cast<uint2*>(qs)[tid] = qv;
  __syncthreads();
  stamp(3);
  // wave w: pixels 8 w .. 8 w + 7; K-step pair (2 j, 2 j + 1) of pixel j
  // covers its quadrants q = h (row pair 0) and q = 2 + h (row pair 1).  Four
  // pixels' operands are read before their 8 products.
  const int ti = r, kh = ti / 5, kw = ti - 5 * kh;  // A row = tap (25: bias, 26..31: 0)
  const float a_fix = ti == 25 ? 1.f : 0.f;
  f32x16 cw = zero16();
#pragma unroll
  for (int jb = 0; jb < 8; jb += 4) {
    float ae[4], ao[4], bv[4];
    int qb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int pl = 8 * wave + jb + u, pg = pbase + pl;
      const int nn = pg / 196, pp = pg - 196 * nn, py = pp / 14, px = pp - 14 * py;
      const float* xr = xs + (nn - n_first) * C2B_XIMG + (2 * py + kh) * C2B_XLD + 2 * px + h + kw;
      ae[u] = ti < 25 ? xr[0] : a_fix;
      ao[u] = ti < 25 ? xr[C2B_XLD] : a_fix;
      bv[u] = dA[pl * 32 + r];
      qb[u] = qs[pl * 32 + r];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cw = mfma32x32x2(ae[u], qb[u] == h ? bv[u] : 0.f, cw);
      cw = mfma32x32x2(ao[u], qb[u] == 2 + h ? bv[u] : 0.f, cw);
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int t = mfma32_row(k, lane);
    if (t < 26) cred[wave * 832 + t * 32 + r] = cw[k];
  }
  __syncthreads();
  stamp(4);
  for (int i = tid; i < 832; i += 512) {
    float sum = 0.f;
#pragma unroll
    for (int wv = 0; wv < 8; ++wv) sum += cred[wv * 832 + i];
    c1.part1[(size_t)db * 832 + i] = sum;
  }
}

// Blocks [0, nd) data, [nd, nd + nc2) filter grad, then the FC SGD: the data
// role is the longest (its operands' round trips at the launch start), so its
// loads go first (data first: 57.2 vs 59.2 us a step, scripts/sessions/r5_s25.steps)
__global__ __launch_bounds__(512) void conv2_bwd_kernel(
    const bf* __restrict__ dy2p, const bf* __restrict__ w2b, const bf* __restrict__ a1p,
    const bf* __restrict__ a1t, const bf* __restrict__ dy2t, int batch, float* __restrict__ da1m,
    float* __restrict__ part2, float* __restrict__ part_db2, int nc2, int nd,
    const mnist::C1Filter c1, const mnist::FcSgd sgd, unsigned long long* __restrict__ prof) {
  __shared__ float smem[C2B_SM];
  const int b = blockIdx.x;
  // prof (labs): per block [start, end] of the constant 100 MHz clock, then 8
  // phase stamps per data block
  unsigned long long t0 = 0;
  if (prof) t0 = __builtin_amdgcn_s_memrealtime();
  if (b < nd) {
    c2b_data_block(b, dy2p, w2b, a1p, batch, da1m, c1, smem,
                   prof ? prof + 2 * gridDim.x + 8 * b : nullptr);
  } else if (b < nd + nc2) {
    // (the filter role keeps its XCD grouping: blocks b and b' share an XCD
    // iff (b - nd) & 7 == (b' - nd) & 7)
    conv2_bwd_filter_body(b - nd, a1t, dy2t, batch, part2, part_db2, smem);
  } else {
    // FC SGD: two units a round (unit pairs take the same path - SHADOW_W1_BLOCKS
    // is even - so the tile path's barrier is met by both halves)
    const int half = threadIdx.x >> 8, nsg = gridDim.x - nc2 - nd;
    for (int u0 = 2 * (b - nc2 - nd); u0 < sgd.nblk; u0 += 2 * nsg) {
      const int u = u0 + half;
      if (u < sgd.nblk) mnist::fc_sgd_role(sgd, u, smem + half * 64 * 65, threadIdx.x & 255);
    }
  }
  if (prof) {
    __syncthreads();
    if (threadIdx.x == 0) {
      prof[2 * b] = t0;
      prof[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// lab: the FC SGD units as a launch of their own
__global__ __launch_bounds__(256) void fc_sgd_kernel(const mnist::FcSgd sgd) {
  __shared__ float tile[64 * 65];
  mnist::fc_sgd_role(sgd, blockIdx.x, tile);
}
}  // namespace mnist16

// ======================================================================
// host launchers
// ======================================================================
namespace mnist16 {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline const bf* C16(const uint16_t* p) { return reinterpret_cast<const bf*>(p); }
static inline bf* M16(uint16_t* p) { return reinterpret_cast<bf*>(p); }

void launch_shadows(const float* w1, const float* w2, uint16_t* w1b, uint16_t* w1t,
                    uint16_t* w2t, uint16_t* w2b, hipStream_t s) {
  shadow_kernel<<<mnist::SHADOW_BLOCKS, 256, 0, s>>>(w1, w2, M16(w1b), M16(w1t), M16(w2t),
                                                            M16(w2b));
}

void launch_conv2_fwd(const uint16_t* a1p, int batch, const uint16_t* w2t, const float* b2,
                      uint16_t* a2p, uint16_t* a2t, uint8_t* idx2, hipStream_t s) {
  if (batch % 8 != 0) throw std::runtime_error("mnist16 conv2_fwd: batch % 8 != 0");
  if (a2t && batch % 16 != 0) throw std::runtime_error("mnist16 conv2_fwd: a2t needs batch % 16");
  const int waves = 2 * (batch * 49 / 8);
  conv2_fwd_kernel<<<cdiv(waves, 4), 256, 0, s>>>(C16(a1p), batch, C16(w2t), b2, M16(a2p),
                                                  a2t ? M16(a2t) : nullptr, idx2);
}

void launch_fc1_fwd_train(const uint16_t* a2p, const uint16_t* w1t, int batch, float* part,
                          hipStream_t s) {
  const int waves = cdiv(batch, 32) * (FC1_OUT / 32) * FC1_SPLITS;
  fc1_fwd_kernel<false, 7><<<cdiv(waves, 4), 256, 0, s>>>(C16(a2p), batch, C16(w1t), nullptr,
                                                          part, batch, FC1_SPLITS, 0u, 1.f);
}

void launch_fc1_fwd_eval(const uint16_t* a2p, int ld, const uint16_t* w1t, const float* b, int M,
                         float* h, uint32_t key, float keep_prob, hipStream_t s) {
  const int waves = cdiv(M, 32) * (FC1_OUT / 32);
  fc1_fwd_kernel<true, 4><<<cdiv(waves, 4), 256, 0, s>>>(C16(a2p), ld, C16(w1t), b, h, M, 1, key,
                                                         keep_prob);
}

void launch_fc1_bwd(const uint16_t* a2p, const uint16_t* a2t, const uint8_t* idx2,
                    const uint16_t* dh16, const uint16_t* dht16, const float* hd, const float* dh,
                    const float* dlog, const uint16_t* w1b, int batch, float* g_w3, float* g_b3,
                    float* g_w4, float* g_b4, uint16_t* dy2p, uint16_t* dy2t, hipStream_t s) {
  if (batch % 32 != 0) throw std::runtime_error("mnist16 fc1_bwd: batch % 32 != 0");
  const int n_dx = cdiv(batch / 32 * (FC1_IN / 32), 4);
  const int n_dw = (FC1_IN / 32) * (FC1_OUT / 32) / 4;
  fc1_bwd_kernel<<<n_dx + n_dw + mnist::SMALL_BLOCKS, 256, 0, s>>>(
      C16(a2p), C16(a2t), idx2, C16(dh16), C16(dht16), hd, dh, dlog, C16(w1b), batch, g_w3, g_b3,
      g_w4, g_b4, M16(dy2p), M16(dy2t));
}

void launch_conv2_bwd_data(const uint16_t* dy2p, const uint16_t* w2b, const uint16_t* a1p,
                           int batch, float* da1m, hipStream_t s,
                           const mnist::FcSgdArgs* fc_sgd) {
  if (batch % 8 != 0) throw std::runtime_error("mnist16 conv2_bwd_data: batch % 8 != 0");
  const int mtiles = batch * 196 / 32;
  const mnist::FcSgd sg = mnist::fc_sgd_args(fc_sgd);
  conv2_bwd_data_kernel<<<cdiv(mtiles, 2) + sg.nblk, 256, 0, s>>>(C16(dy2p), C16(w2b), C16(a1p),
                                                                  batch, da1m, sg);
}

int conv2_filter_groups(int batch) { return cdiv(batch, C2F_IMG); }

void launch_conv2_bwd_filter(const uint16_t* a1t, const uint16_t* dy2t, int batch, float* part2,
                             hipStream_t s, const mnist::C1FilterArgs* c1) {
  const int G = conv2_filter_groups(batch);
  const mnist::C1Filter c = mnist::c1_args(c1);
  const int n1 = c.part1 ? mnist::conv1_filter_blocks(batch) : 0;
  conv2_bwd_filter_kernel<<<25 * G + n1, 512, 0, s>>>(C16(a1t), C16(dy2t), batch, part2,
                                                      part2 + (size_t)G * 51200, 25 * G, c);
}

size_t part2_floats(int batch) { return (size_t)conv2_filter_groups(batch) * (51200 + 256); }

int conv2_bwd_conv1_rows(int batch) { return cdiv(batch * 196, C2B_PIX); }

// labs: per-block clock stamps of the merged conv2 backward (null: off)
static unsigned long long* g_c2b_prof = nullptr;
void set_conv2_bwd_prof(unsigned long long* p) { g_c2b_prof = p; }

void launch_conv2_bwd(const uint16_t* dy2p, const uint16_t* w2b, const uint16_t* a1p,
                      const uint16_t* a1t, const uint16_t* dy2t, int batch, float* da1m,
                      float* part2, hipStream_t s, const mnist::FcSgdArgs* fc_sgd,
                      const mnist::C1FilterArgs* c1) {
  if (batch % 8 != 0) throw std::runtime_error("mnist16 conv2_bwd: batch % 8 != 0");
  const int G = conv2_filter_groups(batch);
  const int nc2 = 25 * G, nd = conv2_bwd_conv1_rows(batch);
  const mnist::FcSgd sg = mnist::fc_sgd_args(fc_sgd);
  mnist::C1Filter c = mnist::c1_args(c1);
  // lab switch (MTA_C2B_LAB): 1 = the FC SGD as a launch of its own after this
  // one, 2 = no conv1 filter-grad epilogue (timing only: conv1 grads unset)
  static const int lab = [] {
    const char* e = getenv("MTA_C2B_LAB");
    return e ? atoi(e) : 0;
  }();
  mnist::FcSgd sg_in = sg;
  if (lab == 1) sg_in.nblk = 0;
  if (lab == 2) c.part1 = nullptr;
  conv2_bwd_kernel<<<nd + nc2 + cdiv(sg_in.nblk, 2), 512, 0, s>>>(
      C16(dy2p), C16(w2b), C16(a1p), C16(a1t), C16(dy2t), batch, da1m, part2,
      part2 + (size_t)G * 51200, nc2, nd, c, sg_in, g_c2b_prof);
  if (lab == 1 && sg.nblk > 0) fc_sgd_kernel<<<sg.nblk, 256, 0, s>>>(sg);
}

}  // namespace mnist16
