// bf16 MFMA implicit-GEMM convolution for wide NHWC layers (C % 64 == 0,
// K % 64 == 0: every ResNet-18 conv but the 3-channel stem), forward and the
// stride-1 backward-data (a forward conv of dY with flipped, transposed taps).
//
// Why a second bf16 path next to conv_tiled.hip's: that family stages K tiles
// of 32 channels, i.e. 2 bf16 MFMA k-steps between barriers, and writes its
// B operand into LDS one bf16 at a time (put_r4) because the HWIO weights are
// co-contiguous.  Here:
//   * the weights are re-laid once per call into bf16 [tap][n][k] (k
//     contiguous) by wcvt_kernel, so B tiles are 16-byte bf16 vectors in and
//     16-byte ds_write_b128 out, no transposes;
//   * a K tile is one tap x 64 channels: 4 k-steps of v_mfma_f32_32x32x16_bf16
//     on TMxTN 32x32 tiles per wave (16 MFMAs per barrier for 128x128);
//   * A is a bf16 copy of the NHWC activations (to_bf16_kernel, written once
//     per conv and kept for the filter gradient): one 16-byte load per 8
//     channels straight into the row-major [row][64 + 8] LDS image (144-byte
//     rows: the ds_read_b128 fragments of 8 consecutive lanes hit disjoint
//     banks).  These kernels are bound by vector-L1 bytes per MFMA, so
//     halving the A bytes is the lever (fp32 activations, converted while
//     staged, remain the fallback when no copy is passed);
//   * double-buffered LDS, next tile's global loads in flight during the
//     current tile's MFMAs, one barrier per K tile, XCD-aware block order;
//   * split-K (gridDim.y) for deep layers writes fp32 slabs, summed
//     deterministically by the caller.
// fp32 accumulate; fp32 in / out (the rest of the generic engine is fp32).
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "ops_generic.h"

namespace gops {
namespace cbf {

constexpr int BK = 64;       // channels per K tile
constexpr int LDK = BK + 8;  // bf16 per LDS row (144 B)
constexpr int NT = 256;      // 4 waves, 2 x 2

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint4 pack8(float4 a, float4 b) {
  bfx8 v;
  v[0] = (__bf16)a.x;
  v[1] = (__bf16)a.y;
  v[2] = (__bf16)a.z;
  v[3] = (__bf16)a.w;
  v[4] = (__bf16)b.x;
  v[5] = (__bf16)b.y;
  v[6] = (__bf16)b.z;
  v[7] = (__bf16)b.w;
  return __builtin_bit_cast(uint4, v);
}

// fp32 -> bf16 (round to nearest even), 8 elements per thread-iteration.
__global__ __launch_bounds__(256) void to_bf16_kernel(const float4* __restrict__ x,
                                                      uint4* __restrict__ y, long long n8) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride)
    y[i] = pack8(x[2 * i], x[2 * i + 1]);
}

// Weights HWIO fp32 [R][S][C][K] -> bf16
//   mode 0 (forward):            Wt[tap][co][ci]            = W[tap][ci][co]
//   mode 1 (stride-1 bwd-data):  Wt[R*S-1-tap][ci][co]      = W[tap][ci][co]
// (mode 1 is the forward weight of the conv dX = conv(dY, W'), whose input
// channels are co and output channels ci.)  32x32 transpose tiles via LDS.
__global__ __launch_bounds__(256) void wcvt_kernel(const float* __restrict__ w, int taps, int C,
                                                   int K, int mode, __bf16* __restrict__ out) {
  __shared__ float t[32][33];
  const int ct = C / 32, kt = K / 32;
  const int b = blockIdx.x;
  const int tap = b / (ct * kt), rem = b % (ct * kt), c0 = (rem / kt) * 32, k0 = (rem % kt) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const float* src = w + (size_t)tap * C * K;
  if (mode == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) t[ty + 8 * i][tx] = src[(size_t)(c0 + ty + 8 * i) * K + k0 + tx];
    __syncthreads();
    __bf16* dst = out + (size_t)tap * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[(size_t)(k0 + ty + 8 * i) * C + c0 + tx] = (__bf16)t[tx][ty + 8 * i];
  } else {
    __bf16* dst = out + (size_t)(taps - 1 - tap) * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t o = (size_t)(c0 + ty + 8 * i) * K + k0 + tx;
      dst[o] = (__bf16)src[o];
    }
  }
}

// All the bf16 weight copies of a model in ONE launch (per training step,
// after the update): jobs[j] = {w, out, taps, C, K, mode, first block, 0} as
// int64, blocks of job j run wcvt_kernel's 32 x 32 tile at (block - first).
// Replaces one wcvt launch per conv call (ResNet-18: 40 launches, ~195 us a
// step, each too small to fill the chip).
__global__ __launch_bounds__(256) void wcvt_batch_kernel(const long long* __restrict__ jobs,
                                                         int njobs) {
  __shared__ float t[32][33];
  const int b = blockIdx.x;
  // job of this block: the first blocks ascend with j, so the jobs starting at
  // or before b are a prefix; every lane tests one job (one load round per 64
  // jobs instead of a dependent load chain through the table)
  int j = 0;
  for (int base = 0; base < njobs; base += 64) {
    const int jj = base + (int)(threadIdx.x & 63);
    const bool le = jj < njobs && jobs[8 * min(jj, njobs - 1) + 6] <= b;
    const int cnt = __popcll(__ballot(le));
    j = base + cnt - 1;
    if (cnt < 64) break;
  }
  j = max(j, 0);
  const long long* J = jobs + 8 * j;
  const float* w = reinterpret_cast<const float*>(J[0]);
  __bf16* out = reinterpret_cast<__bf16*>(J[1]);
  const int taps = (int)J[2], C = (int)J[3], K = (int)J[4], mode = (int)J[5];
  const int lb = b - (int)J[6];
  const int ct = C / 32, kt = K / 32;
  const int tap = lb / (ct * kt), rem = lb % (ct * kt), c0 = (rem / kt) * 32, k0 = (rem % kt) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* src = w + (size_t)tap * C * K;
  if (mode == 2) {  // fp32 stride-1 dgrad weights: flipped taps, ci / co transposed
#pragma unroll
    for (int i = 0; i < 4; ++i) t[ty + 8 * i][tx] = src[(size_t)(c0 + ty + 8 * i) * K + k0 + tx];
    __syncthreads();
    float* dst = reinterpret_cast<float*>(J[1]) + (size_t)(taps - 1 - tap) * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[(size_t)(k0 + ty + 8 * i) * C + c0 + tx] = t[tx][ty + 8 * i];
  } else if (mode == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) t[ty + 8 * i][tx] = src[(size_t)(c0 + ty + 8 * i) * K + k0 + tx];
    __syncthreads();
    __bf16* dst = out + (size_t)tap * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dst[(size_t)(k0 + ty + 8 * i) * C + c0 + tx] = (__bf16)t[tx][ty + 8 * i];
  } else {
    __bf16* dst = out + (size_t)(taps - 1 - tap) * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t o = (size_t)(c0 + ty + 8 * i) * K + k0 + tx;
      dst[o] = (__bf16)src[o];
    }
  }
}

// The flat momentum SGD of a bf16-conv model in ONE launch that also writes
// the bf16 MFMA layouts of the updated conv weights (wcvt_kernel modes 0 and
// 1), so no per-step weight-conversion launch remains ("for bf16
// configs it also writes the bf16 weight shadow").
//  * blocks [0, conv_blocks): one 32 x 32 (ci, co) tile of one tap of a conv
//    weight - SGD of its 1024 floats (rows along co: 128-B loads per
//    half-wave), the bf16 result straight into the dgrad layout
//    Wd[R*S-1-tap][ci][co] and, transposed through LDS, into the forward
//    layout Wt[tap][co][ci];
//  * the other blocks: the remaining flat ranges (BatchNorm, FC, ...),
//    float4 grid-stride per range.
// jobs[j] = {w offset (floats), fwd out, dgrad out, taps, C, K, first block,
// kind}; kind 0: the bf16 forward / dgrad layouts; kind 1 (fp32 model): the
// fp32 stride-1 dgrad weights, flipped and transposed (wflip_kernel's
// layout) into `fwd out`.  ranges[r] = {lo4, hi4, first block, nblocks}
// (float4 units).  Same arithmetic as optim::sgd_momentum_flat_kernel
// (bit-identical updates).
struct SgdWcvtArgs {
  float* w;
  const float* g;
  float* mom;
  float momentum, gscale, l2;
  const float* lr;
  long long* step;
  const long long* jobs;
  int njobs, conv_blocks;
  const long long* ranges;
  int nranges;
};

// index of the entry whose first block (field `f` of an 8- / 4-wide int64
// row) is the last one <= b: one ballot per 64 entries
__device__ __forceinline__ int table_lookup(const long long* tab, int n, int width, int f,
                                            long long b) {
  int j = 0;
  for (int base = 0; base < n; base += 64) {
    const int jj = base + (int)(threadIdx.x & 63);
    const bool le = jj < n && tab[width * min(jj, n - 1) + f] <= b;
    const int cnt = __popcll(__ballot(le));
    j = base + cnt - 1;
    if (cnt < 64) break;
  }
  return max(j, 0);
}

__global__ __launch_bounds__(256) void sgd_wcvt_kernel(const SgdWcvtArgs a) {
  __shared__ float t[32][33];
  const float lr = *a.lr;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (a.step && b == 0 && tid == 0) *a.step += 1;
  if (b < a.conv_blocks) {
    const long long* J = a.jobs + 8 * table_lookup(a.jobs, a.njobs, 8, 6, b);
    const long long woff = J[0];
    __bf16* out0 = reinterpret_cast<__bf16*>(J[1]);
    __bf16* out1 = reinterpret_cast<__bf16*>(J[2]);
    const int taps = (int)J[3], C = (int)J[4], K = (int)J[5];
    const int lb = b - (int)J[6];
    const bool f32flip = J[7] == 1;
    const int ct = C / 32, kt = K / 32;
    const int tap = lb / (ct * kt), rem = lb % (ct * kt), c0 = (rem / kt) * 32, k0 = (rem % kt) * 32;
    const int tx = tid & 31, ty = tid >> 5;
    const size_t base = (size_t)woff + (size_t)tap * C * K;
    float wv[4], gv[4], mv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // all loads of the tile in flight together
      const size_t e = base + (size_t)(c0 + ty + 8 * i) * K + k0 + tx;
      wv[i] = a.w[e];
      gv[i] = a.g[e];
      mv[i] = a.mom[e];
    }
    __bf16* d1 = out1 + (size_t)(taps - 1 - tap) * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t o = (size_t)(c0 + ty + 8 * i) * K + k0 + tx;
      const float ge = __builtin_fmaf(a.l2, wv[i], gv[i] * a.gscale);
      const float m = a.momentum * mv[i] + ge;
      const float w = wv[i] - lr * m;
      a.w[base + o] = w;
      a.mom[base + o] = m;
      t[ty + 8 * i][tx] = w;
      if (!f32flip) d1[o] = (__bf16)w;
    }
    __syncthreads();
    if (f32flip) {
      float* df = reinterpret_cast<float*>(out0) + (size_t)(taps - 1 - tap) * C * K;
#pragma unroll
      for (int i = 0; i < 4; ++i) df[(size_t)(k0 + ty + 8 * i) * C + c0 + tx] = t[tx][ty + 8 * i];
      return;
    }
    __bf16* d0 = out0 + (size_t)tap * C * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) d0[(size_t)(k0 + ty + 8 * i) * C + c0 + tx] = (__bf16)t[tx][ty + 8 * i];
    return;
  }
  const long long rb = b - a.conv_blocks;
  const long long* Rr = a.ranges + 4 * table_lookup(a.ranges, a.nranges, 4, 2, rb);
  const long long lo4 = Rr[0], hi4 = Rr[1], nb = Rr[3];
  float4* W4 = reinterpret_cast<float4*>(a.w);
  float4* M4 = reinterpret_cast<float4*>(a.mom);
  const float4* G4 = reinterpret_cast<const float4*>(a.g);
  const long long stride = nb * 256;
  for (long long i = lo4 + (rb - Rr[2]) * 256 + tid; i < hi4; i += stride) {
    float4 wv = W4[i], gv = G4[i], mv = M4[i];
    gv.x = __builtin_fmaf(a.l2, wv.x, gv.x * a.gscale);
    gv.y = __builtin_fmaf(a.l2, wv.y, gv.y * a.gscale);
    gv.z = __builtin_fmaf(a.l2, wv.z, gv.z * a.gscale);
    gv.w = __builtin_fmaf(a.l2, wv.w, gv.w * a.gscale);
    mv.x = a.momentum * mv.x + gv.x;
    mv.y = a.momentum * mv.y + gv.y;
    mv.z = a.momentum * mv.z + gv.z;
    mv.w = a.momentum * mv.w + gv.w;
    wv.x -= lr * mv.x;
    wv.y -= lr * mv.y;
    wv.z -= lr * mv.z;
    wv.w -= lr * mv.w;
    W4[i] = wv;
    M4[i] = mv;
  }
}

// Forward conv Y[m = (n, oy, ox)][co] = sum_{tap, ci} X[n, iy, ix, ci] Wt[tap][co][ci].
// XT = __bf16: bf16 activation copy (16-byte loads); XT = float: fp32
// activations converted while staged.
template <int BM, int BN, class XT>
struct Loader {
  static constexpr bool XB = sizeof(XT) == 2;
  static constexpr int AR = BM * BK / 8 / NT;  // 8-channel A chunks per thread
  static constexpr int BR = BN * BK / 8 / NT;  // 8-channel B chunks per thread
  ConvShape s;
  const __bf16* wt;
  int cchunks;
  const XT* abase[AR];
  int iy0[AR], ix0[AR];
  bool av[AR];
  const __bf16* bbase[BR];
  float4 ra[XB ? 1 : AR][2];
  uint4 rab[XB ? AR : 1];
  uint4 rb[BR];
  static constexpr int EXTRA = 0;  // bf16 elements of loader-owned LDS (none so far)
  __device__ Loader(const ConvShape& s_, const ConvShape&, const XT* x, const __bf16* wt_, int m0,
                    int n0, __bf16*)
      : s(s_), wt(wt_) {
    cchunks = s.C / BK;
    const int tid = threadIdx.x, c8 = tid & 7;
    const int M = s.N * s.OH * s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + (NT / 8) * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
      abase[i] = x + (size_t)n * s.H * s.W * s.C + 8 * c8;
      iy0[i] = oy * s.stride - s.pad;
      ix0[i] = ox * s.stride - s.pad;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = min(n0 + (tid >> 3) + (NT / 8) * i, s.K - 1);  // K % 64 == 0: never clamps
      bbase[i] = wt + (size_t)n * s.C + 8 * c8;
    }
  }
  __device__ __forceinline__ void load(int kt) {
    const int tap = kt / cchunks, ci0 = (kt - tap * cchunks) * BK;
    const int kh = tap / s.S, kw = tap - kh * s.S;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int iy = iy0[i] + kh, ix = ix0[i] + kw;
      const bool ok = av[i] && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
      const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
      const XT* src = abase[i] + ((size_t)iyc * s.W + ixc) * s.C + ci0;
      if constexpr (XB) {
        const uint4 v = *reinterpret_cast<const uint4*>(src);
        rab[i] = sel(ok, v);
      } else {
        const float4* p = reinterpret_cast<const float4*>(src);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 v0 = p[0], v1 = p[1];
        ra[i][0] = sel(ok, v0);
        ra[i][1] = sel(ok, v1);
      }
    }
    const size_t wo = (size_t)tap * s.K * s.C + ci0;
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = *reinterpret_cast<const uint4*>(bbase[i] + wo);
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x, c8 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v;
      if constexpr (XB)
        v = rab[i];
      else
        v = pack8(ra[i][0], ra[i][1]);
      *reinterpret_cast<uint4*>(As + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(Bs + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = rb[i];
  }
};

// Implicit im2col for a thin-input strided conv (the ResNet stem, 7x7 / s2 /
// 3 channels), replacing the materialised bf16 im2col (154 MB written and
// read twice per step at B = 32): s is the 1x1 GEMM shape over kp = K-dim
// channels, si the image conv.  The k order is per tap row (kh * seg + kw * C
// + ci, seg = S*C rounded up to 8, zero beyond R * seg) as in
// im2col_bf16_kernel: a thread's 8 consecutive k of one tap row are ONE run of
// 8 consecutive image floats (NHWC), fetched as two unaligned 16-byte loads
// and masked to the in-image part.
struct StemGeo {
  int seg, sc;  // padded and real tap-row length (S * C)
  long long nx;  // image elements
  __device__ StemGeo(const ConvShape& si)
      : seg((si.S * si.C + 7) / 8 * 8), sc(si.S * si.C),
        nx((long long)si.N * si.H * si.W * si.C) {}
  // 8 (or 4) consecutive k from k0 (within one tap row) of output pixel
  // (n, iy0 = oy*stride - pad, ix0) of image x
  template <int E>
  __device__ __forceinline__ void fetch(const ConvShape& si, const float* x, int n, int iy0,
                                        int ix0, int k0, bool pix_ok, float* v) const {
    const int kh = k0 / seg, j0 = k0 - kh * seg;
    const int iy = iy0 + kh;
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = 0.f;
    if (!pix_ok || kh >= si.R || iy < 0 || iy >= si.H) return;
    const int jlo = max(0, -ix0) * si.C, jhi = min(sc, (si.W - ix0) * si.C);
    const long long e0 = (((long long)n * si.H + iy) * si.W + ix0) * si.C + j0;
    if (e0 >= 0 && e0 + E <= nx) {
      float r[E];
#pragma unroll
      for (int u = 0; u < E / 4; ++u) {
        const float4 f = *reinterpret_cast<const float4*>(x + e0 + 4 * u);
        r[4 * u] = f.x;
        r[4 * u + 1] = f.y;
        r[4 * u + 2] = f.z;
        r[4 * u + 3] = f.w;
      }
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = (j0 + j >= jlo && j0 + j < jhi) ? r[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j)
        if (j0 + j >= jlo && j0 + j < jhi) v[j] = x[e0 + j];
    }
  }
};

template <int BM, int BN>
struct StemLoader {
  static constexpr int AR = BM * BK / 8 / NT;
  static constexpr int BR = BN * BK / 8 / NT;
  ConvShape s, si;
  StemGeo g;
  const float* x;
  const __bf16* wt;
  int nimg[AR], iy0[AR], ix0[AR];
  bool av[AR];
  const __bf16* bbase[BR];
  uint4 rab[AR];
  uint4 rb[BR];
  static constexpr int EXTRA = 0;
  __device__ StemLoader(const ConvShape& s_, const ConvShape& si_, const float* x_,
                        const __bf16* wt_, int m0, int n0, __bf16*)
      : s(s_), si(si_), g(si_), x(x_), wt(wt_) {
    const int tid = threadIdx.x, c8 = tid & 7;
    const int M = s.N * s.OH * s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + (NT / 8) * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH;
      nimg[i] = t / s.OH;
      iy0[i] = oy * si.stride - si.pad;
      ix0[i] = ox * si.stride - si.pad;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = min(n0 + (tid >> 3) + (NT / 8) * i, s.K - 1);
      bbase[i] = wt + (size_t)n * s.C + 8 * c8;
    }
  }
  __device__ __forceinline__ void load(int kt) {
    const int k0 = kt * BK + 8 * (threadIdx.x & 7);
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      float v[8];
      g.fetch<8>(si, x, nimg[i], iy0[i], ix0[i], k0, av[i], v);
      rab[i] = pack8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = *reinterpret_cast<const uint4*>(bbase[i] + kt * BK);
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x, c8 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      *reinterpret_cast<uint4*>(As + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = rab[i];
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(Bs + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = rb[i];
  }
};

// Space-to-depth stem (conv_fwd_s2d_stem_bf16): the 7x7 / stride-2 / pad-3
// conv over 3 channels, re-cast as a 4x4 / stride-1 conv over the bf16
// space-to-depth image xs [N][OH + 3][OW + 3][16] (s2d_stem_input: pixel
// (Y, X) holds the 2x2 input block at rows 2 (Y - 2) + p, columns
// 2 (X - 2) + q as channels (p * 2 + q) * 3 + ci, 4 zero channels, zero
// outside the image), with the 8x8-extended filter (tap (a, b) <- kernel
// (2a + p - 1, 2b + q - 1), zero off the 7x7).  GEMM K = 16 taps x 16
// channels: K tile kt = tap row a, a thread's 8 consecutive k = half of tap
// (a, c8 / 2)'s channels = ONE aligned 16-byte load, always inside the padded
// image - no masks, no fp32 gather, no conversion (the StemLoader's implicit
// im2col did 2 unaligned fp32 float4 loads + masks + a pack per 8 k).
template <int BM, int BN>
struct S2dLoader {
  static constexpr int AR = BM * BK / 8 / NT;
  static constexpr int BR = BN * BK / 8 / NT;
  static constexpr int EXTRA = 0;
  const __bf16* abase[AR];
  bool av[AR];
  const __bf16* bbase[BR];
  uint4 ra[AR];
  uint4 rb[BR];
  int ws16;  // one s2d image row, in bf16 (16 channels a pixel)
  __device__ S2dLoader(const ConvShape& s, const ConvShape& si, const __bf16* x,
                       const __bf16* wt, int m0, int n0, __bf16*) {
    const int tid = threadIdx.x, c8 = tid & 7;
    const int M = s.N * s.OH * s.OW;
    ws16 = si.W * 16;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + (NT / 8) * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
      abase[i] = x + (((size_t)n * si.H + oy) * si.W + ox + (c8 >> 1)) * 16 + 8 * (c8 & 1);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = min(n0 + (tid >> 3) + (NT / 8) * i, s.K - 1);
      bbase[i] = wt + (size_t)n * s.C + 8 * c8;
    }
  }
  __device__ __forceinline__ void load(int kt) {
#pragma unroll
    for (int i = 0; i < AR; ++i)
      ra[i] = av[i] ? *reinterpret_cast<const uint4*>(abase[i] + (size_t)kt * ws16)
                    : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = *reinterpret_cast<const uint4*>(bbase[i] + kt * BK);
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x, c8 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      *reinterpret_cast<uint4*>(As + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(Bs + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = rb[i];
  }
};

// The same operands with every K tile requested at once: the stem GEMM has
// only 4 K tiles (K = 256) a block, so fwd_kernel's one-tile-ahead pipeline
// waited on 4 dependent load round trips per block at 2 blocks a CU.  Here the
// first load() issues all 4 tiles' A / B loads (64 + 32 VGPRs) and store()
// writes the tile the last load() named (a uniform switch: no dynamic register
// indexing).
template <int BM, int BN>
struct S2dLoaderPre {
  static constexpr int AR = BM * BK / 8 / NT;
  static constexpr int BR = BN * BK / 8 / NT;
  static constexpr int NKT = 4;  // tap rows = K tiles
  static constexpr int EXTRA = 0;
  const __bf16* abase[AR];
  bool av[AR];
  const __bf16* bbase[BR];
  uint4 ra[NKT][AR];
  uint4 rb[NKT][BR];
  int ws16, cur = 0;
  __device__ S2dLoaderPre(const ConvShape& s, const ConvShape& si, const __bf16* x,
                          const __bf16* wt, int m0, int n0, __bf16*) {
    const int tid = threadIdx.x, c8 = tid & 7;
    const int M = s.N * s.OH * s.OW;
    ws16 = si.W * 16;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + (NT / 8) * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
      abase[i] = x + (((size_t)n * si.H + oy) * si.W + ox + (c8 >> 1)) * 16 + 8 * (c8 & 1);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = min(n0 + (tid >> 3) + (NT / 8) * i, s.K - 1);
      bbase[i] = wt + (size_t)n * s.C + 8 * c8;
    }
  }
  __device__ __forceinline__ void load(int kt) {
    cur = kt;
    if (kt != 0) return;
#pragma unroll
    for (int k = 0; k < NKT; ++k) {
#pragma unroll
      for (int i = 0; i < AR; ++i)
        ra[k][i] = av[i] ? *reinterpret_cast<const uint4*>(abase[i] + (size_t)k * ws16)
                         : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int i = 0; i < BR; ++i) rb[k][i] = *reinterpret_cast<const uint4*>(bbase[i] + k * BK);
    }
  }
  template <int K>
  __device__ __forceinline__ void store_k(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x, c8 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      *reinterpret_cast<uint4*>(As + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = ra[K][i];
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(Bs + ((tid >> 3) + (NT / 8) * i) * LDK + 8 * c8) = rb[K][i];
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    switch (cur) {
      case 0: store_k<0>(As, Bs); break;
      case 1: store_k<1>(As, Bs); break;
      case 2: store_k<2>(As, Bs); break;
      default: store_k<3>(As, Bs); break;
    }
  }
};

// K tiles a loader holds at once (fwd_kernel unrolls its loop for them), 0: streamed
template <class LD>
struct FixedNk {
  static constexpr int v = 0;
};
template <int BM, int BN>
struct FixedNk<S2dLoaderPre<BM, BN>> {
  static constexpr int v = S2dLoaderPre<BM, BN>::NKT;
};

// BatchNorm statistics in a bf16-output epilogue (ConvStats): lane (r, h) of
// a wave holds column r of its 32-row tiles; after its own rows are summed
// the two half-waves combine, and lanes h == 0 write the wave's partial row
// prow.  Table layout [2][K / 64][P][64]: the 32 lanes store 128 contiguous
// bytes (a channel-major table made every lane's store its own cache line:
// +3.6 us per halo conv); every (channel, prow) is written exactly once.
__device__ __forceinline__ size_t stats_index(int co, int prow, int P) {
  return ((size_t)(co >> 6) * P + prow) * 64 + (co & 63);
}
__device__ __forceinline__ void stats_store(const ConvStats& cs, int K, int co, int prow, int h,
                                            float s1, float s2) {
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if (h == 0) {
    const size_t i = stats_index(co, prow, cs.P);
    cs.part[i] = s1;
    cs.part[(size_t)K * cs.P + i] = s2;
  }
}

// BatchNorm BACKWARD statistics in a dgrad epilogue (BnBwdStats): the fp32
// dX value v at element e of channel co is the BatchNorm's dY; d = v [y > 0]
// (relu), s1 += d, s2 += d (x - mean) rstd.  Same partial-row table and
// store as the forward statistics (stats_store).
__device__ __forceinline__ float bf16_at(const void* p, size_t e) {
  return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[e] << 16);
}
__device__ __forceinline__ void bnb_store(const BnBwdStats& bb, int C, int co, int prow, int h,
                                          float s1, float s2) {
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if (h == 0) {
    const size_t i = stats_index(co, prow, bb.P);
    bb.part[i] = s1;
    bb.part[(size_t)C * bb.P + i] = s2;
  }
}

template <int BM, int BN, class XT, class LD = Loader<BM, BN, XT>>
__global__ __launch_bounds__(NT) void fwd_kernel(ConvShape s, const XT* __restrict__ x,
                                                 const __bf16* __restrict__ wt,
                                                 const float* __restrict__ bias,
                                                 float* __restrict__ y, int relu, int kps,
                                                 const float* __restrict__ addend,
                                                 __bf16* __restrict__ yb, int ex2,
                                                 const ConvShape si, const ConvStats cs) {
  // ex2 (unsplit): the 1x1 stride-2 backward-data - rows are dY pixels
  // (n, a, b), written to dX pixel (2a, 2b) of the 2x-sized output with the
  // other three pixels of its 2x2 block zero (plus addend everywhere)
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int STAGE = (BM + BN) * LDK;  // bf16 elements
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int M = s.N * s.OH * s.OW;
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;
  const int nk_all = s.R * s.S * (s.C / BK), kb = blockIdx.y * kps;
  const int nk = min(kps, nk_all - kb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5;
  __shared__ __attribute__((aligned(16))) __bf16 xtra[LD::EXTRA > 0 ? LD::EXTRA : 1];
  LD ld(s, si, x, wt, m0, n0, xtra);
  // BatchNorm shift of this lane's output columns, loaded before the main
  // loop: an epilogue load issued after the first stores would make the
  // compiler wait for those stores (vmcnt counts both) before the next ones
  float kcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
    kcol[j] = (yb && cs.part) ? cs.shift[n0 + wn * (BN / 2) + 32 * j + r] : 0.f;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero16();
  auto mma = [&](const __bf16* A, const __bf16* B) {
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bfx8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const bfx8*>(A + (wm * (BM / 2) + 32 * i + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const bfx8*>(B + (wn * (BN / 2) + 32 * j + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (FixedNk<LD>::v > 0) {
    // a loader holding all K tiles in registers: the loop unrolled, so its
    // per-tile stores index the tiles with constants (no scratch)
    constexpr int NK = FixedNk<LD>::v;
    ld.load(0);
    ld.store(smem, smem + BM * LDK);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      const __bf16* A = smem + (kt & 1) * STAGE;
      mma(A, A + BM * LDK);
      if (kt + 1 < NK) {
        __bf16* nxt = smem + ((kt + 1) & 1) * STAGE;
        ld.cur = kt + 1;
        ld.store(nxt, nxt + BM * LDK);
      }
      __syncthreads();
    }
  } else if (nk > 0) {
    ld.load(kb);
    ld.store(smem, smem + BM * LDK);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const __bf16* A = smem + (kt & 1) * STAGE;
      const __bf16* B = A + BM * LDK;
      __bf16* nxt = smem + ((kt + 1) & 1) * STAGE;
      const bool more = kt + 1 < nk;
      if (more) ld.load(kb + kt + 1);
      mma(A, B);
      if (more) ld.store(nxt, nxt + BM * LDK);
      __syncthreads();
    }
  }
  if (ex2) {
    const size_t K = s.K, W2 = 2 * (size_t)s.OW;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (BN / 2) + 32 * j + r;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(q, lane);
          if (m >= M) continue;
          const int b = m % s.OW, t = m / s.OW;  // t = n * OH + a
          const size_t o = ((size_t)(2 * t) * W2 + 2 * b) * K + co;  // (n, 2a, 2b)
          const size_t o2[4] = {o, o + K, o + W2 * K, o + W2 * K + K};
          const float v[4] = {acc[i][j][q], 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) y[o2[e]] = addend ? v[e] + addend[o2[e]] : v[e];
        }
    }
    return;
  }
  y += (size_t)blockIdx.y * M * s.K;
  const bool st = yb && cs.part;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + r;
    const float bv = bias ? bias[co] : 0.f;
    const float kc = kcol[j];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(q, lane);
        if (m >= M) continue;
        float v = acc[i][j][q] + bv;
        if (relu) v = fmaxf(v, 0.f);
        if (addend) v += addend[(size_t)m * s.K + co];  // gradient junction (dX accumulate)
        if (yb) {  // bf16 output (unsplit only): the conv feeds a bf16-input BatchNorm
          const __bf16 hv = (__bf16)v;
          yb[(size_t)m * s.K + co] = hv;
          const float d = (float)hv - kc;
          s1 += d;
          s2 += d * d;
        } else {
          y[(size_t)m * s.K + co] = v;
        }
      }
    if (st) stats_store(cs, s.K, co, (bid % mt) * 2 + wm, h, s1, s2);
  }
}


// ------------------------------------------- 3x3 stride-1 halo forward ----
// The generic kernels above stage a fresh [128 pixels x 64 ch] A tile for
// EACH of the 9 taps (the same activations read 9 times through L2) and keep
// one K tile in flight: on ResNet-18's 3x3 stride-1 layers (forward, and the
// stride-1 dgrad, which is the same conv) they ran 33-40 us a layer at B = 32,
// latency bound.  Here a block owns 128 consecutive output pixels x 64
// output channels and, per 64-channel chunk:
//   * stages the activation HALO once - the contiguous run of input pixels
//     from one stacked image row above the tile to one below (<= 344
//     pixels x 128 B): in NHWC the rows of consecutive images are adjacent,
//     so it is ONE strided copy, done with global_load_lds_dwordx4 (no VGPR
//     staging; 8 pixels per wave-instruction);
//   * reads each tap's A fragments straight out of the halo at a per-lane
//     shifted pixel row (padding taps and the rows of a neighbouring image
//     read a zero row), so the activations cross L2 once per chunk, not 9x;
//   * streams the 9 taps' weight tiles (64 co x 64 ci) through a 4-deep LDS
//     ring, three in flight (counted vmcnt, raw s_barrier: the DMA queue is
//     not drained by the barrier);
//   * 16-byte chunks of every 128-byte LDS row are swizzled through the DMA
//     source address, slot = chunk ^ ((row >> 1) & 7): a ds_read_b128 lane
//     group (16 lanes, one LDS cycle when its 16 x 16 B cover the 64 banks)
//     reads 16 consecutive rows, i.e. both 128-B halves of the bank row x 8
//     slots.  (chunk ^ (row & 7) left every group 2-way conflicted: half of
//     the LDS cycles were SQ_LDS_BANK_CONFLICT.)
// Split-K over channel chunks (deterministic slabs) fills the chip on the
// small-M deep layers.  LDS 75 KiB: two blocks per CU.
namespace h3 {
constexpr int ROWB = 128;  // bytes per LDS row (64 bf16 channels)
constexpr int HCAP = 344;  // halo pixel rows (multiple of 8); row HCAP is all zeros
__device__ uint4 g_zero[4];  // never written: the DMA source of rows outside the tensor

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void glds(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
// halo rows a BM-pixel tile can need: the stacked rows it touches + 2, x W
inline int halo_rows(const ConvShape& s, int bm) { return ((bm + s.W - 2) / s.W + 3) * s.W; }
}  // namespace h3

// EPI: the epilogue kind, one per instantiation (each keeps only its own
// code): 0 fp32 output (+ addend), 1 bf16 output (+ the BatchNorm forward
// statistics, ConvStats), 2 fp32 dX + the BatchNorm backward sums (BnBwdStats,
// + addend)
template <int BM, int BN, int RB, int EPI>
__global__ __launch_bounds__(NT) void conv3_kernel(ConvShape s, const __bf16* __restrict__ x,
                                                   const __bf16* __restrict__ wt,
                                                   float* __restrict__ y, int cps,
                                                   const float* __restrict__ addend,
                                                   __bf16* __restrict__ yb, const ConvStats cs,
                                                   const BnBwdStats bb) {
  using h3::ROWB;
  using h3::HCAP;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GB = BN / 32;  // weight DMA instructions per wave per tap
  constexpr int HB = (HCAP + 1) * ROWB;
  constexpr int BSZ = BN * ROWB;
  static_assert(RB >= 3 && RB <= 4, "ring depth");
  __shared__ __attribute__((aligned(1024))) char smem[HB + RB * BSZ];
  const int M = s.N * s.H * s.W;
  const int W = s.W, H = s.H;
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;
  const int nch = s.C / BK;
  const int cc0 = blockIdx.y * cps, cc1 = min(nch, cc0 + cps);
  const int g_first = m0 / W, g_last = (min(m0 + BM, M) - 1) / W;
  const long long hbase = (long long)(g_first - 1) * W;  // global pixel of halo row 0
  const int npix = (g_last - g_first + 3) * W;
  const int nins = (npix + 7) >> 3;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5, lr = lane >> 3;
  if (tid < 8) *reinterpret_cast<uint4*>(smem + HCAP * ROWB + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
  // this lane's A rows (output pixels)
  int gl[TM], oxs[TM], oys[TM];
  bool mv[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / 2) + 32 * i + r;
    mv[i] = m < M;
    const int mm = mv[i] ? m : m0;
    const int g = mm / W;
    oxs[i] = mm - g * W;
    oys[i] = g % H;
    gl[i] = g - g_first + 1;
  }
  const __bf16* bsrc[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = wave * (BN / 4) + 8 * j + lr;
    bsrc[j] = wt + (size_t)(n0 + row) * s.C + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  auto issue_b = [&](int tap, int cc, int slot) {
    const size_t o = (size_t)tap * s.K * s.C + (size_t)cc * BK;
    char* dst = smem + HB + slot * BSZ + wave * (BN / 4) * ROWB;
#pragma unroll
    for (int j = 0; j < GB; ++j) h3::glds(bsrc[j] + o, dst + 8 * j * ROWB);
  };
  auto issue_halo = [&](int cc) {
    for (int ins = wave; ins < nins; ins += 4) {
      const int p = 8 * ins + lr;
      const long long gp = hbase + p;
      const bool ok = p < npix && gp >= 0 && gp < M;
      const void* src = ok ? (const void*)(x + gp * s.C + (size_t)cc * BK +
                                           8 * ((lane & 7) ^ ((p >> 1) & 7)))
                           : (const void*)h3::g_zero;
      h3::glds(src, smem + ins * 8 * ROWB);
    }
  };
  // BatchNorm shift of this lane's output columns (loaded up front, see
  // fwd_kernel); dgrad feeding a BatchNorm backward: its mean / rstd
  constexpr bool bs = EPI == 2;
  float kcol[TN], bmu[TN], brs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + r;
    kcol[j] = bmu[j] = brs[j] = 0.f;
    if constexpr (EPI == 1) kcol[j] = cs.part ? cs.shift[co] : 0.f;
    if constexpr (EPI == 2) {
      bmu[j] = bb.mean[co];
      brs[j] = bb.rstd[co];
    }
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero16();
  for (int cc = cc0; cc < cc1; ++cc) {
    // the previous chunk's halo and ring reads are done (and the zero row is written)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_halo(cc);
#pragma unroll
    for (int t = 0; t < RB - 1; ++t) issue_b(t, cc, t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // halo and tap t's weights landed (own DMAs; the barrier: every wave's);
      // the (up to RB - 2) taps issued after t may stay in flight
      const int ahead = min(RB - 2, 8 - t);
      if (ahead >= 2)
        h3::wait_vm<2 * GB>();
      else if (ahead == 1)
        h3::wait_vm<GB>();
      else
        h3::wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring slot (t - 1) % RB read
      __builtin_amdgcn_s_barrier();
      if (t + RB - 1 < 9) issue_b(t + RB - 1, cc, (t + RB - 1) % RB);
      const int kh = t / 3, kw = t - 3 * kh;
      int hrow[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int iy = oys[i] + kh - 1, ix = oxs[i] + kw - 1;
        const bool ok = mv[i] && iy >= 0 && iy < H && ix >= 0 && ix < W;
        hrow[i] = ok ? (gl[i] + kh - 1) * W + ix : HCAP;
      }
      const char* B = smem + HB + (t % RB) * BSZ;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int c = 2 * ks + h;
        bfx8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bfx8*>(smem + hrow[i] * ROWB +
                                                ((c ^ ((hrow[i] >> 1) & 7)) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int R = wn * (BN / 2) + 32 * j + r;
          b[j] = *reinterpret_cast<const bfx8*>(B + R * ROWB + ((c ^ ((R >> 1) & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // epilogue: lane (r, h) of 32 x 32 tile (i, j) holds rows 4h + (q & 3) +
  // 8 (q >> 2), column r; per-tile base pointers, the 16 row offsets are
  // wave-uniform multiples of K, and the bounds / addend branches are taken
  // once per tile (per element they were ~40 % of the kernel's instructions)
  y += (size_t)blockIdx.y * M * s.K;
  const size_t K = s.K;
  const bool st = EPI == 1 && cs.part;
  float ss1[TN], ss2[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) ss1[j] = ss2[j] = 0.f;
  if constexpr (EPI == 2) {
    // fp32 dX = a BatchNorm's dY, plus that BatchNorm's backward sums.  Every
    // operand load of every tile (x, y = the ReLU mask source, addend) is
    // issued first from clamped, always-valid rows, then one wait, the sums,
    // and the stores last: a load issued after a store waits for that store
    // too (vmcnt counts both), and a conditional load compiles to a branch
    // plus a wait per element (each measured ~2x on the 128-pixel tiles)
    auto epi2 = [&](auto has_add) {
      constexpr bool ADD = decltype(has_add)::value;
      uint32_t xr[TM][TN][16], yr[TM][TN][16];
      float av[TM][TN][ADD ? 16 : 1];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mb = m0 + wm * (BM / 2) + 32 * i + 4 * h;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int co = n0 + wn * (BN / 2) + 32 * j + r;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int rr = (q & 3) + 8 * (q >> 2);
            // rows past M (the last tile, whose 4-row group base mb may itself
            // be past M) read row M - 1: in bounds, finite, and selected away
            const size_t e = (size_t)min(mb + rr, M - 1) * K + co;
            xr[i][j][q] = reinterpret_cast<const uint16_t*>(bb.x)[e];
            yr[i][j][q] = reinterpret_cast<const uint16_t*>(bb.y)[e];
            if constexpr (ADD) av[i][j][q] = addend[e];
          }
        }
      }
      const uint32_t one = bb.relu ? 0u : 0x3f80u;  // bf16 1.0: no ReLU mask
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mb = m0 + wm * (BM / 2) + 32 * i + 4 * h;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int rr = (q & 3) + 8 * (q >> 2);
            float v = acc[i][j][q];
            if constexpr (ADD) v += av[i][j][q];
            acc[i][j][q] = v;
            const uint32_t ym = one ? one : yr[i][j][q];
            const bool in = mb + rr < M;
            const float d = (in && __uint_as_float(ym << 16) > 0.f) ? v : 0.f;
            const float dx = d * (__uint_as_float(xr[i][j][q] << 16) - bmu[j]) * brs[j];
            ss1[j] += d;
            ss2[j] += in ? dx : 0.f;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mb = m0 + wm * (BM / 2) + 32 * i + 4 * h;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float* p = y + (size_t)mb * K + n0 + wn * (BN / 2) + 32 * j + r;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int rr = (q & 3) + 8 * (q >> 2);
            if (mb + rr < M) p[(size_t)rr * K] = acc[i][j][q];
          }
        }
      }
    };
    if (addend)
      epi2(std::true_type{});
    else
      epi2(std::false_type{});
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bnb_store(bb, s.K, n0 + wn * (BN / 2) + 32 * j + r, (bid % mt) * 2 + wm, h, ss1[j], ss2[j]);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = m0 + wm * (BM / 2) + 32 * i + 4 * h;
    const bool full = m0 + wm * (BM / 2) + 32 * i + 32 <= M;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (BN / 2) + 32 * j + r;
      float* p = y + (size_t)mb * K + co;
      if constexpr (EPI == 1) {  // bf16 output (unsplit, no addend): feeds a bf16-input BatchNorm
        __bf16* pb = yb + (size_t)mb * K + co;
        const float kc = kcol[j];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = (q & 3) + 8 * (q >> 2);
          if (full || mb + rr < M) {
            const __bf16 hv = (__bf16)acc[i][j][q];
            pb[(size_t)rr * K] = hv;
            const float d = (float)hv - kc;
            ss1[j] += d;
            ss2[j] += d * d;
          }
        }
      } else if constexpr (EPI == 2) {
        // (the whole EPI 2 epilogue runs above, before these per-tile loops)
      } else if (full && addend) {
        // all 16 addend loads first, then the stores (interleaved, hipcc waited
        // vmcnt(0) per element: 16 serial round trips)
        const float* ap = addend + (size_t)mb * K + co;
        float av[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) av[q] = ap[(size_t)((q & 3) + 8 * (q >> 2)) * K];
#pragma unroll
        for (int q = 0; q < 16; ++q) p[(size_t)((q & 3) + 8 * (q >> 2)) * K] = acc[i][j][q] + av[q];
      } else if (full) {
#pragma unroll
        for (int q = 0; q < 16; ++q) p[(size_t)((q & 3) + 8 * (q >> 2)) * K] = acc[i][j][q];
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = (q & 3) + 8 * (q >> 2);
          if (mb + rr >= M) continue;
          float v = acc[i][j][q];
          if (addend) v += addend[(size_t)(mb + rr) * K + co];
          p[(size_t)rr * K] = v;
        }
      }
    }
  }
  if (st) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      stats_store(cs, s.K, n0 + wn * (BN / 2) + 32 * j + r, (bid % mt) * 2 + wm, h, ss1[j], ss2[j]);
  }
}

// ------------------------------- 3x3 stride-2 backward-data (halo form) ----
// dX of a 3x3 / stride 2 / pad 1 conv on an even input: output pixel
// (2a + py, 2b + px) takes only the taps of its parity class -
//   py = 0: kh = 1 reading dY row a;  py = 1: kh = 0 reading row a + 1 and
//   kh = 2 reading row a  (likewise px / kw / columns)
// - so a block owns 128 dY-grid pixels (n, a, b) x 64 input channels and
// keeps FOUR accumulator sets, one per class: each of the 9 taps is one
// 128 x 64 x 64 MFMA step into its class, reading the dY halo (the tile's
// stacked rows plus one below) at a per-lane (+1 row / +1 column) shift.
// Same staging as conv3_kernel: halo and weight ring by LDS-DMA, swizzled
// 128-byte rows, zero row for shifts past the image; weights in the
// stride-1 dgrad layout (taps reversed, [tap'][ci][co]).  Replaces the
// phase-split tiled kernel on these layers (45-56 us at B = 32).
template <int BM, int BN, int RB>
__global__ __launch_bounds__(NT) void dgrad3s2_kernel(ConvShape s, const __bf16* __restrict__ dy,
                                                      const __bf16* __restrict__ wt,
                                                      float* __restrict__ dx, int cps,
                                                      const float* __restrict__ addend,
                                                      const BnBwdStats bb) {
  using h3::ROWB;
  using h3::HCAP;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GB = BN / 32;
  constexpr int HB = (HCAP + 1) * ROWB;
  constexpr int BSZ = BN * ROWB;
  static_assert(RB >= 3 && RB <= 4, "ring depth");
  __shared__ __attribute__((aligned(1024))) char smem[HB + RB * BSZ];
  const int OH = s.OH, OW = s.OW;
  const int M = s.N * OH * OW;  // dY-grid pixels
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;  // n: input channel ci
  const int nch = s.K / BK;  // reduction over output channels co
  const int cc0 = blockIdx.y * cps, cc1 = min(nch, cc0 + cps);
  const int g_first = m0 / OW, g_last = (min(m0 + BM, M) - 1) / OW;
  const long long hbase = (long long)g_first * OW;  // global dY pixel of halo row 0
  const int npix = (g_last - g_first + 2) * OW;
  const int nins = (npix + 7) >> 3;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5, lr = lane >> 3;
  if (tid < 8) *reinterpret_cast<uint4*>(smem + HCAP * ROWB + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
  int gl[TM], bs[TM], as[TM];
  bool mv[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / 2) + 32 * i + r;
    mv[i] = m < M;
    const int mm = mv[i] ? m : m0;
    const int g = mm / OW;
    bs[i] = mm - g * OW;
    as[i] = g % OH;
    gl[i] = g - g_first;
  }
  const __bf16* bsrc[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = wave * (BN / 4) + 8 * j + lr;
    bsrc[j] = wt + (size_t)(n0 + row) * s.K + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  auto issue_b = [&](int tap, int cc, int slot) {  // original tap (kh, kw) = (tap / 3, tap % 3)
    const size_t o = (size_t)(8 - tap) * s.C * s.K + (size_t)cc * BK;
    char* dst = smem + HB + slot * BSZ + wave * (BN / 4) * ROWB;
#pragma unroll
    for (int j = 0; j < GB; ++j) h3::glds(bsrc[j] + o, dst + 8 * j * ROWB);
  };
  auto issue_halo = [&](int cc) {
    for (int ins = wave; ins < nins; ins += 4) {
      const int p = 8 * ins + lr;
      const long long gp = hbase + p;
      const bool ok = p < npix && gp < M;
      const void* src = ok ? (const void*)(dy + gp * s.K + (size_t)cc * BK +
                                           8 * ((lane & 7) ^ ((p >> 1) & 7)))
                           : (const void*)h3::g_zero;
      h3::glds(src, smem + ins * 8 * ROWB);
    }
  };
  f32x16 acc[4][TM][TN];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[c][i][j] = zero16();
  for (int cc = cc0; cc < cc1; ++cc) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_halo(cc);
#pragma unroll
    for (int t = 0; t < RB - 1; ++t) issue_b(t, cc, t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ahead = min(RB - 2, 8 - t);
      if (ahead >= 2)
        h3::wait_vm<2 * GB>();
      else if (ahead == 1)
        h3::wait_vm<GB>();
      else
        h3::wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + RB - 1 < 9) issue_b(t + RB - 1, cc, (t + RB - 1) % RB);
      const int kh = t / 3, kw = t - 3 * kh;
      const int cls = (kh != 1 ? 2 : 0) + (kw != 1 ? 1 : 0);  // (py, px)
      const int dh = kh == 0 ? 1 : 0, dw = kw == 0 ? 1 : 0;
      int hrow[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool ok = mv[i] && as[i] + dh < OH && bs[i] + dw < OW;
        hrow[i] = ok ? (gl[i] + dh) * OW + bs[i] + dw : HCAP;
      }
      const char* B = smem + HB + (t % RB) * BSZ;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int c = 2 * ks + h;
        bfx8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bfx8*>(smem + hrow[i] * ROWB +
                                                ((c ^ ((hrow[i] >> 1) & 7)) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int R = wn * (BN / 2) + 32 * j + r;
          b[j] = *reinterpret_cast<const bfx8*>(B + R * ROWB + ((c ^ ((R >> 1) & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[cls][i][j] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[cls][i][j], 0, 0, 0);
      }
    }
  }
  // epilogue: grid pixel m = (n, a, b) -> dX pixels (n, 2a + py, 2b + px);
  // the addend (the gradient join of a downsample block) is loaded for a whole
  // row group before any store: interleaved, hipcc waited vmcnt(0) per element
  // (64 serial round trips a lane; 162 us instead of ~50 at B = 128)
  dx += (size_t)blockIdx.y * s.N * s.H * s.W * s.C;
  const size_t C = s.C, W = s.W;
  // unsplit, dX = a BatchNorm's dY: its backward sums too (bnb_store)
  const bool bst = bb.part != nullptr;
  float bs1[TN], bs2[TN], bmu[TN], brs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int ci = n0 + wn * (BN / 2) + 32 * j + r;
    bs1[j] = bs2[j] = 0.f;
    bmu[j] = bst ? bb.mean[ci] : 0.f;
    brs[j] = bst ? bb.rstd[ci] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int ci = n0 + wn * (BN / 2) + 32 * j + r;
#pragma unroll
      for (int q4 = 0; q4 < 16; q4 += 4) {
        size_t o[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(q4 + u, lane);
          ok[u] = m < M;
          const int mm = ok[u] ? m : 0;
          const int b = mm % OW, g = mm / OW;  // g = n * OH + a
          o[u] = ((size_t)(2 * g) * W + 2 * b) * C + ci;  // (n, 2a, 2b)
        }
        float av[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            av[u][c] = (addend && ok[u]) ? addend[o[u] + (c >> 1) * W * C + (c & 1) * C] : 0.f;
        float xv[4][4], yv[4][4];
        if (bst) {
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const size_t e = o[u] + (c >> 1) * W * C + (c & 1) * C;
              xv[u][c] = bf16_at(bb.x, e);
              yv[u][c] = bf16_at(bb.y, e);  // y = x without a ReLU (host), mask unused
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (!ok[u]) continue;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float v = acc[c][i][j][q4 + u] + av[u][c];
            dx[o[u] + (c >> 1) * W * C + (c & 1) * C] = v;
            if (bst) {
              const float d = (!bb.relu || yv[u][c] > 0.f) ? v : 0.f;
              bs1[j] += d;
              bs2[j] += d * (xv[u][c] - bmu[j]) * brs[j];
            }
          }
        }
      }
    }
  if (bst) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bnb_store(bb, s.C, n0 + wn * (BN / 2) + 32 * j + r, (bid % mt) * 2 + wm, h, bs1[j], bs2[j]);
  }
}

// ----------------------------------------------------- backward-filter ----
// dW[tap][ci][co] = sum_pix X[pix shifted by tap][ci] dY[pix][co].  GEMM
// M = (tap, ci), N = co, reduction over output pixels; block = (128-row M
// tile, co tile, pixel slice z).  The MFMA wants 8 consecutive pixels per lane and
// NHWC keeps channels contiguous, so every thread loads 8 pixels x 4
// channels (8 float4; 64-row tiles: 4 pixels) and writes them transposed as
// 4 [channel][8 (4) pixels] 16 (8)-byte vectors into the [row][64 + 8] LDS
// image - no per-element LDS stores.
// XB: x and dY are bf16 copies (8-byte loads of 4 channels), else fp32.
template <int BM, int BN, bool XB>
struct WgLoader {
  using T = typename std::conditional<XB, __bf16, float>::type;
  using V = typename std::conditional<XB, uint2, float4>::type;  // 4 channels
  static constexpr int GA = BM / 4, GB = BN / 4;          // channel quads per tile
  static constexpr int PA = BK * GA / NT, PB = BK * GB / NT;  // pixels per thread (4 or 8)
  static_assert((PA == 4 || PA == 8) && (PB == 4 || PB == 8), "tile shape");
  ConvShape s;
  const T* x;
  const T* dy;
  int kh, kw, pix0, npix, ca, cb;
  // output-pixel coordinates of this thread's first A pixel, walked forward BK
  // pixels a K tile (load(kt) runs for kt = 0, 1, ... in order): one division
  // set per thread instead of one per tile (conv_tiled.hip PixWalk: the fp32
  // filter gradients' VALU count 4,249 -> 3,571 a wave)
  int wox, woy, wn, dox, doy;
  bool mv;
  V ra[PA], rb[PB];
  // A rows are the flattened (tap, ci) index m = tap * C + ci: a 128-row tile
  // spans two taps of a 64-channel layer, so the dY tile it multiplies is
  // fetched once for both (C % 64 == 0: a channel quad never straddles taps)
  using TX = T;
  using TD = T;
  __device__ WgLoader(const ConvShape& s_, const ConvShape&, const T* x_, const T* dy_, int m0,
                      int n0, int pix0_, int npix_)
      : s(s_), x(x_), dy(dy_), pix0(pix0_), npix(npix_) {
    const int m = m0 + 4 * (threadIdx.x % GA);
    mv = m < s.R * s.S * s.C;
    const int mm = mv ? m : 0, tap = mm / s.C;
    kh = tap / s.S;
    kw = tap % s.S;
    ca = mm % s.C;
    cb = n0 + 4 * (threadIdx.x % GB);
    const int pc = min(pix0 + PA * ((int)threadIdx.x / GA), npix - 1);
    wox = pc % s.OW;
    const int t = pc / s.OW;
    woy = t % s.OH;
    wn = t / s.OH;
    dox = BK % s.OW;
    doy = BK / s.OW;
  }
  __device__ __forceinline__ void load(int kt) {
    const int tid = threadIdx.x;
    V z;
    if constexpr (XB)
      z = make_uint2(0u, 0u);
    else
      z = make_float4(0.f, 0.f, 0.f, 0.f);
    {
      const int p = pix0 + kt * BK + PA * (tid / GA);
      int ox = wox, oy = woy, n = min(wn, s.N - 1);
      wox += dox;  // the next tile's first pixel (past the end: masked, image clamped)
      woy += doy;
      if (wox >= s.OW) {
        wox -= s.OW;
        ++woy;
      }
      while (woy >= s.OH) {
        woy -= s.OH;
        ++wn;
      }
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        const int iy = oy * s.stride - s.pad + kh, ix = ox * s.stride - s.pad + kw;
        const bool ok = mv && p + q < npix && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
        const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
        const V v = *reinterpret_cast<const V*>(x + (((size_t)n * s.H + iyc) * s.W + ixc) * s.C + ca);
        ra[q] = sel(ok, v);
        if (++ox == s.OW) {  // next output pixel (rows past the end are masked)
          ox = 0;
          if (++oy == s.OH) {
            oy = 0;
            n = min(n + 1, s.N - 1);
          }
        }
      }
    }
    {
      const int p = pix0 + kt * BK + PB * (tid / GB);
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const V v = *reinterpret_cast<const V*>(dy + (size_t)min(p + q, npix - 1) * s.K + cb);
        rb[q] = sel(p + q < npix, v);
      }
    }
  }
  // channel c of the P pixels held in r, as P consecutive bf16 (one LDS row run)
  __device__ __forceinline__ static __bf16 chan(const float4& r, int c) {
    return (__bf16)(c == 0 ? r.x : c == 1 ? r.y : c == 2 ? r.z : r.w);
  }
  __device__ __forceinline__ static __bf16 chan(const uint2& r, int c) {
    const uint32_t w = c < 2 ? r.x : r.y;
    return __builtin_bit_cast(__bf16, (uint16_t)(c & 1 ? w >> 16 : w & 0xffffu));
  }
  template <int P>
  __device__ __forceinline__ static void put_col(__bf16* dst, const V (&r)[P], int c) {
    __bf16 v[P];
#pragma unroll
    for (int q = 0; q < P; ++q) v[q] = chan(r[q], c);
    if constexpr (P == 8)
      *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, v);
    else
      *reinterpret_cast<uint2*>(dst) = __builtin_bit_cast(uint2, v);
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x;
    const int ra0 = 4 * (tid % GA), ka = PA * (tid / GA);
    const int rb0 = 4 * (tid % GB), kb = PB * (tid / GB);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      put_col<PA>(As + (ra0 + c) * LDK + ka, ra, c);
      put_col<PB>(Bs + (rb0 + c) * LDK + kb, rb, c);
    }
  }
};

// Stem filter gradient over the implicit im2col (see StemLoader): A rows are
// the kp k-indices, each thread fetches 4 consecutive k (one image run) for
// PA pixels straight from the fp32 image; B = the bf16 dY as in WgLoader.
template <int BM, int BN>
struct StemWgLoader {
  using TX = float;
  using TD = __bf16;
  using LA = WgLoader<BM, BN, false>;  // fp32 A vectors (float4 = 4 k)
  using LB = WgLoader<BM, BN, true>;   // bf16 B vectors (uint2 = 4 channels)
  static constexpr int GA = LA::GA, GB = LB::GB, PA = LA::PA, PB = LB::PB;
  ConvShape s, si;
  StemGeo g;
  const float* x;
  const __bf16* dy;
  int pix0, npix, ka0, cb;
  bool mv;
  float4 ra[PA];
  uint2 rb[PB];
  __device__ StemWgLoader(const ConvShape& s_, const ConvShape& si_, const float* x_,
                          const __bf16* dy_, int m0, int n0, int pix0_, int npix_)
      : s(s_), si(si_), g(si_), x(x_), dy(dy_), pix0(pix0_), npix(npix_) {
    ka0 = m0 + 4 * (threadIdx.x % GA);  // this thread's 4 k (a quad never straddles tap rows)
    mv = ka0 < s.C;
    cb = n0 + 4 * (threadIdx.x % GB);
  }
  __device__ __forceinline__ void load(int kt) {
    const int tid = threadIdx.x;
    {
      const int p = pix0 + kt * BK + PA * (tid / GA);
      const int pc = min(p, npix - 1);
      int ox = pc % s.OW, t = pc / s.OW, oy = t % s.OH, n = t / s.OH;
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        float v[4];
        g.fetch<4>(si, x, n, oy * si.stride - si.pad, ox * si.stride - si.pad, ka0,
                   mv && p + q < npix, v);
        ra[q] = make_float4(v[0], v[1], v[2], v[3]);
        if (++ox == s.OW) {
          ox = 0;
          if (++oy == s.OH) {
            oy = 0;
            n = min(n + 1, s.N - 1);
          }
        }
      }
    }
    {
      const int p = pix0 + kt * BK + PB * (tid / GB);
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const uint2 v = *reinterpret_cast<const uint2*>(dy + (size_t)min(p + q, npix - 1) * s.K + cb);
        rb[q] = sel(p + q < npix, v);
      }
    }
  }
  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
    const int tid = threadIdx.x;
    const int ra0 = 4 * (tid % GA), ka = PA * (tid / GA);
    const int rb0 = 4 * (tid % GB), kb = PB * (tid / GB);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      LA::template put_col<PA>(As + (ra0 + c) * LDK + ka, ra, c);
      LB::template put_col<PB>(Bs + (rb0 + c) * LDK + kb, rb, c);
    }
  }
};

template <int BM, int BN, bool XB, class LD = WgLoader<BM, BN, XB>>
__global__ __launch_bounds__(NT) void wgrad_kernel(
    ConvShape s, const typename LD::TX* __restrict__ x, const typename LD::TD* __restrict__ dy,
    float* __restrict__ part, int kchunk, const ConvShape si) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int STAGE = (BM + BN) * LDK;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int Mw = s.R * s.S * s.C;
  const int mt = (Mw + BM - 1) / BM, ntl = s.K / BN;
  const int tiles = mt * ntl;
  const int z = blockIdx.x / tiles, rem = blockIdx.x % tiles;
  const int m0 = (rem % mt) * BM, n0 = (rem / mt) * BN;
  const int npix = s.N * s.OH * s.OW;
  const int pix0 = z * kchunk * BK;
  const int nk = min(kchunk, (npix - pix0 + BK - 1) / BK);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5;
  LD ld(s, si, x, dy, m0, n0, pix0, npix);
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero16();
  if (nk > 0) {
    ld.load(0);
    ld.store(smem, smem + BM * LDK);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const __bf16* A = smem + (kt & 1) * STAGE;
      const __bf16* B = A + BM * LDK;
      __bf16* nxt = smem + ((kt + 1) & 1) * STAGE;
      const bool more = kt + 1 < nk;
      if (more) ld.load(kt + 1);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bfx8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bfx8*>(A + (wm * (BM / 2) + 32 * i + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const bfx8*>(B + (wn * (BN / 2) + 32 * j + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (more) ld.store(nxt, nxt + BM * LDK);
      __syncthreads();
    }
  }
  float* out = part + (size_t)z * Mw * s.K;  // HWIO flattened: row m = tap * C + ci
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + r;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(q, lane);
        if (m < Mw) out[(size_t)m * s.K + co] = acc[i][j][q];
      }
  }
}

// cs (with outb): BatchNorm statistics of the bf16 outputs, one partial row
// per block (C channels, 256 % (C / 4) == 0: a thread keeps one channel quad)
__global__ __launch_bounds__(256) void slab_sum4_kernel(const float4* __restrict__ part, int nz,
                                                        long long zs, long long n4,
                                                        float4* __restrict__ out,
                                                        const float4* __restrict__ addend,
                                                        uint2* __restrict__ outb,
                                                        const ConvStats cs, int C,
                                                        const BnBwdStats bb) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const bool bs = !outb && bb.part;  // fp32 dX = a BatchNorm's dY: its backward sums
  const bool st = (outb && cs.part) || bs;
  const int cq = C >> 2, tid = threadIdx.x;
  float4 kc = make_float4(0.f, 0.f, 0.f, 0.f), t1 = kc, t2 = kc, mu = kc, rs = kc;
  if (outb && cs.part) kc = *reinterpret_cast<const float4*>(cs.shift + 4 * (tid % cq));
  if (bs) {
    mu = *reinterpret_cast<const float4*>(bb.mean + 4 * (tid % cq));
    rs = *reinterpret_cast<const float4*>(bb.rstd + 4 * (tid % cq));
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = part[i];
    for (int z = 1; z < nz; ++z) {
      const float4 b = part[z * zs + i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    if (addend) {
      const float4 b = addend[i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    if (outb) {
      const __bf16 hv[4] = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w};
      outb[i] = __builtin_bit_cast(uint2, hv);
      if (st) {
        const float d[4] = {(float)hv[0] - kc.x, (float)hv[1] - kc.y, (float)hv[2] - kc.z,
                            (float)hv[3] - kc.w};
        t1.x += d[0]; t1.y += d[1]; t1.z += d[2]; t1.w += d[3];
        t2.x += d[0] * d[0]; t2.y += d[1] * d[1]; t2.z += d[2] * d[2]; t2.w += d[3] * d[3];
      }
    } else {
      out[i] = a;
      if (bs) {
        const float av[4] = {a.x, a.y, a.z, a.w};
        const float mv[4] = {mu.x, mu.y, mu.z, mu.w}, rv[4] = {rs.x, rs.y, rs.z, rs.w};
        // 4 bf16 of x and of y (= x without a ReLU) as one 8-byte load each
        const uint2 xu = reinterpret_cast<const uint2*>(bb.x)[i];
        const uint2 yu = reinterpret_cast<const uint2*>(bb.y)[i];
        const float xv[4] = {__uint_as_float(xu.x << 16), __uint_as_float(xu.x & 0xffff0000u),
                             __uint_as_float(xu.y << 16), __uint_as_float(xu.y & 0xffff0000u)};
        const float yv[4] = {__uint_as_float(yu.x << 16), __uint_as_float(yu.x & 0xffff0000u),
                             __uint_as_float(yu.y << 16), __uint_as_float(yu.y & 0xffff0000u)};
        float d[4], e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          d[c] = (!bb.relu || yv[c] > 0.f) ? av[c] : 0.f;
          e[c] = d[c] * (xv[c] - mv[c]) * rv[c];
        }
        t1.x += d[0]; t1.y += d[1]; t1.z += d[2]; t1.w += d[3];
        t2.x += e[0]; t2.y += e[1]; t2.z += e[2]; t2.w += e[3];
      }
    }
  }
  if (st) {  // threads tid, tid + cq, ... share a channel quad: fixed-order sum
    __shared__ float4 red[2][256];
    red[0][tid] = t1;
    red[1][tid] = t2;
    __syncthreads();
    if (tid < cq) {
      float4 a = red[0][tid], b = red[1][tid];
      for (int t = tid + cq; t < 256; t += cq) {
        a.x += red[0][t].x; a.y += red[0][t].y; a.z += red[0][t].z; a.w += red[0][t].w;
        b.x += red[1][t].x; b.y += red[1][t].y; b.z += red[1][t].z; b.w += red[1][t].w;
      }
      float* part = bs ? bb.part : cs.part;
      const int P = bs ? bb.P : cs.P;
      const size_t i = stats_index(4 * tid, blockIdx.x, P);
      *reinterpret_cast<float4*>(part + i) = a;
      *reinterpret_cast<float4*>(part + (size_t)C * P + i) = b;
    }
  }
}

// In-place first stage for deep, narrow slab stacks (the im2col'd stem's
// filter gradient: 256 slices of 192 x 64): group g of G slices is summed
// into its first slice, so the final slab_sum4 pass (zstride G) reads nz / G
// slices per thread instead of nz on 12 blocks.
__global__ __launch_bounds__(256) void slab_fold4_kernel(float4* __restrict__ part, int nz, int G,
                                                         long long n4) {
  const int z0 = blockIdx.y * G, z1 = min(nz, z0 + G);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = part[z0 * n4 + i];
    for (int z = z0 + 1; z < z1; ++z) {
      const float4 b = part[z * n4 + i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    part[z0 * n4 + i] = a;
  }
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Deep, narrow slab stacks in ONE pass (the fold + sum pair of launches
// before): G lanes per output float4 (lanes i * G .. i * G + G - 1 of a
// block), lane g summing slabs g, g + G, g + 2G, ... in order with 4 loads in
// flight, then a fixed xor tree over the G lanes - the same association on
// every run.  Plain fp32 outputs only (no statistics / addend / bf16 copy).
template <int G>
__global__ __launch_bounds__(256) void slab_sumg4_kernel(const float4* __restrict__ part, int nz,
                                                         long long n4, float4* __restrict__ out) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long i = t / G;
  const int g = (int)(t % G);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int z = g;
    for (; z + 3 * G < nz; z += 4 * G) {
      const float4 v0 = part[(long long)z * n4 + i], v1 = part[(long long)(z + G) * n4 + i];
      const float4 v2 = part[(long long)(z + 2 * G) * n4 + i];
      const float4 v3 = part[(long long)(z + 3 * G) * n4 + i];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; z < nz; z += G) {
      const float4 v = part[(long long)z * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) {
    a.x += __shfl_xor(a.x, m, 64);
    a.y += __shfl_xor(a.y, m, 64);
    a.z += __shfl_xor(a.z, m, 64);
    a.w += __shfl_xor(a.w, m, 64);
  }
  if (g == 0 && i < n4) out[i] = a;
}

// Deterministic sum of nz slabs of n4 float4s into out (fixed association
// order for a given nz).
// outb: bf16 output instead of out
// grid of slab_sum4 (also the partial rows of its BatchNorm statistics)
static inline int slab_blocks(long long n4) {
  long long b = (n4 + 255) / 256;
  return (int)(b > 4096 ? 4096 : b);
}
static void slab_reduce(float* slabs, int nz, long long n4, float* out, hipStream_t st,
                        const float* addend = nullptr, __bf16* outb = nullptr,
                        const ConvStats* stats = nullptr, int C = 0,
                        const BnBwdStats* bstats = nullptr) {
  const long long b = slab_blocks(n4);
  if (nz >= 16 && !addend && !outb && !(stats && stats->part) && !(bstats && bstats->part)) {
    // plain sums of 16+ slabs: G lanes per output keep more loads in flight
    // than one thread walking every slab
    const float4* P4 = reinterpret_cast<const float4*>(slabs);
    float4* O4 = reinterpret_cast<float4*>(out);
    if (nz >= 128)
      slab_sumg4_kernel<16><<<cdiv(n4 * 16, 256), 256, 0, st>>>(P4, nz, n4, O4);
    else if (nz >= 32)
      slab_sumg4_kernel<8><<<cdiv(n4 * 8, 256), 256, 0, st>>>(P4, nz, n4, O4);
    else
      slab_sumg4_kernel<4><<<cdiv(n4 * 4, 256), 256, 0, st>>>(P4, nz, n4, O4);
    return;
  }
  int G = 1;
  if (b < 128 && nz >= 32) {
    G = 8;
    slab_fold4_kernel<<<dim3((int)b, cdiv(nz, G)), 256, 0, st>>>(reinterpret_cast<float4*>(slabs),
                                                                 nz, G, n4);
  }
  ConvStats cs;
  if (stats && stats->part) {
    if (!outb || C % 64 || 256 % (C / 4) || stats->P != b)
      throw std::runtime_error("slab_reduce: BatchNorm statistics layout mismatch");
    cs = *stats;
  }
  BnBwdStats bb;
  if (bstats && bstats->part) {
    if (outb || C % 64 || 256 % (C / 4) || bstats->P != b)
      throw std::runtime_error("slab_reduce: BatchNorm backward statistics layout mismatch");
    bb = *bstats;
  }
  slab_sum4_kernel<<<(int)b, 256, 0, st>>>(reinterpret_cast<const float4*>(slabs), cdiv(nz, G),
                                          n4 * G, n4, reinterpret_cast<float4*>(out),
                                          reinterpret_cast<const float4*>(addend),
                                          reinterpret_cast<uint2*>(outb), cs, C, bb);
}

enum Tile { T128x128, T128x64, T64x128, T64x64 };
static inline int tm(Tile t) { return (t == T128x128 || t == T128x64) ? 128 : 64; }
static inline int tn(Tile t) { return (t == T128x128 || t == T64x128) ? 128 : 64; }

// Largest tile that still gives >= 256 blocks (one per CU); deep layers that
// cannot reach it take 64x64 (or 64x128) tiles plus split-K.
struct Plan {
  Tile t;
  int z, kps;
};
static inline Plan plan(const ConvShape& s, bool epilogue) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const Tile order[4] = {T128x128, T128x64, T64x128, T64x64};
  Tile t = T64x64;
  for (Tile c : order) {
    if (tn(c) > s.K) continue;
    if ((long long)cdiv(M, tm(c)) * cdiv(s.K, tn(c)) >= 256) {
      t = c;
      break;
    }
  }
  const long long blocks = (long long)cdiv(M, tm(t)) * cdiv(s.K, tn(t));
  const int nk = s.R * s.S * (s.C / BK);
  int z = 1;
  if (!epilogue && blocks < 256 && nk >= 8) {
    z = cdiv(512, blocks);
    if (z > nk / 4) z = nk / 4;
    if (z > 8) z = 8;
    if (z < 1) z = 1;
  }
  const int kps = cdiv(nk, z);
  return {t, cdiv(nk, kps), kps};
}

static inline long long wt_elems(const ConvShape& s) { return (long long)s.R * s.S * s.C * s.K; }
// bf16 weight copy at the front of the workspace, split-K slabs after it
static inline long long wt_floats(const ConvShape& s) { return ((wt_elems(s) + 127) / 128) * 64; }

// partial rows of the BatchNorm statistics the forward writes (plan-dependent)
static int stats_rows(const ConvShape& s, bool epilogue) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const Plan p = plan(s, epilogue);
  if (p.z > 1) return slab_blocks(M * s.K / 4);
  return cdiv(M, tm(p.t)) * 2;
}

template <class XT>
static void launch(const ConvShape& s, const XT* x, const __bf16* wt, const float* bias,
                   float* y, bool relu, float* ws, hipStream_t st,
                   const float* addend = nullptr, __bf16* yb = nullptr, int ex2 = 0,
                   const ConvStats* stats = nullptr) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const Plan p = plan(s, bias != nullptr || relu || ex2);  // ex2: never split
  ConvStats cs;
  if (stats && stats->part) {
    if (!yb || bias || relu || ex2 || stats->P != stats_rows(s, false))
      throw std::runtime_error("conv fwd: BatchNorm statistics need a plain bf16-output conv");
    if (p.z == 1) cs = *stats;
  }
  float* slabs = ws + wt_floats(s);
  float* out = p.z > 1 ? slabs : y;
  const float* add = p.z > 1 ? nullptr : addend;  // split-K: added by the slab reduction
  __bf16* ob = p.z > 1 ? nullptr : yb;             // ... and converted there
  const int r = relu ? 1 : 0;
#define GRID(BM_, BN_) dim3(cdiv(M, BM_) * cdiv(s.K, BN_), p.z)
  switch (p.t) {
    case T128x128: fwd_kernel<128, 128, XT><<<GRID(128, 128), NT, 0, st>>>(s, x, wt, bias, out, r, p.kps, add, ob, ex2, s, cs); break;
    case T128x64: fwd_kernel<128, 64, XT><<<GRID(128, 64), NT, 0, st>>>(s, x, wt, bias, out, r, p.kps, add, ob, ex2, s, cs); break;
    case T64x128: fwd_kernel<64, 128, XT><<<GRID(64, 128), NT, 0, st>>>(s, x, wt, bias, out, r, p.kps, add, ob, ex2, s, cs); break;
    default: fwd_kernel<64, 64, XT><<<GRID(64, 64), NT, 0, st>>>(s, x, wt, bias, out, r, p.kps, add, ob, ex2, s, cs); break;
  }
#undef GRID
  if (p.z > 1) slab_reduce(slabs, p.z, M * s.K / 4, y, st, addend, yb, stats, s.K);
}

// halo conv: 3x3, stride 1, pad 1, C and K % 64 == 0, a 128-pixel tile's
// halo within HCAP rows (W <= ~84), 32-bit pixel x channel offsets
static bool conv3_ok(const ConvShape& s) {
  return s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.OH == s.H && s.OW == s.W &&
         s.C % 64 == 0 && s.K % 64 == 0 && h3::halo_rows(s, 128) <= h3::HCAP &&
         (long long)s.N * s.H * s.W * s.C < (1LL << 31);
}
// 64-channel output tiles; split-K over channel chunks up to one block per CU
struct P3 {
  int z, cps, bm;
};
// 128-pixel tiles when they fill the chip; otherwise (the small-M deep
// layers) 64-pixel tiles, split-K over channel chunks only below 128 blocks
// (split-K slabs cost a ~7 us reduction launch per conv)
static inline P3 plan3(const ConvShape& s) {
  const long long M = (long long)s.N * s.H * s.W;
  const int nch = s.C / BK;
  if ((long long)cdiv(M, 128) * (s.K / 64) >= 256) return {1, nch, 128};
  const long long blocks = (long long)cdiv(M, 64) * (s.K / 64);
  int z = 1;
  if (blocks < 128) {
    z = cdiv(256, blocks);
    if (z > nch) z = nch;
  }
  const int cps = cdiv(nch, z);
  return {cdiv(nch, cps), cps, 64};
}
static int stats_rows3(const ConvShape& s) {
  const long long M = (long long)s.N * s.H * s.W;
  const P3 p = plan3(s);
  if (p.z > 1) return slab_blocks(M * s.K / 4);
  return cdiv(M, p.bm) * 2;
}
static void launch3(const ConvShape& s, const __bf16* x, const __bf16* wt, float* y, float* ws,
                    hipStream_t st, const float* addend, __bf16* yb = nullptr,
                    const ConvStats* stats = nullptr, const BnBwdStats* bstats = nullptr) {
  const long long M = (long long)s.N * s.H * s.W;
  const P3 p = plan3(s);
  ConvStats cs;
  if (stats && stats->part) {
    if (!yb || addend || stats->P != stats_rows3(s))
      throw std::runtime_error("conv3: BatchNorm statistics need a plain bf16-output conv");
    if (p.z == 1) cs = *stats;
  }
  BnBwdStats bb;
  if (bstats && bstats->part) {
    if (yb || bstats->P != stats_rows3(s))
      throw std::runtime_error("conv3: BatchNorm backward statistics layout mismatch");
    if (p.z == 1) bb = *bstats;
  }
  float* slabs = ws + wt_floats(s);
  float* out = p.z > 1 ? slabs : y;
  const dim3 grid(cdiv(M, p.bm) * (s.K / 64), p.z);
  const float* add = p.z > 1 ? nullptr : addend;
  __bf16* ob = p.z > 1 ? nullptr : yb;
  const int epi = ob ? 1 : (bb.part ? 2 : 0);
#define C3(BM_, E_) conv3_kernel<BM_, 64, 4, E_><<<grid, NT, 0, st>>>(s, x, wt, out, p.cps, add, ob, cs, bb)
  if (p.bm == 128) {
    if (epi == 1) C3(128, 1); else if (epi == 2) C3(128, 2); else C3(128, 0);
  } else {
    if (epi == 1) C3(64, 1); else if (epi == 2) C3(64, 2); else C3(64, 0);
  }
#undef C3
  if (p.z > 1) slab_reduce(slabs, p.z, M * s.K / 4, y, st, addend, yb, stats, s.K, bstats);
}

// 3x3 / stride 2 / pad 1 dgrad on an even input (the halo form above)
static bool dgrad3s2_ok(const ConvShape& s) {
  return s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.H == 2 * s.OH &&
         s.W == 2 * s.OW && s.C % 64 == 0 && s.K % 64 == 0 &&
         ((128 + s.OW - 2) / s.OW + 2) * s.OW <= h3::HCAP &&
         (long long)s.N * s.H * s.W * s.C < (1LL << 31);
}
// split-K over co chunks up to one block per CU (measured: splitting only
// below 128 blocks - fewer 4x-sized dX slabs - was no faster, 2.70 vs 2.69 ms)
static inline P3 plan3s2(const ConvShape& s) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const long long blocks = (long long)cdiv(M, 64) * (s.C / 64);
  const int nch = s.K / BK;
  int z = 1;
  if (blocks < 256) {
    z = cdiv(256, blocks);
    if (z > nch) z = nch;
  }
  const int cps = cdiv(nch, z);
  return {cdiv(nch, cps), cps, 64};
}
// partial rows of the BatchNorm backward statistics launch3s2 writes
static int stats_rows3s2(const ConvShape& s) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const P3 p = plan3s2(s);
  if (p.z > 1) return slab_blocks((long long)s.N * s.H * s.W * s.C / 4);
  return cdiv(M, 64) * 2;
}
static void launch3s2(const ConvShape& s, const __bf16* dy, const __bf16* wt, float* dx,
                      float* ws, hipStream_t st, const float* addend,
                      const BnBwdStats* bstats = nullptr) {
  const long long M = (long long)s.N * s.OH * s.OW;
  const P3 p = plan3s2(s);
  BnBwdStats bb;
  if (bstats && bstats->part) {
    if (bstats->P != stats_rows3s2(s))
      throw std::runtime_error("dgrad3s2: BatchNorm backward statistics layout mismatch");
    if (p.z == 1) bb = *bstats;
  }
  float* slabs = ws + wt_floats(s);
  float* out = p.z > 1 ? slabs : dx;
  // 64-pixel tiles: with four accumulator classes a 128-pixel tile needed 272
  // registers a lane (one wave per SIMD) and ran 10x slower per tile
  const dim3 grid(cdiv(M, 64) * (s.C / 64), p.z);
  dgrad3s2_kernel<64, 64, 4><<<grid, NT, 0, st>>>(s, dy, wt, out, p.cps,
                                                  p.z > 1 ? nullptr : addend, bb);
  if (p.z > 1)
    slab_reduce(slabs, p.z, (long long)s.N * s.H * s.W * s.C / 4, dx, st, addend, nullptr,
                nullptr, s.C, bstats);
}

// wgrad: tile = (ci, co) per tap; pixel slices fill the chip (~1024 blocks),
// at least 4 K tiles per slice, at most 64 slices
struct WgPlan {
  int bm, bn, z, kchunk;
};
static inline WgPlan wg_plan(const ConvShape& s) {
  // (128-row tiles on the space-to-depth stem's 16 taps x 16 channels, each dY
  // tile feeding 8 taps: its filter gradient 69.2 -> 72.4 us, step neutral;
  // r6_s40.steps)
  const int bm = s.C % 128 == 0 ? 128 : 64;
  const int bn = s.K % 128 == 0 ? 128 : 64;
  const long long tiles = (long long)cdiv((long long)s.R * s.S * s.C, bm) * (s.K / bn);
  const int ktiles = cdiv((long long)s.N * s.OH * s.OW, BK);
  const int target = 1024;
  int z = cdiv(target, tiles);
  if (z > ktiles / 4) z = ktiles / 4;
  // <= 4 output tiles (the im2col'd stem: 192 x 64) need deep pixel splits to
  // fill the chip; otherwise 64 slices (measured: more slices cost more slab
  // traffic than they win on ResNet-18 layer1)
  const int zcap = tiles <= 4 ? 256 : 64;
  if (z > zcap) z = zcap;
  if (z < 1) z = 1;
  const int kchunk = cdiv(ktiles, z);
  return {bm, bn, cdiv(ktiles, kchunk), kchunk};
}

static void convert(const ConvShape& s, const float* w, int mode, __bf16* out, hipStream_t st) {
  const int taps = s.R * s.S;
  wcvt_kernel<<<taps * (s.C / 32) * (s.K / 32), 256, 0, st>>>(w, taps, s.C, s.K, mode, out);
}

// the stride-1 backward-data conv as a forward conv: input dY [N, OH, OW, K],
// output dX [N, H, W, C], padding R - 1 - pad
static inline ConvShape dgrad_shape(const ConvShape& s) {
  ConvShape d;
  d.N = s.N;
  d.H = s.OH;
  d.W = s.OW;
  d.C = s.K;
  d.K = s.C;
  d.R = s.R;
  d.S = s.S;
  d.stride = 1;
  d.pad = s.R - 1 - s.pad;
  d.OH = s.H;
  d.OW = s.W;
  return d;
}

// ------------------------------------------ 3x3 stride-1 filter gradient ----
// dW[kh,kw,ci,co] = sum_{n,y,x} X[n, y+kh-1, x+kw-1, ci] dY[n, y, x, co] for
// the 3x3 / stride-1 / pad-1 layers that make up most of ResNet-18.  The
// generic wgrad above re-fetches (and per-element transposes) the shifted X
// tile once per tap and ran layer 1 at ~86 TFLOP/s (4 x 86 us per step).
// Here a block owns a 64 (ci) x 64 (co) pair for ALL 9 taps and streams
// 64-pixel chunks (TR whole output rows of one image):
//   * the chunk's X halo ((TR + 2) x (W + 2) pixels x 64 ci) and its dY tile
//     (64 pixels x 64 co) are staged once into LDS as plain [pixel][channel]
//     rows (16-byte global loads, 16-byte LDS stores, zero borders);
//   * the MFMA wants 8 consecutive PIXELS of one channel per lane for both
//     operands (the reduction axis is the pixel), which is a column of those
//     images: gfx950's ds_read_b64_tr_b16 delivers it transposed for free
//     (cdna_hip_programming.md T10), and each lane supplies its own pixel-row
//     address, so the tap shift is just an address offset into the halo;
//   * per 16-pixel k-step a wave reads its dY fragment ONCE and reuses it for
//     the 9 taps' MFMAs (9 accumulators of 32 x 32), i.e. 20 transposed reads
//     per 9 v_mfma_f32_32x32x16_bf16;
//   * rows are 192 B apart, so the four rows of a transposed read and the two
//     16-lane groups of a half-wave hit 8 distinct 8-bank windows;
//   * double-buffered LDS stages, the next chunk's global loads in flight
//     during the current chunk's MFMAs, one barrier per chunk;
//   * pixel splits write fp32 slabs [z][tap][ci][co] summed by slab_reduce
//     (deterministic); the split count keeps the slabs near 38 MB.
// ResNet-18 at B = 32, the 13 such layers: 489 us per step vs 658 us for the
// generic wgrad kernels above (scripts/wgrad3_lab.py).
namespace w3 {
constexpr int LD = 96;  // bf16 per LDS pixel row (192 B)
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

// chunk geometry: NPX output pixels (TR whole rows of one image) per chunk;
// 128-pixel chunks for W >= 28 (twice the MFMAs per staging round trip and
// 2 / 3 of the halo re-reads), 64 below (a 7 x 7 image is one 49-pixel chunk)
template <int NPX>
struct Cfg {
  static constexpr int MAXH = NPX == 128 ? 264 : 200;  // halo pixels (W = 64: 4 x 66 / 3 x 66)
  static constexpr int STG = (MAXH + NPX) * LD;
  static constexpr int XR = (MAXH * 8 + NT - 1) / NT;  // 16-byte halo pieces per thread
  static constexpr int YR = NPX * 8 / NT;              // 16-byte dY pieces per thread
  static constexpr int KS = NPX / 16;                  // MFMA k-steps per chunk
};

__device__ __forceinline__ v4s tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)p);
}

__device__ __forceinline__ bfx8 frag(const __bf16* p0, const __bf16* p1) {
  const v8s v = __builtin_shufflevector(tr_read(p0), tr_read(p1), 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bfx8, v);
}

__host__ __device__ __forceinline__ int rows_per_chunk(const ConvShape& s, int npx) {
  const int tr = npx / s.W;
  return tr < s.H ? tr : s.H;
}

__host__ __device__ __forceinline__ int chunk_pixels(const ConvShape& s) {
  return s.W >= 28 ? 128 : 64;
}
}  // namespace w3

// Global -> register prefetch of one chunk (halo + dY tile), and the
// register -> LDS store of it (plain functions: the arrays must stay in VGPRs)
template <int NPX>
struct W3Regs {
  uint4 rx[w3::Cfg<NPX>::XR], ry[w3::Cfg<NPX>::YR];
};

template <int NPX>
__device__ __forceinline__ void w3_load(W3Regs<NPX>& R, const ConvShape& s, const __bf16* x,
                                        const __bf16* dy, int ch, int rpi, int TR, int HW2,
                                        int hpx, int ci0, int co0) {
  using CF = w3::Cfg<NPX>;
  const int tid = threadIdx.x, H = s.H, W = s.W;
  const int n = ch / rpi, r0 = (ch - n * rpi) * TR, nvalid = min(TR, H - r0) * W;
#pragma unroll
  for (int i = 0; i < CF::XR; ++i) {
    const int e = tid + NT * i, hp = e >> 3, c8 = e & 7;
    const int hy = hp / HW2, hx = hp - hy * HW2, y = r0 + hy - 1, xx = hx - 1;
    const bool ok = hp < hpx && y >= 0 && y < H && xx >= 0 && xx < W;
    const int yc = min(max(y, 0), H - 1), xc = min(max(xx, 0), W - 1);
    const uint4 v =
        *reinterpret_cast<const uint4*>(x + (((size_t)n * H + yc) * W + xc) * s.C + ci0 + 8 * c8);
    R.rx[i] = sel(ok, v);
  }
#pragma unroll
  for (int i = 0; i < CF::YR; ++i) {
    const int e = tid + NT * i, p = e >> 3, c8 = e & 7;
    const bool ok = p < nvalid;
    const int pc = min(p, nvalid - 1), py = pc / W, px = pc - py * W;
    const uint4 v = *reinterpret_cast<const uint4*>(
        dy + (((size_t)n * H + r0 + py) * W + px) * s.K + co0 + 8 * c8);
    R.ry[i] = sel(ok, v);
  }
}

template <int NPX>
__device__ __forceinline__ void w3_store(const W3Regs<NPX>& R, __bf16* Xs, __bf16* Ys, int hpx) {
  using CF = w3::Cfg<NPX>;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < CF::XR; ++i) {
    const int e = tid + NT * i, hp = e >> 3;
    if (hp < hpx) *reinterpret_cast<uint4*>(Xs + hp * w3::LD + 8 * (e & 7)) = R.rx[i];
  }
#pragma unroll
  for (int i = 0; i < CF::YR; ++i) {
    const int e = tid + NT * i;
    *reinterpret_cast<uint4*>(Ys + (e >> 3) * w3::LD + 8 * (e & 7)) = R.ry[i];
  }
}

template <int NPX>
__global__ __launch_bounds__(NT) void wgrad3_kernel(ConvShape s, const __bf16* __restrict__ x,
                                                    const __bf16* __restrict__ dy,
                                                    float* __restrict__ out, int cps) {
  using CF = w3::Cfg<NPX>;
  using w3::LD;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * CF::STG];
  const int C = s.C, K = s.K, H = s.H, W = s.W;
  const int TR = w3::rows_per_chunk(s, NPX), HW2 = W + 2, hpx = (TR + 2) * HW2;
  const int cpairs = C / 64, pairs = cpairs * (K / 64);
  const int pair = blockIdx.x % pairs, z = blockIdx.x / pairs;
  const int ci0 = (pair % cpairs) * 64, co0 = (pair / cpairs) * 64;
  const int rpi = (H + TR - 1) / TR, nchunks = s.N * rpi;
  const int c_begin = z * cps, c_end = min(nchunks, c_begin + cps);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;

  // per-lane transposed-read offsets (chunk invariant): lane 4q + p of its
  // 16-lane group G supplies pixel row q of the 4-pixel block, channels
  // 4p .. 4p + 3 of the group's 16; 8 pixels per lane = 2 reads per k-step
  const int G = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int csub = 16 * (G & 1) + 4 * p4, kb = 8 * (G >> 1);
  int aoff[CF::KS][2], boff[CF::KS][2];
#pragma unroll
  for (int ks = 0; ks < CF::KS; ++ks)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pix = 16 * ks + kb + 4 * r + q;
      const int pa = min(pix, TR * W - 1), pr = pa / W, pc = pa - pr * W;  // padded pixels: dY = 0
      aoff[ks][r] = (pr * HW2 + pc) * LD + wm * 32 + csub;
      boff[ks][r] = pix * LD + wn * 32 + csub;
    }
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) toff[t] = ((t / 3) * HW2 + (t % 3)) * LD;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = zero16();
  if (c_begin < c_end) {
    W3Regs<NPX> R;
    w3_load<NPX>(R, s, x, dy, c_begin, rpi, TR, HW2, hpx, ci0, co0);
    w3_store<NPX>(R, smem, smem + CF::MAXH * LD, hpx);
    __syncthreads();
    for (int ch = c_begin; ch < c_end; ++ch) {
      const int stage = (ch - c_begin) & 1;
      const bool more = ch + 1 < c_end;
      if (more) w3_load<NPX>(R, s, x, dy, ch + 1, rpi, TR, HW2, hpx, ci0, co0);
      // the next chunk's global loads are issued here, ahead of this chunk's
      // MFMAs (the scheduler would otherwise sink them to their LDS stores)
      __builtin_amdgcn_sched_barrier(0);
      const __bf16* Xs = smem + stage * CF::STG;
      {
      const __bf16* Ys = Xs + CF::MAXH * LD;
      // fragments of k-step ks + 1 are read while the 9 MFMAs of ks run (one
      // wave per SIMD: nothing else hides the LDS latency)
      bfx8 fb[2], fa[2][9];
      fb[0] = w3::frag(Ys + boff[0][0], Ys + boff[0][1]);
#pragma unroll
      for (int t = 0; t < 9; ++t)
        fa[0][t] = w3::frag(Xs + aoff[0][0] + toff[t], Xs + aoff[0][1] + toff[t]);
#pragma unroll
      for (int ks = 0; ks < CF::KS; ++ks) {
        const int cur = ks & 1, nx = cur ^ 1;
        if (ks + 1 < CF::KS) {
          fb[nx] = w3::frag(Ys + boff[ks + 1][0], Ys + boff[ks + 1][1]);
#pragma unroll
          for (int t = 0; t < 9; ++t)
            fa[nx][t] = w3::frag(Xs + aoff[ks + 1][0] + toff[t], Xs + aoff[ks + 1][1] + toff[t]);
        }
        // keep the next k-step's 20 reads ahead of this k-step's MFMAs (the
        // scheduler otherwise sinks each read next to its MFMA and every
        // MFMA then waits out a full LDS latency)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 9; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][t], fb[cur], acc[t], 0, 0, 0);
      }
      }
      if (more) {
        __bf16* nx = smem + (stage ^ 1) * CF::STG;
        w3_store<NPX>(R, nx, nx + CF::MAXH * LD, hpx);
      }
      __syncthreads();
    }
  }
  // slab store, one tap at a time through LDS so every lane writes 16-byte
  // vectors (4 consecutive co): [64 ci][64 co] fp32 tile per tap, row pitch 68
  float* o = out + (size_t)z * 9 * C * K;
  float* tile = reinterpret_cast<float*>(smem);
  const int col = wn * 32 + (lane & 31);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    __syncthreads();
#pragma unroll
    for (int qq = 0; qq < 16; ++qq) tile[(wm * 32 + mfma32_row(qq, lane)) * 68 + col] = acc[t][qq];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // 64 rows x 16 float4 = 1024 vectors, 4 per thread
      const int e = tid + NT * k, row = e >> 4, c4 = (e & 15) * 4;
      const float4 v = *reinterpret_cast<const float4*>(tile + row * 68 + c4);
      *reinterpret_cast<float4*>(o + ((size_t)t * C + ci0 + row) * K + co0 + c4) = v;
    }
  }
}

static bool wgrad3_ok(const ConvShape& s) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.OH == s.H && s.OW == s.W))
    return false;
  const int npx = w3::chunk_pixels(s);
  if (s.C % 64 || s.K % 64 || s.W > npx) return false;
  const int tr = w3::rows_per_chunk(s, npx);
  return (tr + 2) * (s.W + 2) <= (npx == 128 ? w3::Cfg<128>::MAXH : w3::Cfg<64>::MAXH);
}

static int wgrad3_chunks(const ConvShape& s) {
  const int tr = w3::rows_per_chunk(s, w3::chunk_pixels(s));
  return s.N * ((s.H + tr - 1) / tr);
}

// pixel splits: slabs of ~38 MB in total, >= 1 chunk per split.  Measured at
// B = 32 (scripts/wgrad3_lab.py): the slab writes + their reduction cost ~15 us
// per call at 19 MB, but halving the splits to that leaves the per-block
// chunk chains (load -> 9 x 4 MFMAs -> barrier) too long: 607 vs 489 us per
// step for the 13 layers; 76 MB: 681 us.
static int wgrad3_splits(const ConvShape& s) {
  const int nchunks = wgrad3_chunks(s);
  const long long budget = 9437184LL;
  long long z = (budget + 9LL * s.C * s.K - 1) / (9LL * s.C * s.K);
  z = std::max(1LL, std::min(z, (long long)nchunks));
  const int cps = (int)((nchunks + z - 1) / z);
  return (nchunks + cps - 1) / cps;
}

static void wgrad3(const ConvShape& s, const __bf16* xb, const __bf16* dyb, float* ws, float* dw,
                   hipStream_t st) {
  const int nchunks = wgrad3_chunks(s);
  const int z = wgrad3_splits(s);
  const int cps = (nchunks + z - 1) / z;
  const int blocks = (s.C / 64) * (s.K / 64) * z;
  if (z > 1 && !ws) throw std::runtime_error("wgrad3: split-K needs a workspace");
  float* out = z > 1 ? ws : dw;
  if (w3::chunk_pixels(s) == 128)
    wgrad3_kernel<128><<<blocks, NT, 0, st>>>(s, xb, dyb, out, cps);
  else
    wgrad3_kernel<64><<<blocks, NT, 0, st>>>(s, xb, dyb, out, cps);
  if (z > 1) slab_reduce(ws, z, 9LL * s.C * s.K / 4, dw, st);
}

}  // namespace cbf

bool conv_fwd_bf16_ok(const ConvShape& s) { return s.C % 64 == 0 && s.K % 64 == 0; }
bool conv_bwd_filter_bf16_ok(const ConvShape& s) { return s.C % 64 == 0 && s.K % 64 == 0; }
// 1x1, stride 2, no padding, even input: dX = dY W^T on the even pixels, zero elsewhere
static bool dgrad_1x1s2(const ConvShape& s) {
  return s.R == 1 && s.S == 1 && s.stride == 2 && s.pad == 0 && s.H == 2 * s.OH &&
         s.W == 2 * s.OW;
}
bool conv_bwd_data_bf16_ok(const ConvShape& s) {
  if (s.C % 64 != 0 || s.K % 64 != 0) return false;
  return dgrad_1x1s2(s) || cbf::dgrad3s2_ok(s) ||
         (s.stride == 1 && s.R == s.S && s.pad <= s.R - 1 &&
          s.OH == s.H + 2 * s.pad - s.R + 1 && s.OW == s.W + 2 * s.pad - s.S + 1);
}

long long conv_bf16_ws_floats(const ConvShape& s, bool fwd_epilogue) {
  using namespace cbf;
  long long n = 0;
  auto slab_floats = [](const ConvShape& c, bool epi) {
    const Plan p = plan(c, epi);
    const long long mk = (long long)c.N * c.OH * c.OW * c.K;
    long long f = p.z > 1 ? p.z * mk : 0LL;
    if (conv3_ok(c)) {
      const P3 q = plan3(c);
      if (q.z > 1) f = std::max(f, q.z * mk);
    }
    return f;
  };
  if (conv_fwd_bf16_ok(s)) n = std::max(n, wt_floats(s) + slab_floats(s, fwd_epilogue));
  if (conv_bwd_data_bf16_ok(s)) {
    const ConvShape d = dgrad_shape(s);
    n = std::max(n, wt_floats(d) + slab_floats(d, false));
    if (dgrad3s2_ok(s)) {
      const P3 q = plan3s2(s);
      if (q.z > 1) n = std::max(n, wt_floats(s) + (long long)q.z * s.N * s.H * s.W * s.C);
    }
  }
  if (conv_bwd_filter_bf16_ok(s)) {
    const WgPlan p = wg_plan(s);
    if (p.z > 1) n = std::max(n, (long long)p.z * s.R * s.S * s.C * s.K);
  }
  if (wgrad3_ok(s)) n = std::max(n, (long long)wgrad3_splits(s) * 9 * s.C * s.K);
  return n;
}

// bf16 im2col for thin-input convs (the 3-channel ResNet stem).  Per-tap row
// segments: for tap row kh the S*C inputs X[n, oy s - p + kh, ox s - p + kw,
// ci] (kw, ci) are contiguous in NHWC, so col[m][kh * seg + j] = that run
// (j < S C, zero-padded to seg = roundup(S C, 8)), zero from R seg up to kp
// (% 64).  The conv then runs as a 1x1 conv over kp channels on the kernels
// above (forward and filter gradient) with the weights laid out to match
// (ops/functional.py _ConvIm2colFn).  Thread = 8 consecutive k (one 16-byte
// store, consecutive threads -> consecutive stores); 32-bit index math with
// one divide per coordinate instead of the per-element (kh, kw, ci) divides.
__global__ __launch_bounds__(256) void im2col_bf16_kernel(ConvShape s, const float* __restrict__ x,
                                                          int kp, int seg, uint4* __restrict__ col) {
  const int kq = kp / 8, sq = seg / 8, sc = s.S * s.C;
  const long long nx = (long long)s.N * s.H * s.W * s.C;
  const int total = s.N * s.OH * s.OW * kq;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int m = i / kq, c = i - m * kq;
    const int kh = c / sq, j0 = (c - kh * sq) * 8;
    const int ox = m % s.OW, t = m / s.OW;
    const int oy = t % s.OH, n = t / s.OH;
    const int iy = oy * s.stride - s.pad + kh, ix0 = ox * s.stride - s.pad;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (kh < s.R && iy >= 0 && iy < s.H) {
      const int jlo = max(0, -ix0) * s.C, jhi = min(sc, (s.W - ix0) * s.C);
      const long long rowbase = ((long long)(n * s.H + iy) * s.W + ix0) * s.C;
      const long long e0 = rowbase + j0;
      if (e0 >= 0 && e0 + 8 <= nx) {
        // two 16-byte loads at 4-byte alignment (full speed on gfx950), then
        // the run is masked to the in-image part [jlo, jhi) of the segment
        const float4 a = *reinterpret_cast<const float4*>(x + e0);
        const float4 b = *reinterpret_cast<const float4*>(x + e0 + 4);
        const float r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (j0 + j >= jlo && j0 + j < jhi) ? r[j] : 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j0 + j >= jlo && j0 + j < jhi) v[j] = x[rowbase + j0 + j];
      }
    }
    col[i] = cbf::pack8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  }
}

void im2col_bf16(const ConvShape& s, const float* x, int kp, void* col, hipStream_t st) {
  const int seg = (s.S * s.C + 7) / 8 * 8;
  if (kp % 64 != 0 || kp < s.R * seg) throw std::runtime_error("im2col_bf16: bad kp");
  const long long total = (long long)s.N * s.OH * s.OW * kp / 8;
  if (total >= (1LL << 31) || (long long)s.N * s.H * s.W * s.C >= (1LL << 31))
    throw std::runtime_error("im2col_bf16: tensor too large for 32-bit indexing");
  long long b = (total + 255) / 256;
  if (b > 16384) b = 16384;
  im2col_bf16_kernel<<<(int)b, 256, 0, st>>>(s, x, kp, seg, reinterpret_cast<uint4*>(col));
}

void to_bf16(const float* x, void* y, long long n, hipStream_t st) {
  if (n % 8 != 0) throw std::runtime_error("to_bf16: n % 8 != 0");
  long long b = (n / 8 + 255) / 256;
  if (b > 8192) b = 8192;
  cbf::to_bf16_kernel<<<(int)(b < 1 ? 1 : b), 256, 0, st>>>(
      reinterpret_cast<const float4*>(x), reinterpret_cast<uint4*>(y), n / 8);
}

long long wcvt_blocks(int taps, int C, int K) {
  if (C % 32 || K % 32) throw std::runtime_error("wcvt_blocks: C, K must be multiples of 32");
  return (long long)taps * (C / 32) * (K / 32);
}

void wcvt_batch(const long long* jobs, int njobs, long long nblocks, hipStream_t st) {
  if (njobs <= 0 || nblocks <= 0 || nblocks >= (1LL << 31))
    throw std::runtime_error("wcvt_batch: bad job table");
  cbf::wcvt_batch_kernel<<<(int)nblocks, 256, 0, st>>>(jobs, njobs);
}

void sgd_wcvt(float* w, const float* g, float* mom, float momentum, float gscale, float l2,
              const float* lr, long long* step, const long long* jobs, int njobs,
              long long conv_blocks, const long long* ranges, int nranges, long long range_blocks,
              hipStream_t st) {
  if (njobs < 0 || nranges < 0 || conv_blocks < 0 || range_blocks < 0 ||
      conv_blocks + range_blocks <= 0 || conv_blocks + range_blocks >= (1LL << 31) ||
      (njobs == 0) != (conv_blocks == 0) || (nranges == 0) != (range_blocks == 0))
    throw std::runtime_error("sgd_wcvt: bad job / range table");
  const cbf::SgdWcvtArgs a{w, g, mom, momentum, gscale, l2, lr, step, jobs, njobs,
                           (int)conv_blocks, ranges, nranges};
  cbf::sgd_wcvt_kernel<<<(int)(conv_blocks + range_blocks), 256, 0, st>>>(a);
}

int conv_fwd_stats_rows(const ConvShape& s, bool bf16) {
  using namespace cbf;
  if (!bf16) {
    if (!conv_fwd_tiled_ok(s) && !conv_fwd_tiled_gather_ok(s))
      throw std::runtime_error("conv_fwd_stats_rows: not a tiled-family conv");
    return conv_fwd_tiled_stats_rows(s, false);
  }
  if (!conv_fwd_bf16_ok(s)) throw std::runtime_error("conv_fwd_stats_rows: not a bf16-family conv");
  return conv3_ok(s) ? stats_rows3(s) : stats_rows(s, false);
}

int conv_fwd_stem_stats_rows(const ConvShape& s1) {
  using namespace cbf;
  return cdiv((long long)s1.N * s1.OH * s1.OW, 128) * 2;
}

void conv_fwd_bf16(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
                   bool relu, float* ws, hipStream_t st, const void* xb, const void* wtb,
                   void* yb, const ConvStats* stats) {
  using namespace cbf;
  if (!conv_fwd_bf16_ok(s) || !ws) throw std::runtime_error("conv_fwd_bf16: unsupported shape");
  const __bf16* wt = reinterpret_cast<const __bf16*>(wtb);
  if (!wt) {
    __bf16* wc = reinterpret_cast<__bf16*>(ws);
    convert(s, w, 0, wc, st);
    wt = wc;
  }
  __bf16* ob = reinterpret_cast<__bf16*>(yb);
  // statistics rows are planned for the halo kernel whenever it takes the shape
  if (stats && stats->part && conv3_ok(s) && !(xb && !bias && !relu))
    throw std::runtime_error("conv_fwd_bf16: statistics need the bf16 input of a plain halo conv");
  if (xb && !bias && !relu && conv3_ok(s))
    launch3(s, reinterpret_cast<const __bf16*>(xb), wt, y, ws, st, nullptr, ob, stats);
  else if (xb)
    launch(s, reinterpret_cast<const __bf16*>(xb), wt, bias, y, relu, ws, st, nullptr, ob, 0, stats);
  else
    launch(s, x, wt, bias, y, relu, ws, st, nullptr, ob, 0, stats);
}

// BatchNorm backward statistics rows of the dgrad of s (0: not available -
// the dgrad kinds without the epilogue, or a channel count the slab pass
// cannot keep one quad per thread of)
int conv_bwd_data_stats_rows(const ConvShape& s) {
  using namespace cbf;
  if (!conv_bwd_data_bf16_ok(s) || s.C % 64 != 0 || 256 % (s.C / 4) != 0) return 0;
  if (dgrad3s2_ok(s)) return stats_rows3s2(s);
  if (dgrad_1x1s2(s)) return 0;
  if (conv3_ok(dgrad_shape(s))) return stats_rows3(dgrad_shape(s));
  return 0;
}

void conv_bwd_data_bf16(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                        hipStream_t st, const void* dyb, const float* addend, const void* wtb,
                        const BnBwdStats* bstats) {
  using namespace cbf;
  if (!conv_bwd_data_bf16_ok(s) || !ws) throw std::runtime_error("conv_bwd_data_bf16: unsupported shape");
  if (bstats && bstats->part &&
      (!dyb || bstats->P != conv_bwd_data_stats_rows(s) || bstats->P == 0 || !bstats->x ||
       !bstats->mean || !bstats->rstd || (bstats->relu && !bstats->y)))
    throw std::runtime_error("conv_bwd_data_bf16: BatchNorm backward statistics not available here");
  BnBwdStats bsv;
  if (bstats && bstats->part) {  // the kernels load y unconditionally: y = x without a ReLU
    bsv = *bstats;
    if (!bsv.relu) bsv.y = bsv.x;
    bstats = &bsv;
  }
  const __bf16* wt = reinterpret_cast<const __bf16*>(wtb);
  if (!wt) {
    __bf16* wc = reinterpret_cast<__bf16*>(ws);
    convert(s, w, 1, wc, st);
    wt = wc;
  }
  if (dgrad3s2_ok(s)) {
    if (dyb)
      return launch3s2(s, reinterpret_cast<const __bf16*>(dyb), wt, dx, ws, st, addend, bstats);
    return conv_bwd_data_tiled(s, dy, w, dx, ws, st, true, addend);  // fp32 dY only
  }
  if (dgrad_1x1s2(s)) {  // a 1x1 GEMM over the dY pixels, 2x2-expanding epilogue
    ConvShape d = dgrad_shape(s);
    d.H = d.OH = s.OH;
    d.W = d.OW = s.OW;
    if (dyb)
      launch(d, reinterpret_cast<const __bf16*>(dyb), wt, nullptr, dx, false, ws, st, addend,
             nullptr, 1);
    else
      launch(d, dy, wt, nullptr, dx, false, ws, st, addend, nullptr, 1);
    return;
  }
  if (dyb && conv3_ok(dgrad_shape(s)))
    launch3(dgrad_shape(s), reinterpret_cast<const __bf16*>(dyb), wt, dx, ws, st, addend, nullptr,
            nullptr, bstats);
  else if (dyb)
    launch(dgrad_shape(s), reinterpret_cast<const __bf16*>(dyb), wt, nullptr, dx, false, ws, st,
           addend);
  else
    launch(dgrad_shape(s), dy, wt, nullptr, dx, false, ws, st, addend);
}

void conv_bwd_filter_bf16(const ConvShape& s, const float* x, const float* dy, float* ws,
                          float* dw, hipStream_t st, const void* xb, const void* dyb) {
  using namespace cbf;
  if (!conv_bwd_filter_bf16_ok(s)) throw std::runtime_error("conv_bwd_filter_bf16: unsupported shape");
  if (xb && dyb && wgrad3_ok(s))
    return wgrad3(s, reinterpret_cast<const __bf16*>(xb), reinterpret_cast<const __bf16*>(dyb), ws,
                  dw, st);
  const WgPlan p = wg_plan(s);
  if (p.z > 1 && !ws) throw std::runtime_error("conv_bwd_filter_bf16: split-K needs a workspace");
  float* out = p.z > 1 ? ws : dw;
  const int blocks = cdiv((long long)s.R * s.S * s.C, p.bm) * (s.K / p.bn) * p.z;
  if (xb && dyb) {
    const __bf16* xh = reinterpret_cast<const __bf16*>(xb);
    const __bf16* dh = reinterpret_cast<const __bf16*>(dyb);
    if (p.bm == 128 && p.bn == 128)
      wgrad_kernel<128, 128, true><<<blocks, NT, 0, st>>>(s, xh, dh, out, p.kchunk, s);
    else if (p.bm == 128)
      wgrad_kernel<128, 64, true><<<blocks, NT, 0, st>>>(s, xh, dh, out, p.kchunk, s);
    else if (p.bn == 128)
      wgrad_kernel<64, 128, true><<<blocks, NT, 0, st>>>(s, xh, dh, out, p.kchunk, s);
    else
      wgrad_kernel<64, 64, true><<<blocks, NT, 0, st>>>(s, xh, dh, out, p.kchunk, s);
  } else {
    if (p.bm == 128 && p.bn == 128)
      wgrad_kernel<128, 128, false><<<blocks, NT, 0, st>>>(s, x, dy, out, p.kchunk, s);
    else if (p.bm == 128)
      wgrad_kernel<128, 64, false><<<blocks, NT, 0, st>>>(s, x, dy, out, p.kchunk, s);
    else if (p.bn == 128)
      wgrad_kernel<64, 128, false><<<blocks, NT, 0, st>>>(s, x, dy, out, p.kchunk, s);
    else
      wgrad_kernel<64, 64, false><<<blocks, NT, 0, st>>>(s, x, dy, out, p.kchunk, s);
  }
  if (p.z > 1) slab_reduce(ws, p.z, (long long)s.R * s.S * s.C * s.K / 4, dw, st);
}

// ---- stem over the implicit im2col (StemLoader / StemWgLoader) ----------
// s1: the 1x1 GEMM shape over kp channels (kp % 64 == 0, >= R * seg), si the
// image conv (C * S <= seg, fp32 NHWC image x)
static void stem_check(const ConvShape& s1, const ConvShape& si) {
  const int seg = (si.S * si.C + 7) / 8 * 8;
  if (s1.C % 64 || s1.C < si.R * seg || s1.K % 64 || s1.R != 1 || s1.S != 1 ||
      s1.N != si.N || s1.OH != si.OH || s1.OW != si.OW ||
      (long long)si.N * si.H * si.W * si.C >= (1LL << 31) ||
      (long long)s1.N * s1.OH * s1.OW >= (1LL << 31))
    throw std::runtime_error("stem conv: inconsistent shapes");
}

void conv_fwd_stem_bf16(const ConvShape& s1, const ConvShape& si, const float* x, const void* wtb,
                        void* yb, hipStream_t st, const ConvStats* stats) {
  using namespace cbf;
  stem_check(s1, si);
  const long long M = (long long)s1.N * s1.OH * s1.OW;
  ConvStats cs;
  if (stats && stats->part) {
    if (stats->P != conv_fwd_stem_stats_rows(s1))
      throw std::runtime_error("stem conv: BatchNorm statistics layout mismatch");
    cs = *stats;
  }
  // 128 x 64 tiles: M = 401 K pixels at B = 32 (3136 blocks), no split.
  // (An A operand built from an LDS halo of the block's image rows, staged
  // once as bf16, measured 105 vs 90 us: the halo's 16 KB of LDS halved the
  // blocks per CU and the chunk builds cost more than the L2 gathers saved.)
  const dim3 grid(cdiv(M, 128) * (s1.K / 64), 1);
  fwd_kernel<128, 64, float, StemLoader<128, 64>><<<grid, NT, 0, st>>>(
      s1, x, reinterpret_cast<const __bf16*>(wtb), nullptr, nullptr, 0, s1.C / BK, nullptr,
      reinterpret_cast<__bf16*>(yb), 0, si, cs);
}

void conv_bwd_filter_stem_bf16(const ConvShape& s1, const ConvShape& si, const float* x,
                               const void* dyb, float* ws, float* dw, hipStream_t st) {
  using namespace cbf;
  stem_check(s1, si);
  const WgPlan p = wg_plan(s1);
  if (p.z > 1 && !ws) throw std::runtime_error("stem wgrad: split-K needs a workspace");
  float* out = p.z > 1 ? ws : dw;
  const int blocks = cdiv((long long)s1.C, p.bm) * (s1.K / p.bn) * p.z;
  const __bf16* d = reinterpret_cast<const __bf16*>(dyb);
#define STEM_WG(BM_, BN_)                                                                 \
  wgrad_kernel<BM_, BN_, true, StemWgLoader<BM_, BN_>><<<blocks, NT, 0, st>>>(s1, x, d, out, \
                                                                             p.kchunk, si)
  if (p.bm == 128 && p.bn == 128)
    STEM_WG(128, 128);
  else if (p.bm == 128)
    STEM_WG(128, 64);
  else if (p.bn == 128)
    STEM_WG(64, 128);
  else
    STEM_WG(64, 64);
#undef STEM_WG
  if (p.z > 1) slab_reduce(ws, p.z, (long long)s1.C * s1.K / 4, dw, st);
}

// ---- space-to-depth stem (S2dLoader) -----------------------------------
// si: the 4x4 stride-1 conv over the s2d image (N, OH + 3, OW + 3, 16 -> K);
// s1 its 1x1 GEMM view (N, OH, OW, 256 -> K)
static ConvShape s2d_gemm_shape(const ConvShape& si) {
  ConvShape s1{};
  s1.N = si.N;
  s1.H = s1.OH = si.OH;
  s1.W = s1.OW = si.OW;
  s1.C = 256;
  s1.K = si.K;
  s1.R = s1.S = s1.stride = 1;
  s1.pad = 0;
  return s1;
}
static void s2d_check(const ConvShape& si) {
  if (si.C != 16 || si.R != 4 || si.S != 4 || si.stride != 1 || si.pad != 0 || si.K % 64 ||
      si.OH != si.H - 3 || si.OW != si.W - 3 || (long long)si.N * si.H * si.W * 16 >= (1LL << 31))
    throw std::runtime_error("s2d stem conv: inconsistent shapes");
}

static bool g_s2d_preload = true;  // A/B: S2dLoaderPre (all K tiles at once) vs S2dLoader

void conv_fwd_s2d_stem_bf16(const ConvShape& si, const void* xs, const void* wt8, void* yb,
                            hipStream_t st, const ConvStats* stats) {
  using namespace cbf;
  s2d_check(si);
  const ConvShape s1 = s2d_gemm_shape(si);
  ConvStats cs;
  if (stats && stats->part) {
    if (stats->P != conv_fwd_stem_stats_rows(s1))
      throw std::runtime_error("s2d stem conv: BatchNorm statistics layout mismatch");
    cs = *stats;
  }
  const long long M = (long long)s1.N * s1.OH * s1.OW;
  const dim3 grid(cdiv(M, 128) * (s1.K / 64), 1);
  if (s1.C / BK != S2dLoaderPre<128, 64>::NKT) throw std::runtime_error("s2d stem conv: K tiles");
  if (g_s2d_preload)
    fwd_kernel<128, 64, __bf16, S2dLoaderPre<128, 64>><<<grid, NT, 0, st>>>(
        s1, reinterpret_cast<const __bf16*>(xs), reinterpret_cast<const __bf16*>(wt8), nullptr,
        nullptr, 0, s1.C / BK, nullptr, reinterpret_cast<__bf16*>(yb), 0, si, cs);
  else
    fwd_kernel<128, 64, __bf16, S2dLoader<128, 64>><<<grid, NT, 0, st>>>(
        s1, reinterpret_cast<const __bf16*>(xs), reinterpret_cast<const __bf16*>(wt8), nullptr,
        nullptr, 0, s1.C / BK, nullptr, reinterpret_cast<__bf16*>(yb), 0, si, cs);
}
void s2d_stem_set_preload(bool on) { g_s2d_preload = on; }

// the 4x4 conv's filter gradient over the s2d image: the generic bf16 wgrad
// (rows m = tap * 16 + channel; a channel quad never straddles taps), split-K
// slabs summed into dw8 [256][K]
void conv_bwd_filter_s2d_stem_bf16(const ConvShape& si, const void* xs, const void* dyb,
                                   float* ws, float* dw8, hipStream_t st) {
  using namespace cbf;
  s2d_check(si);
  const WgPlan p = wg_plan(si);
  if (p.z > 1 && !ws) throw std::runtime_error("s2d stem wgrad: split-K needs a workspace");
  float* out = p.z > 1 ? ws : dw8;
  const int blocks = cdiv(256, p.bm) * (si.K / p.bn) * p.z;
  const __bf16* xh = reinterpret_cast<const __bf16*>(xs);
  const __bf16* dh = reinterpret_cast<const __bf16*>(dyb);
  if (p.bm == 128) {
    if (p.bn == 128)
      wgrad_kernel<128, 128, true><<<blocks, NT, 0, st>>>(si, xh, dh, out, p.kchunk, si);
    else
      wgrad_kernel<128, 64, true><<<blocks, NT, 0, st>>>(si, xh, dh, out, p.kchunk, si);
  } else if (p.bn == 128) {
    wgrad_kernel<64, 128, true><<<blocks, NT, 0, st>>>(si, xh, dh, out, p.kchunk, si);
  } else {
    wgrad_kernel<64, 64, true><<<blocks, NT, 0, st>>>(si, xh, dh, out, p.kchunk, si);
  }
  if (p.z > 1) slab_reduce(ws, p.z, 256LL * si.K / 4, dw8, st);
}

size_t s2d_stem_ws_floats(const ConvShape& si) {
  using namespace cbf;
  s2d_check(si);
  const WgPlan p = wg_plan(si);
  return p.z > 1 ? (size_t)p.z * 256 * si.K : 0;
}

}  // namespace gops
