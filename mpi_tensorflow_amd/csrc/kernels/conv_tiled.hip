// LDS-tiled implicit-GEMM convolutions (NHWC activations, HWIO weights, fp32
// storage; fp32 MFMA v_mfma_f32_32x32x2_f32 or, with bf16 = true, operands
// converted to bf16 while staged into LDS and v_mfma_f32_32x32x16_bf16) for the channel counts of
// ResNet-18 and wide layers in general: forward, backward-data (stride-s
// phase decomposition) and backward-filter (split-K slabs).
//
// Why a second conv family next to ops_generic.hip's gather engine: that
// engine decodes (tap, channel) per element per K step (div/mod in the inner
// loop) and stages one float per lane.  Here a K tile is ONE tap x BK
// consecutive channels, so each operand row of a tile is BK contiguous
// floats in memory: the per-row pixel decode and bounds test happen once per
// tap, global loads are float4 along the channel axis, and the LDS image is
// k-major ([BK][BM + pad]) so the 32 lanes of a half-wave read 32 consecutive
// rows of one k for the fp32 MFMA operand (A[i][k] on lane i, B[k][j] on
// lane j).  Block = 256 threads = 2x2 waves, each wave (BM/2)x(BN/2) =
// TMxTN 32x32 MFMA tiles; double-buffered LDS, one barrier per K tile, the
// next tile's global loads in flight during the current tile's MFMAs;
// XCD-aware block order.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "ops_generic.h"

namespace gops {
namespace tiled {

constexpr int BK = 32, NT = 256;

// Operand precision of the MFMA.  fp32 storage everywhere; BF16 converts the
// tiles to bf16 as they are staged into LDS and runs v_mfma_f32_32x32x16_bf16
// (16x the fp32-MFMA rate) with fp32 accumulation.
enum Prec { F32 = 0, BF16 = 1 };
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));

// LDS image of one K tile of an operand with ROWS rows (M or N):
//   F32 : k-major [BK][ROWS] floats - the 32 lanes of a half-wave read 32
//         consecutive rows of one k (the fp32 MFMA takes one k per lane).
//         Unpadded, rows XOR-swizzled by 32 (k & 1) + 8 ((k >> 2) & 3): the
//         two half-waves of a fragment read (k, k + 1) land in opposite bank
//         halves (one pass of the 64-bank array) and a loader store of k = c,
//         c + 4, ..., c + 28 x 8 rows spreads over 32 banks.  ResNet-18 fp32
//         step, same box: 6.39 ms vs 6.44 with a pad of 4 floats (fwd 0.44-0.62
//         vs 1.45-2.2 conflict cycles per LDS instruction, data 1.0 vs 4.0;
//         profiles/r4_resnet18_fp32_pmc.txt).  A swizzle that also spreads the
//         stores over all 64 banks (by (k ^ k >> 2) & 1, (k >> 3) & 3) cost
//         more VALU than it saved (6.65 ms); a pad of 32 made the reads
//         conflict-free but cost a block per CU (6.92 ms)
//   BF16: row-major [ROWS][BK + 8] bf16 - each lane reads one 16-byte
//         fragment (8 consecutive k of its row); the 80-byte row stride makes
//         the ds_read_b128 lane groups conflict-free
// put_k4 stores 4 consecutive k of one row, put_r4 4 consecutive rows of one k.
// KB: k per tile (BK everywhere but the fp32 16-deep filter-gradient variant)
template <int P, int ROWS, int KB = BK>
struct Stage;

template <int ROWS, int KB>
struct Stage<F32, ROWS, KB> {
  static_assert(ROWS % 64 == 0, "F32 stage rows: multiples of 64 (swizzle within 64-row groups)");
  static constexpr int LD = ROWS;
  static constexpr int FLOATS = KB * LD;
  // element (k, row); the swizzle keeps 4-row groups contiguous (put_r4)
  static __device__ __forceinline__ int at(int k, int row) {
    return k * LD + (row ^ ((k & 1) << 5) ^ (((k >> 2) & 3) << 3));
  }
  static __device__ __forceinline__ void put_k4(float* T, int row, int k0, float4 v) {
    T[at(k0 + 0, row)] = v.x;
    T[at(k0 + 1, row)] = v.y;
    T[at(k0 + 2, row)] = v.z;
    T[at(k0 + 3, row)] = v.w;
  }
  static __device__ __forceinline__ void put_r4(float* T, int row0, int k, float4 v) {
    *reinterpret_cast<float4*>(T + at(k, row0)) = v;
  }
};

template <int ROWS, int KB>
struct Stage<BF16, ROWS, KB> {
  static constexpr int LDK = KB + 8;  // bf16 elements per row
  static constexpr int FLOATS = ROWS * LDK / 2;
  static __device__ __forceinline__ void put_k4(float* T, int row, int k0, float4 v) {
    const __bf16 h[4] = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(T) + row * LDK + k0) =
        __builtin_bit_cast(uint2, h);
  }
  static __device__ __forceinline__ void put_r4(float* T, int row0, int k, float4 v) {
    __bf16* b = reinterpret_cast<__bf16*>(T) + row0 * LDK + k;
    b[0] = (__bf16)v.x;
    b[LDK] = (__bf16)v.y;
    b[2 * LDK] = (__bf16)v.z;
    b[3 * LDK] = (__bf16)v.w;
  }
};

template <int BM, int BN, int P = F32, int KB = BK>
struct Geo {
  static constexpr int TM = BM / 64, TN = BN / 64;  // MFMA tiles per wave
  static constexpr int A_FLOATS = Stage<P, BM, KB>::FLOATS;
  static constexpr int STAGE = A_FLOATS + Stage<P, BN, KB>::FLOATS;
  static constexpr int SMEM = 2 * STAGE;
};

// The MFMAs of one staged K tile for the wave's TMxTN 32x32 sub-tiles.
template <int BM, int BN, int P, int KB = BK>
__device__ __forceinline__ void mma_tile(const float* As, const float* Bs, int wm, int wn,
                                         int lane, f32x16 (&acc)[BM / 64][BN / 64]) {
  using G = Geo<BM, BN, P, KB>;
  const int r = lane & 31, h = lane >> 5;
  if constexpr (P == F32) {
    using SA = Stage<F32, BM, KB>;
    using SB = Stage<F32, BN, KB>;
#pragma unroll
    for (int ks = 0; ks < KB / 2; ++ks) {
      float a[G::TM], b[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) a[i] = As[SA::at(2 * ks + h, wm * (BM / 2) + 32 * i + r)];
#pragma unroll
      for (int j = 0; j < G::TN; ++j) b[j] = Bs[SB::at(2 * ks + h, wn * (BN / 2) + 32 * j + r)];
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j) acc[i][j] = mfma32x32x2(a[i], b[j], acc[i][j]);
    }
  } else {
    constexpr int LDK = Stage<BF16, BM, KB>::LDK;
    const __bf16* A = reinterpret_cast<const __bf16*>(As);
    const __bf16* B = reinterpret_cast<const __bf16*>(Bs);
#pragma unroll
    for (int ks = 0; ks < KB / 16; ++ks) {
      bfx8 a[G::TM], b[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
        a[i] = *reinterpret_cast<const bfx8*>(A + (wm * (BM / 2) + 32 * i + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
        b[j] = *reinterpret_cast<const bfx8*>(B + (wn * (BN / 2) + 32 * j + r) * LDK + 16 * ks + 8 * h);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
}

// Double-buffered main loop over K tiles [k0, k0 + nk).  L provides
//   load(kt)       : issue the global loads of K tile kt into its registers
//   store<P>(A, B) : write those registers into the LDS stage (Stage<P, .>)
template <int BM, int BN, int P, int KB = BK, class L>
__device__ __forceinline__ void mainloop(L& ld, float* smem, int k0, int nk,
                                         f32x16 (&acc)[BM / 64][BN / 64]) {
  using G = Geo<BM, BN, P, KB>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = zero16();
  if (nk <= 0) return;
  ld.load(k0);
  ld.template store<P>(smem, smem + G::A_FLOATS);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* cur = smem + (kt & 1) * G::STAGE;
    float* nxt = smem + ((kt + 1) & 1) * G::STAGE;
    const bool more = kt + 1 < nk;
    if (more) ld.load(k0 + kt + 1);
    mma_tile<BM, BN, P, KB>(cur, cur + G::A_FLOATS, wm, wn, lane, acc);
    if (more) ld.template store<P>(nxt, nxt + G::A_FLOATS);
    __syncthreads();
  }
}

__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
  return sel(ok, v);
}

// ------------------------------------------------------------- forward ----
// Y[m = (n, oy, ox)][co] = sum_{kh, kw, ci} X[n, oy s - p + kh, ox s - p + kw, ci] W[kh, kw, ci, co]
// K tile kt = (tap, 32-channel chunk).  Requires C % 32 == 0, K % 4 == 0.
template <int BM, int BN>
struct FwdLoader {
  static constexpr int AR = BM * BK / 4 / NT;  // float4 of A per thread
  static constexpr int BR = BN * BK / 4 / NT;  // float4 of B per thread
  ConvShape s;
  const float* x;
  const float* w;
  int n0, cchunks;
  // A rows of this thread: pixel base pointer and top-left input coords
  const float* abase[AR];
  int iy0[AR], ix0[AR];
  bool av[AR];
  float4 ra[AR], rb[BR];
  bool bv[BR];
  __device__ FwdLoader(const ConvShape& s_, const float* x_, const float* w_, int m0, int n0_)
      : s(s_), x(x_), w(w_), n0(n0_) {
    cchunks = s.C / BK;
    const int tid = threadIdx.x, c4 = tid & 7;
    const int M = s.N * s.OH * s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
      abase[i] = x + (size_t)n * s.H * s.W * s.C + 4 * c4;
      iy0[i] = oy * s.stride - s.pad;
      ix0[i] = ox * s.stride - s.pad;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + 4 * (tid % (BN / 4));
      bv[i] = n < s.K;
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
      ra[i] = sel4(ok, *reinterpret_cast<const float4*>(abase[i] + ((size_t)iyc * s.W + ixc) * s.C + ci0));
    }
    const int tid = threadIdx.x;
    const float* wb = w + (size_t)(tap * s.C + ci0) * s.K + min(n0 + 4 * (tid % (BN / 4)), s.K - 4);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      rb[i] = sel4(bv[i], *reinterpret_cast<const float4*>(wb + (size_t)k * s.K));
    }
  }
  template <int P>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x, c4 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i) Stage<P, BM>::put_k4(As, (tid >> 3) + 32 * i, 4 * c4, ra[i]);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      Stage<P, BN>::put_r4(Bs, 4 * (tid % (BN / 4)), k, rb[i]);
    }
  }
};

// Forward over the flattened (kh, kw, ci) reduction axis for channel counts
// that are not a multiple of 32 (the 3-channel ResNet stem: 147 = 7x7x3, five
// K tiles, the last zero-padded): each thread gathers 4 consecutive k of its
// rows as scalars (the (kh, kw, ci) decode once per K tile, the pixel decode
// once per thread); the weight rows are the HWIO rows kk, float4 along co.
// Requires K % 4 == 0.
template <int BM, int BN>
struct FwdGatherLoader {
  static constexpr int AR = BM * BK / 4 / NT;
  static constexpr int BR = BN * BK / 4 / NT;
  ConvShape s;
  const float* x;
  const float* w;
  int n0, ktot;
  const float* abase[AR];
  int iy0[AR], ix0[AR];
  bool av[AR];
  float4 ra[AR], rb[BR];
  bool bv[BR];
  __device__ FwdGatherLoader(const ConvShape& s_, const float* x_, const float* w_, int m0,
                             int n0_)
      : s(s_), x(x_), w(w_), n0(n0_) {
    ktot = s.R * s.S * s.C;
    const int tid = threadIdx.x;
    const int M = s.N * s.OH * s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      av[i] = m < M;
      const int mm = av[i] ? m : 0;
      const int ox = mm % s.OW, t = mm / s.OW, oy = t % s.OH, n = t / s.OH;
      abase[i] = x + (size_t)n * s.H * s.W * s.C;
      iy0[i] = oy * s.stride - s.pad;
      ix0[i] = ox * s.stride - s.pad;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) bv[i] = n0 + 4 * (tid % (BN / 4)) < s.K;
  }
  __device__ __forceinline__ void load(int kt) {
    const int tid = threadIdx.x, kb = kt * BK + 4 * (tid & 7);
    int dy[4], dx[4], ci[4];
    bool kv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // (kh, kw, ci) of this thread's 4 k
      const int kk = min(kb + u, ktot - 1);
      kv[u] = kb + u < ktot;
      const int tap = kk / s.C;
      ci[u] = kk - tap * s.C;
      dy[u] = tap / s.S;
      dx[u] = tap - dy[u] * s.S;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int iy = iy0[i] + dy[u], ix = ix0[i] + dx[u];
        const bool ok = av[i] && kv[u] && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
        // clamped pixel: the load is always in bounds, the value selected away
        const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
        const float e = abase[i][((size_t)iyc * s.W + ixc) * s.C + ci[u]];
        v[u] = ok ? e : 0.f;
      }
      ra[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
    const float* wb = w + min(n0 + 4 * (tid % (BN / 4)), s.K - 4);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = kt * BK + tid / (BN / 4) + (NT / (BN / 4)) * i;
      const float4 e = *reinterpret_cast<const float4*>(wb + (size_t)min(k, ktot - 1) * s.K);
      rb[i] = sel4(bv[i] && k < ktot, e);
    }
  }
  template <int P>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x, c4 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i) Stage<P, BM>::put_k4(As, (tid >> 3) + 32 * i, 4 * c4, ra[i]);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      Stage<P, BN>::put_r4(Bs, 4 * (tid % (BN / 4)), k, rb[i]);
    }
  }
};

// GATHER: FwdGatherLoader over the flattened reduction axis, else FwdLoader
// cs (unsplit launches): the consuming BatchNorm's statistics of the stored
// values, shifted by cs.shift, in the [2][K / 64][P][64] partial-row table of
// the bf16 family (row (m tile, wm) per wave, P = 2 x m tiles); the two
// half-waves combine their rows and lanes h == 0 store 32 contiguous floats
template <int BM, int BN, int P, bool GATHER = false>
__global__ __launch_bounds__(NT) void fwd_kernel(ConvShape s, const float* __restrict__ x,
                                                 const float* __restrict__ w,
                                                 const float* __restrict__ bias,
                                                 float* __restrict__ y, int relu, int kps,
                                                 const ConvStats cs,
                                                 const float* __restrict__ addend) {
  // split-K (gridDim.y > 1, no bias / ReLU): slice z of kps K tiles writes a
  // raw slab y + z * M * K, summed by slab_sum4 afterwards
  using G = Geo<BM, BN, P>;
  __shared__ float smem[G::SMEM];
  const int M = s.N * s.OH * s.OW;
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;
  const int nk = GATHER ? (s.R * s.S * s.C + BK - 1) / BK : s.R * s.S * (s.C / BK);
  const int kb = blockIdx.y * kps;
  using LD = typename std::conditional<GATHER, FwdGatherLoader<BM, BN>, FwdLoader<BM, BN>>::type;
  LD ld(s, x, w, m0, n0);
  f32x16 acc[G::TM][G::TN];
  mainloop<BM, BN, P>(ld, smem, kb, min(kps, nk - kb), acc);
  y += (size_t)blockIdx.y * M * s.K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave & 1, wn = wave >> 1;
  const bool st = cs.part != nullptr;
#pragma unroll
  for (int j = 0; j < G::TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + (lane & 31);
    const bool cok = co < s.K;
    const float b = (bias && cok) ? bias[co] : 0.f;
    const float kc = (st && cok) ? cs.shift[co] : 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(r, lane);
        if (m >= M || !cok) continue;
        float v = acc[i][j][r] + b;
        if (relu) v = fmaxf(v, 0.f);
        if (addend) v += addend[(size_t)m * s.K + co];  // gradient join (dgrad as forward)
        y[(size_t)m * s.K + co] = v;
        const float d = v - kc;
        s1 += d;
        s2 += d * d;
      }
    if (st) {  // both half-waves hold the same column
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if ((lane >> 5) == 0 && cok) {
        const size_t e = ((size_t)(co >> 6) * cs.P + (bid % mt) * 2 + wm) * 64 + (co & 63);
        cs.part[e] = s1;
        cs.part[(size_t)s.K * cs.P + e] = s2;
      }
    }
  }
}

// ------------------------------------------------------- backward-data ----
// dX[n, iy, ix, ci] = sum_{kh, kw, co} dY[n, oy, ox, co] W[kh, kw, ci, co] over
// oy = (iy + p - kh) / s when exact.  Phase decomposition: input pixels with
// (iy mod s, ix mod s) = (py, px) only receive taps kh = (py + p) mod s (mod s)
// and likewise kw, so each phase is a dense implicit GEMM over its own tap
// list (no zero MFMA work for stride 2).  Block z-dimension = phase.
// K tile = (phase tap, 32-channel chunk of co).  Requires K % 32 == 0, C % 4 == 0.
// DT: element type of dY in global memory (float, or __bf16 when the
// gradient arrives as the bf16 output of a bf16-input BatchNorm backward)
template <int BM, int BN, class DT = float>
struct DataLoader {
  static constexpr int AR = BM * BK / 4 / NT;
  static constexpr int BR = BN * BK / 4 / NT;
  ConvShape s;
  const DT* dy;
  const float* w;
  int n0, cchunks, nkw, kh0, kw0;
  const DT* abase[AR];
  int qy[AR], qx[AR];  // iy + p, ix + p
  bool av[AR];
  float4 ra[AR], rb[BR];
  bool bv[BR];
  __device__ DataLoader(const ConvShape& s_, const DT* dy_, const float* w_, int m0, int n0_,
                        int py, int px, int PH, int PW, int nkw_, int kh0_, int kw0_)
      : s(s_), dy(dy_), w(w_), n0(n0_), nkw(nkw_), kh0(kh0_), kw0(kw0_) {
    cchunks = s.K / BK;
    const int tid = threadIdx.x, c4 = tid & 7;
    const int M = s.N * PH * PW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      const int mm = m < M ? m : 0;
      const int jx = mm % PW, t = mm / PW, jy = t % PH, n = t / PH;
      const int iy = jy * s.stride + py, ix = jx * s.stride + px;
      av[i] = m < M && iy < s.H && ix < s.W;
      abase[i] = dy + (size_t)n * s.OH * s.OW * s.K + 4 * c4;
      qy[i] = iy + s.pad;
      qx[i] = ix + s.pad;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) bv[i] = n0 + (tid >> 3) + 32 * i < s.C;
  }
  __device__ __forceinline__ void load(int kt) {
    const int tp = kt / cchunks, co0 = (kt - tp * cchunks) * BK;
    const int kh = kh0 + (tp / nkw) * s.stride, kw = kw0 + (tp % nkw) * s.stride;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int oy = (qy[i] - kh) / s.stride, ox = (qx[i] - kw) / s.stride;  // exact by phase
      const bool ok = av[i] && qy[i] >= kh && qx[i] >= kw && oy < s.OH && ox < s.OW;
      const int oyc = min(max(oy, 0), s.OH - 1), oxc = min(max(ox, 0), s.OW - 1);
      const DT* src = abase[i] + ((size_t)oyc * s.OW + oxc) * s.K + co0;
      float4 v;
      if constexpr (sizeof(DT) == 2) {
        const uint2 u = *reinterpret_cast<const uint2*>(src);
        v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                        __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        v = *reinterpret_cast<const float4*>(src);
      }
      ra[i] = sel4(ok, v);
    }
    // B[k = co][n = ci] = W[kh, kw, ci, co]: float4 along co for one ci
    const int tid = threadIdx.x, c4 = tid & 7;
    const float* wb = w + (size_t)(kh * s.S + kw) * s.C * s.K + co0 + 4 * c4;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int ci = min(n0 + (tid >> 3) + 32 * i, s.C - 1);
      rb[i] = sel4(bv[i], *reinterpret_cast<const float4*>(wb + (size_t)ci * s.K));
    }
  }
  template <int P>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x, c4 = tid & 7;
#pragma unroll
    for (int i = 0; i < AR; ++i) Stage<P, BM>::put_k4(As, (tid >> 3) + 32 * i, 4 * c4, ra[i]);
#pragma unroll
    for (int i = 0; i < BR; ++i) Stage<P, BN>::put_k4(Bs, (tid >> 3) + 32 * i, 4 * c4, rb[i]);
  }
};

template <int BM, int BN, int P, class DT>
__device__ __forceinline__ void data_body(const ConvShape& s, const DT* __restrict__ dy,
                                          const float* __restrict__ w, float* __restrict__ dx,
                                          int kps, const float* __restrict__ addend) {
  // addend (unsplit only): a gradient that joins dX at this tensor, added in
  // the epilogue instead of by a separate elementwise pass
  // split-K over gridDim.z: slice z writes the raw slab dx + z * N*H*W*C
  using G = Geo<BM, BN, P>;
  __shared__ float smem[G::SMEM];
  const int sd = s.stride;
  const int phase = blockIdx.y, py = phase / sd, px = phase % sd;
  const int PH = (s.H - py + sd - 1) / sd, PW = (s.W - px + sd - 1) / sd;
  // taps of this phase: kh = (py + p) mod s, + s, ... < R
  const int kh0 = ((py + s.pad) % sd + sd) % sd, kw0 = ((px + s.pad) % sd + sd) % sd;
  const int nkh = kh0 < s.R ? (s.R - kh0 + sd - 1) / sd : 0;
  const int nkw = kw0 < s.S ? (s.S - kw0 + sd - 1) / sd : 0;
  const int M = s.N * PH * PW;
  // the grid is sized for the largest phase (py = px = 0)
  const int mt = (s.N * ((s.H + sd - 1) / sd) * ((s.W + sd - 1) / sd) + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;
  if (m0 >= M) return;  // phases with fewer pixels than the grid covers
  DataLoader<BM, BN, DT> ld(s, dy, w, m0, n0, py, px, PH, PW, nkw > 0 ? nkw : 1, kh0, kw0);
  f32x16 acc[G::TM][G::TN];
  const int nk = nkh * nkw * (s.K / BK), kb = blockIdx.z * kps;
  mainloop<BM, BN, P>(ld, smem, kb, min(kps, nk - kb), acc);
  dx += (size_t)blockIdx.z * s.N * s.H * s.W * s.C;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave & 1, wn = wave >> 1;
  // addend loads of 4 rows are issued before their stores (interleaved, hipcc
  // waited vmcnt(0) per element)
#pragma unroll
  for (int j = 0; j < G::TN; ++j) {
    const int ci = n0 + wn * (BN / 2) + 32 * j + (lane & 31);
    if (ci >= s.C) continue;
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int r4 = 0; r4 < 16; r4 += 4) {
        size_t o[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(r4 + u, lane);
          const int mm = m < M ? m : 0;
          const int jx = mm % PW, t = mm / PW, jy = t % PH, n = t / PH;
          const int iy = jy * sd + py, ix = jx * sd + px;
          ok[u] = m < M && iy < s.H && ix < s.W;
          o[u] = (((size_t)n * s.H + iy) * s.W + ix) * s.C + ci;
        }
        float av[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) av[u] = (addend && ok[u]) ? addend[o[u]] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (ok[u]) dx[o[u]] = acc[i][j][r4 + u] + av[u];
      }
  }
}

template <int BM, int BN, int P>
__global__ __launch_bounds__(NT) void data_kernel(ConvShape s, const float* __restrict__ dy,
                                                  const float* __restrict__ w,
                                                  float* __restrict__ dx, int kps,
                                                  const float* __restrict__ addend) {
  data_body<BM, BN, P, float>(s, dy, w, dx, kps, addend);
}
template <int BM, int BN, int P>
__global__ __launch_bounds__(NT) void data_b16_kernel(ConvShape s, const __bf16* __restrict__ dy,
                                                      const float* __restrict__ w,
                                                      float* __restrict__ dx, int kps,
                                                      const float* __restrict__ addend) {
  data_body<BM, BN, P, __bf16>(s, dy, w, dx, kps, addend);
}

// ----------------------------------------------------- backward-filter ----
// XCD-aware split-K order.  Block b runs on XCD (b + o) mod 8 and each XCD
// dispatches its blocks in id order, so with the slice count a multiple of 8
// XCD x gets the slices z = x (mod 8), each with all of its tiles back to back:
// every tap / channel tile of a pixel slice reads that slice's X and dY rows,
// which then come from one L2 instead of up to eight (the 56x56 layer's nine
// tap blocks of a slice otherwise landed on nine consecutive ids: eight XCDs).
__device__ __forceinline__ int xcd_slice_bid(int bid, int tiles, bool xcd) {
  if (!xcd || gridDim.x % (8 * tiles)) return bid;
  const int x = bid & 7, idx = bid >> 3;
  return (x + 8 * (idx / tiles)) * tiles + idx % tiles;
}

// dW[tap][ci][co] = sum_{pix} X[pix shifted by tap][ci] dY[pix][co]; per
// block: one tap, a BM x BN (ci x co) tile, one split-K slice of the pixels;
// K tile = 32 output pixels.  Both operands load float4 along their channel
// axis straight into the k-major LDS image.  Requires C % 4 == 0, K % 4 == 0.
// Output-pixel coordinates of one A row of the filter-gradient loaders, walked
// forward BK pixels a K tile: mainloop calls load(kt) for kt = k0, k0 + 1, ...
// in order, so the four runtime integer divisions per row per tile (~200 VALU
// instructions a K tile per wave, more than the tile's 16 MFMAs could hide)
// happen once per thread.  Past the last pixel the walk runs on (n >= N); the
// loaders clamp the image index and mask the row by its pixel index.
struct PixWalk {
  int n, oy, ox;
  __device__ __forceinline__ void init(const ConvShape& s, int pix) {
    ox = pix % s.OW;
    const int t = pix / s.OW;
    oy = t % s.OH;
    n = t / s.OH;
  }
  __device__ __forceinline__ void step(const ConvShape& s, int dox, int doy) {
    ox += dox;
    oy += doy;
    if (ox >= s.OW) {
      ox -= s.OW;
      ++oy;
    }
    while (oy >= s.OH) {
      oy -= s.OH;
      ++n;
    }
  }
};

template <int BM, int BN, int KB = BK>
struct FilterLoader {
  static constexpr int AR = BM * KB / 4 / NT;
  static constexpr int BR = BN * KB / 4 / NT;
  ConvShape s;
  const float* x;
  const float* dy;
  int m0, n0, kh, kw, pix0, npix, dox, doy;
  PixWalk pw[AR];
  float4 ra[AR], rb[BR];
  __device__ FilterLoader(const ConvShape& s_, const float* x_, const float* dy_, int m0_, int n0_,
                          int tap, int pix0_, int npix_)
      : s(s_), x(x_), dy(dy_), m0(m0_), n0(n0_), pix0(pix0_), npix(npix_) {
    kh = tap / s.S;
    kw = tap % s.S;
    dox = KB % s.OW;
    doy = KB / s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      pw[i].init(s, min(pix0 + (int)threadIdx.x / (BM / 4) + (NT / (BM / 4)) * i, npix - 1));
  }
  __device__ __forceinline__ void load(int kt) {  // kt = k0, k0 + 1, ... in order
    const int tid = threadIdx.x;
    const int ma = 4 * (tid % (BM / 4)), nb = 4 * (tid % (BN / 4));
    const int ci = min(m0 + ma, s.C - 4), co = min(n0 + nb, s.K - 4);
    const bool cv = m0 + ma < s.C, kv = n0 + nb < s.K;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = tid / (BM / 4) + (NT / (BM / 4)) * i;
      const int pix = pix0 + kt * KB + k;
      const int n = min(pw[i].n, s.N - 1);
      const int iy = pw[i].oy * s.stride - s.pad + kh, ix = pw[i].ox * s.stride - s.pad + kw;
      const bool ok = cv && pix < npix && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
      const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
      ra[i] = sel4(ok, *reinterpret_cast<const float4*>(
                           x + (((size_t)n * s.H + iyc) * s.W + ixc) * s.C + ci));
      pw[i].step(s, dox, doy);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      const int pix = pix0 + kt * KB + k;
      const bool ok = kv && pix < npix;
      rb[i] = sel4(ok, *reinterpret_cast<const float4*>(dy + (size_t)min(pix, npix - 1) * s.K + co));
    }
  }
  template <int P>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = tid / (BM / 4) + (NT / (BM / 4)) * i;
      Stage<P, BM, KB>::put_r4(As, 4 * (tid % (BM / 4)), k, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      Stage<P, BN, KB>::put_r4(Bs, 4 * (tid % (BN / 4)), k, rb[i]);
    }
  }
};

template <int BM, int BN, int P, int KB = BK>
__global__ __launch_bounds__(NT) void filter_kernel(ConvShape s, const float* __restrict__ x,
                                                    const float* __restrict__ dy,
                                                    float* __restrict__ part, int kchunk_tiles,
                                                    bool xcd) {
  using G = Geo<BM, BN, P, KB>;
  __shared__ float smem[G::SMEM];
  const int mt = (s.C + BM - 1) / BM, nt = (s.K + BN - 1) / BN;
  const int taps = s.R * s.S;
  const int tiles = mt * nt * taps;
  const int bid = xcd_slice_bid(blockIdx.x, tiles, xcd);
  const int z = bid / tiles, rem = bid % tiles;
  const int tap = rem % taps, t2 = rem / taps;
  const int m0 = (t2 % mt) * BM, n0 = (t2 / mt) * BN;
  const int npix = s.N * s.OH * s.OW;
  const int pix0 = z * kchunk_tiles * KB;
  const int nk = min(kchunk_tiles, (npix - pix0 + KB - 1) / KB);
  FilterLoader<BM, BN, KB> ld(s, x, dy, m0, n0, tap, pix0, npix);
  f32x16 acc[G::TM][G::TN];
  mainloop<BM, BN, P, KB>(ld, smem, 0, nk, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave & 1, wn = wave >> 1;
  const size_t slab = (size_t)taps * s.C * s.K;
#pragma unroll
  for (int j = 0; j < G::TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + (lane & 31);
    if (co >= s.K) continue;
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = m0 + wm * (BM / 2) + 32 * i + mfma32_row(r, lane);
        if (ci >= s.C) continue;
        part[z * slab + ((size_t)tap * s.C + ci) * s.K + co] = acc[i][j][r];
      }
  }
}

// Backward-filter for channel counts that are not a multiple of 4 (the
// 3-channel ResNet stem, LeNet's 6-channel conv): M = R*S*C rows (tap, ci)
// in one GEMM (no per-tap grid split, so a 3-channel layer does not waste a
// 64-row tile per tap); A elements are scalar gathers whose (tap, ci) decode
// is done once per thread, the pixel decode once per K tile row.
template <int BM, int BN>
struct FilterGatherLoader {
  static constexpr int AR = BM * BK / 4 / NT;
  static constexpr int BR = BN * BK / 4 / NT;
  ConvShape s;
  const float* x;
  const float* dy;
  int n0, pix0, npix, dox, doy;
  int dh[4], dw[4], ci[4];  // this thread's 4 A columns (m = ma + j)
  bool mv[4];
  PixWalk pw[AR];
  float4 ra[AR], rb[BR];
  __device__ FilterGatherLoader(const ConvShape& s_, const float* x_, const float* dy_, int m0,
                                int n0_, int pix0_, int npix_)
      : s(s_), x(x_), dy(dy_), n0(n0_), pix0(pix0_), npix(npix_) {
    dox = BK % s.OW;
    doy = BK / s.OW;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      pw[i].init(s, min(pix0 + (int)threadIdx.x / (BM / 4) + (NT / (BM / 4)) * i, npix - 1));
    const int Mw = s.R * s.S * s.C;
    const int ma = m0 + 4 * (threadIdx.x % (BM / 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = ma + j;
      mv[j] = m < Mw;
      const int mm = mv[j] ? m : 0;
      ci[j] = mm % s.C;
      const int tap = mm / s.C;
      dh[j] = tap / s.S - s.pad;
      dw[j] = tap % s.S - s.pad;
    }
  }
  __device__ __forceinline__ void load(int kt) {
    const int tid = threadIdx.x;
    const int nb = 4 * (tid % (BN / 4));
    const int co = min(n0 + nb, s.K - 4);
    const bool kv = n0 + nb < s.K;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = tid / (BM / 4) + (NT / (BM / 4)) * i;
      const int pix = pix0 + kt * BK + k;
      const int oy = pw[i].oy, ox = pw[i].ox;
      const float* img = x + (size_t)min(pw[i].n, s.N - 1) * s.H * s.W * s.C;
      pw[i].step(s, dox, doy);
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int iy = oy * s.stride + dh[j], ix = ox * s.stride + dw[j];
        const bool ok = mv[j] && pix < npix && iy >= 0 && iy < s.H && ix >= 0 && ix < s.W;
        const int iyc = min(max(iy, 0), s.H - 1), ixc = min(max(ix, 0), s.W - 1);
        const float e = img[((size_t)iyc * s.W + ixc) * s.C + ci[j]];
        v[j] = ok ? e : 0.f;
      }
      ra[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      const int pix = pix0 + kt * BK + k;
      rb[i] = sel4(kv && pix < npix,
                   *reinterpret_cast<const float4*>(dy + (size_t)min(pix, npix - 1) * s.K + co));
    }
  }
  template <int P>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = tid / (BM / 4) + (NT / (BM / 4)) * i;
      Stage<P, BM>::put_r4(As, 4 * (tid % (BM / 4)), k, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = tid / (BN / 4) + (NT / (BN / 4)) * i;
      Stage<P, BN>::put_r4(Bs, 4 * (tid % (BN / 4)), k, rb[i]);
    }
  }
};

template <int BM, int BN, int P>
__global__ __launch_bounds__(NT) void filter_gather_kernel(ConvShape s, const float* __restrict__ x,
                                                           const float* __restrict__ dy,
                                                           float* __restrict__ part,
                                                           int kchunk_tiles, bool xcd) {
  using G = Geo<BM, BN, P>;
  __shared__ float smem[G::SMEM];
  const int Mw = s.R * s.S * s.C;
  const int mt = (Mw + BM - 1) / BM, nt = (s.K + BN - 1) / BN;
  const int bid = xcd_slice_bid(blockIdx.x, mt * nt, xcd);
  const int z = bid / (mt * nt), rem = bid % (mt * nt);
  const int m0 = (rem % mt) * BM, n0 = (rem / mt) * BN;
  const int npix = s.N * s.OH * s.OW;
  const int pix0 = z * kchunk_tiles * BK;
  const int nk = min(kchunk_tiles, (npix - pix0 + BK - 1) / BK);
  FilterGatherLoader<BM, BN> ld(s, x, dy, m0, n0, pix0, npix);
  f32x16 acc[G::TM][G::TN];
  mainloop<BM, BN, P>(ld, smem, 0, nk, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave & 1, wn = wave >> 1;
#pragma unroll
  for (int j = 0; j < G::TN; ++j) {
    const int co = n0 + wn * (BN / 2) + 32 * j + (lane & 31);
    if (co >= s.K) continue;
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + 32 * i + mfma32_row(r, lane);
        if (m < Mw) part[(size_t)z * Mw * s.K + (size_t)m * s.K + co] = acc[i][j][r];
      }
  }
}

__device__ __forceinline__ void add4(float4& a, const float4 b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}

// Deep, narrow slab stacks (the thin gather-path filter gradients of LeNet:
// 128 slices of a few hundred floats, 1-3 blocks of slab_sum4_kernel whose
// threads each walk a 128-long chain of dependent L2 loads, ~26 us): block =
// 64 float4 outputs x 4 slice groups, 4 independent partial sums per thread
// (16 loads in flight), groups combined through LDS in a fixed order, so the
// result is deterministic for a given nz.
__global__ __launch_bounds__(256) void slab_sum4_deep_kernel(const float4* __restrict__ part,
                                                             int nz, long long n4,
                                                             float4* __restrict__ out) {
  __shared__ float4 red[4][64];
  const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + o;
  float4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int z = g;
    for (; z + 12 < nz; z += 16) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = part[(long long)(z + 4 * u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) add4(a[u], v[u]);
    }
    for (; z < nz; z += 4) add4(a[0], part[(long long)z * n4 + i]);
  }
  add4(a[0], a[1]);
  add4(a[2], a[3]);
  add4(a[0], a[2]);
  red[g][o] = a[0];
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 r = red[0][o];
    add4(r, red[1][o]);
    add4(r, red[2][o]);
    add4(r, red[3][o]);
    out[i] = r;
  }
}

// Deterministic slab reduction, float4-vectorised (n % 4 == 0).
__global__ __launch_bounds__(256) void slab_sum4_kernel(const float4* __restrict__ part, int nz,
                                                        long long n4, float4* __restrict__ out,
                                                        const float4* __restrict__ addend) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = part[i];
    for (int z = 1; z < nz; ++z) {
      const float4 b = part[z * n4 + i];
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
    out[i] = a;
  }
}

// slab_sum4 for a split-K forward whose output feeds a BatchNorm: also the
// shifted statistics of the summed values, one partial row per block in the
// [2][C / 64][P][64] table (P = grid; 256 % (C / 4) == 0, so every thread
// keeps one channel quad; threads sharing a quad are combined in a fixed order)
__global__ __launch_bounds__(256) void slab_sum4_stats_kernel(const float4* __restrict__ part,
                                                              int nz, long long n4,
                                                              float4* __restrict__ out,
                                                              const ConvStats cs, int C) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int cq = C >> 2, tid = threadIdx.x;
  const float4 kc = *reinterpret_cast<const float4*>(cs.shift + 4 * (tid % cq));
  float4 t1 = make_float4(0.f, 0.f, 0.f, 0.f), t2 = t1;
  for (long long i = (long long)blockIdx.x * blockDim.x + tid; i < n4; i += stride) {
    float4 a = part[i];
    for (int z = 1; z < nz; ++z) {
      const float4 b = part[z * n4 + i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    out[i] = a;
    const float dx = a.x - kc.x, dy = a.y - kc.y, dz = a.z - kc.z, dw = a.w - kc.w;
    t1.x += dx; t1.y += dy; t1.z += dz; t1.w += dw;
    t2.x += dx * dx; t2.y += dy * dy; t2.z += dz * dz; t2.w += dw * dw;
  }
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
    const int co = 4 * tid;
    const size_t e = ((size_t)(co >> 6) * cs.P + blockIdx.x) * 64 + (co & 63);
    *reinterpret_cast<float4*>(cs.part + e) = a;
    *reinterpret_cast<float4*>(cs.part + (size_t)C * cs.P + e) = b;
  }
}

// ------------------------------------ fp32 3x3 stride-1 halo conv ----
// The fp32 port of conv_bf16.hip's conv3_kernel (forward and stride-1 dgrad
// of ResNet-18's 3x3 layers).  The tiled fwd_kernel above re-stages the A
// tile through L2 for each of the 9 taps, one K tile in flight: on the
// 56x56x64 layer at B = 32 it ran 100 us, 47 % of the fp32 MFMA rate.  Here a
// block owns BM consecutive output pixels x BN output channels and, per
// CH-channel chunk (CH = 32: 128-byte LDS rows, the bf16 kernel's geometry;
// CH = 16: 64-byte rows, so 128-column weight tiles still fit two blocks a CU):
//   * stages the activation halo once (the stacked image rows from one above
//     the tile to one below) with global_load_lds_dwordx4;
//   * reads each tap's A fragments out of it at per-lane shifted rows
//     (padding taps read an all-zero row);
//   * streams the 9 taps' weight tiles [BN out][32 in] through an RB-deep LDS
//     ring, RB - 1 in flight.
// 16-byte pieces are XOR-swizzled by the row's bank line (h3f::Geo) through the
// DMA source address, so a ds_read_b128 lane group reads 16 rows conflict-free.  MFMA
// v_mfma_f32_32x32x2f32: lane (r, h) of a fragment read takes chunk 2c + h
// (channels 8c + 4h .. + 3) and element e feeds MFMA e, so MFMA e of group c
// reduces the channel pair {8c + e, 8c + 4 + e} on both operands.
// Weights: wt[tap'][out][in] (in contiguous) read at tap' = 8 - t: the
// forward passes the stride-1 dgrad copy (wflip_kernel / the SGD's kind-1
// job: W[8 - t] transposed), the dgrad the original HWIO weights (W[8 - t]
// with in = the conv's K is already [out = C][in = K]).
// LDS (HCAP + 1) x 4 CH + RB x BN x 4 CH bytes: 77 KiB at (BN 64, CH 32),
// 54 KiB at (BN 128, CH 16), RB = 4: two blocks a CU.  Split-K over channel
// chunks (blockIdx.y, slabs) for small M.
namespace h3f {
// halo pixel rows, a multiple of every RPI (the DMA fills whole groups of RPI
// rows, so the last group of a halo of <= HCAP pixels ends at or below row
// HCAP - 1); row HCAP is all zeros
constexpr int HCAP = 352;
__device__ uint4 g_zero[4];  // never written: the DMA source of rows outside the tensor
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void glds(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
inline int halo_rows(const ConvShape& s, int bm) { return ((bm + s.W - 2) / s.W + 3) * s.W; }
// LDS row geometry of a CH-channel chunk: NCK 16-byte pieces a row, the piece
// index XOR-swizzled by the row's 256-byte bank line (RPL rows a line), so a
// ds_read_b128 lane group (16 consecutive rows, one piece each) is conflict-free
template <int CH>
struct Geo {
  static constexpr int ROWB = CH * 4;
  static constexpr int NCK = CH / 4;
  static constexpr int RPL = 256 / ROWB;
  static constexpr int RPI = 64 / NCK;  // rows one wave-wide DMA instruction fills
  __device__ static __forceinline__ int swz(int row) { return (row / RPL) & (NCK - 1); }
};
}  // namespace h3f

// HC: halo rows of the LDS image (h3f::HCAP, or fewer for a smaller footprint)
template <int BM, int BN, int RB, int CH, int HC = h3f::HCAP>
__global__ __launch_bounds__(NT) void conv3f_kernel(ConvShape s, const float* __restrict__ x,
                                                    const float* __restrict__ wt,
                                                    float* __restrict__ y, int cps,
                                                    const float* __restrict__ addend) {
  constexpr int HCAP = HC;
  using G3 = h3f::Geo<CH>;
  constexpr int ROWB = G3::ROWB, NCK = G3::NCK, RPI = G3::RPI;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GB = (BN / 4) / RPI;  // weight DMA instructions per wave per tap
  constexpr int HB = (HCAP + 1) * ROWB;
  constexpr int BSZ = BN * ROWB;
  static_assert(RB >= 3 && RB <= 4, "ring depth");
  static_assert(GB >= 1 && (BN / 4) % RPI == 0, "weight rows per wave");
  static_assert(HCAP % RPI == 0, "halo DMA groups end below the zero row");
  __shared__ __attribute__((aligned(1024))) char smem[HB + RB * BSZ];
  const int M = s.N * s.H * s.W;
  const int W = s.W, H = s.H;
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;
  const int nch = s.C / CH;
  const int cc0 = blockIdx.y * cps, cc1 = min(nch, cc0 + cps);
  const int g_first = m0 / W, g_last = (min(m0 + BM, M) - 1) / W;
  const long long hbase = (long long)(g_first - 1) * W;  // global pixel of halo row 0
  const int npix = (g_last - g_first + 3) * W;
  const int nins = (npix + RPI - 1) / RPI;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5, lr = lane / NCK, lp = lane % NCK;
  if (tid < NCK) *reinterpret_cast<uint4*>(smem + HCAP * ROWB + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
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
  const float* bsrc[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = wave * (BN / 4) + RPI * j + lr;
    bsrc[j] = wt + (size_t)(n0 + row) * s.C + 4 * (lp ^ G3::swz(row));
  }
  auto issue_b = [&](int tap, int cc, int slot) {
    const size_t o = (size_t)(8 - tap) * s.K * s.C + (size_t)cc * CH;
    char* dst = smem + HB + slot * BSZ + wave * (BN / 4) * ROWB;
#pragma unroll
    for (int j = 0; j < GB; ++j) h3f::glds(bsrc[j] + o, dst + RPI * j * ROWB);
  };
  auto issue_halo = [&](int cc) {
    for (int ins = wave; ins < nins; ins += 4) {
      const int p = RPI * ins + lr;
      const long long gp = hbase + p;
      const bool ok = p < npix && gp >= 0 && gp < M;
      const void* src = ok ? (const void*)(x + gp * s.C + (size_t)cc * CH + 4 * (lp ^ G3::swz(p)))
                           : (const void*)h3f::g_zero;
      h3f::glds(src, smem + ins * RPI * ROWB);
    }
  };
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
      const int ahead = min(RB - 2, 8 - t);
      if (ahead >= 2)
        h3f::wait_vm<2 * GB>();
      else if (ahead == 1)
        h3f::wait_vm<GB>();
      else
        h3f::wait_vm<0>();
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
      for (int c = 0; c < CH / 8; ++c) {
        const int ck = 2 * c + h;
        float4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const float4*>(smem + hrow[i] * ROWB +
                                                  ((ck ^ G3::swz(hrow[i])) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int R = wn * (BN / 2) + 32 * j + r;
          b[j] = *reinterpret_cast<const float4*>(B + R * ROWB + ((ck ^ G3::swz(R)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = mfma32x32x2(a[i].x, b[j].x, acc[i][j]);
            acc[i][j] = mfma32x32x2(a[i].y, b[j].y, acc[i][j]);
            acc[i][j] = mfma32x32x2(a[i].z, b[j].z, acc[i][j]);
            acc[i][j] = mfma32x32x2(a[i].w, b[j].w, acc[i][j]);
          }
      }
    }
  }
  // epilogue (conv_bf16.hip conv3_kernel EPI 0): lane (r, h) of 32 x 32 tile
  // (i, j) holds rows 4h + (q & 3) + 8 (q >> 2), column r; the addend (a
  // gradient join, unsplit only) loaded for the tile before its stores
  y += (size_t)blockIdx.y * M * s.K;
  const size_t K = s.K;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = m0 + wm * (BM / 2) + 32 * i + 4 * h;
    const bool full = m0 + wm * (BM / 2) + 32 * i + 32 <= M;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (BN / 2) + 32 * j + r;
      float* p = y + (size_t)mb * K + co;
      if (full && addend) {
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
}

// Stride-1 backward-data as a forward conv of dY (fp32): dX = conv(dY, W')
// with pad R - 1 - pad and W'[kh][kw][co][ci] = W[R-1-kh][S-1-kw][ci][co].
// The forward kernel's operands are both float4 rows into LDS; the dgrad
// kernel stages W through 4 scalar LDS stores per float4 (its k = co is the
// contiguous axis) and measured 119-129 us against 96-104 us forward on the
// same ResNet-18 shapes.  One 32 x 32 LDS tile transpose per (tap, ci, co)
// block: coalesced reads along co, coalesced writes along ci.
// ----------------------- fp32 3x3 stride-2 backward-data (halo form) ----
// conv_bf16.hip dgrad3s2_kernel's design on conv3f_kernel's fp32 staging: dX
// of a 3x3 / stride 2 / pad 1 conv on an even input, output pixel
// (2a + py, 2b + px) taking only the taps of its parity class -
//   py = 0: kh = 1 on dY row a;  py = 1: kh = 0 on row a + 1, kh = 2 on row a
// (likewise px / kw / columns).  A block owns BM dY-grid pixels (n, a, b) x
// BN input channels and keeps four accumulator sets, one per class; the dY
// halo (the tile's stacked rows plus one below) is staged once per CH-channel
// chunk of the reduction (the output channels) and each tap reads it at a
// per-lane (+1 row / +1 column) shift, the zero row past the image.  B: the
// HWIO weights themselves, [tap][ci][co] (rows = input channels, the output
// channels contiguous) through the RB-deep ring.  Split-K over the output-
// channel chunks (blockIdx.y, slabs).  Replaces the phase-split data_kernel.
template <int BM, int BN, int RB, int CH>
__global__ __launch_bounds__(NT) void dgrad3s2f_kernel(ConvShape s, const float* __restrict__ dy,
                                                       const float* __restrict__ w,
                                                       float* __restrict__ dx, int cps,
                                                       const float* __restrict__ addend) {
  using h3f::HCAP;
  using G3 = h3f::Geo<CH>;
  constexpr int ROWB = G3::ROWB, NCK = G3::NCK, RPI = G3::RPI;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GB = (BN / 4) / RPI;  // weight DMA instructions per wave per tap
  constexpr int HB = (HCAP + 1) * ROWB;
  constexpr int BSZ = BN * ROWB;
  static_assert(RB >= 3 && RB <= 4, "ring depth");
  static_assert(GB >= 1 && (BN / 4) % RPI == 0, "weight rows per wave");
  static_assert(HCAP % RPI == 0, "halo DMA groups end below the zero row");
  __shared__ __attribute__((aligned(1024))) char smem[HB + RB * BSZ];
  const int OH = s.OH, OW = s.OW;
  const int M = s.N * OH * OW;  // dY-grid pixels
  const int mt = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid % mt) * BM, n0 = (bid / mt) * BN;  // n: input channel ci
  const int nch = s.K / CH;
  const int cc0 = blockIdx.y * cps, cc1 = min(nch, cc0 + cps);
  const int g_first = m0 / OW, g_last = (min(m0 + BM, M) - 1) / OW;
  const long long hbase = (long long)g_first * OW;  // global dY pixel of halo row 0
  const int npix = (g_last - g_first + 2) * OW;
  const int nins = (npix + RPI - 1) / RPI;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int r = lane & 31, h = lane >> 5, lr = lane / NCK, lp = lane % NCK;
  if (tid < NCK) *reinterpret_cast<uint4*>(smem + HCAP * ROWB + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
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
  const float* bsrc[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = wave * (BN / 4) + RPI * j + lr;
    bsrc[j] = w + (size_t)(n0 + row) * s.K + 4 * (lp ^ G3::swz(row));
  }
  auto issue_b = [&](int tap, int cc, int slot) {
    const size_t o = (size_t)tap * s.C * s.K + (size_t)cc * CH;
    char* dst = smem + HB + slot * BSZ + wave * (BN / 4) * ROWB;
#pragma unroll
    for (int j = 0; j < GB; ++j) h3f::glds(bsrc[j] + o, dst + RPI * j * ROWB);
  };
  auto issue_halo = [&](int cc) {
    for (int ins = wave; ins < nins; ins += 4) {
      const int p = RPI * ins + lr;
      const long long gp = hbase + p;
      const bool ok = p < npix && gp < M;
      const void* src = ok ? (const void*)(dy + gp * s.K + (size_t)cc * CH + 4 * (lp ^ G3::swz(p)))
                           : (const void*)h3f::g_zero;
      h3f::glds(src, smem + ins * RPI * ROWB);
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
    // the previous chunk's halo and ring reads are done (and the zero row is written)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_halo(cc);
#pragma unroll
    for (int t = 0; t < RB - 1; ++t) issue_b(t, cc, t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ahead = min(RB - 2, 8 - t);
      if (ahead >= 2)
        h3f::wait_vm<2 * GB>();
      else if (ahead == 1)
        h3f::wait_vm<GB>();
      else
        h3f::wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring slot (t - 1) % RB read
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
      for (int c = 0; c < CH / 8; ++c) {
        const int ck = 2 * c + h;
        float4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const float4*>(smem + hrow[i] * ROWB +
                                                  ((ck ^ G3::swz(hrow[i])) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int R = wn * (BN / 2) + 32 * j + r;
          b[j] = *reinterpret_cast<const float4*>(B + R * ROWB + ((ck ^ G3::swz(R)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[cls][i][j] = mfma32x32x2(a[i].x, b[j].x, acc[cls][i][j]);
            acc[cls][i][j] = mfma32x32x2(a[i].y, b[j].y, acc[cls][i][j]);
            acc[cls][i][j] = mfma32x32x2(a[i].z, b[j].z, acc[cls][i][j]);
            acc[cls][i][j] = mfma32x32x2(a[i].w, b[j].w, acc[cls][i][j]);
          }
      }
    }
  }
  // epilogue: grid pixel m = (n, a, b) -> dX pixels (n, 2a + py, 2b + px);
  // the addend (a gradient join, unsplit only) of four rows loaded before
  // their stores (vmcnt counts both: interleaved, every load would wait for
  // the stores ahead of it)
  dx += (size_t)blockIdx.y * s.N * s.H * s.W * s.C;
  const size_t C = s.C, W = s.W;
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
          const int g = mm / OW, b = mm - g * OW;  // g = n * OH + a
          o[u] = ((size_t)(2 * g) * W + 2 * b) * C + ci;  // (n, 2a, 2b)
        }
        float av[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            av[u][c] = addend && ok[u] ? addend[o[u] + ((c >> 1) * W + (c & 1)) * C] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (!ok[u]) continue;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            dx[o[u] + ((c >> 1) * W + (c & 1)) * C] = acc[c][i][j][q4 + u] + av[u][c];
        }
      }
    }
}

__global__ __launch_bounds__(256) void wflip_kernel(const float* __restrict__ w,
                                                    float* __restrict__ wt, int R, int S, int C,
                                                    int K) {
  __shared__ float t[32][33];
  const int tap = blockIdx.z, ci0 = blockIdx.y * 32, co0 = blockIdx.x * 32;
  const int kh = tap / S, kw = tap - kh * S;
  const float* src = w + (size_t)((R - 1 - kh) * S + (S - 1 - kw)) * C * K;
  float* dst = wt + (size_t)tap * K * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int r = ty; r < 32; r += 8) {
    const int ci = ci0 + r, co = co0 + tx;
    t[r][tx] = (ci < C && co < K) ? src[(size_t)ci * K + co] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int r = ty; r < 32; r += 8) {
    const int co = co0 + r, ci = ci0 + tx;
    if (co < K && ci < C) dst[(size_t)co * C + ci] = t[tx][r];
  }
}

// ------------------------------------------------------------ dispatch ----
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Block tile from the GEMM's M and N: 128-wide where the dimension allows it.
enum Tile { T128x128, T128x64, T64x128, T64x64 };
// 128-row tiles only with >= 256 blocks of them (bf16).  fp32 never: on the
// ResNet-18 56x56 layers (M = 100352) 64-row tiles measured 116.4 -> 103.8 us
// forward and 145.5 -> 129.0 us dgrad (the 128x64 grid, 784 blocks, overran
// the 768 resident slots by 16).  (TiledPlan m128_min_*)
static inline long long m128_min(bool bf16) {
  return bf16 ? tiled_plan().m128_min_bf16 : tiled_plan().m128_min_f32;
}
// narrow: 64-column tiles even for N > 64 (fp32 stride-2 dgrad and 1x1 stride-2
// forward of ResNet-18: 99.0 -> 84.0 / 33.3 -> 20.0 us dgrad at 128 channels,
// 98.0 -> 92.4 / 35.9 -> 29.1 at 256, 1x1 forward 14.4 -> 12.3 / 20.8 -> 17.0;
// the stride-1 3x3 layers were slower with them, 95.7 -> 103.2 us forward)
static inline Tile pick(long long M, int N, bool bf16, bool narrow = false) {
  const bool bm = M >= m128_min(bf16), bn = N > 64 && !(narrow && !bf16);
  if (bn) return bm ? T128x128 : T64x128;
  return bm ? T128x64 : T64x64;
}

#define TILED_DISPATCH_P(P, t, KERNEL, GRID, ...)                                        \
  switch (t) {                                                                            \
    case T128x128: KERNEL<128, 128, P><<<GRID(128, 128), NT, 0, st>>>(__VA_ARGS__); break; \
    case T128x64: KERNEL<128, 64, P><<<GRID(128, 64), NT, 0, st>>>(__VA_ARGS__); break;    \
    case T64x128: KERNEL<64, 128, P><<<GRID(64, 128), NT, 0, st>>>(__VA_ARGS__); break;    \
    default: KERNEL<64, 64, P><<<GRID(64, 64), NT, 0, st>>>(__VA_ARGS__); break;           \
  }
#define TILED_DISPATCH(t, KERNEL, GRID, ...)                  \
  if (bf16) {                                                 \
    TILED_DISPATCH_P(BF16, t, KERNEL, GRID, __VA_ARGS__)      \
  } else {                                                    \
    TILED_DISPATCH_P(F32, t, KERNEL, GRID, __VA_ARGS__)       \
  }

}  // namespace tiled

TiledPlan& tiled_plan() {
  static TiledPlan plan;
  return plan;
}

bool conv_fwd_tiled_ok(const ConvShape& s) { return s.C % 32 == 0 && s.K % 4 == 0; }
// the gather-loader forward: thin inputs with a reduction axis of >= 2 K tiles
// (the ResNet stem); smaller ones stay on the direct / gather engines
bool conv_fwd_tiled_gather_ok(const ConvShape& s) {
  return s.C % 32 != 0 && s.K % 4 == 0 && s.R * s.S * s.C >= 64;
}
bool conv_bwd_data_tiled_ok(const ConvShape& s) { return s.K % 32 == 0 && s.C % 4 == 0; }
bool conv_bwd_filter_tiled_ok(const ConvShape& s) { return s.K % 4 == 0; }  // C % 4: vector path

namespace tiled {
static inline int tile_m(Tile t) { return (t == T128x128 || t == T128x64) ? 128 : 64; }
static inline int tile_n(Tile t) { return (t == T128x128 || t == T64x128) ? 128 : 64; }

// split targets (blocks to aim for): TiledPlan ksplit_target (forward / dgrad)
// and wgsplit_target (filter gradient)
static inline int ksplit_target() { return tiled_plan().ksplit_target; }
static inline int wgsplit_target() { return tiled_plan().wgsplit_target; }
// split-K factor for a GEMM with `blocks` output tiles of nk K tiles each:
// deep layers (few tiles, long K) get enough blocks to fill 256 CUs twice
static inline int ksplit(long long blocks, int nk) {
  // measured (ResNet-18, B=32): filling the chip beats the extra slab traffic
  // (a 256-block / 8-slice cap cost +15 % step time in fp32 and bf16)
  if (blocks >= 512 || nk < 8) return 1;
  int z = cdiv(ksplit_target(), blocks);
  if (z > nk / 4) z = nk / 4;
  if (z > 16) z = 16;
  if (z < 1) z = 1;
  const int kps = cdiv(nk, z);
  return cdiv(nk, kps);
}
static inline void fwd_plan(const ConvShape& s, bool epilogue, bool bf16, Tile& t, int& z,
                            int& kps) {
  const long long M = (long long)s.N * s.OH * s.OW;
  t = pick(M, s.K, bf16, s.R == 1 && s.S == 1 && s.stride == 2);
  const int nk = s.C % BK == 0 ? s.R * s.S * (s.C / BK) : cdiv(s.R * s.S * s.C, BK);
  z = epilogue ? 1 : ksplit((long long)cdiv(M, tile_m(t)) * cdiv(s.K, tile_n(t)), nk);
  kps = cdiv(nk, z);
}
static inline void data_plan(const ConvShape& s, bool bf16, Tile& t, int& z, int& kps) {
  const int sd = s.stride;
  const long long Mph = (long long)s.N * ((s.H + sd - 1) / sd) * ((s.W + sd - 1) / sd);
  t = pick(Mph * sd * sd, s.C, bf16, sd == 2);
  const int ntap = cdiv(s.R, sd) * cdiv(s.S, sd);  // taps of the richest phase
  const int nk = ntap * (s.K / BK);
  z = ksplit((long long)cdiv(Mph, tile_m(t)) * cdiv(s.C, tile_n(t)) * sd * sd, nk);
  kps = cdiv(nk, z);
}
static inline long long slab_grid(long long n) {
  const long long b = (n / 4 + 255) / 256;
  return b > 4096 ? 4096 : b;
}
static inline void slab_sum(const float* part, int z, long long n, float* out, hipStream_t st,
                            const float* addend = nullptr) {
  const long long b = slab_grid(n);
  if (b < 64 && z >= 16 && !addend) {  // deep, narrow stack: spread the slices over the block
    slab_sum4_deep_kernel<<<cdiv(n / 4, 64), 256, 0, st>>>(reinterpret_cast<const float4*>(part),
                                                            z, n / 4, reinterpret_cast<float4*>(out));
    return;
  }
  slab_sum4_kernel<<<(int)b, 256, 0, st>>>(reinterpret_cast<const float4*>(part), z, n / 4,
                                          reinterpret_cast<float4*>(out),
                                          reinterpret_cast<const float4*>(addend));
}
}  // namespace tiled

// fp32 stride-1 dgrad through the forward kernel (see wflip_kernel): the
// forward shape over dY and the floats of the flipped weight ahead of its
// split-K workspace.  TiledPlan dgrad_fwd = false: the phase-decomposed dgrad
static bool dgrad_fwd_ok(const ConvShape& s) {
  return tiled_plan().dgrad_fwd && s.stride == 1 && s.R == s.S && s.pad <= s.R - 1 && 2 * s.pad == s.R - 1 &&
         s.K % tiled::BK == 0 && s.C % 4 == 0 && s.OH == s.H && s.OW == s.W;
}
static ConvShape dgrad_fwd_shape(const ConvShape& s) {
  return ConvShape{s.N, s.OH, s.OW, s.K, s.C, s.R, s.S, 1, s.R - 1 - s.pad, s.H, s.W};
}
static long long dgrad_fwd_ws_floats(const ConvShape& s) {
  const long long wf = ((long long)s.R * s.S * s.C * s.K + 3) / 4 * 4;
  return wf + conv_fwd_tiled_ws_floats(dgrad_fwd_shape(s), false);
}

// fp32 3x3 stride-1 halo conv (conv3f_kernel): block rows, channel-chunk split
// TiledPlan halo_f32_wide: 128-column tiles on 16-channel chunks where K allows
struct C3fPlan {
  int bm, bn, ch, z, cps;
  bool small;  // 64 x 64 on 16-channel chunks with a 288-row halo and a 3-deep ring
};
constexpr int C3F_SMALL_ROWS = 288;
static bool conv3f_plan(const ConvShape& s, C3fPlan& p) {
  using namespace tiled;
  if (!tiled_plan().halo_f32) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.OH == s.H && s.OW == s.W))
    return false;
  if (s.C % 32 || s.K % 64 || (long long)s.N * s.H * s.W * std::max(s.C, s.K) >= (1LL << 31))
    return false;
  const long long M = (long long)s.N * s.H * s.W;
  const bool wide = tiled_plan().halo_f32_wide && s.K % 128 == 0;
  p.bn = wide ? 128 : 64;
  p.ch = wide || tiled_plan().halo_f32_ch == 16 ? 16 : 32;
  const int nch = s.C / p.ch;
  // blocks launched with bm-row tiles (channel-chunk split-K below 512 tiles)
  auto grid = [&](int bm, int& z, int& cps) {
    const long long blocks = cdiv(M, bm) * (s.K / p.bn);
    z = 1;
    if (blocks < 512) z = (int)std::min<long long>(nch, cdiv(ksplit_target(), blocks));
    cps = cdiv(nch, z);
    z = cdiv(nch, cps);
    return blocks * z;
  };
  // block rows (TiledPlan halo_f32_bm; 0 = auto): 128 when that launches at
  // least as many blocks as 64 without adding a split-K 64 does not need (the
  // 14x14 layer: the same split count, fewer halo re-reads: conv_lab 88.5 ->
  // 80.2 us), else 64 (the 56x56 layer would fill under one round of four
  // blocks a CU, the 7x7 one gets fewer blocks, the 28x28 one a split for
  // nothing: 88.5 vs 89.3 us; r6_s29.steps)
  int z64, c64, z128, c128;
  const long long b64 = grid(64, z64, c64), b128 = grid(128, z128, c128);
  const int want = tiled_plan().halo_f32_bm;
  p.bm = want == 128 || (want == 0 && b128 >= b64 && (z64 > 1 || z128 == 1)) ? 128 : 64;
  if (h3f::halo_rows(s, p.bm) > h3f::HCAP) p.bm = 64;
  if (h3f::halo_rows(s, p.bm) > h3f::HCAP) return false;
  p.z = p.bm == 128 ? z128 : z64;
  p.cps = p.bm == 128 ? c128 : c64;
  // TiledPlan halo_f32_small: 30.5 KiB of LDS, five blocks a CU instead of four
  p.small = tiled_plan().halo_f32_small && p.bm == 64 && p.bn == 64 && p.ch == 16 &&
            h3f::halo_rows(s, 64) <= C3F_SMALL_ROWS;
  return true;
}
bool conv3f_ok(const ConvShape& s) {
  C3fPlan p;
  return conv3f_plan(s, p);
}
long long conv3f_ws_floats(const ConvShape& s) {
  C3fPlan p;
  if (!conv3f_plan(s, p) || p.z == 1) return 0;
  return (long long)p.z * s.N * s.H * s.W * s.K;
}
// wt: [9][K][C] read at tap 8 - t (see conv3f_kernel)
void conv3f(const ConvShape& s, const float* x, const float* wt, float* y, float* ws,
            hipStream_t st, const float* addend) {
  using namespace tiled;
  C3fPlan p;
  if (!conv3f_plan(s, p)) throw std::runtime_error("conv3f: unsupported shape");
  if (p.z > 1 && !ws) throw std::runtime_error("conv3f: split-K needs a workspace");
  const long long M = (long long)s.N * s.H * s.W;
  float* out = p.z > 1 ? ws : y;
  const float* add = p.z > 1 ? nullptr : addend;
  const dim3 grid(cdiv(M, p.bm) * (s.K / p.bn), p.z);
#define C3F(BM_, BN_, CH_) conv3f_kernel<BM_, BN_, 4, CH_><<<grid, NT, 0, st>>>(s, x, wt, out, p.cps, add)
  if (p.bn == 128) {
    if (p.bm == 128)
      C3F(128, 128, 16);
    else
      C3F(64, 128, 16);
  } else if (p.small) {
    conv3f_kernel<64, 64, 3, 16, C3F_SMALL_ROWS><<<grid, NT, 0, st>>>(s, x, wt, out, p.cps, add);
  } else if (p.ch == 16) {  // 64-byte rows: 38 KiB of LDS, four blocks a CU
    if (p.bm == 128)
      C3F(128, 64, 16);
    else
      C3F(64, 64, 16);
  } else if (p.bm == 128) {
    C3F(128, 64, 32);
  } else {
    C3F(64, 64, 32);
  }
#undef C3F
  if (p.z > 1) slab_sum(ws, p.z, M * s.K, y, st, addend);
}

// fp32 3x3 stride-2 dgrad on the halo kernel (dgrad3s2f_kernel): 64 x 64 tiles
// on 16-channel chunks (38 KiB of LDS), channel-chunk split-K below 512 tiles
struct D3s2fPlan {
  int z, cps;
};
static bool dgrad3s2f_plan(const ConvShape& s, D3s2fPlan& p) {
  using namespace tiled;
  if (!tiled_plan().halo_f32_s2) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.H == 2 * s.OH && s.W == 2 * s.OW))
    return false;
  if (s.C % 64 || s.K % 16 || (long long)s.N * s.H * s.W * std::max(s.C, s.K) >= (1LL << 31))
    return false;
  if (((64 + s.OW - 2) / s.OW + 2) * s.OW > h3f::HCAP) return false;  // halo rows
  const long long blocks = cdiv((long long)s.N * s.OH * s.OW, 64) * (s.C / 64);
  const int nch = s.K / 16;
  const int target = tiled_plan().ksplit_s2 > 0 ? tiled_plan().ksplit_s2 : ksplit_target();
  p.z = 1;
  if (blocks < 512) p.z = (int)std::min<long long>(nch, cdiv(target, blocks));
  p.cps = cdiv(nch, p.z);
  p.z = cdiv(nch, p.cps);
  return true;
}
static long long dgrad3s2f_ws_floats(const ConvShape& s) {
  D3s2fPlan p;
  if (!dgrad3s2f_plan(s, p) || p.z == 1) return 0;
  return (long long)p.z * s.N * s.H * s.W * s.C;
}

// workspace for either operand precision (the plans differ in tile shape)
long long conv_fwd_tiled_ws_floats(const ConvShape& s, bool epilogue) {
  long long n = conv3f_ws_floats(s);
  for (const bool b : {false, true}) {
    tiled::Tile t;
    int z, kps;
    tiled::fwd_plan(s, epilogue, b, t, z, kps);
    if (z > 1) n = std::max(n, (long long)z * s.N * s.OH * s.OW * s.K);
  }
  return n;
}

long long conv_bwd_data_tiled_ws_floats(const ConvShape& s) {
  long long n = dgrad_fwd_ok(s) ? dgrad_fwd_ws_floats(s) : 0;
  n = std::max(n, dgrad3s2f_ws_floats(s));
  if (dgrad_fwd_ok(s)) n = std::max(n, conv3f_ws_floats(dgrad_fwd_shape(s)));
  for (const bool b : {false, true}) {
    tiled::Tile t;
    int z, kps;
    tiled::data_plan(s, b, t, z, kps);
    if (z > 1) n = std::max(n, (long long)z * s.N * s.H * s.W * s.C);
  }
  return n;
}

int conv_fwd_tiled_stats_rows(const ConvShape& s, bool bf16) {
  using namespace tiled;
  const long long M = (long long)s.N * s.OH * s.OW;
  Tile t;
  int z, kps;
  fwd_plan(s, false, bf16, t, z, kps);
  return z > 1 ? (int)slab_grid(M * s.K) : cdiv(M, tile_m(t)) * 2;
}

static void conv_fwd_tiled_impl(const ConvShape& s, const float* x, const float* w,
                                const float* bias, float* y, bool relu, float* ws,
                                hipStream_t st, bool bf16, const ConvStats* stats,
                                const float* addend);

void conv_fwd_tiled(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
                    bool relu, float* ws, hipStream_t st, bool bf16, const ConvStats* stats) {
  conv_fwd_tiled_impl(s, x, w, bias, y, relu, ws, st, bf16, stats, nullptr);
}

static void conv_fwd_tiled_impl(const ConvShape& s, const float* x, const float* w,
                                const float* bias, float* y, bool relu, float* ws,
                                hipStream_t st, bool bf16, const ConvStats* stats,
                                const float* addend) {
  using namespace tiled;
  const long long M = (long long)s.N * s.OH * s.OW;
  Tile t;
  int z, kps;
  fwd_plan(s, bias != nullptr || relu, bf16, t, z, kps);
  if (z > 1 && !ws) throw std::runtime_error("conv_fwd_tiled: split-K needs a workspace");
  ConvStats cs;
  if (stats && stats->part) {
    if (bias || relu || s.K % 64 || 256 % (s.K / 4) ||
        stats->P != conv_fwd_tiled_stats_rows(s, bf16))
      throw std::runtime_error("conv_fwd_tiled: BatchNorm statistics layout mismatch");
    if (z == 1) cs = *stats;
  }
  float* out = z > 1 ? ws : y;
#define GRID(BM_, BN_) dim3(cdiv(M, BM_) * cdiv(s.K, BN_), z)
  if (s.C % BK != 0) {  // gather loader (fp32 operands only)
    if (bf16) throw std::runtime_error("conv_fwd_tiled: the gather forward is fp32");
#define F32G F32, true
    TILED_DISPATCH_P(F32G, t, fwd_kernel, GRID, s, x, w, bias, out, relu ? 1 : 0, kps, cs,
                     z > 1 ? nullptr : addend)
#undef F32G
  } else {
    TILED_DISPATCH(t, fwd_kernel, GRID, s, x, w, bias, out, relu ? 1 : 0, kps, cs,
                   z > 1 ? nullptr : addend)
  }
#undef GRID
  if (z > 1) {
    if (addend && stats && stats->part)
      throw std::runtime_error("conv_fwd_tiled: statistics with an addend");
    if (stats && stats->part)
      slab_sum4_stats_kernel<<<(int)slab_grid(M * s.K), 256, 0, st>>>(
          reinterpret_cast<const float4*>(ws), z, M * s.K / 4, reinterpret_cast<float4*>(y),
          *stats, s.K);
    else
      slab_sum(ws, z, M * s.K, y, st, addend);
  }
}

void conv_bwd_data_tiled(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                         hipStream_t st, bool bf16, const float* addend, const void* dyb,
                         const float* wflip) {
  using namespace tiled;
  if (!bf16 && dy && ws && dgrad_fwd_ok(s)) {
    const ConvShape f = dgrad_fwd_shape(s);
    if (conv3f_ok(f)) {  // the halo kernel reads W itself, taps reversed (conv3f_kernel)
      conv3f(f, dy, w, dx, ws, st, addend);
      return;
    }
    float* fws = ws + ((long long)s.R * s.S * s.C * s.K + 3) / 4 * 4;
    const float* wt = wflip;  // kept current by the step's SGD (gops::sgd_wcvt)
    if (!wt) {
      wflip_kernel<<<dim3(cdiv(s.K, 32), cdiv(s.C, 32), s.R * s.S), 256, 0, st>>>(w, ws, s.R, s.S,
                                                                                 s.C, s.K);
      wt = ws;
    }
    conv_fwd_tiled_impl(f, dy, wt, nullptr, dx, false, fws, st, false, nullptr, addend);
    return;
  }
  D3s2fPlan dp;
  if (!bf16 && dy && dgrad3s2f_plan(s, dp)) {
    if (dp.z > 1 && !ws) throw std::runtime_error("dgrad3s2f: split-K needs a workspace");
    const dim3 grid(cdiv((long long)s.N * s.OH * s.OW, 64) * (s.C / 64), dp.z);
    dgrad3s2f_kernel<64, 64, 4, 16><<<grid, NT, 0, st>>>(s, dy, w, dp.z > 1 ? ws : dx, dp.cps,
                                                         dp.z > 1 ? nullptr : addend);
    if (dp.z > 1) slab_sum(ws, dp.z, (long long)s.N * s.H * s.W * s.C, dx, st, addend);
    return;
  }
  const int sd = s.stride;
  const long long Mph = (long long)s.N * ((s.H + sd - 1) / sd) * ((s.W + sd - 1) / sd);
  Tile t;
  int z, kps;
  data_plan(s, bf16, t, z, kps);
  if (z > 1 && !ws) throw std::runtime_error("conv_bwd_data_tiled: split-K needs a workspace");
  float* out = z > 1 ? ws : dx;
  // phases no tap reaches (odd pixels of a 1x1 stride-2 conv) run zero K
  // tiles and write zeros
#define GRID(BM_, BN_) dim3(cdiv(Mph, BM_) * cdiv(s.C, BN_), sd * sd, z)
  if (!dy && dyb) {  // dY only as bf16: bf16 loads, converted in registers
    const __bf16* d16 = reinterpret_cast<const __bf16*>(dyb);
    TILED_DISPATCH(t, data_b16_kernel, GRID, s, d16, w, out, kps, z > 1 ? nullptr : addend)
  } else {
    TILED_DISPATCH(t, data_kernel, GRID, s, dy, w, out, kps, z > 1 ? nullptr : addend)
  }
#undef GRID
  if (z > 1) slab_sum(ws, z, (long long)s.N * s.H * s.W * s.C, dx, st, addend);
}

namespace tiled {
static inline Tile filter_tile(const ConvShape& s) {  // ci x co tiles
  // 64-wide ci tiles: ResNet-18 fp32 filter gradients 136 -> 122 (28x28), 112 -> 103
  // (14x14), 116 -> 102 us (7x7), step 6.96 -> 6.78 ms; twice the tiles, so half
  // the split-K slices (the bf16 models take the conv_bf16 filter kernels).
  // TiledPlan wg64 = false: 128-wide ci tiles from C >= 128 (the old plan)
  const bool bm = s.C >= 128 && !tiled_plan().wg64, bn = s.K > 64 && !tiled_plan().wg_n64;
  return bm ? (bn ? T128x128 : T128x64) : (bn ? T64x128 : T64x64);
}
static inline int filter_blocks_per_split(const ConvShape& s) {
  const Tile t = filter_tile(s);
  const int BM = (t == T128x128 || t == T128x64) ? 128 : 64;
  const int BN = (t == T128x128 || t == T64x128) ? 128 : 64;
  return cdiv(s.C, BM) * cdiv(s.K, BN) * s.R * s.S;
}
}  // namespace tiled

namespace tiled {
// slices launched (padded to a multiple of 8 for the XCD order) and the K
// tiles of each
static int filter_splits(const ConvShape& s, int& kchunk) {
  const int ktiles = cdiv((long long)s.N * s.OH * s.OW, BK);
  const bool vec = s.C % 4 == 0;
  const int tiles = vec ? filter_blocks_per_split(s) : cdiv(s.R * s.S * s.C, 64) * cdiv(s.K, 64);
  // blocks to aim for (TiledPlan wgsplit_target).  With the walked pixel
  // coordinates (PixWalk) fewer, longer slices pay: ResNet-18 fp32 filter
  // gradients in conv_lab 1934 / 1805 / 1836 / 1901 us a step at 2048 / 1024 /
  // 768 / 512 blocks, the full step 5.69 / 5.75 / 5.65 ms at 2048 / 1024 / 768
  // (r6_s26 / r6_s27.steps, two runs each); with the halo convs on 16-channel
  // chunks and the stride-2 halo dgrad the order changed: 5.50 / 5.46 / 5.58 ms
  // at 768 / 1024 / 640 (r6_s32.steps), so 1024
  int z = cdiv(wgsplit_target(), tiles);
  if (z < 1) z = 1;
  if (z > ktiles) z = ktiles;
  // gather-path slice cap: the ResNet stem's filter gradient (3 tiles of 64 x 64,
  // 12544 K tiles) went 271 -> 197 us from 128 to 256 slices (512: 196, 1024: 198)
  const int gcap = tiled_plan().gcap;
  // vector-path slice cap (TiledPlan vcap).  conv_lab fp32: the 56x56x64 filter
  // gradient (9 tiles) 152.2 -> 132.3 -> 120.8 us at caps 64 -> 128 -> 256 (all
  // layers 2076 -> 1994 / 1979 us); ResNet-18 fp32 step 5.93 -> 5.845 / 5.82 ms
  // (r6_s22.steps, two runs each), so 256
  const int vcap = tiled_plan().vcap;
  if (z > (vec ? vcap : gcap)) z = vec ? vcap : gcap;
  kchunk = cdiv(ktiles, z);
  const int zr = cdiv(ktiles, kchunk);
  // XCD-aware slice order (xcd_slice_bid) wants a multiple of 8 slices: the
  // padding slices have no pixels and write zero slabs
  if (tiled_plan().wg_xcd && zr > 8) return (zr + 7) / 8 * 8;
  return zr;
}
}  // namespace tiled

int conv_filter_tiled_splits(const ConvShape& s) {
  int kchunk;
  return tiled::filter_splits(s, kchunk);
}

void conv_bwd_filter_tiled(const ConvShape& s, const float* x, const float* dy, float* part,
                           float* dw, hipStream_t st, bool bf16) {
  using namespace tiled;
  int kchunk;
  const int z = filter_splits(s, kchunk);
  const bool xcd = tiled_plan().wg_xcd;
  const int taps = s.R * s.S;
  if (s.C % 4 != 0) {  // (tap, ci) gather rows, 64x64 tiles
    const int Mw = taps * s.C;
    if (bf16)
      filter_gather_kernel<64, 64, BF16><<<cdiv(Mw, 64) * cdiv(s.K, 64) * z, NT, 0, st>>>(
          s, x, dy, z == 1 ? dw : part, kchunk, xcd);
    else
      filter_gather_kernel<64, 64, F32><<<cdiv(Mw, 64) * cdiv(s.K, 64) * z, NT, 0, st>>>(
          s, x, dy, z == 1 ? dw : part, kchunk, xcd);
    if (z > 1) slab_sum(part, z, (long long)Mw * s.K, dw, st);
    return;
  }
  const Tile t = filter_tile(s);
#define GRID(BM_, BN_) dim3(cdiv(s.C, BM_) * cdiv(s.K, BN_) * taps * z)
  // 16-pixel K tiles (the same slices in twice the tiles): 64 x 128 in 24 KiB of
  // LDS, five blocks a CU instead of three - filter gradients 1806 -> 1773 us a
  // step, ResNet-18 fp32 5.412 / 5.413 -> 5.379 / 5.387 ms (r6_s43.steps)
  if (!bf16 && t == T64x128 && tiled_plan().wg_bk16) {
    filter_kernel<64, 128, F32, 16><<<GRID(64, 128), NT, 0, st>>>(s, x, dy, z == 1 ? dw : part,
                                                                 2 * kchunk, xcd);
  } else if (!bf16 && t == T64x64 && tiled_plan().wg_bk16_64) {
    filter_kernel<64, 64, F32, 16><<<GRID(64, 64), NT, 0, st>>>(s, x, dy, z == 1 ? dw : part,
                                                               2 * kchunk, xcd);
  } else {
    TILED_DISPATCH(t, filter_kernel, GRID, s, x, dy, z == 1 ? dw : part, kchunk, xcd)
  }
#undef GRID
  if (z > 1) slab_sum(part, z, (long long)taps * s.C * s.K, dw, st);
}

}  // namespace gops
