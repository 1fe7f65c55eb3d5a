// Generic LDS-tiled fp32 MFMA GEMM tile engine for gfx950.
//
// One workgroup computes a BM x BN output tile (BM = 32*WM, BN = 32*WN) over
// the K range [k_begin, k_end) with WM*WN*WK waves:
//   * wave (wm, wn, wk) owns the 32x32 sub-tile (wm, wn) and the K slice
//     kk in [wk*BK/WK, (wk+1)*BK/WK) of every staged K tile;
//   * operands are gathered from global memory by the problem's functors
//     (implicit GEMM: im2col, transposes, pooling-aware row orders and zero
//     padding live in the functor and are never materialised).  Each thread
//     gathers a FIXED set of (row, k-in-tile) slots for every K tile, so the
//     expensive part of the address (pixel decode, bounds) is computed ONCE
//     per slot into a context (`a_ctx`/`b_ctx`) before the K loop; the per
//     tile `a_get`/`b_get` only adds the tile's uniform K offset;
//   * the next K tile is fetched into registers while the MFMAs run on the
//     current one (issue-early / write-late, cdna_hip_programming.md T14),
//     into a double-buffered LDS image As[k][m] / Bs[k][n] (+1 float row pad:
//     conflict-free staging writes and MFMA operand reads), ONE barrier per
//     K tile;
//   * K-split partial accumulators (WK > 1) are summed through LDS and the
//     owner wave (wk == 0) returns the 32x32 tile in the MFMA C/D layout.
//
// Math: v_mfma_f32_32x32x2_f32 = exact fp32 products, fp32 accumulation in
// K order (cdna_hip_programming.md §3 "FP32-input MFMA").
#pragma once

#include "common.h"

namespace gemm {

// A_KC: consecutive threads walk K when gathering A (A stored K-contiguous);
// otherwise they walk M.  B_NC: consecutive threads walk N for B; otherwise K.
template <int WM, int WN, int WK, int BK, bool A_KC, bool B_NC>
struct Cfg {
  static constexpr int BM = 32 * WM;
  static constexpr int BN = 32 * WN;
  static constexpr int NW = WM * WN * WK;
  static constexpr int NT = 64 * NW;
  static constexpr int LDA = BM + 1;
  static constexpr int LDB = BN + 1;
  static constexpr int RA = BM * BK / NT;  // A slots per thread
  static constexpr int RB = BK * BN / NT;
  static constexpr int STAGE_FLOATS = BK * LDA + BK * LDB;
  static constexpr int SMEM_FLOATS_TILE = 2 * STAGE_FLOATS;
  static constexpr int SMEM_FLOATS_RED = (WK > 1) ? (WK - 1) * WM * WN * 64 * 16 : 0;
  static constexpr int SMEM_FLOATS =
      SMEM_FLOATS_TILE > SMEM_FLOATS_RED ? SMEM_FLOATS_TILE : SMEM_FLOATS_RED;
  static constexpr int SMEM_BYTES = SMEM_FLOATS * 4;
  static_assert(BK % 32 == 0, "BK must be a multiple of 32");
  static_assert(BM * BK % NT == 0 && BK * BN % NT == 0, "tile not divisible by threads");
  static_assert(BK % (2 * WK) == 0, "K slice per wave must be a multiple of 2");
  static_assert(!A_KC || NT % 32 == 0, "A_KC mapping");
  static_assert(A_KC || NT % BM == 0, "A_MC mapping needs NT % BM == 0");
  static_assert(B_NC ? NT % BN == 0 : NT % 32 == 0, "B mapping");

  // slot -> (m_local, k_local) for A, (k_local, n_local) for B
  __device__ static __forceinline__ void a_slot(int tid, int i, int& ml, int& kl) {
    const int e = tid + i * NT;
    if (A_KC) {
      kl = e % 32 + (e / (32 * BM)) * 32;
      ml = (e / 32) % BM;
    } else {
      ml = e % BM;
      kl = e / BM;
    }
  }
  __device__ static __forceinline__ void b_slot(int tid, int i, int& kl, int& nl) {
    const int e = tid + i * NT;
    if (B_NC) {
      nl = e % BN;
      kl = e / BN;
    } else {
      kl = e % 32 + (e / (32 * BN)) * 32;
      nl = (e / 32) % BN;
    }
  }
};

// Runs the tile.  Returns true on the owner wave (wk == 0); `acc` then holds
// the full-K result of sub-tile (wm, wn): register r of lane l is element
// (m0 + 32*wm + mfma32_row(r, l), n0 + 32*wn + (l & 31)).
// Requires (k_end - k_begin) % BK == 0 (problems zero-fill past their K).
template <int WM, int WN, int WK, int BK, class Prob>
__device__ __forceinline__ bool run_tile(const Prob& p, float* smem, int m0, int n0, int k_begin,
                                         int k_end, f32x16& acc, int& wm, int& wn) {
  using CF = Cfg<WM, WN, WK, BK, Prob::A_KC, Prob::B_NC>;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  wm = wave % WM;
  wn = (wave / WM) % WN;
  const int wk = wave / (WM * WN);

  typename Prob::ACtx ac[CF::RA];
  typename Prob::BCtx bc[CF::RB];
  int a_off[CF::RA], b_off[CF::RB];
#pragma unroll
  for (int i = 0; i < CF::RA; ++i) {
    int ml, kl;
    CF::a_slot(tid, i, ml, kl);
    ac[i] = p.a_ctx(m0 + ml, kl);
    a_off[i] = kl * CF::LDA + ml;
  }
#pragma unroll
  for (int i = 0; i < CF::RB; ++i) {
    int kl, nl;
    CF::b_slot(tid, i, kl, nl);
    bc[i] = p.b_ctx(kl, n0 + nl);
    b_off[i] = kl * CF::LDB + nl;
  }

  acc = zero16();
  float ra[CF::RA];
  float rb[CF::RB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < CF::RA; ++i) ra[i] = p.a_get(ac[i], k0);
#pragma unroll
    for (int i = 0; i < CF::RB; ++i) rb[i] = p.b_get(bc[i], k0);
  };
  auto store = [&](int buf) {
    float* As = smem + buf * CF::STAGE_FLOATS;
    float* Bs = As + BK * CF::LDA;
#pragma unroll
    for (int i = 0; i < CF::RA; ++i) As[a_off[i]] = ra[i];
#pragma unroll
    for (int i = 0; i < CF::RB; ++i) Bs[b_off[i]] = rb[i];
  };

  int cur = 0;
  if (k_begin < k_end) {
    load(k_begin);
    store(0);
  }
  __syncthreads();
  constexpr int KS = BK / WK;
  const int khalf = lane >> 5;
  for (int k0 = k_begin; k0 < k_end; k0 += BK) {
    const bool more = k0 + BK < k_end;
    if (more) load(k0 + BK);
    const float* As = smem + cur * CF::STAGE_FLOATS;
    const float* Aw = As + wm * 32 + (lane & 31) + (wk * KS + khalf) * CF::LDA;
    const float* Bw = As + BK * CF::LDA + wn * 32 + (lane & 31) + (wk * KS + khalf) * CF::LDB;
#pragma unroll
    for (int kk = 0; kk < KS; kk += 2) acc = mfma32x32x2(Aw[kk * CF::LDA], Bw[kk * CF::LDB], acc);
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  if constexpr (WK > 1) {
    float* red = smem;  // tile buffers are dead after the final barrier
    const int sub = wm + WM * wn;
    if (wk > 0) {
      float* dst = red + (((wk - 1) * WM * WN + sub) * 16) * 64 + lane;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64] = acc[r];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int g = 1; g < WK; ++g) {
        const float* src = red + (((g - 1) * WM * WN + sub) * 16) * 64 + lane;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += src[r * 64];
      }
    }
    return wk == 0;
  } else {
    return true;
  }
}

// One-shot variant for short K ranges (KT = (k_end-k_begin)/BK tiles, known at
// compile time): EVERY K tile of the block is gathered into LDS up front (all
// global loads in flight together, one barrier), then the MFMAs run without
// further synchronisation.  Trades LDS (KT stage buffers) for the serial
// per-tile latency chain of run_tile - the right shape for the small-M FC
// GEMMs of the MNIST step (K per block 224..512).
template <int WM, int WN, int WK, int BK, int KT, class Prob>
__device__ __forceinline__ bool run_tile_oneshot(const Prob& p, float* smem, int m0, int n0,
                                                 int k_begin, f32x16& acc, int& wm, int& wn) {
  using CF = Cfg<WM, WN, WK, BK, Prob::A_KC, Prob::B_NC>;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  wm = wave % WM;
  wn = (wave / WM) % WN;
  const int wk = wave / (WM * WN);
  {
    float ra[KT][CF::RA];
    float rb[KT][CF::RB];
#pragma unroll
    for (int i = 0; i < CF::RA; ++i) {
      int ml, kl;
      CF::a_slot(tid, i, ml, kl);
      const auto c = p.a_ctx(m0 + ml, kl);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) ra[kt][i] = p.a_get(c, k_begin + kt * BK);
    }
#pragma unroll
    for (int i = 0; i < CF::RB; ++i) {
      int kl, nl;
      CF::b_slot(tid, i, kl, nl);
      const auto c = p.b_ctx(kl, n0 + nl);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) rb[kt][i] = p.b_get(c, k_begin + kt * BK);
    }
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      float* As = smem + kt * CF::STAGE_FLOATS;
      float* Bs = As + BK * CF::LDA;
#pragma unroll
      for (int i = 0; i < CF::RA; ++i) {
        int ml, kl;
        CF::a_slot(tid, i, ml, kl);
        As[kl * CF::LDA + ml] = ra[kt][i];
      }
#pragma unroll
      for (int i = 0; i < CF::RB; ++i) {
        int kl, nl;
        CF::b_slot(tid, i, kl, nl);
        Bs[kl * CF::LDB + nl] = rb[kt][i];
      }
    }
  }
  __syncthreads();
  acc = zero16();
  constexpr int KS = BK / WK;
  const int khalf = lane >> 5;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const float* As = smem + kt * CF::STAGE_FLOATS;
    const float* Aw = As + wm * 32 + (lane & 31) + (wk * KS + khalf) * CF::LDA;
    const float* Bw = As + BK * CF::LDA + wn * 32 + (lane & 31) + (wk * KS + khalf) * CF::LDB;
#pragma unroll
    for (int kk = 0; kk < KS; kk += 2) acc = mfma32x32x2(Aw[kk * CF::LDA], Bw[kk * CF::LDB], acc);
  }
  if constexpr (WK > 1) {
    __syncthreads();
    float* red = smem;
    const int sub = wm + WM * wn;
    if (wk > 0) {
      float* dst = red + (((wk - 1) * WM * WN + sub) * 16) * 64 + lane;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64] = acc[r];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int g = 1; g < WK; ++g) {
        const float* src = red + (((g - 1) * WM * WN + sub) * 16) * 64 + lane;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += src[r * 64];
      }
    }
    return wk == 0;
  } else {
    return true;
  }
}

// ------------------------------------------------- plain matrix operands ----
// A row-major [M][lda] walked along K (A_KC) with rows >= M reading zero.
struct RowMajorA {
  struct Ctx {
    const float* p;
    bool v;
  };
  const float* a;
  int lda, M;
  __device__ __forceinline__ Ctx ctx(int m, int kl) const {
    return {a + (size_t)(m < M ? m : 0) * lda + kl, m < M};
  }
  __device__ __forceinline__ float get(const Ctx& c, int k0) const {
    const float v = c.p[k0];  // always a valid address (row clamped to 0)
    return c.v ? v : 0.f;
  }
};

}  // namespace gemm
