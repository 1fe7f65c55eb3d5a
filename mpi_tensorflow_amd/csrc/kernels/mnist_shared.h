// Device helpers and constants shared by the fp32 (mnist.hip) and bf16
// (mnist_bf16.hip) MNIST kernel sets.
#pragma once
#include "common.h"
#include "mnist.h"

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
// dlog, db3 = sum dh.  Block blk owns hidden units [64 blk, 64 blk + 64); its
// 4 waves take every 4th row.  dlog is staged in LDS 64 rows at a time (one
// coalesced pass; the rows are then LDS broadcasts): read straight from
// global memory they were 80 dependent broadcast loads per 8 rows (8.2 us
// for the role alone).  Row order per thread: rg, rg + 4, rg + 8, ...
constexpr int FC1_SMALL_SMEM = 64 * NCLS + 4 * (NCLS + 1) * 64;  // floats
__device__ __forceinline__ void fc1_small_grads(int blk, const float* hd, const float* dh,
                                                const float* dlog, int batch, float* g_w4,
                                                float* g_b4, float* g_b3, float* smem) {
  const int tid = threadIdx.x, jl = tid & 63, rg = tid >> 6;
  const int j = blk * 64 + jl;
  float* dl = smem;              // [64][NCLS]: this chunk's dlog rows
  float* s = smem + 64 * NCLS;   // [4][NCLS + 1][64]: row-group partials
  float acc[NCLS + 1];
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) acc[c] = 0.f;
  for (int r0 = 0; r0 < batch; r0 += 64) {
    const int rows = min(64, batch - r0);
    float hv[16], dv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int n = min(r0 + rg + 4 * u, batch - 1);
      hv[u] = hd[(size_t)n * FC1_OUT + j];
      dv[u] = dh[(size_t)n * FC1_OUT + j];
    }
    if (r0 > 0) __syncthreads();  // the previous chunk's rows are consumed
    for (int i = tid; i < rows * NCLS; i += 256) dl[i] = dlog[(size_t)r0 * NCLS + i];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = rg + 4 * u;
      if (r < rows) {
#pragma unroll
        for (int c = 0; c < NCLS; ++c) acc[c] += hv[u] * dl[r * NCLS + c];
        acc[NCLS] += dv[u];
      }
    }
  }
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
  if (blk == 0 && tid < 64) {  // db4: rows strided over the wave, all loads in flight
    float v[NCLS];
#pragma unroll
    for (int c = 0; c < NCLS; ++c) v[c] = 0.f;
    for (int n = tid; n < batch; n += 64) {
#pragma unroll
      for (int c = 0; c < NCLS; ++c) v[c] += dlog[n * NCLS + c];
    }
#pragma unroll
    for (int c = 0; c < NCLS; ++c) {
      const float t = wave_sum(v[c]);
      if (tid == 0) g_b4[c] = t;
    }
  }
}

// ------------------------------------------------ conv1 filter gradient ----
// Sparse: each pooled gradient reaches exactly one pre-pool pixel (its argmax),
// so dW1[t][co] = sum over pooled (n,py,px) of dA1m * x[argmax pixel + tap]
// (reference mpipy.py:155-157 conv1, B7).  Unit = (image, band of 14 / SPLIT
// pooled rows) -> one 832-float partial row part1[unit] (800 weights + 32
// biases); thread = (co, position group), NT / 32 groups.  All of a thread's
// (gradient, argmax) pairs are loaded up front (one latency round); the two
// groups of a wave are combined by a lane shuffle, the NT / 64 wave partials
// in a fixed order through LDS.  Run as its own 256-thread kernel or as the
// 512-thread role blocks appended to a conv2 filter-gradient launch: SPLIT = 7
// (pairs of pooled rows) where the conv2 part fills the chip, SPLIT = 1 (whole
// images: batch units) where the conv2 part leaves batch CUs free (Winograd).
constexpr int C1F_SPLIT = 7;  // default: pooled-row pairs per image (mnist.h)
template <int SPLIT, int NW = 8>
constexpr int c1f_smem() {  // floats for NW waves: image rows + wave partials
  return (2 * (14 / SPLIT) + 4) * 32 + NW * (26 * 32 + 1);
}
constexpr int C1F_SMEM = c1f_smem<C1F_SPLIT>();

struct C1Filter {  // conv1 filter-grad role arguments (part1 == nullptr: off)
  const float* data;
  const long long* step;
  int n_local;
  const float* da1m;
  const uint8_t* idx1;
  float* part1;
};

C1Filter c1_args(const C1FilterArgs* a);  // host (mnist.hip)

template <int NT, int SPLIT = C1F_SPLIT>
__device__ inline void conv1_filter_unit(int unit, int batch, const C1Filter& c, float* smem) {
  static_assert(14 % SPLIT == 0, "SPLIT divides the 14 pooled rows");
  constexpr int PR = 14 / SPLIT, POS = PR * 14, XR = 2 * PR + 4;
  constexpr int NG = NT / 32, PER_T = (POS + NG - 1) / NG, NW = NT / 64;  // smem: c1f_smem<SPLIT, NW>
  float* xs = smem;            // rows 2*PR*band-2 .. +XR-1 of the padded image
  float* red = smem + XR * 32;  // [NW][26 * 32 + 1]
  const int n = unit / SPLIT, band = unit % SPLIT;
  const long long off = batch_offset_dev(c.step, c.n_local, batch);
  const float* x = c.data + (off + n) * 784;
  const int tid = threadIdx.x, co = tid & 31, grp = tid >> 5, wave = tid >> 6;
  const int y0 = 2 * PR * band - 2;  // first image row held in xs
  for (int i = tid; i < XR * 32; i += NT) {
    const int yy = y0 + i / 32, xx = i % 32 - 2;
    xs[i] = (yy >= 0 && yy < 28 && xx >= 0 && xx < 28) ? x[yy * 28 + xx] : 0.f;
  }
  float v[PER_T];
  int q[PER_T];
#pragma unroll
  for (int j = 0; j < PER_T; ++j) {
    const int p = grp + NG * j;
    v[j] = 0.f;
    q[j] = 0;
    if (p < POS) {
      const int py = PR * band + p / 14, px = p % 14;
      const int e = ((n * 14 + py) * 14 + px) * 32 + co;
      v[j] = c.da1m[e];
      q[j] = c.idx1[e];
    }
  }
  __syncthreads();
  float acc[26];
#pragma unroll
  for (int t = 0; t < 26; ++t) acc[t] = 0.f;
#pragma unroll
  for (int j = 0; j < PER_T; ++j) {
    const int p = grp + NG * j;
    if (p < POS && v[j] != 0.f) {
      const int py = PR * band + p / 14, px = p % 14;
      const int ly = 2 * py + (q[j] >> 1) - y0 - 2;  // row in xs of tap kh = 0
      const int lx = 2 * px + (q[j] & 1);            // col in xs (padded by 2) of kw = 0
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc[kh * 5 + kw] += v[j] * xs[(ly + kh) * 32 + lx + kw];
      acc[25] += v[j];
    }
  }
#pragma unroll
  for (int t = 0; t < 26; ++t) acc[t] += __shfl_xor(acc[t], 32, 64);
  if ((tid & 32) == 0) {
#pragma unroll
    for (int t = 0; t < 26; ++t) red[wave * (26 * 32 + 1) + t * 32 + co] = acc[t];
  }
  __syncthreads();
  for (int i = tid; i < 26 * 32; i += NT) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w * (26 * 32 + 1) + i];
    c.part1[(size_t)unit * 832 + i] = s;
  }
}

// momentum SGD on 4 floats: g = gs g + lc w (rank-sum scale 1/N, L2);
// m = mu m + g; w -= lr m (the expression forms of optim::sgd_momentum_flat,
// so every SGD path of the step rounds identically)
__device__ __forceinline__ void sgd4(float4& wv, float4& mv, float4 gv, float lc, float lr,
                                     float mu, float gs = 1.f) {
  // explicit fma: the same rounding in every kernel that inlines this (a
  // free contraction of g * gs + lc * w may fuse either product)
  gv.x = __builtin_fmaf(lc, wv.x, gv.x * gs);
  gv.y = __builtin_fmaf(lc, wv.y, gv.y * gs);
  gv.z = __builtin_fmaf(lc, wv.z, gv.z * gs);
  gv.w = __builtin_fmaf(lc, wv.w, gv.w * gs);
  mv.x = mu * mv.x + gv.x;
  mv.y = mu * mv.y + gv.y;
  mv.z = mu * mv.z + gv.z;
  mv.w = mu * mv.w + gv.w;
  wv.x -= lr * mv.x;
  wv.y -= lr * mv.y;
  wv.z -= lr * mv.z;
  wv.w -= lr * mv.w;
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
static_assert(SHADOW_W1_BLOCKS % 2 == 0, "fc_sgd_role: unit pairs of a 512-thread block");
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

// ---------------------------------------------- world-1 FC SGD role ----
// Single-rank step: every FC gradient is final when fc1 backward ends, so the
// momentum SGD of the FC bucket (flat [0, n4) float4s, all of it under the L2
// term, reference mpipy.py:58-65) runs as extra blocks of the conv2 bwd-data
// launch that follows.  That kernel is MFMA / vector-L1 bound on 196 blocks
// and leaves ~60 CUs idle, which these HBM-streaming blocks fill; the SGD
// launch at the end of the step then only finishes the conv parameters.
struct FcSgd {
  float* w;
  const float* g;
  float* m;
  long long n4;  // float4s; 0 = role off
  float l2, mu;
  const float* lr;
  int nblk;  // extra blocks appended to the grid
  // bf16 engine, single rank: the fc1 weight's bf16 MFMA shadows (layouts of
  // shadow_block below) are written by the same threads that update it, so
  // the next step's conv1 launch only re-derives the small conv2 shadows.
  // fc1 weight = float4s [w1_off4, w1_off4 + W1_F4) of the bucket, updated in
  // SHADOW_W1_BLOCKS 64 x 64 tiles (LDS transpose for w1t); the other blocks
  // stream the rest of the bucket.
  __bf16* w1b;
  __bf16* w1t;
  long long w1_off4;
  float gs;  // gradient scale (1 / ranks: the bucket holds the rank sum)
  // fused fc1 weight gradient (FcSgdArgs::a2): the fc1 weight's float4s are
  // skipped by the streaming units and updated by fc1_dw_sgd tiles
  const float* a2;
  const float* dh;
  int batch;
};
constexpr int FC_SGD_UNROLL = 4;
constexpr long long W1_F4 = (long long)FC1_IN * FC1_OUT / 4;
FcSgd fc_sgd_args(const FcSgdArgs* a);  // host: role off when a == nullptr (mnist.hip)

// one 64 x 64 tile of the fc1 weight: momentum SGD + both bf16 shadows (tid:
// the thread's index in its 256-thread unit; every unit of a block runs one)
__device__ inline void fc_sgd_w1_tile(const FcSgd& a, int L, float lr, float* tile, int tid) {
  const int i0 = (L % (FC1_IN / 64)) * 64, j0 = (L / (FC1_IN / 64)) * 64;
  const int row = tid >> 2, ck = tid & 3;
  const size_t e0 = (size_t)a.w1_off4 * 4 + (size_t)(i0 + row) * FC1_OUT + j0 + 16 * ck;
  float4* W4 = reinterpret_cast<float4*>(a.w + e0);
  float4* M4 = reinterpret_cast<float4*>(a.m + e0);
  const float4* G4 = reinterpret_cast<const float4*>(a.g + e0);
  float4 wv[4], gv[4], mv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    wv[u] = W4[u];
    gv[u] = G4[u];
    mv[u] = M4[u];
  }
  float v[16];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    sgd4(wv[u], mv[u], gv[u], a.l2, lr, a.mu, a.gs);
    W4[u] = wv[u];
    M4[u] = mv[u];
    v[4 * u] = wv[u].x;
    v[4 * u + 1] = wv[u].y;
    v[4 * u + 2] = wv[u].z;
    v[4 * u + 3] = wv[u].w;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) tile[row * 65 + 16 * ck + e] = v[e];
  shadow_store16(a.w1b + ((size_t)((j0 >> 4) + ck) * FC1_IN + i0 + row) * 16, v);
  __syncthreads();
  const int col = tid >> 2;
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = tile[(16 * ck + e) * 65 + col];
  shadow_store16(a.w1t + ((size_t)((i0 >> 4) + ck) * FC1_OUT + j0 + col) * 16, v);
}

// blk: index among the role's blocks; tile: >= 64 x 65 floats of LDS (the
// unit's own) when a.w1b is set
// tid: the thread's index in its 256-thread unit (a 512-thread block runs two
// units; with a.w1b the two take the same path - SHADOW_W1_BLOCKS is even - so
// the tile path's barrier is met by both)
__device__ __forceinline__ void fc_sgd_role(const FcSgd& a, int blk, float* tile,
                                   int tid = (int)threadIdx.x) {
  float4* W4 = reinterpret_cast<float4*>(a.w);
  float4* M4 = reinterpret_cast<float4*>(a.m);
  const float4* G4 = reinterpret_cast<const float4*>(a.g);
  const float lr = *a.lr;
  long long n4 = a.n4;
  int nb = a.nblk;
  if (a.w1b) {
    if (blk < SHADOW_W1_BLOCKS) {
      fc_sgd_w1_tile(a, blk, lr, tile, tid);
      return;
    }
    blk -= SHADOW_W1_BLOCKS;
    nb -= SHADOW_W1_BLOCKS;
    n4 -= W1_F4;  // the rest of the bucket, the fc1 weight's float4s skipped
  }
  if (a.a2) n4 -= W1_F4;  // the fc1 weight: fc1_dw_sgd tiles
  const bool skip = a.w1b || a.a2;
  const long long stride = (long long)nb * 256;
  auto at = [&](long long f) { return (skip && f >= a.w1_off4) ? f + W1_F4 : f; };
  // U float4s per thread per round, every load of a round in flight together
  for (long long i0 = (long long)blk * 256 + tid; i0 < n4; i0 += stride * FC_SGD_UNROLL) {
    float4 wv[FC_SGD_UNROLL], gv[FC_SGD_UNROLL], mv[FC_SGD_UNROLL];
#pragma unroll
    for (int u = 0; u < FC_SGD_UNROLL; ++u) {
      const long long i = at(min(i0 + u * stride, n4 - 1));
      wv[u] = W4[i];
      gv[u] = G4[i];
      mv[u] = M4[i];
    }
#pragma unroll
    for (int u = 0; u < FC_SGD_UNROLL; ++u) {
      if (i0 + u * stride < n4) {
        const long long i = at(i0 + u * stride);
        sgd4(wv[u], mv[u], gv[u], a.l2, lr, a.mu, a.gs);
        W4[i] = wv[u];
        M4[i] = mv[u];
      }
    }
  }
}

}  // namespace mnist
