// Fused fp32 HIP kernel set for the reference MNIST CNN on gfx950.
//
// Reference graph (/root/reference/mpipy.py:155-167, loss :54-58, optimizer
// :59-66) and the TF ops each kernel replaces (SURVEY.md §2.4 F1-F12, B1-B7,
// U1-U2, E1-E2):
//
//   conv_pool_fwd<conv1>   F1-F3  conv5x5(1->32)+bias+ReLU+maxpool2 (+argmax)
//   fc1_fwd                F8     3136x512 GEMM, split-K partial slabs (train)
//                                 or bias+ReLU(+dropout) epilogue (eval)
//   fc_head                F8-F11, B1  split-K reduce, bias, ReLU, dropout,
//                                 fc2, softmax-xent, dlogits, dhidden
//   fc1_bwd                B1-B4  roles: dW1 (=a2^T dh), dX (=dh W1^T with the
//                                 pool2/ReLU2 backward scatter fused), dW2/db
//   conv2_fwd_v3           F4-F6  conv2 from an LDS halo tile (+W2 transpose)
//   conv2_bwd_data_l2      B6     L2-direct bwd-data over the channel-major
//                                 dY2 image (ReLU1 mask fused)
//   conv2_bwd_filter       B5     bwd-filter with L2-direct NHWC operands
//                                 (+db2 on the centre tap)
//   conv1_bwd_filter       B7     sparse VALU filter grad through pool1 argmax
//   grad_finalize          B2     deterministic slab reduction
//   fc_head_eval           E1-E2  logits, argmax, on-device error count
//
// Activations are NHWC fp32, weights keep the TF layouts (HWIO, [in, out]).
// Every GEMM-shaped op runs on v_mfma_f32_32x32x2_f32 through gemm_core.h.
#include <stdexcept>
#include <type_traits>
#include <string>

#include "common.h"
#include "gemm_core.h"
#include "mnist.h"
#include "mnist_shared.h"
#include "wino.h"

namespace mnist {


// ----------------------------------------------------------- geometry ----
template <int H_, int W_, int CIN_, int COUT_, int KS_, int PAD_, int BK_>
struct ConvGeo {
  static constexpr int H = H_, W = W_, CIN = CIN_, COUT = COUT_, KS = KS_, PAD = PAD_;
  static constexpr int PH = H / 2, PW = W / 2;
  static constexpr int K = KS * KS * CIN;
  static constexpr int BK = BK_;
  static constexpr int KPAD = (K + BK - 1) / BK * BK;
};
using Conv1 = ConvGeo<28, 28, 1, 32, 5, 2, 32>;


// --------------------------------------------- conv + bias + relu + pool ----
// GEMM view: M = pre-pool pixels ordered (n, py, px, quadrant) so that the 4
// pixels of one 2x2 pooling window are 4 consecutive C rows = 4 consecutive
// accumulator registers of ONE lane (rows (r&3) + 8(r>>2) + 4(l>>5)); the
// pool is then a register max, no LDS, no extra pass.  N = Cout, K = taps*Cin.
template <class G>
struct ConvPoolFwdProb {
  static constexpr bool A_KC = true, B_NC = true;
  struct ACtx {
    const float* p;  // input at (n, 0, 0, ci) of this slot's image
    int y, x, kl;
    bool v;
  };
  struct BCtx {
    const float* p;
    int kl;
  };
  const float* x;
  const float* w;
  int batch;
  __device__ __forceinline__ ACtx a_ctx(int m, int kl) const {
    const int q = m & 3, pix = m >> 2;
    const int px = pix % G::PW, t = pix / G::PW, py = t % G::PH, n = t / G::PH;
    const int y = 2 * py + (q >> 1), xx = 2 * px + (q & 1);
    const bool v = n < batch;
    const int ci = kl % G::CIN;
    return {x + (size_t)(v ? n : 0) * G::H * G::W * G::CIN + ci, y, xx, kl, v};
  }
  // unconditional load from a clamped (always valid) address + select: a
  // guarded load would compile to an exec-mask branch per element
  __device__ __forceinline__ float a_get(const ACtx& c, int k0) const {
    const int k = k0 + c.kl;
    const int tap = k / G::CIN;
    const int kh = tap / G::KS, kw = tap % G::KS;
    const int iy = c.y + kh - G::PAD, ix = c.x + kw - G::PAD;
    const bool ok = c.v && k < G::K && iy >= 0 && iy < G::H && ix >= 0 && ix < G::W;
    const int iyc = min(max(iy, 0), G::H - 1), ixc = min(max(ix, 0), G::W - 1);
    const float v = c.p[(iyc * G::W + ixc) * G::CIN];
    return ok ? v : 0.f;
  }
  __device__ __forceinline__ BCtx b_ctx(int kl, int n) const { return {w + kl * G::COUT + n, kl}; }
  __device__ __forceinline__ float b_get(const BCtx& c, int k0) const {
    const int k = k0 + c.kl;
    const float v = c.p[(min(k, G::K - 1) - c.kl) * G::COUT];
    return k < G::K ? v : 0.f;
  }
};

template <class G, int WM, int WN, int WK>
__global__ __launch_bounds__(64 * WM * WN * WK) void conv_pool_fwd_kernel(
    const float* __restrict__ data, const long long* step_ptr, int n_local, int batch,
    const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ out,
    uint8_t* __restrict__ argmax, __bf16* __restrict__ out_p, __bf16* __restrict__ out_t,
    int ld_batch, float* __restrict__ out_pad, const ShadowPtrs sh, int conv_blocks) {
  // out_p / out_t (bf16 engine, layouts in mnist_bf16.h): pooled output as
  // the zero-bordered K-packed image [C/16][ld_batch][PH+4][PW+4][16] and as
  // [n][PH+4][C][MNIST16_T_LD], instead of the fp32 NHWC `out`.  out_pad
  // (fp32 engine, optional): a zero-bordered NHWC copy [n][PH+4][PW+4][C]
  // whose border is never written (bounds-check-free conv2 filter operand)
  // blocks beyond `conv_blocks` (bf16 train step) re-derive the bf16 weight
  // shadows from the fp32 master weights (mnist_shared.h shadow_block): the
  // first consumer is the NEXT launch (conv2), so they ride in this grid
  // instead of costing a launch of their own
  using CF = gemm::Cfg<WM, WN, WK, G::BK, true, true>;
  static_assert(64 * WM * WN * WK == 256, "shadow role needs 256-thread blocks");
  constexpr int SM = CF::SMEM_FLOATS > SHADOW_SMEM_FLOATS ? CF::SMEM_FLOATS : SHADOW_SMEM_FLOATS;
  __shared__ float smem[SM];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  if (bid >= conv_blocks) {  // sh.w1b == nullptr: conv2 shadows only (the SGD wrote fc1's)
    shadow_block(bid - conv_blocks + (sh.w1b ? 0 : SHADOW_W1_BLOCKS), sh, smem);
    return;
  }
  const long long off = batch_offset_dev(step_ptr, n_local, batch);
  ConvPoolFwdProb<G> p{data + off * (G::H * G::W * G::CIN), w, batch};
  const int M = batch * G::PH * G::PW * 4;
  const int mt = (M + CF::BM - 1) / CF::BM;
  const int m0 = (bid % mt) * CF::BM, n0 = (bid / mt) * CF::BN;
  f32x16 acc;
  int wm, wn;
  bool own = gemm::run_tile<WM, WN, WK, G::BK>(p, smem, m0, n0, 0, G::KPAD, acc, wm, wn);
  if (!own) return;
  const int lane = threadIdx.x & 63;
  const int co = n0 + 32 * wn + (lane & 31);
  const float b = bias[co];
  const int P = batch * G::PH * G::PW;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int pooled = ((m0 + 32 * wm) >> 2) + 2 * g + (lane >> 5);
    float v = acc[4 * g];
    int q = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      if (acc[4 * g + j] > v) {  // strict: first max wins (TF MaxPool order)
        v = acc[4 * g + j];
        q = j;
      }
    }
    if (pooled < P) {
      const float o = fmaxf(v + b, 0.f);
      if (out_p) {
        constexpr int PP = G::PH + 4, PQ = G::PW + 4;
        const int px = pooled % G::PW, t = pooled / G::PW, py = t % G::PH, n = t / G::PH;
        out_p[(((size_t)(co >> 4) * ld_batch + n) * PP + py + 2) * PQ * 16 + (px + 2) * 16 +
              (co & 15)] = (__bf16)o;
        if (out_t)
          out_t[((size_t)(n * PP + py + 2) * G::COUT + co) * MNIST16_T_LD + px + 2] = (__bf16)o;
      } else {
        out[pooled * G::COUT + co] = o;
        if (out_pad) {
          const int px = pooled % G::PW, t = pooled / G::PW, py = t % G::PH, n = t / G::PH;
          out_pad[((size_t)(n * (G::PH + 4) + py + 2) * (G::PW + 4) + px + 2) * G::COUT + co] = o;
        }
      }
      if (argmax) argmax[pooled * G::COUT + co] = (uint8_t)q;
    }
  }
}

// ------------------------------------------------------------- fc1 fwd ----
struct Fc1FwdProb {
  static constexpr bool A_KC = true, B_NC = true;
  using ACtx = gemm::RowMajorA::Ctx;
  struct BCtx {
    const float* p;
  };
  gemm::RowMajorA A;
  const float* w;  // [3136][512]
  __device__ __forceinline__ ACtx a_ctx(int m, int kl) const { return A.ctx(m, kl); }
  __device__ __forceinline__ float a_get(const ACtx& c, int k0) const { return A.get(c, k0); }
  __device__ __forceinline__ BCtx b_ctx(int kl, int n) const { return {w + kl * FC1_OUT + n}; }
  __device__ __forceinline__ float b_get(const BCtx& c, int k0) const {
    return c.p[k0 * FC1_OUT];
  }
};

// train: split-K partial slabs part[z][m][n]; eval: h = relu(acc + b) (+dropout)
template <int WM, int WN, int WK, int BK, bool EVAL, int ONESHOT_KT = 0>
__global__ __launch_bounds__(64 * WM * WN * WK) void fc1_fwd_kernel(
    const float* __restrict__ a, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, int M, int kchunk, uint32_t drop_key, float keep_prob) {
  using CF = gemm::Cfg<WM, WN, WK, BK, true, true>;
  constexpr int SM1 = ONESHOT_KT > 0 ? ONESHOT_KT * CF::STAGE_FLOATS : CF::SMEM_FLOATS;
  constexpr int SM = SM1 > CF::SMEM_FLOATS_RED ? SM1 : CF::SMEM_FLOATS_RED;
  __shared__ float smem[SM];
  Fc1FwdProb p{{a, FC1_IN, M}, w};
  const int mt = (M + CF::BM - 1) / CF::BM;
  const int z = blockIdx.y;
  const int bid = blockIdx.x;
  const int m0 = (bid % mt) * CF::BM, n0 = (bid / mt) * CF::BN;
  const int kb = z * kchunk, ke = min(FC1_IN, kb + kchunk);
  f32x16 acc;
  int wm, wn;
  bool own;
  if constexpr (ONESHOT_KT > 0)
    own = gemm::run_tile_oneshot<WM, WN, WK, BK, ONESHOT_KT>(p, smem, m0, n0, kb, acc, wm, wn);
  else
    own = gemm::run_tile<WM, WN, WK, BK>(p, smem, m0, n0, kb, ke, acc, wm, wn);
  if (!own) return;
  const int lane = threadIdx.x & 63;
  const int n = n0 + 32 * wn + (lane & 31);
  const float b = EVAL ? bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + 32 * wm + mfma32_row(r, lane);
    if (m >= M) continue;
    if (EVAL) {
      float h = fmaxf(acc[r] + b, 0.f);
      if (keep_prob < 1.f) {
        h = dropout_keep(drop_key, (uint32_t)(m * FC1_OUT + n), keep_prob) ? h / keep_prob : 0.f;
      }
      out[(size_t)m * FC1_OUT + n] = h;
    } else {
      out[((size_t)z * M + m) * FC1_OUT + n] = acc[r];
    }
  }
}

// fc1 forward (train) over the feature-major a2t [3136][batch] that the
// Winograd conv2 forward writes: both MFMA operands come straight from
// L2 / MALL with lanes on their contiguous axis (a2t rows along the batch,
// W1 rows along the 512 outputs: one 128-B line per half-wave load), so there
// is no LDS staging, no transpose and no barrier before the products.
// Block = (32 rows, 32 outputs, split of 3136 / FC1T_SPLITS features); its 4
// waves take consecutive quarters of the split (49 k-steps each, every load
// issued up front, two accumulator chains) and meet once in LDS; wave 0
// writes the split's partial slab part[split][row][512] (the head sums them).
constexpr int FC1T_SPLITS = 8;
constexpr int FC1T_KW = FC1_IN / FC1T_SPLITS / 4;  // 98 features per wave
static_assert(FC1T_KW % 2 == 0 && FC1_IN % (FC1T_SPLITS * 4) == 0, "fc1_fwd_t split");

__global__ __launch_bounds__(256) void fc1_fwd_t_kernel(const float* __restrict__ a2t,
                                                        const float* __restrict__ w,
                                                        int batch, float* __restrict__ part) {
  __shared__ float red[3][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i = lane & 31, h = lane >> 5;
  const int nt = blockIdx.x % (FC1_OUT / 32), bt = blockIdx.x / (FC1_OUT / 32);
  const int z = blockIdx.y;
  const int n0 = 32 * nt, b0 = 32 * bt;
  const int kb = z * (FC1_IN / FC1T_SPLITS) + wave * FC1T_KW;
  constexpr int ST = FC1T_KW / 2;  // 49 MFMA k-steps
  const float* ap = a2t + (size_t)(kb + h) * batch + b0 + i;
  const float* bp = w + (size_t)(kb + h) * FC1_OUT + n0 + i;
  float av[ST], bv[ST];
#pragma unroll
  for (int t = 0; t < ST; ++t) {
    av[t] = ap[(size_t)2 * t * batch];
    bv[t] = bp[(size_t)2 * t * FC1_OUT];
  }
  f32x16 c0 = zero16(), c1 = zero16();
#pragma unroll
  for (int t = 0; t < ST; ++t) {
    if (t & 1)
      c1 = mfma32x32x2(av[t], bv[t], c1);
    else
      c0 = mfma32x32x2(av[t], bv[t], c0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) c0[r] += c1[r];
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave - 1][r][lane] = c0[r];
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = c0[r] + red[0][r][lane] + red[1][r][lane] + red[2][r][lane];
      const int row = b0 + mfma32_row(r, lane);
      part[((size_t)z * batch + row) * FC1_OUT + n0 + i] = v;
    }
  }
}

// -------------------------------------------------------------- fc head ----
// One workgroup per batch row: reduce fc1 split-K slabs, bias, ReLU, dropout,
// fc2 (512x10, too thin for MFMA: VALU dot products), softmax cross-entropy
// forward AND backward (dlogits = (softmax - onehot) / B), then
// dhidden = dlogits W2^T through the dropout and ReLU masks.
template <int NS>  // split-K slabs of the fc1 forward (FC1_SPLITS, FC1T_SPLITS)
__global__ __launch_bounds__(256) void fc_head_train_kernel(
    const float* __restrict__ part, const float* __restrict__ b3, const float* __restrict__ w4,
    const float* __restrict__ b4, const int* __restrict__ labels, int n_local,
    const long long* step_ptr, int batch, float keep_prob, uint32_t seed, uint32_t rank,
    float base_lr, float lr_decay, float* __restrict__ hd_out, float* __restrict__ dh_out,
    float* __restrict__ dlog_out, float* __restrict__ loss_rows, float* __restrict__ lr_out,
    int* __restrict__ correct, __bf16* __restrict__ dh16, __bf16* __restrict__ dht16) {
  // dh16 / dht16 (bf16 engine): the K-packed MFMA operands of fc1 dX / dW1
  __shared__ float red[4][NCLS];
  __shared__ float dlog_s[NCLS];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long step = step_ptr ? *step_ptr : 0;
  const long long off = batch_offset_dev(step_ptr, n_local, batch);
  const uint32_t key = dropout_key(seed, rank, (uint32_t)step, 0u);
  const float scale = 1.f / keep_prob;
  // the label and fc2 bias used after the logit reduction: loaded now, not
  // as a dependent round trip after the barrier
  const int label = labels[off + row];
  const float b4l = lane < NCLS ? b4[lane] : 0.f;
  // issue every slab load up front (one latency round, not 14)
  float ps[2][NS];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int q = 0; q < NS; ++q)
      ps[u][q] = part[((size_t)q * batch + row) * FC1_OUT + tid + 256 * u];
  float w4r[2][NCLS];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int c = 0; c < NCLS; ++c) w4r[u][c] = w4[(tid + 256 * u) * NCLS + c];
  float z[2], hd[2];
  bool kp[2];
  float lg[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) lg[c] = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = tid + 256 * u;
    float s = b3[j];
#pragma unroll
    for (int q = 0; q < NS; ++q) s += ps[u][q];
    z[u] = s;
    const float h = fmaxf(s, 0.f);
    kp[u] = dropout_keep(key, (uint32_t)(row * FC1_OUT + j), keep_prob);
    hd[u] = kp[u] ? h * scale : 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) lg[c] += hd[u] * w4r[u][c];
  }
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {
    float v = wave_sum(lg[c]);
    if (lane == 0) red[wv][c] = v;
  }
  __syncthreads();
  if (tid < 64) {
    float logit = -INFINITY;
    if (lane < NCLS) logit = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane] + b4l;
    const float mx = wave_max(logit);
    const float e = lane < NCLS ? __expf(logit - mx) : 0.f;
    const float se = wave_sum(e);
    const float p = e / se;
    const float lab_logit = wave_sum(lane == label ? logit : 0.f);
    if (lane < NCLS) dlog_s[lane] = (p - (lane == label ? 1.f : 0.f)) / (float)batch;
    const unsigned long long bal = __ballot(lane < NCLS && logit == mx);
    const int am = __ffsll((long long)bal) - 1;
    if (lane == 0) {
      loss_rows[row] = (logf(se) + mx) - lab_logit;  // logsumexp - logit[label]
      if (correct) atomicAdd(correct, am == label ? 1 : 0);
      if (row == 0 && lr_out) {
        const float e2 = (float)((step * batch) / n_local);
        lr_out[0] = base_lr * powf(lr_decay, e2);
      }
    }
  }
  __syncthreads();
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) dl[c] = dlog_s[c];
  if (tid < NCLS) dlog_out[row * NCLS + tid] = dl[tid];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = tid + 256 * u;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) d += dl[c] * w4r[u][c];
    d = (kp[u] && z[u] > 0.f) ? d * scale : 0.f;
    hd_out[row * FC1_OUT + j] = hd[u];
    dh_out[row * FC1_OUT + j] = d;
    if (dh16) {  // K-packed layouts of mnist_bf16.h
      dh16[((j >> 4) * batch + row) * 16 + (j & 15)] = (__bf16)d;
      dht16[((row >> 4) * FC1_OUT + j) * 16 + (row & 15)] = (__bf16)d;
    }
  }
}

// eval head: logits = h W2 + b, argmax vs label -> error count (E1/E2)
__global__ __launch_bounds__(256) void fc_head_eval_kernel(const float* __restrict__ h,
                                                           const float* __restrict__ w4,
                                                           const float* __restrict__ b4,
                                                           const int* __restrict__ labels, int M,
                                                           float* __restrict__ logits_out,
                                                           int* __restrict__ errors) {
  // one wave per row, 4 rows per block
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float lg[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) lg[c] = 0.f;
#pragma unroll
  for (int jj = 0; jj < FC1_OUT / 64; ++jj) {
    const int j = lane + 64 * jj;
    const float hv = h[(size_t)row * FC1_OUT + j];
#pragma unroll
    for (int c = 0; c < NCLS; ++c) lg[c] += hv * w4[j * NCLS + c];
  }
  float best = -INFINITY;
  int bi = 0;
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {
    const float v = wave_sum(lg[c]) + b4[c];
    if (logits_out && lane == 0) logits_out[(size_t)row * NCLS + c] = v;
    if (v > best) {
      best = v;
      bi = c;
    }
  }
  if (lane == 0 && labels && errors) {
    if (bi != labels[row]) atomicAdd(errors, 1);
  }
}

// ------------------------------------------------------------- fc1 bwd ----
// One launch, three block roles; every block is 4 waves and no operand goes
// through LDS (the previous LDS-staged version was a serial chain of 8 K tiles,
// 17.6 us in graph replay):
//  * dX   dA2 = dh W1^T (M = batch, N = 3136, K = 512), one 32x32 tile per
//         block, K split over the 4 waves (128 each).  Both operands have k
//         contiguous, but the fp32 MFMA wants one k per lane with lanes on
//         rows, so each wave loads its rows coalesced (float4, lanes along k,
//         all 32 loads in flight) and transposes them through a wave-private
//         LDS image (no block barrier).  Loading the fragments directly
//         (32 rows = 32 cache lines per wave load) measured 11 us; the
//         staged form touches 8x fewer lines.  Partial tiles are summed
//         through LDS; wave 0 applies the ReLU2 mask and scatters through the
//         pool2 argmax into dY2 (NHWC, filter-grad operand) and dY2t
//         (channel-major, bwd-data operand).
//  * dW1  M = 3136 features, N = 512, K = batch; block = 32 features x 256
//         hidden (each wave 32x64 with one shared A fragment); lanes on the
//         contiguous axis of a2 / dh (one 128-B line per half-wave), K in
//         chunks of 32 MFMA steps with all loads of a chunk in flight.
//  * fc2 weight / bias and fc1 bias grads (fc1_small_grads).
// Logical block ids are XCD-remapped so the two M tiles of a dX N tile (same
// W1 rows) and the two halves of a dW1 M tile (same a2 columns) share an L2.
constexpr int FC1BWD_DW_BLOCKS = (FC1_IN / 32) * (FC1_OUT / 256);  // 196

constexpr int FC1DX_LD = 33;                     // LDS row (k) length: 32 rows + 1
constexpr int FC1DX_WAVE = 2 * 64 * FC1DX_LD;    // per-wave LDS: A and B, 64 k each

__device__ __forceinline__ void fc1_bwd_dx(int L, const float* __restrict__ a2,
                                           const uint8_t* __restrict__ idx2,
                                           const float* __restrict__ dh,
                                           const float* __restrict__ w1, int batch,
                                           float* __restrict__ dy2, float* __restrict__ dy2t,
                                           float* smem) {
  const int n_m = batch / 32;
  const int mt = L % n_m, nt = L / n_m;
  const int m0 = mt * 32, n0 = nt * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  // wave-private LDS transpose: coalesced float4 row loads (lanes along k,
  // 4 rows x 256 B per wave load) -> k-major [64][33] images -> one k per lane
  float* TA = smem + wave * FC1DX_WAVE;
  float* TB = TA + 64 * FC1DX_LD;
  const int lr = lane >> 4, lk = (lane & 15) * 4;
  const float* ap = dh + (size_t)(m0 + lr) * FC1_OUT + wave * 128 + lk;
  const float* bp = w1 + (size_t)(n0 + lr) * FC1_OUT + wave * 128 + lk;
  // epilogue operands of this wave's 4 accumulator registers (k = 4 wave + j),
  // issued first so their latency hides under the MFMAs (the scheduler
  // otherwise sinks them behind the products)
  const int fi = n0 + r;  // (py, px, co) flat feature index
  float relu_in[4];
  int qsel[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = m0 + mfma32_row(4 * wave + j, lane);
    relu_in[j] = a2[(size_t)n * FC1_IN + fi];
    qsel[j] = idx2[(size_t)n * FC1_IN + fi];
  }
  float4 a[2][8], b[2][8];
#pragma unroll
  for (int rho = 0; rho < 2; ++rho)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[rho][i] = *reinterpret_cast<const float4*>(ap + (size_t)4 * i * FC1_OUT + 64 * rho);
      b[rho][i] = *reinterpret_cast<const float4*>(bp + (size_t)4 * i * FC1_OUT + 64 * rho);
    }
  __builtin_amdgcn_sched_barrier(0);
  f32x16 c0 = zero16(), c1 = zero16();
#pragma unroll
  for (int rho = 0; rho < 2; ++rho) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 4 * i + lr;
      TA[(lk + 0) * FC1DX_LD + row] = a[rho][i].x;
      TA[(lk + 1) * FC1DX_LD + row] = a[rho][i].y;
      TA[(lk + 2) * FC1DX_LD + row] = a[rho][i].z;
      TA[(lk + 3) * FC1DX_LD + row] = a[rho][i].w;
      TB[(lk + 0) * FC1DX_LD + row] = b[rho][i].x;
      TB[(lk + 1) * FC1DX_LD + row] = b[rho][i].y;
      TB[(lk + 2) * FC1DX_LD + row] = b[rho][i].z;
      TB[(lk + 3) * FC1DX_LD + row] = b[rho][i].w;
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      const float av = TA[(2 * t + h) * FC1DX_LD + r], bv = TB[(2 * t + h) * FC1DX_LD + r];
      if (t & 1)
        c1 = mfma32x32x2(av, bv, c1);
      else
        c0 = mfma32x32x2(av, bv, c0);
    }
  }
  // K reduction over the 4 waves through LDS (each wave's own region, now
  // free), then every wave finishes 4 of the 16 accumulator registers
#pragma unroll
  for (int k = 0; k < 16; ++k) TA[k * 64 + lane] = c0[k] + c1[k];
  __syncthreads();
  const int co = fi & 63, pp = fi >> 6, py = pp / 7, px = pp % 7;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * wave + j;
    const int n = m0 + mfma32_row(k, lane);
    float g = smem[k * 64 + lane] + smem[FC1DX_WAVE + k * 64 + lane] +
              smem[2 * FC1DX_WAVE + k * 64 + lane] + smem[3 * FC1DX_WAVE + k * 64 + lane];
    if (relu_in[j] <= 0.f) g = 0.f;  // ReLU2 inactive at the argmax
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int y = 2 * py + dy, x = 2 * px;
      const float v0 = (qsel[j] == 2 * dy) ? g : 0.f, v1 = (qsel[j] == 2 * dy + 1) ? g : 0.f;
      dy2[((n * 14 + y) * 14 + x) * 64 + co] = v0;
      dy2[((n * 14 + y) * 14 + x + 1) * 64 + co] = v1;
      // x + 2 is even and MNIST32_T_LD is even: one 8-byte store per row pair
      if (dy2t != nullptr)
        *reinterpret_cast<float2*>(dy2t + ((size_t)(n * 64 + co) * 18 + y + 2) * MNIST32_T_LD +
                                   x + 2) = make_float2(v0, v1);
    }
  }
}

// one wave's 32 x 64 part of dW1 tile L (32 features x 256 hidden; wave w of
// 4 takes hidden columns 64 w .. 64 w + 63): c0 / c1 = columns n0 .. n0 + 31 /
// n0 + 32 .. n0 + 63, rows m0 + mfma32_row(k, lane)
__device__ __forceinline__ void fc1_dw_tile(int L, const float* __restrict__ a2,
                                            const float* __restrict__ dh, int batch, int wave,
                                            f32x16& c0, f32x16& c1, int& m0, int& n0) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  m0 = (L >> 1) * 32;
  n0 = (L & 1) * 256 + wave * 64;
  const float* ap = a2 + m0 + r;
  const float* bp = dh + n0 + r;
  c0 = zero16();
  c1 = zero16();
  for (int k0 = 0; k0 < batch; k0 += 64) {  // 32 MFMA steps (k = k0 + 2t + h)
    float av[32], b0[32], b1[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      const int kc = min(k0 + 2 * t + h, batch - 1);
      av[t] = ap[(size_t)kc * FC1_IN];
      b0[t] = bp[kc * FC1_OUT];
      b1[t] = bp[kc * FC1_OUT + 32];
    }
    // all 96 loads issued before the first product: left to itself the
    // scheduler interleaves them with the MFMA chain (one load + wait per
    // MFMA), exposing the L2-miss latency several times over (12 us alone)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 32; ++t)
      if (k0 + 2 * t + h >= batch) av[t] = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      c0 = mfma32x32x2(av[t], b0[t], c0);
      c1 = mfma32x32x2(av[t], b1[t], c1);
    }
  }
}

__device__ __forceinline__ void fc1_bwd_dw(int L, const float* __restrict__ a2,
                                           const float* __restrict__ dh, int batch,
                                           float* __restrict__ g_w3, int wave) {
  f32x16 c0, c1;
  int m0, n0;
  fc1_dw_tile(L, a2, dh, batch, wave, c0, c1, m0, n0);
  const int lane = threadIdx.x & 63, r = lane & 31;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int m = m0 + mfma32_row(k, lane);
    g_w3[(size_t)m * FC1_OUT + n0 + r] = c0[k];
    g_w3[(size_t)m * FC1_OUT + n0 + 32 + r] = c1[k];
  }
}

// single rank: dW1 tile L formed and applied at once - momentum SGD of those
// fc1 weights (the sgd4 expression forms, so the parameters match the
// gradient-buffer path bit for bit).  The weight / momentum loads follow the
// products, one accumulator at a time: issued ahead of them they took the
// final SGD launch to 232 VGPRs, halving its occupancy (12.2 -> 15.7 us).
// (Half-tile units - one accumulator per wave, buffer-descriptor addressing,
// 89 VGPRs, 392 blocks - measured 13.2 us: the shorter chains did not pay
// for the doubled operand traffic and block count.)
// tid: index in the 256-thread unit
// (Negative, round 6: the weights / momentum of the tile requested into LDS
// with global_load_lds before the products - no VGPRs - so the SGD would not
// wait for two HBM / MALL round trips after the MFMAs: the launch went 11.5
// -> 13.4 us, r6_s1.)
// (Also negative: the first accumulator's weights / momentum requested before
// the products took the launch to 240 VGPRs, one wave a SIMD.)
__device__ __forceinline__ void fc1_dw_sgd(const FcSgd& a, int L, int tid) {
  const int lane = tid & 63, r = lane & 31, wave = tid >> 6;
  float* w = a.w + (size_t)a.w1_off4 * 4;
  float* mo = a.m + (size_t)a.w1_off4 * 4;
  f32x16 c0, c1;
  int m0, n0;
  fc1_dw_tile(L, a.a2, a.dh, a.batch, wave, c0, c1, m0, n0);
  const float lr = *a.lr;
  auto apply = [&](const f32x16 c, int col) {
    float wv[16], mv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const size_t e = (size_t)(m0 + mfma32_row(k, lane)) * FC1_OUT + col;
      wv[k] = w[e];
      mv[k] = mo[e];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float g = __builtin_fmaf(a.l2, wv[k], c[k] * a.gs);
      mv[k] = a.mu * mv[k] + g;
      wv[k] -= lr * mv[k];
      const size_t e = (size_t)(m0 + mfma32_row(k, lane)) * FC1_OUT + col;
      w[e] = wv[k];
      mo[e] = mv[k];
    }
  };
  apply(c0, n0 + r);
  apply(c1, n0 + 32 + r);
}

__global__ __launch_bounds__(256) void fc1_bwd_kernel(
    const float* __restrict__ a2, const uint8_t* __restrict__ idx2, const float* __restrict__ dh,
    const float* __restrict__ hd, const float* __restrict__ dlog, const float* __restrict__ w1,
    int batch, float* __restrict__ g_w3, float* __restrict__ g_b3, float* __restrict__ g_w4,
    float* __restrict__ g_b4, float* __restrict__ dy2, float* __restrict__ dy2t, int roles) {
  // dy2: NHWC [n][14][14][64]; dy2t: channel-major, zero-bordered
  // [n][64][18][MNIST32_T_LD] (its border is never written)
  constexpr int S_DX = 4 * FC1DX_WAVE, S_SMALL = FC1_SMALL_SMEM;
  __shared__ float smem[S_DX > S_SMALL ? S_DX : S_SMALL];
  // the grid holds the blocks of the roles asked for, in the order dX, dW1,
  // small (launch_fc1_bwd)
  const int n_dx = (roles & 1) ? (batch / 32) * (FC1_IN / 32) : 0;
  const int n_dw = (roles & 2) ? FC1BWD_DW_BLOCKS : 0;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if (L < n_dx)
    fc1_bwd_dx(L, a2, idx2, dh, w1, batch, dy2, dy2t, smem);
  else if (L < n_dx + n_dw)
    fc1_bwd_dw(L - n_dx, a2, dh, batch, g_w3, threadIdx.x >> 6);
  else
    fc1_small_grads(L - n_dx - n_dw, hd, dh, dlog, batch, g_w4, g_b4, g_b3, smem);
}

// FC weight gradients from GATHERED factors (SCHED_FACTORS): dW1 = A^T DH,
// dW2 = HD^T DLOG, db1 = sum DH, db2 = sum DLOG over the rows of every rank
// (rows = N x batch, rank-major; the rank's own slot written in place by its
// forward / head kernels, the rest by one grouped all-gather).  Same dW / small
// block roles as fc1_bwd_kernel with K = rows, so the result is the exact
// global sum, formed in one fixed order identically on every rank.
__global__ __launch_bounds__(256) void fc1_bwd_weights_kernel(
    const float* __restrict__ a2, const float* __restrict__ dh, const float* __restrict__ hd,
    const float* __restrict__ dlog, int rows, float* __restrict__ g_w3, float* __restrict__ g_b3,
    float* __restrict__ g_w4, float* __restrict__ g_b4) {
  __shared__ float smem[FC1_SMALL_SMEM];
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if (L < FC1BWD_DW_BLOCKS)
    fc1_bwd_dw(L, a2, dh, rows, g_w3, threadIdx.x >> 6);
  else
    fc1_small_grads(L - FC1BWD_DW_BLOCKS, hd, dh, dlog, rows, g_w4, g_b4, g_b3, smem);
}

// ------------------------------------------ conv2: dedicated MFMA kernels ----
// The three conv2 products are the bulk of the step's FLOPs (3 x 1.28 GFLOP at
// B = 64).  They bypass the generic gather engine:
//  * fwd and bwd-data stage the block's input halo tile in LDS ONCE (pixel
//    stride 33 / 65 floats: the 32 lanes of a half-wave read 32 different
//    pixels of one channel conflict-free) and read every tap's A operand
//    straight from that image - no im2col, no per-K-tile restaging;
//  * the B operand (weights, L2 resident) is read straight from global memory
//    with lanes on the contiguous channel axis (128 B per half-wave), one tap
//    ahead in registers;
//  * bwd-filter has channels on the lanes for BOTH operands, so it needs no
//    LDS at all: coalesced 128 B loads of a1 and dY2 feed the MFMAs directly.
constexpr int C2_XS_ROWS = 8, C2_XS_COLS = 18;


// conv2 forward + bias + ReLU + 2x2 maxpool (+argmax).  Block = (image, pair of
// pooled rows); 4 waves = 2 (M: 32 pre-pool pixels = 8 pooling windows) x 2
// (N: 32 output channels), one wave per SIMD, each wave owning the FULL K
// (800) of its tile with two independent accumulator chains (even / odd
// channel pairs) so consecutive MFMAs never wait on each other's result and
// no cross-wave K reduction (barrier + LDS round trip) is needed.  A operands
// come from the LDS halo tile, B (weights, L2 resident) one tap ahead in
// registers.  Also writes W2T[t][co][ci] for bwd-data when w2t != nullptr.
constexpr int C2_XS = C2_XS_ROWS * C2_XS_COLS * 33;
// FUSED: the input image rows of the block (8 pg - 6 .. 8 pg + 13, columns
// -2 .. 30, zero outside the 28 x 28 image)
constexpr int C12_IMG_ROWS = 20, C12_IMG_LD = 33;

// conv1 of the fused train forward (launch_conv12_fwd): the block computes the
// pooled conv1 rows its conv2 halo needs (a1 rows 4 pg - 2 .. 4 pg + 5, ~2x
// recompute of a 25-tap conv) straight into the halo tile, and writes the rows
// it owns (4 pg .. 4 pg + 3) to a1 / a1pf / idx1 for the backward pass.  Same
// GEMM view as conv_pool_fwd_kernel: M = pre-pool pixels (window, quadrant),
// N = 32 channels, K = 25 taps (-> 32), one 32 x 32 MFMA tile per 8 windows.
// NT: block size (256 or 512); the conv1 MFMA tiles run on waves 0-3 only
// Sink: where the pooled conv1 values go - zero(tid, NT) clears the block's
// halo tile, put(y, x, co, o, qq, own) stores a1 row y, column x (own: a row
// this block writes out for the backward pass).
struct HaloF32 {  // fp32 engines: the fp32 halo tile + a1 / idx1 / a1pf
  const C12In& c1;
  float* xs;
  int n, y0;
  __device__ __forceinline__ void zero(int tid, int nt) const {
    for (int i = tid; i < C2_XS; i += nt) xs[i] = 0.f;
  }
  __device__ __forceinline__ void put(int y, int x, int co, float o, int qq, bool own) const {
    xs[((y - y0) * C2_XS_COLS + x + 2) * 33 + co] = o;
    if (own) {
      const size_t pi = ((size_t)(n * 14 + y) * 14 + x) * 32 + co;
      c1.a1[pi] = o;
      c1.idx1[pi] = (uint8_t)qq;
      c1.a1pf[((size_t)(n * 18 + y + 2) * 18 + x + 2) * 32 + co] = o;
    }
  }
};

template <int NT, class Sink>
__device__ __forceinline__ void conv1_into_halo_t(const C12In& c1, int batch, int n, int pg,
                                                  float* __restrict__ img, const Sink& sink) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long off = batch_offset_dev(c1.step, c1.n_local, batch);
  const float* xin = c1.data + (off + n) * 784;
  const int iy0 = 8 * pg - 6;
  constexpr int NIMG = C12_IMG_ROWS * C12_IMG_LD;  // 660
  constexpr int NJ = (NIMG + NT - 1) / NT;
  float iv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = tid + NT * j;
    const int r = i / C12_IMG_LD, c = i % C12_IMG_LD, iy = iy0 + r, ix = c - 2;
    const bool ok = i < NIMG && iy >= 0 && iy < 28 && ix >= 0 && ix < 28;
    const float v = xin[min(max(iy, 0), 27) * 28 + min(max(ix, 0), 27)];
    iv[j] = ok ? v : 0.f;
  }
  const int co = lane & 31, kh2 = lane >> 5;
  float wb[13];
#pragma unroll
  for (int st = 0; st < 13; ++st) {
    const int k = 2 * st + kh2;
    const float v = c1.w1[min(k, 24) * 32 + co];
    wb[st] = k < 25 ? v : 0.f;
  }
  const float bias = c1.b1[co];
  sink.zero(tid, NT);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = tid + NT * j;
    if (i < NIMG) img[i] = iv[j];
  }
  __syncthreads();
  constexpr int NW = NT / 64;  // every wave runs conv1 tiles (pairs t, t + NW)
  const int y0 = 4 * pg - 2;  // a1 row of halo row 0
  const int ya = max(y0, 0), yb = min(y0 + C2_XS_ROWS, 14);
  const int nwin = (yb - ya) * 14, ntile = (nwin + 7) / 8;
  // A-operand base of tile t for this lane (vw: the lane's window exists)
  auto tile_base = [&](int t, bool& vw) {
    const int m = lane & 31, wi = t * 8 + (m >> 2), q = m & 3;
    vw = wi < nwin;
    const int wic = vw ? wi : 0;
    const int py = 2 * (ya + wic / 14) + (q >> 1), px = 2 * (wic % 14) + (q & 1);
    return img + (py - 2 - iy0) * C12_IMG_LD + px;  // + kh * LD + kw
  };
  auto epilogue = [&](int t, const f32x16& acc) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int wj = t * 8 + 2 * g + (lane >> 5);
      float v = acc[4 * g];
      int qq = 0;
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        if (acc[4 * g + j] > v) {  // strict: first max wins (TF MaxPool order)
          v = acc[4 * g + j];
          qq = j;
        }
      }
      if (wj < nwin) {
        const int y = ya + wj / 14, x = wj % 14;
        // own: the rows this block writes out
        sink.put(y, x, co, fmaxf(v + bias, 0.f), qq, y >= 4 * pg && y < 4 * pg + 4);
      }
    }
  };
  // tiles t and t + NW of this wave as two interleaved accumulator chains:
  // consecutive MFMAs are independent, and each tile's sum keeps the K order of
  // the standalone conv1 kernel (same results).  With 8 waves (the Winograd
  // forward's 512 threads) the 14 tiles take 2 per wave instead of 4.
  for (int t = wave; t < ntile; t += 2 * NW) {
    const bool two = t + NW < ntile;
    bool v0, v1;
    const float* ib0 = tile_base(t, v0);
    const float* ib1 = tile_base(two ? t + NW : t, v1);
    f32x16 acc0 = zero16(), acc1 = zero16();
    // 13 k-steps cover the 25 taps (k 25 is a zero pair); the standalone
    // kernel's k 26 .. 31 only add exact zeros, so the sums still match it
#pragma unroll
    for (int st = 0; st < 13; ++st) {
      const int k = 2 * st + kh2, kc = min(k, 24), o = (kc / 5) * C12_IMG_LD + kc % 5;
      const float a0 = ib0[o], a1v = ib1[o];
      acc0 = mfma32x32x2((v0 && k < 25) ? a0 : 0.f, wb[st], acc0);
      acc1 = mfma32x32x2((v1 && k < 25) ? a1v : 0.f, wb[st], acc1);
    }
    epilogue(t, acc0);
    if (two) epilogue(t + NW, acc1);
  }
}

// Winograd forward: the halo tile plus the owned rows' argmax taps in LDS
// (q1 [4 rows][14][32]); the owned a1 / a1pf / idx1 rows go out at the end of
// the kernel (halo_flush_owned) as coalesced float4 / u32 stores, so no
// global store of the conv1 epilogue waits in front of the phase barrier.
struct HaloF32Tile {
  float* xs;
  uint8_t* q1;
  int y0, yo;  // a1 row of halo row 0, first owned a1 row (4 pg)
  __device__ __forceinline__ void zero(int tid, int nt) const {
    for (int i = tid; i < C2_XS; i += nt) xs[i] = 0.f;
  }
  __device__ __forceinline__ void put(int y, int x, int co, float o, int qq, bool own) const {
    xs[((y - y0) * C2_XS_COLS + x + 2) * 33 + co] = o;
    if (own) q1[((y - yo) * 14 + x) * 32 + co] = (uint8_t)qq;
  }
};
constexpr int C12_Q1_BYTES = 4 * 14 * 32;

// the owned rows 4 pg .. 4 pg + 3 (clipped at 14) from the halo tile: f4 is
// this thread's float4 index, nt4 the stride (448 float4 per 4 rows)
__device__ __forceinline__ void halo_flush_owned(const C12In& c1, const float* xs,
                                                 const uint8_t* q1, int n, int pg, int f4,
                                                 int nt4) {
  const int yo = 4 * pg, nf = min(4, 14 - yo) * 14 * 8;
  for (int e = f4; e < nf; e += nt4) {
    const int c = 4 * (e & 7), pix = e >> 3, r = pix / 14, x = pix % 14;
    const float* s = xs + ((r + 2) * C2_XS_COLS + x + 2) * 33 + c;
    const float4 v = make_float4(s[0], s[1], s[2], s[3]);
    const size_t pi = ((size_t)(n * 14 + yo + r) * 14 + x) * 32 + c;
    *reinterpret_cast<float4*>(c1.a1 + pi) = v;
    *reinterpret_cast<float4*>(c1.a1pf + ((size_t)(n * 18 + yo + r + 2) * 18 + x + 2) * 32 + c) = v;
    *reinterpret_cast<uint32_t*>(c1.idx1 + pi) = *reinterpret_cast<const uint32_t*>(q1 + pix * 32 + c);
  }
}

template <int NT = 256>
__device__ __forceinline__ void conv1_into_halo(const C12In& c1, int batch, int n, int pg,
                                                float* __restrict__ xs, float* __restrict__ img) {
  conv1_into_halo_t<NT>(c1, batch, n, pg, img, HaloF32{c1, xs, n, 4 * pg - 2});
}

// FUSED (train): conv1 is computed into the halo tile (conv1_into_halo)
// instead of a separate conv1 launch staging a1 through global memory.
template <bool FUSED>
__global__ __launch_bounds__(256) void conv2_fwd_v3_kernel(
    const float* __restrict__ a1, int batch, const float* __restrict__ w2,
    const float* __restrict__ b2, float* __restrict__ out, uint8_t* __restrict__ argmax,
    float* __restrict__ w2t, const C12In c1) {
  __shared__ float xs[C2_XS];
  __shared__ float img[FUSED ? C12_IMG_ROWS * C12_IMG_LD : 1];
  const int n = blockIdx.x >> 2, pg = blockIdx.x & 3, pr0 = 2 * pg;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (w2t) {  // 51200 floats over all blocks
    for (int i = blockIdx.x * 256 + tid; i < 51200; i += gridDim.x * 256) {
      const int ci = i & 31, co = (i >> 5) & 63, t = i >> 11;
      w2t[i] = w2[(t * 32 + ci) * 64 + co];
    }
  }
  if constexpr (FUSED) {
    conv1_into_halo(c1, batch, n, pg, xs, img);
  } else {  // stage the halo tile: all loads in flight first, then the LDS writes
    constexpr int NS = C2_XS_ROWS * C2_XS_COLS * 32 / 256;  // 18
    float sv[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = tid + 256 * j;
      const int ci = i & 31, c = (i >> 5) % C2_XS_COLS, r = (i >> 5) / C2_XS_COLS;
      const int y = 2 * pr0 - 2 + r, x = c - 2;
      const bool ok = y >= 0 && y < 14 && x >= 0 && x < 14;
      const float v = a1[((n * 14 + min(max(y, 0), 13)) * 14 + min(max(x, 0), 13)) * 32 + ci];
      sv[j] = ok ? v : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = tid + 256 * j;
      const int ci = i & 31, c = (i >> 5) % C2_XS_COLS, r = (i >> 5) / C2_XS_COLS;
      xs[(r * C2_XS_COLS + c) * 33 + ci] = sv[j];
    }
  }
  const int msub = wave & 1, nsub = wave >> 1;
  const int m = msub * 32 + (lane & 31);
  const int win = m >> 2, q = m & 3;
  int ly = 0, lx = 0;
  if (win < 14) {
    ly = 2 * (win / 7) + (q >> 1);
    lx = 2 * (win % 7) + (q & 1);
  }
  const int abase = (ly * C2_XS_COLS + lx) * 33 + (lane >> 5);
  const int co = nsub * 32 + (lane & 31);
  const float* wp = w2 + (lane >> 5) * 64 + co;  // + (t*32 + 2c) * 64
  float bc[16], bn[16], ac[16], an[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) bc[c] = wp[(2 * c) * 64];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 16; ++c) ac[c] = xs[abase + 2 * c];
  f32x16 acc0 = zero16(), acc1 = zero16();
#pragma unroll
  for (int t = 0; t < 25; ++t) {
    if (t + 1 < 25) {
      const int kh = (t + 1) / 5, kw = (t + 1) % 5;
      const float* xa = xs + abase + (kh * C2_XS_COLS + kw) * 33;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        bn[c] = wp[((t + 1) * 32 + 2 * c) * 64];
        an[c] = xa[2 * c];
      }
    }
    // keep the next tap's loads issued HERE (the scheduler would otherwise sink
    // them next to their use and expose the L2 latency on every MFMA)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      acc0 = mfma32x32x2(ac[c], bc[c], acc0);
      acc1 = mfma32x32x2(ac[c + 1], bc[c + 1], acc1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      bc[c] = bn[c];
      ac[c] = an[c];
    }
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc0[r] + acc1[r];
  const float bias = b2[co];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int w_ = msub * 8 + 2 * g + (lane >> 5);
    float v = acc[4 * g];
    int qq = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      if (acc[4 * g + j] > v) {  // strict: first max wins (TF MaxPool order)
        v = acc[4 * g + j];
        qq = j;
      }
    }
    const int pr = pr0 + w_ / 7, pc = w_ % 7;
    if (w_ < 14 && pr < 7) {
      const int o = ((n * 7 + pr) * 7 + pc) * 64 + co;
      out[o] = fmaxf(v + bias, 0.f);
      if (argmax) argmax[o] = (uint8_t)qq;
    }
  }
}


// ------------------------------ bf16 engine: conv1 + conv2 in ONE launch ----
// The bf16 twin of conv2_fwd_v3_kernel<true> (BASELINE config 2): each block
// (image, pair of pooled conv2 rows) recomputes the pooled conv1 rows of its
// halo on fp32 MFMA (conv1_into_halo_t, the standalone conv1's K order) and
// stores them bf16-rounded into a bf16 LDS halo; the rows it owns go out in
// the bf16 engine's layouts (a1p / a1t / idx1, mnist_bf16.h).  conv2 then runs
// on v_mfma_f32_32x32x16_bf16 with A fragments from that halo (one
// ds_read_b128 per k-step) and B from the w2t shadow (which the previous
// step's SGD wrote, or refresh_shadows), in the K order and with the two
// accumulator chains of mnist16::conv2_fwd_kernel, so a2 / idx2 equal the
// two-launch path's.  One launch and one a1 round trip through memory fewer.
constexpr int XB_LD = 40;  // bf16 per halo pixel (32 channels + 8: 16-B aligned rows)
constexpr int XB_ELEMS = C2_XS_ROWS * C2_XS_COLS * XB_LD;

// bf16 twin of HaloF32Tile: the halo tile plus the owned rows' argmax taps in
// LDS; halo_b16_flush_owned writes the owned a1p / a1t / idx1 rows at the end
// of the kernel (16-B a1p segments, 4-B a1t column pairs, u32 idx1 words)
// instead of 2-byte scattered stores inside the conv1 epilogue
struct HaloB16Tile {
  __bf16* xb;
  uint8_t* q1;
  int y0, yo;
  __device__ __forceinline__ void zero(int tid, int nt) const {
    uint4* z = reinterpret_cast<uint4*>(xb);
    for (int i = tid; i < XB_ELEMS / 8; i += nt) z[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  __device__ __forceinline__ void put(int y, int x, int co, float o, int qq, bool own) const {
    xb[((y - y0) * C2_XS_COLS + x + 2) * XB_LD + co] = (__bf16)o;
    if (own) q1[((y - yo) * 14 + x) * 32 + co] = (uint8_t)qq;
  }
};

__device__ __forceinline__ void halo_b16_flush_owned(const C12In& c1, const __bf16* xb,
                                                     const uint8_t* q1, __bf16* a1p, __bf16* a1t,
                                                     int n, int pg, int batch, int tid, int nt) {
  const int yo = 4 * pg, nr = min(4, 14 - yo);
  // a1p [2][B][18][18][16]: per (row, plane) 14 pixels x 16 channels contiguous
  for (int e = tid; e < nr * 56; e += nt) {
    const int hh = e & 1, x = (e >> 1) % 14, pl = (e / 28) & 1, r = e / 56;
    const uint4 v = *reinterpret_cast<const uint4*>(
        xb + ((r + 2) * C2_XS_COLS + x + 2) * XB_LD + pl * 16 + hh * 8);
    *reinterpret_cast<uint4*>(a1p + (((size_t)pl * batch + n) * 18 + yo + r + 2) * 18 * 16 +
                              (x + 2) * 16 + hh * 8) = v;
  }
  // a1t [B][18][32][MNIST16_T_LD]: per (row, channel) 14 columns at x + 2
  for (int e = tid; e < nr * 32; e += nt) {
    const int co = e & 31, r = e >> 5;
    const __bf16* src = xb + ((r + 2) * C2_XS_COLS + 2) * XB_LD + co;
    uint32_t* dst = reinterpret_cast<uint32_t*>(
        a1t + ((size_t)(n * 18 + yo + r + 2) * 32 + co) * MNIST16_T_LD + 2);
#pragma unroll
    for (int x = 0; x < 14; x += 2) {
      const uint32_t lo = __builtin_bit_cast(uint16_t, src[x * XB_LD]);
      const uint32_t hi = __builtin_bit_cast(uint16_t, src[(x + 1) * XB_LD]);
      dst[x >> 1] = lo | (hi << 16);
    }
  }
  // idx1 [B][14][14][32] bytes
  for (int e = tid; e < nr * 14 * 8; e += nt) {
    const int pix = e >> 3, c = 4 * (e & 7);
    *reinterpret_cast<uint32_t*>(c1.idx1 + ((size_t)(n * 14 + yo) * 14 + pix) * 32 + c) =
        *reinterpret_cast<const uint32_t*>(q1 + pix * 32 + c);
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void conv12_fwd_bf16_kernel(
    const C12In c1, int batch, const __bf16* __restrict__ w2t, const float* __restrict__ b2,
    __bf16* __restrict__ a1p, __bf16* __restrict__ a1t, __bf16* __restrict__ a2p,
    __bf16* __restrict__ a2t, uint8_t* __restrict__ idx2) {
  __shared__ __attribute__((aligned(16))) __bf16 xb[XB_ELEMS];
  __shared__ float img[C12_IMG_ROWS * C12_IMG_LD];
  __shared__ __attribute__((aligned(4))) uint8_t q1[C12_Q1_BYTES];
  const int n = blockIdx.x >> 2, pg = blockIdx.x & 3;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  conv1_into_halo_t<256>(c1, batch, n, pg, img, HaloB16Tile{xb, q1, 4 * pg - 2, 4 * pg});
  // A rows of this wave: pre-pool pixel m = (window, quadrant) of the block's
  // 14 windows (rows 56..63 of the second tile are padding, read pixel 0)
  const int msub = wave & 1, nsub = wave >> 1;
  const int m = msub * 32 + r, win = m >> 2, q = m & 3;
  int ly = 0, lx = 0;
  if (win < 14) {
    ly = 2 * (win / 7) + (q >> 1);
    lx = 2 * (win % 7) + (q & 1);
  }
  const __bf16* ap = xb + (ly * C2_XS_COLS + lx) * XB_LD + 8 * h;
  const __bf16* bp = w2t + (nsub * 32 + r) * 16 + 8 * h;
  constexpr int D = 5;
  bf16x8 rb[D];
#pragma unroll
  for (int d = 0; d < D; ++d) rb[d] = *reinterpret_cast<const bf16x8*>(bp + d * 1024);
  __syncthreads();  // the halo tile is complete
  f32x16 acc0 = zero16(), acc1 = zero16();
  // K-step ks = (tap t = ks / 2, channel half s = ks % 2), mnist16::kloop order
#pragma unroll
  for (int ks = 0; ks < 50; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int k = ks + d, t = k >> 1, sh = k & 1, kh = t / 5, kw = t % 5;
      const bf16x8 a =
          *reinterpret_cast<const bf16x8*>(ap + (kh * C2_XS_COLS + kw) * XB_LD + 16 * sh);
      const bf16x8 b = rb[d];
      if (k + D < 50) rb[d] = *reinterpret_cast<const bf16x8*>(bp + (k + D) * 1024);
      __builtin_amdgcn_sched_barrier(0);
      if (d & 1)
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc1, 0, 0, 0);
      else
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const int co = nsub * 32 + r;
  const float bias = b2[co];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float v = acc0[4 * g] + acc1[4 * g];
    int qq = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float u = acc0[4 * g + j] + acc1[4 * g + j];
      if (u > v) {  // strict: first max wins (TF MaxPool order)
        v = u;
        qq = j;
      }
    }
    const int w_ = msub * 8 + 2 * g + h;  // pooling window of registers 4g..4g+3
    const int pr = 2 * pg + w_ / 7, pc = w_ % 7;
    if (w_ < 14 && pr < 7) {
      const int i = (pr * 7 + pc) * 64 + co;
      const __bf16 out = (__bf16)fmaxf(v + bias, 0.f);
      a2p[((size_t)(i >> 4) * batch + n) * 16 + (i & 15)] = out;
      idx2[(size_t)n * FC1_IN + i] = (uint8_t)qq;
      a2t[((size_t)(n >> 4) * FC1_IN + i) * 16 + (n & 15)] = out;
    }
  }
  halo_b16_flush_owned(c1, xb, q1, a1p, a1t, n, pg, batch, tid, 256);
}

// ------------------------------------- conv2 forward, Winograd F(2x2,5x5) ----
// Transformed filters (wino.h), stored in MFMA fragment order so that one
// 16x16x4 B fragment is 256 contiguous bytes and a point's fragments sit at
// small immediate offsets from one base (p = 6 a + b):
//   U  (forward, K = ci, N = co):  [p][s = ci/4][q = co/16][ci%4][co%16]
//   Ud (bwd-data, rotated filter, K = co, N = ci): [p][s = co/4][q = ci/16][co%4][ci%16]
// One thread per (ci, co); both written from the same 25 loads.
__host__ __device__ __forceinline__ int wino_u_index(int p, int ci, int co) {
  return (((p * 8 + (ci >> 2)) * 4 + (co >> 4)) * 4 + (ci & 3)) * 16 + (co & 15);
}
__host__ __device__ __forceinline__ int wino_ud_index(int p, int ci, int co) {
  return (((p * 16 + (co >> 2)) * 2 + (ci >> 4)) * 4 + (co & 3)) * 16 + (ci & 15);
}
__global__ __launch_bounds__(256) void conv2_wino_weights_kernel(const float* __restrict__ w2,
                                                                 float* __restrict__ U,
                                                                 float* __restrict__ Ud) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // ci * 64 + co
  if (i >= 2048) return;
  const int ci = i >> 6, co = i & 63;
  float g[25], r[25], u[36];
#pragma unroll
  for (int t = 0; t < 25; ++t) g[t] = w2[t * 2048 + i];  // HWIO (t, ci, co)
  wino::filter_tile(g, u);
#pragma unroll
  for (int p = 0; p < 36; ++p) U[wino_u_index(p, ci, co)] = u[p];
  if (Ud) {
#pragma unroll
    for (int t = 0; t < 25; ++t) r[t] = g[24 - t];
    wino::filter_tile(r, u);
#pragma unroll
    for (int p = 0; p < 36; ++p) Ud[wino_ud_index(p, ci, co)] = u[p];
  }
}

// Output-transform weights per point: kWinoCoef[p][i * 2 + j]
struct WinoCoef {
  float c[36][4];
};
__host__ __device__ constexpr WinoCoef make_wino_coef() {
  WinoCoef w{};
  for (int p = 0; p < 36; ++p)
    for (int o = 0; o < 4; ++o) w.c[p][o] = wino::out_coef(p / 6, p % 6, o >> 1, o & 1);
  return w;
}
__constant__ WinoCoef kWinoCoef = make_wino_coef();

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// conv2 forward + bias + ReLU + 2x2 maxpool (+argmax) by Winograd F(2x2,5x5).
// Block = (image, pair of pooled rows) as conv2_fwd_v3_kernel: 14 pool
// windows = 14 Winograd tiles (M padded to 16).  Phases:
//   1. a1 halo tile in LDS (FUSED: conv1 recomputed into it, conv1_into_halo)
//   2. input transform: V[p][ci][tile] (36 x 32 x 16 floats) in LDS
//   3. 36 batched products [16 tiles x 32 ci] x [32 ci x 64 co] on
//      v_mfma_f32_16x16x4_f32; wave = (co quarter, half of the points), each
//      point folded into the four 2x2 outputs right after its 8 k-steps (the
//      output transform is linear), B = U[p] straight from L2, one pair ahead
//   4. the two halves' partial outputs summed through LDS, then bias + ReLU +
//      pool + argmax from registers
// FLOP per image: 36 x 49 x 32 x 64 x 2 = 7.2 M (direct: 20.1 M).
constexpr int WV_FLOATS = 36 * 32 * 16;  // V image; reused for the cross-wave sums

// 512 threads = 8 waves, two per SIMD: the transform runs one item per thread
// and each SIMD interleaves two waves' MFMA streams (wave = co quarter x half
// of the 36 points).  B fragments of the next point pair are loaded into the
// other of two register sets while the current pair's MFMAs run.
constexpr int WNT = 512, WNW = WNT / 64;

// halo image rows: the 8 of the block's windows + 6 zero rows that the two
// padding tiles (14, 15) transform (zeros in, zeros out: no selects)
constexpr int WX_ROWS = C2_XS_ROWS + 6, WX_FLOATS = WX_ROWS * C2_XS_COLS * 33;

// PROF (labs): per-wave s_memtime at the phase boundaries -> prof[block][wave][5]
template <bool FUSED, bool PROF = false>
__global__ __launch_bounds__(WNT) void conv2_fwd_wino_kernel(
    const float* __restrict__ a1, int batch, const float* __restrict__ w2,
    const float* __restrict__ U, const float* __restrict__ b2, float* __restrict__ out,
    uint8_t* __restrict__ argmax, float* __restrict__ w2t, const C12In c1,
    unsigned long long* __restrict__ prof = nullptr, float* __restrict__ out_t = nullptr) {
  // out_t (optional): the pooled output also feature-major, a2t [3136][batch]
  // (the fc1 forward's MFMA operand, fc1_fwd_t_kernel)
  unsigned long long stamp[5];
  if constexpr (PROF) stamp[0] = __builtin_amdgcn_s_memtime();
  __shared__ float xs[WX_FLOATS];
  __shared__ float img[FUSED ? C12_IMG_ROWS * C12_IMG_LD : 1];
  __shared__ float V[WV_FLOATS];
  __shared__ __attribute__((aligned(4))) uint8_t q1[FUSED ? C12_Q1_BYTES : 4];
  const int n = blockIdx.x >> 2, pg = blockIdx.x & 3, pr0 = 2 * pg;
  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform in an SGPR: the point index p, its output-transform weights
  // (scalar loads) and the fragment bases are then scalar
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (w2t) {  // W2T[t][co][ci] for the direct bwd-data kernel: 51200 floats over all blocks
    for (int i = blockIdx.x * WNT + tid; i < 51200; i += gridDim.x * WNT) {
      const int ci = i & 31, co = (i >> 5) & 63, t = i >> 11;
      w2t[i] = w2[(t * 32 + ci) * 64 + co];
    }
  }
  for (int i = C2_XS + tid; i < WX_FLOATS; i += WNT) xs[i] = 0.f;
  if constexpr (FUSED) {
    conv1_into_halo_t<WNT>(c1, batch, n, pg, img, HaloF32Tile{xs, q1, 4 * pg - 2, 4 * pg});
  } else {
    constexpr int NS = C2_XS_ROWS * C2_XS_COLS * 32 / WNT;  // 9
    float sv[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = tid + WNT * j;
      const int ci = i & 31, c = (i >> 5) % C2_XS_COLS, r = (i >> 5) / C2_XS_COLS;
      const int y = 2 * pr0 - 2 + r, x = c - 2;
      const bool ok = y >= 0 && y < 14 && x >= 0 && x < 14;
      const float v = a1[((n * 14 + min(max(y, 0), 13)) * 14 + min(max(x, 0), 13)) * 32 + ci];
      sv[j] = ok ? v : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = tid + WNT * j;
      const int ci = i & 31, c = (i >> 5) % C2_XS_COLS, r = (i >> 5) / C2_XS_COLS;
      xs[(r * C2_XS_COLS + c) * 33 + ci] = sv[j];
    }
  }
  // the first point pair's B fragments (U, L2) load under the input transform
  const int qw = wave & 3, ph = wave >> 2;
  const float* ub = U + qw * 64 + lane;  // fragment (s, qw) of point p at (32 p + 4 s) * 64
  auto loadb2 = [&](int p0, float(&b)[16]) {
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int k = 0; k < 8; ++k) b[pt * 8 + k] = ub[(32 * (p0 + pt) + 4 * k) * 64];
  };
  float bA[16], bB[16];
  loadb2(18 * ph, bA);
  __syncthreads();
  if constexpr (PROF) stamp[1] = __builtin_amdgcn_s_memtime();
  // 2. input transform, one (ci, tile) item per thread.  Tile t = (pooled row
  // 2 pg + t / 7, col t % 7): its 6x6 window starts at halo row 2 (t / 7),
  // halo col 2 (t % 7).  Tiles 14, 15 are zero.
  {
    const int t = tid & 15, ci = tid >> 4;
    float d[36], v[36];
    const int r0 = t < 14 ? 2 * (t / 7) : C2_XS_ROWS, c0 = t < 14 ? 2 * (t % 7) : 0;
    const float* src = xs + (r0 * C2_XS_COLS + c0) * 33 + ci;
#pragma unroll
    for (int yy = 0; yy < 6; ++yy)
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) d[yy * 6 + xx] = src[(yy * C2_XS_COLS + xx) * 33];
    wino::input_tile(d, v);
    float* vp = V + ci * 16 + t;
#pragma unroll
    for (int p = 0; p < 36; ++p) vp[p * 512] = v[p];
  }
  __syncthreads();
  if constexpr (PROF) stamp[2] = __builtin_amdgcn_s_memtime();
  // 3. batched products.  16x16x4 fragment maps: A lane l = V[tile l & 15][ci
  // 4 s + l >> 4]; B lane l = U[ci 4 s + l >> 4][co 16 q + l & 15]; C lane l,
  // reg j = (tile 4 (l >> 4) + j, co 16 q + l & 15).
  // Wave w owns co quarter q = w & 3 and the 18 points of half ph = w >> 2
  // (144 MFMAs per wave, every wave the same), two points at a time (one
  // accumulator chain each, interleaved); each point is
  // folded into the four 2x2 outputs right after its 8 k-steps.  The two
  // halves' partials meet once (LDS) and the ph = 0 waves finish bias, ReLU,
  // pool and argmax straight from their registers: no (tile, co) re-read of
  // all eight waves' partial outputs.
  f32x4 y[4];  // [output i*2+j] for (tiles, co quarter qw)
#pragma unroll
  for (int o = 0; o < 4; ++o) y[o] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int p0 = 18 * ph + 2 * i;
    float(&cur)[16] = (i & 1) ? bB : bA;
    float(&nxt)[16] = (i & 1) ? bA : bB;
    if (i < 8) loadb2(p0 + 2, nxt);
    __builtin_amdgcn_sched_barrier(0);
    float av[16];
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int k = 0; k < 8; ++k) av[pt * 8 + k] = V[(p0 + pt) * 512 + k * 64 + lane];
    // one accumulator chain per point (k order 0..7), the two points' MFMAs
    // interleaved
    f32x4 acc[2];
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) acc[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) acc[pt] = mfma16x16x4(av[pt * 8 + k], cur[pt * 8 + k], acc[pt]);
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int o = 0; o < 4; ++o) y[o] += kWinoCoef.c[p0 + pt][o] * acc[pt];
    __builtin_amdgcn_sched_barrier(0);
  }
  // 4. the two point halves' partials summed once (half 1 -> LDS -> half 0),
  // then bias + ReLU + 2x2 pool + argmax from the half-0 waves' registers
  if constexpr (PROF) stamp[3] = __builtin_amdgcn_s_memtime();
  __syncthreads();  // every wave is done reading V
  float* R = V;     // [qw][o][reg][lane]
  if (ph == 1) {
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int j = 0; j < 4; ++j) R[((qw * 4 + o) * 4 + j) * 64 + lane] = y[o][j];
  }
  __syncthreads();
  if (ph == 0) {
    const int co = 16 * qw + (lane & 15);
    const float bias = b2[co];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 4 * (lane >> 4) + j;  // tile = pooling window of the block
      float v[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) v[o] = y[o][j] + R[((qw * 4 + o) * 4 + j) * 64 + lane];
      float m = v[0];
      int qq = 0;
#pragma unroll
      for (int o = 1; o < 4; ++o) {
        if (v[o] > m) {  // strict: first max wins (TF MaxPool order)
          m = v[o];
          qq = o;
        }
      }
      const int pr = pr0 + t / 7, pc = t % 7;
      if (t < 14 && pr < 7) {
        const int fi = (pr * 7 + pc) * 64 + co;
        const int oi = n * FC1_IN + fi;
        const float o = fmaxf(m + bias, 0.f);
        out[oi] = o;
        if (argmax) argmax[oi] = (uint8_t)qq;
        if (out_t) out_t[(size_t)fi * batch + n] = o;
      }
    }
  } else if constexpr (FUSED) {
    // the half-1 waves write the owned conv1 rows while half 0 runs the epilogue
    halo_flush_owned(c1, xs, q1, n, pg, tid - WNT / 2, WNT / 2);
  }
  if constexpr (PROF) {
    stamp[4] = __builtin_amdgcn_s_memtime();
    if ((tid & 63) == 0)
      for (int k = 0; k < 5; ++k) prof[((size_t)blockIdx.x * WNW + wave) * 5 + k] = stamp[k];
  }
}

// ------------------------------------ conv2 bwd-data, Winograd F(2x2,5x5) ----
// dA1 = dY2 (x) rot180(W2) with the channel roles swapped: the forward form
// on the NHWC dY2 image dy2 [n][14][14][64] (fc1 backward's coalesced output,
// the filter gradient's operand) with the filters Ud [36][64][32].  Each
// half's input band (8 pixel rows x 14 columns x 32 channels) is fetched with
// coalesced float4 loads - both halves' issued at the start - and staged
// channel-major with zero borders in LDS (WB_FLOATS), from which the
// (tile, channel) threads read their 6 x 6 windows.  A channel-major
// zero-bordered copy written by fc1 backward instead cost its dX role 2.7 us
// of 8-byte scattered stores; per-thread window loads straight from the NHWC
// image (36 single floats) were 3.3 us slower than from that copy.  Block = (image,
// pair of 2x2-tile rows) = 14 tiles (M 16), N = 32 input channels of conv2,
// K = 64 in two halves of 32 (the transformed image V is 72 KB per half).
// Waves = (ci half, quarter of the 36 points), each point's 8 k-steps per K
// half folded into the 2x2 outputs at once; the four quarters' partials are
// summed in order by the epilogue threads.  Half 1's input windows are loaded
// under half 0's products.  Epilogue: the ReLU1 mask (a1 > 0), NHWC da1m.
// Optional FC SGD (single rank): every conv block, once its own work is done,
// updates a 1/(2 x blocks) slice of the FC bucket (two 256-thread units).
// Appended role blocks instead waited for a free CU behind the conv blocks
// (one conv block fills a CU: 8 waves at 150 VGPRs), a serial tail of their
// whole duration (bwd-data 24 us in the step vs 15 alone).
// c1.part1 != nullptr: each block also computes the conv1 filter-gradient
// partial of its band of a1 rows (4 pg .. 4 pg + 3) straight from the dA1
// values it just produced (part1[n * 4 + pg], the conv1_filter_unit math):
// no second pass over dA1 and no role blocks in the filter-gradient launch.
// the staged input band of one K half: [32 ch][8 rows][18 cols] (pixel rows
// 4 pg - 2 .. 4 pg + 5, columns -2 .. 15; zero outside the image)
constexpr int WB_ROWS = 8, WB_COLS = 18, WB_FLOATS = 32 * WB_ROWS * WB_COLS;
constexpr int WD_SMEM = WV_FLOATS + WB_FLOATS;  // bwd-data body LDS (floats)

// Block body (blk of nblk, threads 0 .. WNT - 1, smem: WD_SMEM floats): the
// standalone kernel below, or the bwd-data role of the merged conv2 backward
// launch
template <bool PROF, bool FC = true>
__device__ __forceinline__ void bwd_data_wino_block(
    int blk, int nblk, const float* __restrict__ dy2, const float* __restrict__ Ud,
    const float* __restrict__ a1, int batch, float* __restrict__ da1m, const FcSgd& sgd,
    const C1Filter& c1, unsigned long long* __restrict__ prof, float* smem) {
  // PROF (labs): s_memtime per wave -> prof[block][wave][7]: start, half 0
  // transform / products, half 1 transform / products, dA1 written, end
  unsigned long long stamp[7];
  if constexpr (PROF) stamp[0] = __builtin_amdgcn_s_memtime();
  float* V = smem;
  float* SB = smem + WV_FLOATS;  // staged input band (WB_FLOATS)
  // this block's FC SGD slice (sgd.nblk = 2 x blocks units), after its conv work
  auto fc_sgd_tail = [&]() {
    if (!FC || sgd.n4 == 0) return;
    const int half = threadIdx.x >> 8, t = threadIdx.x & 255;
    if (sgd.a2)  // fused fc1 dW1 + SGD tiles, first halves of every block first
      for (int d = half * nblk + blk; d < FC1BWD_DW_BLOCKS; d += 2 * nblk)
        fc1_dw_sgd(sgd, d, t);
    fc_sgd_role(sgd, 2 * blk + half, nullptr, t);
  };
  const int n = blk >> 2, pg = blk & 3;
  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform in an SGPR: the point index p, its output-transform weights
  // (scalar loads) and the fragment bases are then scalar
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wave = (ci half qw = wave & 1, point quarter pq = wave >> 1: points 9 pq ..
  // 9 pq + 8): 72 MFMAs per wave per K half, every wave the same
  const int qw = wave & 1, pq = wave >> 1;
  f32x4 y[4];
#pragma unroll
  for (int o = 0; o < 4; ++o) y[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  // input bands: 2 x (8 rows x 14 columns x 8 float4) = 2 x 896 float4, both
  // halves' coalesced loads issued now (rows outside the image read a clamped
  // row and stage zeros); a (tile, channel) item per thread reads its 6 x 6
  // window from the staged band
  const int it_t = tid & 15, it_c = tid >> 4;
  const int it_tr = 2 * pg + it_t / 7, it_tc = it_t % 7;
  const bool it_ok = it_t < 14 && it_tr < 7;
  const int y0b = 4 * pg - 2;  // image row of band row 0
  constexpr int BAND4 = WB_ROWS * 14 * 8, BJ = (BAND4 + WNT - 1) / WNT;  // 896 float4, 2 / thread
  float4 bq[2][BJ];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int f = min(tid + WNT * j, BAND4 - 1), c4 = f & 7, pix = f >> 3;
      const int y = min(max(y0b + pix / 14, 0), 13), x = pix % 14;
      bq[hh][j] = *reinterpret_cast<const float4*>(dy2 + ((size_t)(n * 14 + y) * 14 + x) * 64 +
                                                   32 * hh + 4 * c4);
    }
  auto stage = [&](int hh) {  // band hh -> SB (zero borders); no barrier
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int f = tid + WNT * j;
      if (f < BAND4) {
        const int c4 = f & 7, pix = f >> 3, r = pix / 14, x = pix % 14;
        const bool ok = y0b + r >= 0 && y0b + r < 14;
        float* d = SB + ((4 * c4) * WB_ROWS + r) * WB_COLS + x + 2;
        d[0] = ok ? bq[hh][j].x : 0.f;
        d[WB_ROWS * WB_COLS] = ok ? bq[hh][j].y : 0.f;
        d[2 * WB_ROWS * WB_COLS] = ok ? bq[hh][j].z : 0.f;
        d[3 * WB_ROWS * WB_COLS] = ok ? bq[hh][j].w : 0.f;
      }
    }
    // the 2 + 2 zero columns of every (channel, row): 32 x 8 x 4 = 1024 cells
    for (int e = tid; e < 32 * WB_ROWS * 4; e += WNT) {
      const int col = e & 3, cr = e >> 2;
      SB[cr * WB_COLS + (col < 2 ? col : WB_COLS - 4 + col)] = 0.f;
    }
  };
  auto load_in = [&](float (&d)[36]) {  // this thread's window from the staged band
    const float* src = SB + (it_c * WB_ROWS + 2 * (it_ok ? it_tr : 2 * pg) - 4 * pg) * WB_COLS +
                       2 * (it_ok ? it_tc : 0);
#pragma unroll
    for (int yy = 0; yy < 6; ++yy)
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) d[yy * 6 + xx] = src[yy * WB_COLS + xx];
  };
  stage(0);
  __syncthreads();
  float din[36];
  load_in(din);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    {  // input transform
      float v[36];
      wino::input_tile(din, v);
#pragma unroll
      for (int p = 0; p < 36; ++p) V[(p * 32 + it_c) * 16 + it_t] = it_ok ? v[p] : 0.f;
    }
    __syncthreads();
    if constexpr (PROF) stamp[1 + 2 * half] = __builtin_amdgcn_s_memtime();
    // fragment (s, qw) of point p, s in [8 half, 8 half + 8): ub + p * 2048 + s * 128
    const float* ub = Ud + half * 1024 + qw * 64 + lane;
    auto loadb3 = [&](int p0, float(&b)[24]) {
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
#pragma unroll
        for (int k = 0; k < 8; ++k) b[pt * 8 + k] = ub[(p0 + pt) * 2048 + k * 128];
    };
    float bA[24], bB[24];
    loadb3(9 * pq, bA);
    // half 1's band into the staging buffer (every thread read its half-0
    // window before the barrier above); read back after the next barrier
    if (half == 0) stage(1);
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // three points at a time
      const int p0 = 9 * pq + 3 * i;
      float(&cur)[24] = (i & 1) ? bB : bA;
      float(&nxt)[24] = (i & 1) ? bA : bB;
      if (i < 2) loadb3(p0 + 3, nxt);
      __builtin_amdgcn_sched_barrier(0);
      float av[24];
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
#pragma unroll
        for (int k = 0; k < 8; ++k) av[pt * 8 + k] = V[(p0 + pt) * 512 + k * 64 + lane];
      f32x4 acc[3];  // one chain per point (k order), three interleaved
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) acc[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int pt = 0; pt < 3; ++pt)
          acc[pt] = mfma16x16x4(av[pt * 8 + k], cur[pt * 8 + k], acc[pt]);
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
#pragma unroll
        for (int o = 0; o < 4; ++o) y[o] += kWinoCoef.c[p0 + pt][o] * acc[pt];
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PROF) stamp[2 + 2 * half] = __builtin_amdgcn_s_memtime();
    __syncthreads();  // V is rewritten by the next half / the reduction
    if (half == 0) load_in(din);
  }
  // every wave's partial outputs -> R [qw][pq][o][reg][lane]; the epilogue
  // threads sum the four point quarters in order
  float* R = V;
  auto rix = [&](int pq_, int o, int q, int j) { return (((q * 4 + pq_) * 4 + o) * 4 + j) * 64; };
#pragma unroll
  for (int o = 0; o < 4; ++o)
#pragma unroll
    for (int j = 0; j < 4; ++j) R[rix(pq, o, qw, j) + lane] = y[o][j];
  // conv1 band: the padded input rows 8 pg - 2 .. 8 pg + 9 (x 32 columns)
  // staged next to R while the sums are read; argmax codes loaded early
  constexpr int C1X = 12 * 32;
  float* xs1 = V + 2 * 4 * 4 * 4 * 64;
  float* red1 = xs1 + C1X;  // [7 waves][26 * 32 + 1]
  const bool do_c1 = c1.part1 != nullptr;
  const int ci = tid & 31, t = tid >> 5;
  const int tr = 2 * pg + t / 7, tc = t % 7;
  const bool own = t < 14 && tr < 7;
  int q1[4] = {0, 0, 0, 0};
  // the ReLU1 mask operands, loaded before the barrier (a load issued after
  // the dA1 stores below would wait for them: vmcnt counts both)
  float a1v[4] = {0.f, 0.f, 0.f, 0.f};
  if (own) {
#pragma unroll
    for (int o = 0; o < 4; ++o)
      a1v[o] = a1[((size_t)(n * 14 + 2 * tr + (o >> 1)) * 14 + 2 * tc + (o & 1)) * 32 + ci];
  }
  if (do_c1) {
    const long long off = batch_offset_dev(c1.step, c1.n_local, batch);
    const float* x = c1.data + (off + n) * 784;
    const int y0 = 8 * pg - 2;
    if (tid < C1X) {
      const int yy = y0 + tid / 32, xx = tid % 32 - 2;
      xs1[tid] = (yy >= 0 && yy < 28 && xx >= 0 && xx < 28) ? x[yy * 28 + xx] : 0.f;
    }
    if (own) {
#pragma unroll
      for (int o = 0; o < 4; ++o)
        q1[o] = c1.idx1[((size_t)(n * 14 + 2 * tr + (o >> 1)) * 14 + 2 * tc + (o & 1)) * 32 + ci];
    }
  }
  __syncthreads();
  float g1[4] = {0.f, 0.f, 0.f, 0.f};
  if (own) {
    const int q = ci >> 4, l = (t >> 2) * 16 + (ci & 15), j = t & 3;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) sum += R[rix(w, o, q, j) + l];
      const size_t oi =
          ((size_t)(n * 14 + 2 * tr + (o >> 1)) * 14 + 2 * tc + (o & 1)) * 32 + ci;
      g1[o] = a1v[o] > 0.f ? sum : 0.f;
      da1m[oi] = g1[o];
    }
  }
  if constexpr (PROF) stamp[5] = __builtin_amdgcn_s_memtime();
  if (do_c1) {
    // dW1[t][ci] += dA1 * x[argmax pixel + tap] over the thread's 4 positions
    float acc[26];
#pragma unroll
    for (int k = 0; k < 26; ++k) acc[k] = 0.f;
    if (own) {
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        if (g1[o] != 0.f) {
          const int py = 2 * tr + (o >> 1), px = 2 * tc + (o & 1);
          const int ly = 2 * py + (q1[o] >> 1) - 8 * pg;  // xs1 row of tap kh = 0
          const int lx = 2 * px + (q1[o] & 1);            // xs1 col of tap kw = 0
#pragma unroll
          for (int kh = 0; kh < 5; ++kh)
#pragma unroll
            for (int kw = 0; kw < 5; ++kw) acc[kh * 5 + kw] += g1[o] * xs1[(ly + kh) * 32 + lx + kw];
          acc[25] += g1[o];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 26; ++k) acc[k] += __shfl_xor(acc[k], 32, 64);  // tiles 2w, 2w + 1
    if (wave < 7 && (tid & 32) == 0) {
#pragma unroll
      for (int k = 0; k < 26; ++k) red1[wave * (26 * 32 + 1) + k * 32 + ci] = acc[k];
    }
    __syncthreads();
    for (int i = tid; i < 26 * 32; i += WNT) {
      float sv = 0.f;
#pragma unroll
      for (int w = 0; w < 7; ++w) sv += red1[w * (26 * 32 + 1) + i];
      c1.part1[(size_t)(n * 4 + pg) * 832 + i] = sv;
    }
  }
  if constexpr (PROF) {
    stamp[6] = do_c1 ? __builtin_amdgcn_s_memtime() : stamp[5];
    if (lane == 0)
      for (int k = 0; k < 7; ++k) prof[((size_t)blk * WNW + wave) * 7 + k] = stamp[k];
  }
  fc_sgd_tail();
}

template <bool PROF = false>
__global__ __launch_bounds__(WNT) void conv2_bwd_data_wino_kernel(
    const float* __restrict__ dy2, const float* __restrict__ Ud, const float* __restrict__ a1,
    int batch, float* __restrict__ da1m, const FcSgd sgd, const C1Filter c1,
    unsigned long long* __restrict__ prof = nullptr) {
  __shared__ float smem[WD_SMEM];
  bwd_data_wino_block<PROF>(blockIdx.x, gridDim.x, dy2, Ud, a1, batch, da1m, sgd, c1, prof, smem);
}

// ------------------------------------------ Winograd conv2 bwd-filter ----
// dW2 = G^T [ sum_tiles V (.) (AT^T dY AT) ] G per (ci, co) - the gradient of
// the forward transform in wino.h: for each of the 36 points p = (a, b) the
// product M_p[ci][co] = sum_tiles V_p[tile][ci] dY'_p[tile][co] is a GEMM
// over the tiles (2.78x fewer MFMAs than the 25-tap form), dY' = AT^T dY AT of
// the tile's 2x2 pre-pool gradient (dy2).  Block = (group of 2 images, 16 ci,
// 16 co) and all 36 points, so the output transform runs in-block and the
// partials are ordinary tap slabs part2[g][t][ci][co] (grad_finalize /
// sgd_finalize unchanged).  12 waves = (point row a, half of the tile rows):
// three per SIMD, so each SIMD's matrix pipe interleaves three MFMA streams
// (6 waves, one per row, measured 19-28 K cycles in the main loop: 1.5 waves
// per SIMD left the pipe idle behind each wave's LDS -> VALU -> MFMA chain):
//   1. the group's a1 (16 ci, zero border) and dY2 (16 co) slices -> LDS, one
//      round of float4 loads
//   2. the MFMA k index runs over tiles as (row set m, column tx, quad kq):
//      lane quad kq walks tile row 4 m + kq from tx = 0 to 6 (the wave's half:
//      row sets 2 h, 2 h + 1), so the column
//      transform slides - each step reads only the 2 new columns (5 nonzero
//      BT rows, one ds_read_b64 each) - then the row transform gives the 6
//      points' V, two ds_read_b64 give the 2x2 dY -> dY' (row a), and 6
//      v_mfma_f32_16x16x4_f32 run (points (a, 0..5)); 14 k-steps, no
//      staging buffers and no barriers in the loop.  The compiler pairs the
//      b64 reads into ds_read2_b64 (16-lane bank groups, 32 banks): a row of
//      18 floats per channel puts the 16 channels' pairs on distinct banks
//      (a 20-float row measured 1,446 conflict cycles per wave)
//   3. S_ah[kw] = sum_b G[b][kw] M_h[a][b] per wave -> LDS, then dW[kh][kw] =
//      sum_a G[a][kh] (S_a0 + S_a1)[kw] (no FMA contraction) -> part2; the ci-tile-0
//      blocks also write the group's db2 partial
// The conv1 filter grad runs as whole-image role blocks after the conv2
// blocks.
constexpr int WF_IMG = 2, WF_ROWS = 7 * WF_IMG, WF_SETS = (WF_ROWS + 3) / 4;
constexpr int WF_NT = 768;
constexpr int WF_XLD = 18;                        // floats per (image row, ci)
constexpr int WF_XS = WF_IMG * 18 * 16 * WF_XLD;  // [img][row][ci][col]
constexpr int WF_DLD = 18;                        // floats per (dY row, co): 14 + 4
constexpr int WF_DS = WF_IMG * 14 * 16 * WF_DLD;  // [img][row][co][col]
constexpr int WF_SMEM = WF_XS + WF_DS;
static_assert(6 * 2 * 5 * 4 * 64 <= WF_SMEM, "S_ah reduction reuses the slices");

template <int A>
__device__ __forceinline__ void wino_wgrad_row(const float* __restrict__ xs,
                                               const float* __restrict__ dys, int nimg,
                                               int lane, int half, f32x4 (&acc)[6]) {
  const int kq = lane >> 4, ch = lane & 15;
  constexpr float al0 = wino::kAT[0][A], al1 = wino::kAT[1][A];
#pragma unroll 1
  for (int m = half * (WF_SETS / 2); m < (half + 1) * (WF_SETS / 2); ++m) {
    const int R = 4 * m + kq, Rc = min(R, WF_ROWS - 1);
    const int img = Rc / 7, ty = Rc - 7 * img;
    const bool ok = R < WF_ROWS && img < nimg;  // pad rows: dY' = 0
    const float* xrow = xs + ((img * 18 + 2 * ty) * 16 + ch) * WF_XLD;
    const float* drow = dys + ((img * 14 + 2 * ty) * 16 + ch) * WF_DLD;
    // column pair pc of the window: t[c] = sum_i BT[A][i] x[2 ty + i][2 pc + c]
    auto colpair = [&](int pc, float& c0, float& c1) {
      c0 = 0.f;
      c1 = 0.f;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        if (wino::kBT[A][i] == 0.f) continue;
        const float2 x = *reinterpret_cast<const float2*>(xrow + i * 16 * WF_XLD + 2 * pc);
        c0 += wino::kBT[A][i] * x.x;
        c1 += wino::kBT[A][i] * x.y;
      }
    };
    float t[6];
    colpair(0, t[0], t[1]);
    colpair(1, t[2], t[3]);
#pragma unroll
    for (int tx = 0; tx < 7; ++tx) {
      if (tx > 0) {
        t[0] = t[2];
        t[1] = t[3];
        t[2] = t[4];
        t[3] = t[5];
      }
      colpair(tx + 2, t[4], t[5]);
      float v[6];
      wino::bt6<1, 1>(t, v);
      const int ds = 2 * tx;
      const float2 d0 = *reinterpret_cast<const float2*>(drow + ds);
      const float2 d1 = *reinterpret_cast<const float2*>(drow + 16 * WF_DLD + ds);
      float r0 = al0 * d0.x + al1 * d1.x, r1 = al0 * d0.y + al1 * d1.y;
      r0 = ok ? r0 : 0.f;
      r1 = ok ? r1 : 0.f;
      const float u[6] = {r0, r0 + r1, r0 - r1, r0 + 2.f * r1, r0 - 0.5f * r1, r1};
#pragma unroll
      for (int b = 0; b < 6; ++b) acc[b] = mfma16x16x4(v[b], u[b], acc[b]);
    }
  }
}

// PROF: per-wave s_memtime stamps at the phase boundaries -> prof[block][wave][5]
// (scripts/wino_lab.py --phases; never used by the executor)
// Block body (blk): the standalone kernel below, or the filter-gradient role
// of the merged conv2 backward launch (blk = block index - bwd-data blocks, a
// multiple of 8: the XCD-aware group mapping is kept)
constexpr int WF_SMEM_ALL = WF_SMEM > c1f_smem<1, WF_NT / 64>() ? WF_SMEM : c1f_smem<1, WF_NT / 64>();
template <bool PROF>
__device__ __forceinline__ void bwd_filter_wino_block(
    int blk, int batch, const float* __restrict__ a1p, const float* __restrict__ dy2,
    float* __restrict__ part2, float* __restrict__ part_db2, int nwg, const C1Filter& c1,
    unsigned long long* __restrict__ prof, float* smem) {
  unsigned long long stamp[5];
  if constexpr (PROF) stamp[0] = __builtin_amdgcn_s_memtime();
  if (blk >= nwg) {  // conv1 filter-grad role (its dA1 is final)
    conv1_filter_unit<WF_NT, 1>(blk - nwg, batch, c1, smem);
    return;
  }
  // XCD-aware: the 8 (ci, co) tiles of an image group share one XCD's L2
  const int ngroups = nwg / 8, bid = blk;
  int g, sub;
  if (ngroups % 8 == 0) {
    const int x = bid & 7, idx = bid >> 3;
    g = x + 8 * (idx >> 3);
    sub = idx & 7;
  } else {
    g = bid >> 3;
    sub = bid & 7;
  }
  const int ci_t = sub & 1, co_t = sub >> 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int arow = wave % 6, half = wave / 6;
  const int n0 = g * WF_IMG, nimg = min(WF_IMG, batch - n0);
  float* xs = smem;
  float* dys = smem + WF_XS;
  // 1. slices -> LDS (every load issued before the first store)
  {
    constexpr int NX = WF_IMG * 324 * 4, ND = WF_IMG * 196 * 4;  // float4s
    constexpr int PX = (NX + WF_NT - 1) / WF_NT, PD = (ND + WF_NT - 1) / WF_NT;
    float4 vx[PX], vd[PD];
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = min(tid + j * WF_NT, NX - 1), pix = i >> 2, img = pix / 324;
      const int n = min(n0 + img, batch - 1);  // clamped: images past the batch are masked
      vx[j] = *reinterpret_cast<const float4*>(
          a1p + ((size_t)n * 324 + (pix - 324 * img)) * 32 + ci_t * 16 + 4 * (i & 3));
    }
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const int i = min(tid + j * WF_NT, ND - 1), pix = i >> 2, img = pix / 196;
      const int n = min(n0 + img, batch - 1);
      vd[j] = *reinterpret_cast<const float4*>(
          dy2 + ((size_t)n * 196 + (pix - 196 * img)) * 64 + co_t * 16 + 4 * (i & 3));
    }
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = tid + j * WF_NT;
      if (i < NX) {
        const int pix = i >> 2, img = pix / 324, pp = pix - 324 * img, row = pp / 18;
        const int col = pp - 18 * row, c0 = 4 * (i & 3);
        float* d = xs + ((img * 18 + row) * 16 + c0) * WF_XLD + col;
        d[0] = vx[j].x;
        d[WF_XLD] = vx[j].y;
        d[2 * WF_XLD] = vx[j].z;
        d[3 * WF_XLD] = vx[j].w;
      }
    }
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const int i = tid + j * WF_NT;
      if (i < ND) {
        const int pix = i >> 2, img = pix / 196, pp = pix - 196 * img, row = pp / 14;
        const int col = pp - 14 * row, c0 = 4 * (i & 3);
        float* d = dys + ((img * 14 + row) * 16 + c0) * WF_DLD + col;
        d[0] = vd[j].x;
        d[WF_DLD] = vd[j].y;
        d[2 * WF_DLD] = vd[j].z;
        d[3 * WF_DLD] = vd[j].w;
      }
    }
  }
  __syncthreads();
  if constexpr (PROF) stamp[1] = __builtin_amdgcn_s_memtime();
  // 2. the wave's point row
  f32x4 acc[6];
#pragma unroll
  for (int b = 0; b < 6; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  switch (arow) {
    case 0: wino_wgrad_row<0>(xs, dys, nimg, lane, half, acc); break;
    case 1: wino_wgrad_row<1>(xs, dys, nimg, lane, half, acc); break;
    case 2: wino_wgrad_row<2>(xs, dys, nimg, lane, half, acc); break;
    case 3: wino_wgrad_row<3>(xs, dys, nimg, lane, half, acc); break;
    case 4: wino_wgrad_row<4>(xs, dys, nimg, lane, half, acc); break;
    default: wino_wgrad_row<5>(xs, dys, nimg, lane, half, acc); break;
  }
  if constexpr (PROF) stamp[2] = __builtin_amdgcn_s_memtime();
  float db = 0.f;  // db2 partial: thread (co, dY row stripe), ci-tile-0 blocks
  if (ci_t == 0 && tid < 256) {
    const int co = tid & 15;
    for (int L = tid >> 4; L < nimg * 14; L += 16) {
      const float* dl = dys + (L * 16 + co) * WF_DLD;
#pragma unroll
      for (int x = 0; x < 14; ++x) db += dl[x];
    }
  }
  float* dbr = smem + 6 * 2 * 5 * 4 * 64;  // db2 stripes [16][16], after red
  __syncthreads();  // the slices are reused below
  // 3. S_ah[kw] = sum_b G[b][kw] M_h[a][b]   (this wave's a, h)
  float* red = smem;  // [a][h][kw][j][lane]
  {
#pragma clang fp contract(off)
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sv = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b)
          if (wino::kG[b][kw] != 0.f) sv += wino::kG[b][kw] * acc[b][j];
        red[(((arow * 2 + half) * 5 + kw) * 4 + j) * 64 + lane] = sv;
      }
  }
  if (ci_t == 0 && tid < 256) dbr[tid] = db;
  __syncthreads();
  if constexpr (PROF) stamp[3] = __builtin_amdgcn_s_memtime();
  if (tid < 256) {  // dW[kh][kw] = sum_a G[a][kh] S_a[kw] for element (j, lane')
#pragma clang fp contract(off)
    const int j = tid >> 6, l = tid & 63;
    float S[6][5];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw)
        S[a][kw] = red[(((a * 2) * 5 + kw) * 4 + j) * 64 + l] +
                   red[(((a * 2 + 1) * 5 + kw) * 4 + j) * 64 + l];
    const int ci = ci_t * 16 + 4 * (l >> 4) + j, co = co_t * 16 + (l & 15);
    float* out = part2 + (size_t)g * 51200 + ci * 64 + co;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        float sv = 0.f;
#pragma unroll
        for (int a = 0; a < 6; ++a)
          if (wino::kG[a][kh] != 0.f) sv += wino::kG[a][kh] * S[a][kw];
        out[(kh * 5 + kw) * 2048] = sv;
      }
  }
  if (ci_t == 0 && tid < 16) {  // db2: one row per group (rows 4 g + 1..3 zero)
    float sv = 0.f;
#pragma unroll
    for (int st = 0; st < 16; ++st) sv += dbr[st * 16 + tid];
    const int co = co_t * 16 + tid;
    part_db2[(g * 4) * 64 + co] = sv;
#pragma unroll
    for (int r = 1; r < 4; ++r) part_db2[(g * 4 + r) * 64 + co] = 0.f;
  }
  if constexpr (PROF) {
    stamp[4] = __builtin_amdgcn_s_memtime();
    if (lane == 0)
      for (int k = 0; k < 5; ++k) prof[((size_t)blk * (WF_NT / 64) + wave) * 5 + k] = stamp[k];
  }
}

template <bool PROF>
__global__ __launch_bounds__(WF_NT) void conv2_bwd_filter_wino_kernel(
    int batch, const float* __restrict__ a1p, const float* __restrict__ dy2,
    float* __restrict__ part2, float* __restrict__ part_db2, int nwg, const C1Filter c1,
    unsigned long long* __restrict__ prof) {
  __shared__ float smem[WF_SMEM_ALL];
  bwd_filter_wino_block<PROF>(blockIdx.x, batch, a1p, dy2, part2, part_db2, nwg, c1, prof, smem);
}

// Both Winograd conv2 backward products in ONE launch (they depend only on
// fc1 backward): blocks [0, nd) run the bwd-data body on their first WNT
// threads (the surplus waves end at once - a barrier waits only for the
// waves still alive), the rest the filter-gradient body.  One block per CU
// either way (LDS, VGPRs); a CU moves on to its next block as soon as it
// is done, so there is no launch boundary and no drain between the two.
// No FC SGD tail here (its registers would spill at 768 threads): with the
// FC SGD in the bwd-data launch the executor keeps the two launches.
// ---- xGMI FC role (mnist.h XgmiStepArgs): slice blk = blockIdx.x of this
// rank's FC segment - sum every rank's grads (rank order), momentum SGD on
// this rank's params / momentum, barrier, then copy the same slice of every
// other segment from its owner.  Run by xgmi_step_kernel, or as the first
// blocks of the merged conv2 backward launch (conv2_bwd_wino_kernel: the FC
// exchange overlaps the conv backward on the other CUs).
constexpr int XS_UNROLL = 2;
// as role blocks of the conv2 backward launch: few, so they hand their CUs
// back within the launch's first round of conv blocks (512 blocks = 2 exact
// rounds on 256 CUs; every CU held longer costs a third round)
constexpr int XS_FC_ROLE_BLOCKS = 16;

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
  return a;
}

// labs (XgmiStepArgs::prof): stamp i of this block
__device__ __forceinline__ void xs_stamp(const XgmiStepArgs& a, int i) {
  if (a.prof && threadIdx.x == 0) a.prof[6 * blockIdx.x + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ void xgmi_fc_role(const XgmiStepArgs& a, unsigned* ep) {
  const xgmi::Sync& s = a.sync;
  const int n = s.nranks, me = s.rank, tid = threadIdx.x, nt = blockDim.x;
  const float lr = *a.lr;
  // peer-visible bytes go through system-scope loads / stores (kernels/xgmi.h)
  const long long fcb = a.fc4 * 16;
  xgmi::Rsrc gr[xgmi::kMaxRanks], wr[xgmi::kMaxRanks];
#pragma unroll
  for (int r = 0; r < xgmi::kMaxRanks; ++r)
    if (r < n) {
      gr[r] = xgmi::rsrc(a.g[r], fcb);
      wr[r] = xgmi::rsrc(a.w[r], fcb);
    }
  const unsigned e = xgmi::next_epoch(s, ep);
  xs_stamp(a, 1);
  xgmi::barrier(s, 0, e, /*release=*/true);  // the grads come from fc1 backward
  xs_stamp(a, 2);
  const long long lo = (long long)blockIdx.x * a.per4;
  const long long hi = lo + a.per4 < a.seg4 ? lo + a.per4 : a.seg4;
  long long t0 = xgmi::now_ticks();
  const long long base = (long long)me * a.seg4;
  float4* W4 = reinterpret_cast<float4*>(a.w[me]);
  float4* M4 = reinterpret_cast<float4*>(a.mom);
  for (long long i0 = lo + tid; i0 < hi; i0 += (long long)nt * XS_UNROLL) {
    float4 v[xgmi::kMaxRanks][XS_UNROLL], wv[XS_UNROLL], mv[XS_UNROLL];
#pragma unroll
    for (int u = 0; u < XS_UNROLL; ++u) {
      const bool ok = i0 + nt * u < hi;
      const unsigned off = (unsigned)((base + i0 + nt * u) * 16);
#pragma unroll
      for (int r = 0; r < xgmi::kMaxRanks; ++r)
        if (r < n && ok) v[r][u] = xgmi::ld4_peer(s, r, gr[r], off);
      if (ok) {
        wv[u] = W4[base + i0 + nt * u];
        mv[u] = M4[base + i0 + nt * u];
      }
    }
#pragma unroll
    for (int u = 0; u < XS_UNROLL; ++u) {
      if (i0 + nt * u >= hi) continue;
      float4 sv = v[0][u];
#pragma unroll
      for (int r = 1; r < xgmi::kMaxRanks; ++r)
        if (r < n) sv = add4(sv, v[r][u]);
      sgd4(wv[u], mv[u], sv, a.l2, lr, a.momentum, a.gscale);
      const long long i = base + i0 + nt * u;
      xgmi::st4_sys(wr[me], (unsigned)(i * 16), wv[u]);  // the peers gather it
      M4[i] = mv[u];
    }
  }
  xgmi::link_floor(s, t0, a.seg4 * 16);
  xs_stamp(a, 3);
  xgmi::barrier(s, 1, e, false);
  xs_stamp(a, 4);
  if (a.fc_in_bwd) return;  // the step launch gathers (xgmi_fc_gather)
  t0 = xgmi::now_ticks();
  // every other rank's slice at once (one round trip per XS_UNROLL float4s,
  // not one per rank)
  for (long long i0 = lo + tid; i0 < hi; i0 += (long long)nt * XS_UNROLL) {
    float4 v[xgmi::kMaxRanks][XS_UNROLL];
#pragma unroll
    for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u)
        if (r < n && r != me && i0 + nt * u < hi)
          v[r][u] = xgmi::ld4_sys(wr[r], (unsigned)(((long long)r * a.seg4 + i0 + nt * u) * 16));
#pragma unroll
    for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u)
        if (r < n && r != me && i0 + nt * u < hi) W4[(long long)r * a.seg4 + i0 + nt * u] = v[r][u];
  }
  xgmi::link_floor(s, t0, a.seg4 * 16);
}

// The gather half on its own (fc_in_bwd: the conv2 backward launch's role
// blocks did the exchange + SGD and passed their closing barrier, so every
// peer's segment is final): block gb of ng copies slice gb of every other
// rank's segment.  No barrier: a peer rewrites its segment only after the next
// step's arrival barrier, which this rank reaches after this launch.
__device__ void xgmi_fc_gather(const XgmiStepArgs& a, int gb, int ng) {
  const xgmi::Sync& s = a.sync;
  const int n = s.nranks, me = s.rank, tid = threadIdx.x;
  const long long fcb = a.fc4 * 16;
  const long long per = ((a.seg4 + ng - 1) / ng + 255) / 256 * 256;
  const long long lo = (long long)gb * per, hi = lo + per < a.seg4 ? lo + per : a.seg4;
  const long long t0 = xgmi::now_ticks();
  float4* W4 = reinterpret_cast<float4*>(a.w[me]);
  xgmi::Rsrc wr[xgmi::kMaxRanks];
#pragma unroll
  for (int r = 0; r < xgmi::kMaxRanks; ++r)
    if (r < n) wr[r] = xgmi::rsrc(a.w[r], fcb);
  // every other rank's slice at once (one round trip, not one per rank)
  for (long long i0 = lo + tid; i0 < hi; i0 += 256 * XS_UNROLL) {
    float4 v[xgmi::kMaxRanks][XS_UNROLL];
#pragma unroll
    for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u)
        if (r < n && r != me && i0 + 256 * u < hi)
          v[r][u] = xgmi::ld4_sys(wr[r], (unsigned)(((long long)r * a.seg4 + i0 + 256 * u) * 16));
#pragma unroll
    for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u)
        if (r < n && r != me && i0 + 256 * u < hi)
          W4[(long long)r * a.seg4 + i0 + 256 * u] = v[r][u];
  }
  xgmi::link_floor(s, t0, a.seg4 * 16);
}

__global__ __launch_bounds__(WF_NT) void conv2_bwd_wino_kernel(
    int nd, const float* __restrict__ Ud,
    const float* __restrict__ a1, int batch, float* __restrict__ da1m,
    const C1Filter c1, const float* __restrict__ a1p, const float* __restrict__ dy2,
    float* __restrict__ part2, float* __restrict__ part_db2, int nwg, const XgmiStepArgs xfc,
    unsigned long long* __restrict__ prof) {
  // one LDS pool for either role
  __shared__ float smem[WD_SMEM > WF_SMEM_ALL ? WD_SMEM : WF_SMEM_ALL];
  // prof (labs): per block [start, end] of the constant 100 MHz clock
  const unsigned long long t0 = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  struct Stamp {
    unsigned long long* p;
    unsigned long long t0;
    __device__ ~Stamp() {
      if (p && threadIdx.x == 0) {
        p[2 * blockIdx.x] = t0;
        p[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }
  } stamp{prof, t0};
  // world > 1 over xGMI: the first xfc.nfc blocks exchange + update the FC
  // bucket (its grads are final after fc1 backward) while the conv blocks run
  if ((int)blockIdx.x < xfc.nfc) {
    xgmi_fc_role(xfc, reinterpret_cast<unsigned*>(smem));
    return;
  }
  const int b = (int)blockIdx.x - xfc.nfc;
  if (b < nd) {
    if (threadIdx.x >= WNT) return;
    bwd_data_wino_block<false, false>(b, nd, dy2, Ud, a1, batch, da1m, FcSgd{}, c1, nullptr, smem);
  } else {
    bwd_filter_wino_block<false>(b - nd, batch, a1p, dy2, part2, part_db2, nwg, C1Filter{},
                                 nullptr, smem);
  }
}

// conv2 bwd-filter: dW2[t][ci][co] = sum_pix a1[pix shifted by tap t][ci] dY2[pix][co].
// Block = (tap, group of 4 images); 8 waves = 2 (N: co halves) x 4 (one image
// each, summed through LDS).  A[m = ci][k = pixel], B[k = pixel][co]: both
// gathered straight from L2 with channels on lanes, one image row ahead.  The
// centre tap's blocks also sum dY2 per channel (db2).
constexpr int C2F_IPW = 2;                   // images per wave
constexpr int C2F_GROUPS_IMG = 4 * C2F_IPW;  // images per block (4 image slots)

template <int C2F_DEPTH, bool CENTRE_ONLY>
__device__ void conv2_bwd_filter_v3(int bid, int batch, const float* __restrict__ a1p,
                                    const float* __restrict__ dy2, float* __restrict__ part2,
                                    float* __restrict__ part_db2, float* smem) {
  // XCD-aware mapping (blocks b, b+8, ... share an XCD's L2): every tap of an
  // image group runs on ONE XCD, so the group's a1/dY2 tiles are fetched into
  // that L2 once instead of into all eight.
  const int ngroups = (batch + C2F_GROUPS_IMG - 1) / C2F_GROUPS_IMG;
  int t, g;
  if (ngroups % 8 == 0) {
    const int x = bid & 7, idx = bid >> 3;
    t = idx % 25;
    g = x + 8 * (idx / 25);
  } else {
    t = bid % 25;
    g = bid / 25;
  }
  const int kh = t / 5, kw = t % 5;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsub = wave & 1, ih = wave >> 1;
  const int ci = lane & 31, kpar = lane >> 5;
  const int co = nsub * 32 + (lane & 31);
  f32x16 acc = zero16(), acc1 = zero16();
  float dbs = 0.f;
  // this wave's images: n0 + 4 i (i < C2F_IPW); rows of all of them form one
  // continuous prefetch pipeline (longer waves amortise the first-load latency
  // and the LDS-reduction epilogue)
  const int n0 = g * C2F_GROUPS_IMG + ih;
  if (n0 < batch) {
    const int nimg = min(C2F_IPW, (batch - n0 + 3) / 4);
    // a1p is zero-bordered ([n][18][18][32]): input pixel (y + kh - 2, x + kw
    // - 2) is padded pixel (y + kh, x + kw), always in range, and the 7
    // fragments of a row sit at compile-time offsets from one row pointer
    auto fetch = [&](int rr, float* A, float* Bv) {
      const int n = n0 + 4 * (rr / 14), y = rr % 14;
      const float* an = a1p + ((size_t)(n * 18 + y + kh) * 18 + kpar + kw) * 32 + ci;
      const float* dn = dy2 + ((size_t)n * 196 + y * 14 + kpar) * 64 + co;
#pragma unroll
      for (int xp = 0; xp < 7; ++xp) {
        A[xp] = an[2 * xp * 32];
        Bv[xp] = dn[2 * xp * 64];
      }
    };
    // C2F_DEPTH image rows in flight: row rr's fragments are moved out of
    // their ring slot and the slot is refilled with row rr + C2F_DEPTH
    // BEFORE row rr's MFMAs issue, so the loads have C2F_DEPTH rows of MFMA
    // work (7 MFMAs each) to land (measured: consuming in place and refilling
    // after the MFMAs, one row less of cover, was 1 us slower).  Only the
    // centre tap (which visits every dY2 element once) sums the bias grad.
    float ra[C2F_DEPTH][7], rb[C2F_DEPTH][7];
    const int nrows = 14 * nimg;
#pragma unroll
    for (int d = 0; d < C2F_DEPTH; ++d)
      if (d < nrows) fetch(d, ra[d], rb[d]);
    auto rows = [&](auto centre) {
      for (int rr = 0; rr < nrows; rr += C2F_DEPTH) {
#pragma unroll
        for (int d = 0; d < C2F_DEPTH; ++d) {
          const int row = rr + d;
          if (row < nrows) {
            float av[7], bv[7];
#pragma unroll
            for (int xp = 0; xp < 7; ++xp) {
              av[xp] = ra[d][xp];
              bv[xp] = rb[d][xp];
            }
            if (row + C2F_DEPTH < nrows) fetch(row + C2F_DEPTH, ra[d], rb[d]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int xp = 0; xp < 7; ++xp) {
              if (xp & 1)
                acc1 = mfma32x32x2(av[xp], bv[xp], acc1);
              else
                acc = mfma32x32x2(av[xp], bv[xp], acc);
              if constexpr (decltype(centre)::value) dbs += bv[xp];
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    };
    if (!CENTRE_ONLY || t == 12)
      rows(std::true_type{});
    else
      rows(std::false_type{});
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += acc1[r];
  // sum the four images (ih) through LDS, write one slab per block
  float* red = smem;
  if (ih > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(((ih - 1) * 2 + nsub) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (ih == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = acc[r];
#pragma unroll
      for (int j = 0; j < 3; ++j) s += red[((j * 2 + nsub) * 16 + r) * 64 + lane];
      const int row = t * 32 + mfma32_row(r, lane);  // (t, ci)
      part2[((size_t)g * 800 + row) * 64 + co] = s;
    }
  }
  if (t == 12) {  // centre tap visits every pixel exactly once: db2 partial
    dbs += __shfl_xor(dbs, 32, 64);
    if (kpar == 0) part_db2[(g * 4 + ih) * 64 + co] = dbs;
  }
}

// conv2 bwd-data, L2-direct: every wave owns a 32 (pixels) x 32 (ci) tile over
// half of K (co 0-31 / 32-63, the two halves of a wave pair summed through
// LDS) and streams its fragments straight from L2 into a 16-deep register
// ring.  M covers the batch in (n, y, x) order, so no tile is padded (the
// LDS-halo kernel above computes 30 % padding rows).  The A operand comes from
// dy2t, dY2 stored channel-major with a zero border ([n][co][18][20], written
// by fc1 backward): the 32 lanes of a half-wave read ~2 runs of consecutive
// floats of one channel plane per tap, bounds-check free; B = W2T[t][co][ci]
// (written by the conv2 forward kernel).  Measured 19.6 us vs 24.2 us for the
// halo kernel at B = 64 (in-graph).  (A K-permuted float4 variant of this
// structure touches one 128-B line per lane per load and runs slower: for
// fp32 MFMA the limit is cache lines per MFMA, not load instructions.)
constexpr int P32_LD = MNIST32_T_LD;
constexpr int A1T_PLANE = 18 * P32_LD;

template <int D, int NKS, class F>
__device__ __forceinline__ void kloop32(F&& frag, f32x16& c0, f32x16& c1) {
  float ra[D], rb[D];
#pragma unroll
  for (int d = 0; d < D; ++d) frag(d, ra[d], rb[d]);
#pragma unroll
  for (int ks = 0; ks < NKS; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (ks + d < NKS) {
        const float a = ra[d], b = rb[d];
        if (ks + D + d < NKS) frag(ks + D + d, ra[d], rb[d]);
        __builtin_amdgcn_sched_barrier(0);
        if (d & 1)
          c1 = mfma32x32x2(a, b, c1);
        else
          c0 = mfma32x32x2(a, b, c0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

__global__ __launch_bounds__(256) void conv2_bwd_data_l2_kernel(const float* __restrict__ dy2t,
                                                                const float* __restrict__ w2t,
                                                                const float* __restrict__ a1,
                                                                int batch,
                                                                float* __restrict__ da1m,
                                                                const FcSgd sgd) {
  __shared__ float red[2][16][64];
  const int nconv = gridDim.x - sgd.nblk;
  if ((int)blockIdx.x >= nconv) {
    fc_sgd_role(sgd, blockIdx.x - nconv, nullptr);  // fp32: no shadows
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int mtiles = batch * 49 / 8;
  const int mt_raw = xcd_remap(blockIdx.x, nconv) * 2 + (wave & 1), kk = wave >> 1;
  const int mt = min(mt_raw, mtiles - 1);
  const int m = mt * 32 + r, n = m / 196, p = m % 196, y = p / 14, x = p % 14;
  // padded source pixel of tap (kh, kw): (y + 4 - kh, x + 4 - kw)
  const float* ap = dy2t + ((size_t)(n * 64 + 32 * kk + h) * 18 + y + 4) * P32_LD + x + 4;
  const float* bp = w2t + (32 * kk + h) * 32 + r;
  f32x16 c0 = zero16(), c1 = zero16();
  kloop32<16, 400>(
      [&](int ks, float& a, float& b) {  // tap t, channel pair s
        const int t = ks >> 4, s2 = 2 * (ks & 15), kh = t / 5, kw = t % 5;
        a = ap[s2 * A1T_PLANE - kh * P32_LD - kw];
        b = bp[(t * 64 + s2) * 32];
      },
      c0, c1);
  if (kk == 1) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[wave & 1][k][lane] = c0[k] + c1[k];
  }
  __syncthreads();
  if (kk == 1 || mt_raw >= mtiles) return;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int mm = mt * 32 + mfma32_row(k, lane);
    const float g = c0[k] + c1[k] + red[wave & 1][k][lane];
    const size_t o = (size_t)mm * 32 + r;  // (n, y, x, ci) flat
    da1m[o] = a1[o] > 0.f ? g : 0.f;
  }
}

template <int DEPTH, bool CENTRE_ONLY>
__global__ __launch_bounds__(512) void conv2_bwd_filter_kernel(int batch,
                                                              const float* __restrict__ a1p,
                                                              const float* __restrict__ dy2,
                                                              float* __restrict__ part2,
                                                              float* __restrict__ part_db2,
                                                              int nc2, const C1Filter c1) {
  constexpr int SM = 3 * 2 * 16 * 64 > C1F_SMEM ? 3 * 2 * 16 * 64 : C1F_SMEM;
  __shared__ float smem[SM];
  if ((int)blockIdx.x >= nc2) {  // conv1 filter-grad role (its dA1 is final)
    conv1_filter_unit<512>(blockIdx.x - nc2, batch, c1, smem);
    return;
  }
  conv2_bwd_filter_v3<DEPTH, CENTRE_ONLY>(blockIdx.x, batch, a1p, dy2, part2, part_db2, smem);
}

// ------------------------------------------------------ conv1 bwd filter ----
// standalone 256-thread form of mnist_shared.h conv1_filter_unit (the executor
// runs it as a role of the conv2 filter-gradient launch)
__global__ __launch_bounds__(256) void conv1_bwd_filter_kernel(int batch, const C1Filter c) {
  __shared__ float smem[C1F_SMEM];
  conv1_filter_unit<256>(blockIdx.x, batch, c, smem);
}

// ------------------------------------------------------------ finalize ----
// sum of the conv2 filter-grad slabs at float4 i, in group order z = 0, 1, ...
// (the one order every path uses, so world 1 and world > 1 agree bit for bit);
// the loads of up to 32 groups are issued together
__device__ __forceinline__ float4 slab_sum4(const float4* __restrict__ p2, int ngroups) {
  float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
  int z = 0;
  for (; z + 32 <= ngroups; z += 32) {
    float4 v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = p2[(size_t)(z + u) * 12800];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      sv.x += v[u].x;
      sv.y += v[u].y;
      sv.z += v[u].z;
      sv.w += v[u].w;
    }
  }
  for (; z < ngroups; ++z) {
    const float4 v = p2[(size_t)z * 12800];
    sv.x += v.x;
    sv.y += v.y;
    sv.z += v.z;
    sv.w += v.w;
  }
  return sv;
}

// conv2: one thread per dW2 float4 summing the G image-group slabs in group
// order (slab_sum4, shared with sgd_finalize);
// db2 from the 4G centre-tap partials.  conv1: one wave per output (lanes
// stride over the per-block slabs) + wave reduction.
__global__ __launch_bounds__(256) void grad_finalize_kernel(
    const float* __restrict__ part2, const float* __restrict__ part_db2, int ngroups,
    const float* __restrict__ part1, int nblk1, float* __restrict__ g_w2,
    float* __restrict__ g_b2, float* __restrict__ g_w1, float* __restrict__ g_b1) {
  constexpr int B2 = 51200 / 4 / 256;  // 50 blocks of float4
  if ((int)blockIdx.x < B2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const float4 sv = slab_sum4(reinterpret_cast<const float4*>(part2) + i, ngroups);
    reinterpret_cast<float4*>(g_w2)[i] = sv;
    return;
  }
  if ((int)blockIdx.x < B2 + 16) {  // db2: one wave per channel
    const int co = ((int)blockIdx.x - B2) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    float s = 0.f;
    for (int z = lane; z < 4 * ngroups; z += 64) s += part_db2[z * 64 + co];
    s = wave_sum(s);
    if (lane == 0) g_b2[co] = s;
    return;
  }
  const int o = ((int)blockIdx.x - B2 - 16) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= 832) return;
  float s = 0.f;
#pragma unroll 8
  for (int b = lane; b < nblk1; b += 64) s += part1[(size_t)b * 832 + o];
  s = wave_sum(s);
  if (lane == 0) {
    if (o < 800)
      g_w1[o] = s;
    else
      g_b1[o - 800] = s;
  }
}

}  // namespace mnist

// ======================================================================
// host launchers
// ======================================================================
namespace mnist {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// conv1: 128x32 tiles (4 waves stacked in M), K = 25 -> 32 (one K tile)
#define C1_WM 4
#define C1_WN 1
#define C1_WK 1

void launch_conv1_fwd(const float* data, const long long* step, int n_local, int batch,
                      const float* w, const float* b, float* out, uint8_t* argmax,
                      hipStream_t s, float* out_pad) {
  const int M = batch * 14 * 14 * 4;
  const int mt = cdiv(M, 32 * C1_WM), nt = 32 / (32 * C1_WN);
  conv_pool_fwd_kernel<Conv1, C1_WM, C1_WN, C1_WK>
      <<<mt * nt, 64 * C1_WM * C1_WN * C1_WK, 0, s>>>(data, step, n_local, batch, w, b, out,
                                                      argmax, nullptr, nullptr, 0, out_pad,
                                                      ShadowPtrs{}, mt * nt);
}

void launch_conv1_fwd_bf16(const float* data, const long long* step, int n_local, int batch,
                           const float* w, const float* b, uint16_t* a1p, uint16_t* a1t,
                           uint8_t* argmax, int ld_batch, hipStream_t s, const float* w3,
                           const float* w2, uint16_t* w1b, uint16_t* w1t, uint16_t* w2tb,
                           uint16_t* w2b) {
  const int M = batch * 14 * 14 * 4;
  const int mt = cdiv(M, 32 * C1_WM), nt = 32 / (32 * C1_WN);
  auto B16 = [](uint16_t* p) { return reinterpret_cast<__bf16*>(p); };
  const ShadowPtrs sh{w3, w2, B16(w1b), B16(w1t), B16(w2tb), B16(w2b)};
  const int extra = (w2tb ? SHADOW_W2_BLOCKS : 0) + (w1b ? SHADOW_W1_BLOCKS : 0);
  if (w1b && !w2tb) throw std::runtime_error("conv1_fwd_bf16: fc1 shadows without conv2 shadows");
  conv_pool_fwd_kernel<Conv1, C1_WM, C1_WN, C1_WK>
      <<<mt * nt + extra, 64 * C1_WM * C1_WN * C1_WK, 0, s>>>(
          data, step, n_local, batch, w, b, nullptr, argmax, B16(a1p), B16(a1t), ld_batch, nullptr,
          sh, mt * nt);
}

void launch_conv2_fwd(const float* a1, int batch, const float* w, const float* b, float* out,
                      uint8_t* argmax, float* w2t, hipStream_t s) {
  conv2_fwd_v3_kernel<false><<<batch * 4, 256, 0, s>>>(a1, batch, w, b, out, argmax, w2t, C12In{});
}

void launch_conv12_fwd(const C12In& c1, int batch, const float* w2, const float* b2, float* a2,
                       uint8_t* idx2, float* w2t, hipStream_t s) {
  if (!c1.data || !c1.w1 || !c1.b1 || !c1.a1 || !c1.a1pf || !c1.idx1)
    throw std::runtime_error("conv12_fwd: missing conv1 operand");
  conv2_fwd_v3_kernel<true><<<batch * 4, 256, 0, s>>>(nullptr, batch, w2, b2, a2, idx2, w2t, c1);
}

void launch_conv12_fwd_bf16(const C12In& c1, int batch, const uint16_t* w2tb, const float* b2,
                            uint16_t* a1p, uint16_t* a1t, uint16_t* a2p, uint16_t* a2t,
                            uint8_t* idx2, hipStream_t s) {
  if (!c1.data || !c1.w1 || !c1.b1 || !c1.idx1 || !w2tb || !a1p || !a1t || !a2p || !a2t || !idx2)
    throw std::runtime_error("conv12_fwd_bf16: missing operand");
  if (batch % 16 != 0) throw std::runtime_error("conv12_fwd_bf16: batch % 16 != 0");
  auto B16 = [](uint16_t* p) { return reinterpret_cast<__bf16*>(p); };
  conv12_fwd_bf16_kernel<<<batch * 4, 256, 0, s>>>(
      c1, batch, reinterpret_cast<const __bf16*>(w2tb), b2, B16(a1p), B16(a1t), B16(a2p),
      B16(a2t), idx2);
}

void launch_conv2_wino_weights(const float* w2, float* U, float* Ud, hipStream_t s) {
  conv2_wino_weights_kernel<<<2048 / 256, 256, 0, s>>>(w2, U, Ud);
}

void launch_conv12_fwd_wino(const C12In& c1, int batch, const float* w2, const float* U,
                            const float* b2, float* a2, uint8_t* idx2, float* w2t, hipStream_t s,
                            unsigned long long* prof, float* a2t) {
  if (!c1.data || !c1.w1 || !c1.b1 || !c1.a1 || !c1.a1pf || !c1.idx1 || !U)
    throw std::runtime_error("conv12_fwd_wino: missing operand");
  if (prof)
    conv2_fwd_wino_kernel<true, true><<<batch * 4, WNT, 0, s>>>(nullptr, batch, w2, U, b2, a2, idx2,
                                                                w2t, c1, prof, a2t);
  else
    conv2_fwd_wino_kernel<true><<<batch * 4, WNT, 0, s>>>(nullptr, batch, w2, U, b2, a2, idx2, w2t,
                                                          c1, nullptr, a2t);
}

void launch_conv2_fwd_wino(const float* a1, int batch, const float* w2, const float* U,
                           const float* b, float* out, uint8_t* argmax, float* w2t,
                           hipStream_t s) {
  conv2_fwd_wino_kernel<false><<<batch * 4, WNT, 0, s>>>(a1, batch, w2, U, b, out, argmax, w2t,
                                                         C12In{});
}

int fc1_train_splits() { return FC1_SPLITS; }
int fc1_train_t_splits() { return FC1T_SPLITS; }

void launch_fc1_fwd_train(const float* a2, const float* w, int batch, float* part,
                          hipStream_t s) {
  // 64x32 tiles, 2-way in-block K split, 14 split-K slabs of 224 (7 K tiles)
  const int kchunk = FC1_IN / FC1_SPLITS;
  dim3 grid(cdiv(batch, 64) * (FC1_OUT / 32), FC1_SPLITS);
  fc1_fwd_kernel<2, 1, 2, 32, false, FC1_IN / FC1_SPLITS / 32>
      <<<grid, 256, 0, s>>>(a2, w, nullptr, part, batch, kchunk, 0u, 1.f);
}

void launch_fc1_fwd_eval(const float* a2, const float* w, const float* b, int M, float* h,
                         uint32_t key, float keep_prob, hipStream_t s) {
  dim3 grid(cdiv(M, 64) * (FC1_OUT / 64), 1);
  fc1_fwd_kernel<2, 2, 1, 64, true><<<grid, 256, 0, s>>>(a2, w, b, h, M, FC1_IN, key, keep_prob);
}

void launch_fc_head_train(const float* part, const float* b3, const float* w4, const float* b4,
                          const int* labels, int n_local, const long long* step, int batch,
                          float keep_prob, uint32_t seed, uint32_t rank, float base_lr,
                          float lr_decay, float* hd, float* dh, float* dlog, float* loss_rows,
                          float* lr_out, int* correct, hipStream_t s, uint16_t* dh16,
                          uint16_t* dht16, int splits) {
#define HEAD(NS_)                                                                              \
  fc_head_train_kernel<NS_><<<batch, 256, 0, s>>>(part, b3, w4, b4, labels, n_local, step, batch, \
                                                  keep_prob, seed, rank, base_lr, lr_decay, hd, dh, \
                                                  dlog, loss_rows, lr_out, correct,              \
                                                  reinterpret_cast<__bf16*>(dh16),               \
                                                  reinterpret_cast<__bf16*>(dht16))
  if (splits == FC1T_SPLITS)
    HEAD(FC1T_SPLITS);
  else if (splits == FC1_SPLITS)
    HEAD(FC1_SPLITS);
  else
    throw std::runtime_error("fc_head_train: unsupported slab count");
#undef HEAD
}

void launch_fc1_fwd_train_t(const float* a2t, const float* w, int batch, float* part,
                            hipStream_t s) {
  if (batch <= 0 || batch % 32) throw std::runtime_error("fc1_fwd_t: batch % 32 != 0");
  fc1_fwd_t_kernel<<<dim3((FC1_OUT / 32) * (batch / 32), FC1T_SPLITS), 256, 0, s>>>(a2t, w, batch,
                                                                                   part);
}

void launch_fc_head_eval(const float* h, const float* w4, const float* b4, const int* labels,
                         int M, float* logits, int* errors, hipStream_t s) {
  fc_head_eval_kernel<<<cdiv(M, 4), 256, 0, s>>>(h, w4, b4, labels, M, logits, errors);
}

void launch_fc1_bwd(const float* a2, const uint8_t* idx2, const float* dh, const float* hd,
                    const float* dlog, const float* w1, int batch, float* g_w3, float* g_b3,
                    float* g_w4, float* g_b4, float* dy2, float* dy2t, hipStream_t s,
                    int roles) {
  if (batch <= 0 || batch % 32 != 0) throw std::runtime_error("fc1_bwd: batch % 32 != 0");
  if (roles <= 0 || roles > 7) throw std::runtime_error("fc1_bwd: roles must be a mask in 1..7");
  const int grid = ((roles & 1) ? (batch / 32) * (FC1_IN / 32) : 0) +
                   ((roles & 2) ? FC1BWD_DW_BLOCKS : 0) + ((roles & 4) ? SMALL_BLOCKS : 0);
  fc1_bwd_kernel<<<grid, 256, 0, s>>>(a2, idx2, dh, hd, dlog, w1, batch, g_w3, g_b3, g_w4, g_b4,
                                      dy2, dy2t, roles);
}

void launch_fc1_bwd_weights(const float* a2, const float* dh, const float* hd, const float* dlog,
                            int rows, float* g_w3, float* g_b3, float* g_w4, float* g_b4,
                            hipStream_t s) {
  if (rows <= 0 || rows % 32 != 0) throw std::runtime_error("fc1_bwd_weights: rows % 32 != 0");
  fc1_bwd_weights_kernel<<<FC1BWD_DW_BLOCKS + SMALL_BLOCKS, 256, 0, s>>>(
      a2, dh, hd, dlog, rows, g_w3, g_b3, g_w4, g_b4);
}

int conv2_filter_splits(int batch) { return cdiv(batch, C2F_GROUPS_IMG); }


FcSgd fc_sgd_args(const FcSgdArgs* a) {
  FcSgd r{};
  if (a == nullptr || a->n == 0) return r;
  if (a->n % 4) throw std::runtime_error("fc_sgd: FC bucket not a multiple of 4 floats");
  r = FcSgd{a->w, a->g, a->m, a->n / 4, a->l2, a->momentum, a->lr, 0, nullptr, nullptr, 0,
            a->gscale, nullptr, nullptr, 0};
  const long long per_blk = 256LL * FC_SGD_UNROLL * a->rounds;
  if (a->a2) {
    if (a->w1b || a->dh == nullptr || a->batch <= 0)
      throw std::runtime_error("fc_sgd: fused dW1 needs a2, dh, batch and no bf16 shadows");
    if (a->w1 % 4 || a->w1 + (long long)FC1_IN * FC1_OUT > a->n)
      throw std::runtime_error("fc_sgd: fc1 weight misaligned or outside the FC bucket");
    r.a2 = a->a2;
    r.dh = a->dh;
    r.batch = a->batch;
    r.w1_off4 = a->w1 / 4;
    // the streaming units cover the bucket minus the fc1 weight (its tiles are
    // extra blocks of the launch)
    r.nblk = (int)((r.n4 - W1_F4 + per_blk - 1) / per_blk);
    return r;
  }
  if (a->w1b) {
    if (a->w1 % 4 || a->w1 + (long long)FC1_IN * FC1_OUT > a->n)
      throw std::runtime_error("fc_sgd: fc1 weight misaligned or outside the FC bucket");
    r.w1b = reinterpret_cast<__bf16*>(a->w1b);
    r.w1t = reinterpret_cast<__bf16*>(a->w1t);
    r.w1_off4 = a->w1 / 4;
    const long long rest = r.n4 - W1_F4;
    r.nblk = SHADOW_W1_BLOCKS + (int)((rest + per_blk - 1) / per_blk);
    return r;
  }
  r.nblk = (int)((r.n4 + per_blk - 1) / per_blk);
  return r;
}

void launch_conv2_bwd_data_l2(const float* dy2t, const float* w2t, const float* a1, int batch,
                              float* da1m, hipStream_t s, const FcSgdArgs* fc_sgd) {
  if (batch % 8 != 0) throw std::runtime_error("conv2_bwd_data_l2: batch % 8 != 0");
  const int mtiles = batch * 49 / 8;
  const FcSgd sg = fc_sgd_args(fc_sgd);
  if (sg.a2) throw std::runtime_error("conv2_bwd_data_l2: no fused dW1 SGD (Winograd launch only)");
  conv2_bwd_data_l2_kernel<<<cdiv(mtiles, 2) + sg.nblk, 256, 0, s>>>(dy2t, w2t, a1, batch, da1m,
                                                                     sg);
}

void launch_conv2_bwd_data_wino(const float* dy2, const float* Ud, const float* a1, int batch,
                                float* da1m, hipStream_t s, const FcSgdArgs* fc_sgd,
                                const C1FilterArgs* c1, unsigned long long* prof) {
  FcSgd sg = fc_sgd_args(fc_sgd);
  if (sg.w1b) throw std::runtime_error("conv2_bwd_data_wino: the fp32 FC SGD has no shadows");
  // the FC SGD runs in 256-thread units, two per (conv) block
  sg.nblk = 2 * batch * 4;
  if (prof)
    conv2_bwd_data_wino_kernel<true><<<batch * 4, WNT, 0, s>>>(dy2, Ud, a1, batch, da1m, sg,
                                                              c1_args(c1), prof);
  else
    conv2_bwd_data_wino_kernel<false><<<batch * 4, WNT, 0, s>>>(dy2, Ud, a1, batch, da1m, sg,
                                                               c1_args(c1));
}

void launch_conv2_bwd_filter(const float* a1p, const float* dy2, int batch, float* part2,
                             hipStream_t s, const C1FilterArgs* c1) {
  const int G = conv2_filter_splits(batch);
  float* db = part2 + (size_t)G * 51200;
  const C1Filter c = c1_args(c1);
  const int n1 = c.part1 ? conv1_filter_blocks(batch) : 0;
  conv2_bwd_filter_kernel<3, true><<<25 * G + n1, 512, 0, s>>>(batch, a1p, dy2, part2, db, 25 * G,
                                                                c);
}

int conv1_filter_blocks(int batch, int split) {
  if (split != C1F_SPLIT && split != 1 && split != 4)
    throw std::runtime_error("conv1 filter split: 1, 4 (Winograd bwd-data bands) or 7");
  return batch * split;
}

int conv2_wino_filter_groups(int batch) { return cdiv(batch, WF_IMG); }
size_t part2_floats_wino(int batch) {
  return (size_t)conv2_wino_filter_groups(batch) * (51200 + 256);
}

void launch_conv2_bwd_filter_wino(const float* a1p, const float* dy2, int batch, float* part2,
                                  hipStream_t s, const C1FilterArgs* c1) {
  const int G = conv2_wino_filter_groups(batch);
  const C1Filter c = c1_args(c1);
  const int n1 = c.part1 ? conv1_filter_blocks(batch, 1) : 0;
  conv2_bwd_filter_wino_kernel<false><<<8 * G + n1, WF_NT, 0, s>>>(
      batch, a1p, dy2, part2, part2 + (size_t)G * 51200, 8 * G, c, nullptr);
}

// labs: per-block clock stamps of the merged conv2 backward (null: off)
static unsigned long long* g_c2bw_prof = nullptr;

void launch_conv2_bwd_wino(const float* Ud, const float* a1, const float* a1p, const float* dy2,
                           int batch, float* da1m, float* part2, hipStream_t s,
                           const C1FilterArgs* c1, const XgmiStepArgs* xfc) {
  const int nd = batch * 4;
  const int G = conv2_wino_filter_groups(batch);
  XgmiStepArgs xa{};
  if (xfc) {
    xa = *xfc;
    xgmi_fc_plan(xa, WF_NT, XS_FC_ROLE_BLOCKS);
  }
  conv2_bwd_wino_kernel<<<xa.nfc + nd + 8 * G, WF_NT, 0, s>>>(
      nd, Ud, a1, batch, da1m, c1_args(c1), a1p, dy2, part2, part2 + (size_t)G * 51200, 8 * G, xa,
      g_c2bw_prof);
}

void set_conv2_bwd_wino_prof(unsigned long long* p) { g_c2bw_prof = p; }

void launch_conv2_bwd_filter_wino_prof(const float* a1p, const float* dy2, int batch,
                                       float* part2, unsigned long long* prof, hipStream_t s) {
  const int G = conv2_wino_filter_groups(batch);
  conv2_bwd_filter_wino_kernel<true><<<8 * G, WF_NT, 0, s>>>(
      batch, a1p, dy2, part2, part2 + (size_t)G * 51200, 8 * G, C1Filter{}, prof);
}

C1Filter c1_args(const C1FilterArgs* a) {
  if (a == nullptr) return C1Filter{};
  return C1Filter{a->data, a->step, a->n_local, a->da1m, a->idx1, a->part1};
}

void launch_conv1_bwd_filter(const float* data, const long long* step, int n_local, int batch,
                             const float* da1m, const uint8_t* idx1, float* part1,
                             hipStream_t s) {
  conv1_bwd_filter_kernel<<<conv1_filter_blocks(batch), 256, 0, s>>>(
      batch, C1Filter{data, step, n_local, da1m, idx1, part1});
}

// ------------------------------------------------- SGD of the step ----
// The last launch of a train step: momentum SGD (U1) of the parameters whose
// gradients are final, plus the derived weights the NEXT step reads, so no
// launch of its own re-derives them.
//  * world 1: the conv filter-grad slab reductions of grad_finalize_kernel
//    are fused into the SGD (a kernel boundary plus one dependent HBM round
//    trip saved: 6.6 + 4.9 us -> 9.4 us at B = 64); the FC bucket was updated
//    by the conv2 bwd-data launch's role blocks (fc.n4 == 0 here).
//  * world > 1: the conv grads were finalized before their all-reduce, so
//    the conv part reads the rank sums from the flat buffer (x 1/N); the FC
//    bucket, when this launch owns it, runs fc_sgd_role (bf16: also the fc1
//    weight's shadows, in 64 x 64 tiles).
// Roles (blocks): [0, fc.nblk) FC bucket; then, when conv is on, 128
// (Winograd: per (ci, co quarter), + the U / Ud transforms) or 50 (flat, +
// the bf16 conv2 shadows) conv2-weight blocks, 16 conv2-bias blocks (one wave
// per channel), 208 conv1 blocks (one wave per weight / bias).  Each slab sum
// runs in the order of grad_finalize_kernel.
struct SgdFinArgs {
  FcSgd fc;  // FC bucket role (fc.n4 == 0: off)
  float* w;
  const float* g;
  float* mom;
  int conv;  // conv parameters updated by this launch
  int flat;  // conv grads from g (world > 1) instead of the slabs
  int off_w2, off_b2, off_w1, off_b1;
  const float* part2;
  const float* part_db2;
  int ngroups;
  const float* part1;
  int nblk1;
  float momentum, gscale;
  const float* lr;
  long long* step;  // bumped once (nullptr: no bump)
  // Winograd conv2 (optional): the updated conv2 filters' transforms for the
  // NEXT step's forward (U) and bwd-data (Ud), layouts of wino_u_index
  float* U;
  float* Ud;
  // bf16 engine (optional): the updated conv2 weights' bf16 shadows w2t / w2b
  // (mnist_bf16.h layouts) for the NEXT step's fused forward and bwd-data
  __bf16* w2t;
  __bf16* w2b;
  unsigned long long* prof;  // lab: per-block start / end clock (set_sgd_prof)
};

__device__ __forceinline__ void sgd_elem(float* w, float* m, float g, float lr, float mu) {
  const float mv = mu * *m + g;
  *m = mv;
  *w -= lr * mv;
}

// dW2 float4 i (HWIO order): slab sum in group order (slab_sum4), or
// the all-reduced flat gradient
__device__ __forceinline__ float4 conv2_grad4(const SgdFinArgs& a, int i) {
  if (a.flat) return reinterpret_cast<const float4*>(a.g + a.off_w2)[i];
  return slab_sum4(reinterpret_cast<const float4*>(a.part2) + i, a.ngroups);
}

// conv2 weights of one input channel ci and 16 output channels (block b: ci
// = b / 4, co quarter b % 4; 25 taps x 4 float4s = 100 threads): gradient,
// SGD, then the Winograd transforms of the updated 5x5 filters (U and Ud).
// 128 blocks with short sums: with 32 blocks of 2 taps x 32 groups a thread
// waited on 8 rounds of 8 loads (9.1 us SGD).
__device__ void sgd_conv2_wino(const SgdFinArgs& a, int blk, float lr) {
  __shared__ float wl[25 * 16];
  const int tid = threadIdx.x, ci = blk >> 2, cq = blk & 3;
  if (tid < 100) {
    const int t = tid >> 2, c4 = tid & 3;
    const int i = (t * 32 + ci) * 16 + cq * 4 + c4;  // float4 index in the HWIO block
    float4* wp = reinterpret_cast<float4*>(a.w + a.off_w2) + i;
    float4* mp = reinterpret_cast<float4*>(a.mom + a.off_w2) + i;
    float4 wv = *wp, mv = *mp;  // issued ahead of the slab loads
    const float4 sv = conv2_grad4(a, i);
    sgd4(wv, mv, sv, 0.f, lr, a.momentum, a.gscale);
    *wp = wv;
    *mp = mv;
    *reinterpret_cast<float4*>(wl + t * 16 + 4 * c4) = wv;
  }
  __syncthreads();
  if (tid < 32) {
    const int cl = tid & 15, co = cq * 16 + cl;
    float g[25], u[36];
    if (tid < 16) {
#pragma unroll
      for (int t = 0; t < 25; ++t) g[t] = wl[t * 16 + cl];
      wino::filter_tile(g, u);
#pragma unroll
      for (int p = 0; p < 36; ++p) a.U[wino_u_index(p, ci, co)] = u[p];
    } else {
#pragma unroll
      for (int t = 0; t < 25; ++t) g[t] = wl[(24 - t) * 16 + cl];
      wino::filter_tile(g, u);
#pragma unroll
      for (int p = 0; p < 36; ++p) a.Ud[wino_ud_index(p, ci, co)] = u[p];
    }
  }
}

// conv2 weights: 51200 floats = 50 blocks x 256 threads x float4
__device__ void sgd_conv2_flat(const SgdFinArgs& a, int blk, float lr) {
  const int tid = threadIdx.x;
  const int i = blk * 256 + tid;
  float4* wp = reinterpret_cast<float4*>(a.w + a.off_w2) + i;
  float4* mp = reinterpret_cast<float4*>(a.mom + a.off_w2) + i;
  float4 wv = *wp, mv = *mp;
  const float4 s = conv2_grad4(a, i);
  sgd4(wv, mv, s, 0.f, lr, a.momentum, a.gscale);
  *wp = wv;
  *mp = mv;
  if (a.w2t) {  // HWIO (t * 32 + ci) * 64 + co: 4 consecutive co
    const int idx = 4 * i, t = idx >> 11, ci = (idx >> 6) & 31, co = idx & 63;
    const float v[4] = {wv.x, wv.y, wv.z, wv.w};
    __bf16 hb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hb[e] = (__bf16)v[e];
      a.w2t[((t * 2 + (ci >> 4)) * 64 + co + e) * 16 + (ci & 15)] = hb[e];
    }
    // w2b: the 4 co are consecutive within one 16-channel group (8-byte store)
    *reinterpret_cast<uint2*>(a.w2b + ((t * 4 + (co >> 4)) * 32 + ci) * 16 + (co & 15)) =
        __builtin_bit_cast(uint2, hb);
  }
}

__device__ __forceinline__ void sgd_finalize_body(const SgdFinArgs& a, float* tile);

__global__ __launch_bounds__(256) void sgd_finalize_kernel(const SgdFinArgs a) {
  __shared__ float tile[SHADOW_SMEM_FLOATS];  // fc1 shadow tiles (bf16, world > 1)
  if (!a.prof) {
    sgd_finalize_body(a, tile);
    return;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  sgd_finalize_body(a, tile);
  __syncthreads();
  if (threadIdx.x == 0) {
    a.prof[2 * blockIdx.x] = t0;
    a.prof[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__device__ __forceinline__ void sgd_finalize_body(const SgdFinArgs& a, float* tile) {
  const float lr = *a.lr;
  const int tid = threadIdx.x;
  int blk = blockIdx.x;
  if (a.step && blk == 0 && tid == 0) *a.step += 1;
  const int ndw = a.fc.a2 ? FC1BWD_DW_BLOCKS : 0;  // fused dW1 + SGD tiles first
  if (blk < ndw) {
    fc1_dw_sgd(a.fc, blk, tid);
    return;
  }
  blk -= ndw;
  if (blk < a.fc.nblk) {
    fc_sgd_role(a.fc, blk, tile);
    return;
  }
  blk -= a.fc.nblk;
  const int nconv2 = a.U ? 128 : 50;
  if (blk < nconv2) {
    if (a.U)
      sgd_conv2_wino(a, blk, lr);
    else
      sgd_conv2_flat(a, blk, lr);
    return;
  }
  blk -= nconv2;
  const int lane = tid & 63;
  // (gscale: the conv bias / conv1 grads go through the sgd4 form
  // fma(0, w, g * gs), as in optim::sgd_momentum_flat)
  if (blk < 16) {  // conv2 bias: one wave per channel
    const int co = blk * 4 + (tid >> 6);
    float s = 0.f;
    if (a.flat) {
      s = a.g[a.off_b2 + co];
    } else {
      for (int z = lane; z < 4 * a.ngroups; z += 64) s += a.part_db2[z * 64 + co];
      s = wave_sum(s);
    }
    if (lane == 0) {
      float* w = a.w + a.off_b2 + co;
      sgd_elem(w, a.mom + a.off_b2 + co, __builtin_fmaf(0.f, *w, s * a.gscale), lr, a.momentum);
    }
    return;
  }
  blk -= 16;
  // conv1 weights + bias: 4 consecutive parameters a wave (16 a block, so the
  // launch fits one round of 2 blocks per CU), their partial rows as one
  // float4 per row; each parameter's sum runs in the same order as one wave
  // per parameter did
  const int o0 = (blk * 4 + (tid >> 6)) * 4;
  if (o0 >= 832) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.flat) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = o0 + k;
      s[k] = a.g[o < 800 ? a.off_w1 + o : a.off_b1 + (o - 800)];
    }
  } else {
#pragma unroll 8
    for (int b = lane; b < a.nblk1; b += 64) {
      const float4 v = *reinterpret_cast<const float4*>(a.part1 + (size_t)b * 832 + o0);
      s[0] += v.x;
      s[1] += v.y;
      s[2] += v.z;
      s[3] += v.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = o0 + k;
      const int off = o < 800 ? a.off_w1 + o : a.off_b1 + (o - 800);
      sgd_elem(a.w + off, a.mom + off, __builtin_fmaf(0.f, a.w[off], s[k] * a.gscale), lr,
               a.momentum);
    }
  }
}

static unsigned long long* g_sgd_prof = nullptr;

void launch_sgd_step(const SgdStepArgs& s_, hipStream_t s) {
  const SgdStepArgs& p = s_;
  if ((p.w2tb == nullptr) != (p.w2b == nullptr) || (p.w2tb && p.wino_u))
    throw std::runtime_error("sgd_step: bf16 conv2 shadows need both layouts, no Winograd");
  if ((p.wino_u == nullptr) != (p.wino_ud == nullptr))
    throw std::runtime_error("sgd_step: Winograd filters need both U and Ud");
  if (p.off_w2 % 4 || p.fc_end % 4)
    throw std::runtime_error("sgd_step: misaligned flat segments");
  SgdFinArgs a{};
  if (p.fc_end > 0) {
    FcSgdArgs f{p.w, p.g, p.mom, p.fc_end, p.l2, p.momentum, p.lr, p.fc_rounds};
    f.w1b = p.w1b;
    f.w1t = p.w1t;
    f.w1 = p.off_w1fc;
    f.gscale = p.gscale;
    f.a2 = p.a2;
    f.dh = p.dh;
    f.batch = p.batch;
    a.fc = fc_sgd_args(&f);
  }
  a.w = p.w;
  a.g = p.g;
  a.mom = p.mom;
  a.conv = p.conv ? 1 : 0;
  a.flat = p.part2 == nullptr ? 1 : 0;
  a.off_w2 = p.off_w2;
  a.off_b2 = p.off_b2;
  a.off_w1 = p.off_w1;
  a.off_b1 = p.off_b1;
  a.part2 = p.part2;
  a.part_db2 = p.part2 ? p.part2 + (size_t)p.ngroups * 51200 : nullptr;
  a.ngroups = p.ngroups;
  a.part1 = p.part1;
  a.nblk1 = p.nblk1;
  a.momentum = p.momentum;
  a.gscale = p.gscale;
  a.lr = p.lr;
  a.step = p.step;
  a.U = p.wino_u;
  a.Ud = p.wino_ud;
  a.w2t = reinterpret_cast<__bf16*>(p.w2tb);
  a.w2b = reinterpret_cast<__bf16*>(p.w2b);
  const int conv_blocks = p.conv ? (p.wino_u ? 128 : 50) + 16 + cdiv(832, 16) : 0;
  const int grid = (a.fc.a2 ? FC1BWD_DW_BLOCKS : 0) + a.fc.nblk + conv_blocks;
  if (grid == 0) throw std::runtime_error("sgd_step: nothing to update");
  a.prof = g_sgd_prof;
  sgd_finalize_kernel<<<grid, 256, 0, s>>>(a);
}

void set_sgd_prof(unsigned long long* p) { g_sgd_prof = p; }

// ------------------------------------------- xGMI peer-to-peer step sync ----
// (mnist.h XgmiStepArgs).  Two block roles: [0, nfc) FC segment slices (slice
// b = float4s [b * per4, (b + 1) * per4) of the segment); [nfc, nfc + ncv)
// conv blocks, each looping over the "virtual" blocks v = b, b + ncv, ... of
// sgd_finalize_kernel's conv partition: 128 (Winograd) or 50 (flat) conv2
// weight blocks, 16 conv2-bias blocks, 208 conv1 blocks.  Few blocks on
// purpose: a block waiting at a barrier holds its CU slot, and the grid stays
// small beside whatever else the GPU runs.  Every block takes part in both
// barriers (arrival; "reduced / done reading"), so a rank leaves the kernel
// only when every peer has read its grads.
constexpr int XS_FC_BLOCKS = 64, XS_CONV_BLOCKS = 32;

// conv virtual block v: the flat float offset of this thread's output (conv2:
// a float4 index into the conv2 weight, returned in *i4) or -1
struct XsConvItem {
  int kind;  // 0 conv2 weight (float4 i4), 1 scalar (bias / conv1) at off
  int i4, off;
};

__device__ __forceinline__ XsConvItem xs_conv_item(const XgmiStepArgs& a, int v, int tid) {
  const int nconv2 = a.wino_u ? 128 : 50;
  if (v < nconv2) {
    int i = -1;
    if (a.wino_u) {
      if (tid < 100) i = ((tid >> 2) * 32 + (v >> 2)) * 16 + (v & 3) * 4 + (tid & 3);
    } else {
      i = v * 256 + tid;
    }
    return XsConvItem{0, i, -1};
  }
  v -= nconv2;
  if (v < 16) return XsConvItem{1, -1, a.off_b2 + v * 4 + (tid >> 6)};
  const int o = (v - 16) * 4 + (tid >> 6);
  if (o >= 832) return XsConvItem{1, -1, -1};
  return XsConvItem{1, -1, o < 800 ? a.off_w1 + o : a.off_b1 + (o - 800)};
}

__global__ __launch_bounds__(256) void xgmi_step_kernel(const XgmiStepArgs a) {
  __shared__ unsigned ep;
  __shared__ float wl[25 * 16];
  xs_stamp(a, 0);
  struct End {
    const XgmiStepArgs& a;
    __device__ ~End() { xs_stamp(a, 5); }
  } end{a};
  const xgmi::Sync& s = a.sync;
  const int n = s.nranks, me = s.rank, tid = threadIdx.x, lane = tid & 63;
  const float lr = *a.lr;
  if (a.fc_in_bwd && (int)blockIdx.x < a.ngather) {  // ---- the FC gather
    xs_stamp(a, 1);  // (labs: the role in slot 1's gap; gather blocks stamp 1 at once)
    xgmi_fc_gather(a, blockIdx.x, a.ngather);
    return;
  }
  if (a.fc_local && a.fa2 && (int)blockIdx.x < a.nfc) {
    // ---- FC bucket from the gathered factors: the fc1 weight tiles (dW1 over
    // every rank's rows + SGD, fc1_dw_sgd), then the rest of the bucket
    // streamed (its grads from launch_fc1_small_grads)
    FcSgd f{};
    f.w = a.w[me];
    f.g = a.g[me];
    f.m = a.mom;
    f.n4 = a.fc4;
    f.l2 = a.l2;
    f.mu = a.momentum;
    f.lr = a.lr;
    f.nblk = a.nfc - FC1BWD_DW_BLOCKS;
    f.w1_off4 = a.off_w3 / 4;
    f.gs = a.gscale;
    f.a2 = a.fa2;
    f.dh = a.fdh;
    f.batch = a.frows;
    if ((int)blockIdx.x < FC1BWD_DW_BLOCKS)
      fc1_dw_sgd(f, blockIdx.x, tid);
    else
      fc_sgd_role(f, blockIdx.x - FC1BWD_DW_BLOCKS, nullptr, tid);
    return;
  }
  if (a.fc_local && (int)blockIdx.x < a.nfc) {  // ---- FC bucket, grads already global sums
    float4* W4 = reinterpret_cast<float4*>(a.w[me]);
    float4* M4 = reinterpret_cast<float4*>(a.mom);
    const float4* G4 = reinterpret_cast<const float4*>(a.g[me]);
    const long long stride = (long long)a.nfc * 256;
    for (long long i0 = (long long)blockIdx.x * 256 + tid; i0 < a.fc4; i0 += stride * XS_UNROLL) {
      float4 wv[XS_UNROLL], mv[XS_UNROLL], gv[XS_UNROLL];
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u) {
        const long long i = min(i0 + stride * u, a.fc4 - 1);
        wv[u] = W4[i];
        mv[u] = M4[i];
        gv[u] = G4[i];
      }
#pragma unroll
      for (int u = 0; u < XS_UNROLL; ++u) {
        const long long i = i0 + stride * u;
        if (i >= a.fc4) continue;
        sgd4(wv[u], mv[u], gv[u], a.l2, lr, a.momentum, a.gscale);
        W4[i] = wv[u];
        M4[i] = mv[u];
      }
    }
    return;
  }
  if ((int)blockIdx.x < a.nfc) {  // ---- FC bucket: this rank's segment, then the gather
    xgmi_fc_role(a, &ep);
    if (a.prof && threadIdx.x == 0) a.prof[6 * blockIdx.x] |= 1ull << 60;  // role tag: FC
    return;
  }
  // ---- conv parameters (replicated update)
  const unsigned e = xgmi::next_epoch(s, &ep);
  const int cb = (int)blockIdx.x - (a.fc_in_bwd ? a.ngather : a.nfc);
  const int nvirt = (a.wino_u ? 128 : 50) + 16 + 208;
  // every rank's conv grads, system-scope (kernels/xgmi.h): conv2 weight
  // float4s from off_w2, scalars (conv2 bias, conv1) from the buffer start.
  // With the exchange buffer the half of this launch's epoch parity: a block
  // slot writes that half again two launches on, after the next launch's
  // arrival barrier, which no peer's block passes before it has read this one
  // - so no closing barrier
  const bool dbuf = a.xc[0] != nullptr;
  const long long cbytes = 4LL * (a.off_b1 + 32);
  xgmi::Rsrc gr[xgmi::kMaxRanks];
#pragma unroll
  for (int r = 0; r < xgmi::kMaxRanks; ++r)
    if (r < n) gr[r] = xgmi::rsrc(dbuf ? a.xc[r] + (e & 1) * a.cstride : a.g[r], cbytes);
  // this rank's slab reductions (grad_finalize_kernel forms) into its grads,
  // written through for the peers
  for (int v = cb; v < nvirt; v += a.ncv) {
    const XsConvItem it = xs_conv_item(a, v, tid);
    if (it.kind == 0) {
      if (it.i4 >= 0)
        xgmi::st4_sys(gr[me], (unsigned)(4 * a.off_w2 + 16 * it.i4),
                      slab_sum4(reinterpret_cast<const float4*>(a.part2) + it.i4, a.ngroups));
      continue;
    }
    float sl = 0.f;
    if (it.off >= a.off_b2 && it.off < a.off_b2 + 64) {
      const int co = it.off - a.off_b2;
      const float* part_db2 = a.part2 + (size_t)a.ngroups * 51200;
      for (int z = lane; z < 4 * a.ngroups; z += 64) sl += part_db2[z * 64 + co];
      sl = wave_sum(sl);
    } else if (it.off >= 0) {
      const int o = it.off < a.off_b1 ? it.off - a.off_w1 : 800 + (it.off - a.off_b1);
#pragma unroll 8
      for (int b = lane; b < a.nblk1; b += 64) sl += a.part1[(size_t)b * 832 + o];
      sl = wave_sum(sl);
    }
    if (it.off >= 0 && lane == 0) xgmi::st_sys(gr[me], (unsigned)(4 * it.off), sl);
  }
  xs_stamp(a, 1);
  xgmi::barrier(s, 0, e, false);
  xs_stamp(a, 2);
  for (int v = cb; v < nvirt; v += a.ncv) {
    const XsConvItem it = xs_conv_item(a, v, tid);
    if (it.kind == 1) {
      if (it.off >= 0 && lane == 0) {
        float sv = xgmi::ld_peer(s, 0, gr[0], (unsigned)(4 * it.off));
#pragma unroll
        for (int r = 1; r < xgmi::kMaxRanks; ++r)
          if (r < n) sv += xgmi::ld_peer(s, r, gr[r], (unsigned)(4 * it.off));
        float* w = a.w[me] + it.off;
        sgd_elem(w, a.mom + it.off, __builtin_fmaf(0.f, *w, sv * a.gscale), lr, a.momentum);
      }
      continue;
    }
    float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (it.i4 >= 0) {
      float4* wp = reinterpret_cast<float4*>(a.w[me] + a.off_w2) + it.i4;
      float4* mp = reinterpret_cast<float4*>(a.mom + a.off_w2) + it.i4;
      wv = *wp;
      float4 mv = *mp;
      const unsigned off = (unsigned)(4 * a.off_w2 + 16 * it.i4);
      float4 sv = xgmi::ld4_peer(s, 0, gr[0], off);
#pragma unroll
      for (int r = 1; r < xgmi::kMaxRanks; ++r)
        if (r < n) sv = add4(sv, xgmi::ld4_peer(s, r, gr[r], off));
      sgd4(wv, mv, sv, 0.f, lr, a.momentum, a.gscale);
      *wp = wv;
      *mp = mv;
    }
    if (a.wino_u) {  // the next step's Winograd transforms (sgd_conv2_wino)
      const int ci = v >> 2, cq = v & 3;
      __syncthreads();  // wl of the previous virtual block is consumed
      if (tid < 100) *reinterpret_cast<float4*>(wl + (tid >> 2) * 16 + 4 * (tid & 3)) = wv;
      __syncthreads();
      if (tid < 32) {
        const int cl = tid & 15, co = cq * 16 + cl;
        float g[25], u[36];
        if (tid < 16) {
#pragma unroll
          for (int t = 0; t < 25; ++t) g[t] = wl[t * 16 + cl];
          wino::filter_tile(g, u);
#pragma unroll
          for (int p = 0; p < 36; ++p) a.wino_u[wino_u_index(p, ci, co)] = u[p];
        } else {
#pragma unroll
          for (int t = 0; t < 25; ++t) g[t] = wl[(24 - t) * 16 + cl];
          wino::filter_tile(g, u);
#pragma unroll
          for (int p = 0; p < 36; ++p) a.wino_ud[wino_ud_index(p, ci, co)] = u[p];
        }
      }
    }
  }
  if (a.step && cb == 0 && tid == 0) *a.step += 1;
  xs_stamp(a, 3);
  if (!dbuf) xgmi::barrier(s, 1, e, false);
  xs_stamp(a, 4);
}

void xgmi_fc_plan(XgmiStepArgs& a, int threads, int max_blocks) {
  const int n = a.sync.nranks;
  if (n < 1 || a.fc4 <= 0 || a.fc4 % n) throw std::runtime_error("xgmi: FC bucket not split evenly");
  a.seg4 = a.fc4 / n;
  const long long unit = (long long)threads * XS_UNROLL;
  const long long per = (a.seg4 + max_blocks - 1) / max_blocks;
  a.per4 = (int)((per + unit - 1) / unit * unit);
  // a multiple of 8: blocks after the role keep blockIdx % 8 (their XCD mapping)
  a.nfc = (int)((a.seg4 + a.per4 - 1) / a.per4 + 7) / 8 * 8;
}

static unsigned long long* g_xs_prof = nullptr;
void set_xgmi_step_prof(unsigned long long* p) { g_xs_prof = p; }

long long xgmi_conv_floats(long long off_b1) { return (off_b1 + 32 + 63) / 64 * 64; }

void launch_xgmi_step(const XgmiStepArgs& in, hipStream_t s) {
  XgmiStepArgs a = in;
  a.prof = g_xs_prof;
  const int n = a.sync.nranks;
  if (n < 1 || n > xgmi::kMaxRanks || !a.sync.flags || !a.sync.epoch || !a.sync.error || !a.lr)
    throw std::runtime_error("xgmi_step: communicator / lr not set up");
  for (int r = 0; r < n; ++r)
    if (!a.g[r] || !a.w[r] || (!a.sync.emulate && !a.sync.peer_flags[r]))
      throw std::runtime_error("xgmi_step: rank " + std::to_string(r) + " not mapped");
  if (a.fc4 <= 0 || a.fc4 % n) throw std::runtime_error("xgmi_step: FC bucket not split evenly");
  if (a.xc[0] != nullptr) {
    for (int r = 0; r < n; ++r)
      if (!a.xc[r]) throw std::runtime_error("xgmi_step: conv exchange buffer of a rank not mapped");
    if (a.cstride < xgmi_conv_floats(a.off_b1))
      throw std::runtime_error("xgmi_step: conv exchange buffer too small");
  }
  if ((a.wino_u == nullptr) != (a.wino_ud == nullptr))
    throw std::runtime_error("xgmi_step: Winograd transforms need both U and Ud");
  if (!a.part2 || !a.part1 || a.ngroups <= 0 || a.nblk1 <= 0 || a.off_w2 % 4)
    throw std::runtime_error("xgmi_step: conv slabs / offsets");
  if (a.fc_local && a.fa2) {
    // fc1 weight tiles + the rest of the bucket in streaming units
    if (!a.fdh || a.frows <= 0 || a.off_w3 % 4 || a.off_w3 / 4 + W1_F4 > a.fc4)
      throw std::runtime_error("xgmi_step: FC factors / fc1 weight offset");
    a.fc_in_bwd = 0;
    a.nfc = FC1BWD_DW_BLOCKS + (int)((a.fc4 - W1_F4 + 256 * FC_SGD_UNROLL - 1) / (256 * FC_SGD_UNROLL));
    a.ngather = 0;
  } else if (a.fc_local) {
    // the FC grads are global sums: a local streaming SGD of the whole bucket
    a.fc_in_bwd = 0;
    a.nfc = a.sync.lean ? 32 : 256;
    a.ngather = 0;
  } else if (a.fc_in_bwd) {
    // the exchange + SGD ran in the conv2 backward launch; this one gathers
    a.fc4 = in.fc4;
    a.seg4 = a.fc4 / n;
    a.nfc = 0;
    a.ngather = a.sync.lean ? 16 : 256;
  } else {
    // latency-bound loads when the links are fast: many blocks (few when the
    // ranks share a GPU)
    xgmi_fc_plan(a, 256, a.sync.lean ? XS_FC_BLOCKS : 4 * XS_FC_BLOCKS);
    a.ngather = 0;
  }
  // one block per conv unit (latency-bound slab sums: they want the whole
  // chip), or XS_CONV_BLOCKS looping over them when the ranks share a GPU
  a.ncv = a.sync.lean ? XS_CONV_BLOCKS : (a.wino_u ? 128 : 50) + 16 + 208;
  xgmi_step_kernel<<<a.nfc + a.ngather + a.ncv, 256, 0, s>>>(a);
}

// SCHED_XGMI_FAC: every peer's factor rows over its link (see XgmiFacArgs).
// Block b copies slice b of every (buffer, peer) slot, all of a thread's loads
// in flight together.  No closing barrier: a peer rewrites its slot only in its
// next step's forward, after its step launch's conv barrier, which waits for
// this rank's step launch - queued behind this copy.
__device__ void xgmi_fac_gather_block(const XgmiFacArgs& a, int gb, int ngb, unsigned* ep) {
  const xgmi::Sync& s = a.sync;
  const int n = s.nranks, me = s.rank, tid = threadIdx.x;
  const unsigned e = xgmi::next_epoch(s, ep);
  xgmi::barrier(s, 0, e, /*release=*/true);  // the rows come from the forward / head kernels
  const long long t0 = xgmi::now_ticks();
  long long bytes = 0;
#pragma unroll
  for (int k = 0; k < XgmiFacArgs::kBufs; ++k) {
    const long long n4 = a.slot4[k];
    bytes += n4 * 16;
    if (n4 == 0) continue;
    const long long per = ((n4 + ngb - 1) / ngb + 255) / 256 * 256;
    const long long lo = (long long)gb * per, hi = min(lo + per, n4);
    float4* mine = reinterpret_cast<float4*>(a.buf[k][me]);
    for (long long i0 = lo + tid; i0 < hi; i0 += 256 * XS_UNROLL) {
      float4 v[xgmi::kMaxRanks][XS_UNROLL];
#pragma unroll
      for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
        for (int u = 0; u < XS_UNROLL; ++u)
          if (r < n && r != me && i0 + 256 * u < hi) {
            const xgmi::Rsrc rs = xgmi::rsrc(a.buf[k][r], (unsigned long long)n * n4 * 16);
            v[r][u] = xgmi::ld4_sys(rs, (unsigned)(((long long)r * n4 + i0 + 256 * u) * 16));
          }
#pragma unroll
      for (int r = 0; r < xgmi::kMaxRanks; ++r)
#pragma unroll
        for (int u = 0; u < XS_UNROLL; ++u)
          if (r < n && r != me && i0 + 256 * u < hi) mine[(long long)r * n4 + i0 + 256 * u] = v[r][u];
    }
  }
  xgmi::link_floor(s, t0, bytes);
}

__global__ __launch_bounds__(256) void xgmi_fac_gather_kernel(const XgmiFacArgs a) {
  __shared__ unsigned ep;
  xgmi_fac_gather_block(a, blockIdx.x, gridDim.x, &ep);
}

// fc1 dX blocks | factor gather blocks (the gather's barrier slots are its
// own block indices 0 .. ngb - 1: the flag protocol is per block index)
__global__ __launch_bounds__(256) void fc1_bwd_dx_fac_kernel(
    const float* __restrict__ a2, const uint8_t* __restrict__ idx2, const float* __restrict__ dh,
    const float* __restrict__ w1, int batch, float* __restrict__ dy2, float* __restrict__ dy2t,
    int ngb, const XgmiFacArgs f) {
  __shared__ float smem[4 * FC1DX_WAVE];
  if ((int)blockIdx.x < ngb) {
    xgmi_fac_gather_block(f, blockIdx.x, ngb, reinterpret_cast<unsigned*>(smem));
    return;
  }
  const int nb = (int)gridDim.x - ngb;
  const int L = xcd_remap((int)blockIdx.x - ngb, nb);
  fc1_bwd_dx(L, a2, idx2, dh, w1, batch, dy2, dy2t, smem);
}

static void check_fac(const XgmiFacArgs& a) {
  const int n = a.sync.nranks;
  if (n < 1 || n > xgmi::kMaxRanks || !a.sync.flags || !a.sync.epoch || !a.sync.error)
    throw std::runtime_error("xgmi_fac_gather: communicator not set up");
  for (int k = 0; k < XgmiFacArgs::kBufs; ++k)
    for (int r = 0; r < n; ++r)
      if (a.slot4[k] > 0 && !a.buf[k][r])
        throw std::runtime_error("xgmi_fac_gather: a rank's factor buffer is not mapped");
}

void launch_fc1_bwd_dx_fac_gather(const float* a2, const uint8_t* idx2, const float* dh,
                                  const float* w1, int batch, float* dy2, float* dy2t,
                                  const XgmiFacArgs& f, hipStream_t s) {
  if (batch <= 0 || batch % 32 != 0) throw std::runtime_error("fc1_bwd: batch % 32 != 0");
  check_fac(f);
  // 196 dX blocks at B = 64 + 56 gather blocks: one round on 256 CUs
  const int ndx = (batch / 32) * (FC1_IN / 32);
  const int ngb = f.sync.lean ? 16 : std::max(16, std::min(128, 256 - ndx));
  fc1_bwd_dx_fac_kernel<<<ngb + ndx, 256, 0, s>>>(a2, idx2, dh, w1, batch, dy2, dy2t, ngb, f);
}

__global__ __launch_bounds__(256) void fc1_small_grads_kernel(const float* __restrict__ dh,
                                                              const float* __restrict__ hd,
                                                              const float* __restrict__ dlog,
                                                              int rows, float* __restrict__ g_b3,
                                                              float* __restrict__ g_w4,
                                                              float* __restrict__ g_b4) {
  __shared__ float smem[FC1_SMALL_SMEM];
  fc1_small_grads(blockIdx.x, hd, dh, dlog, rows, g_w4, g_b4, g_b3, smem);
}

void launch_fc1_small_grads(const float* dh, const float* hd, const float* dlog, int rows,
                            float* g_b3, float* g_w4, float* g_b4, hipStream_t s) {
  if (rows <= 0 || rows % 32 != 0) throw std::runtime_error("fc1_small_grads: rows % 32 != 0");
  fc1_small_grads_kernel<<<SMALL_BLOCKS, 256, 0, s>>>(dh, hd, dlog, rows, g_b3, g_w4, g_b4);
}

void launch_xgmi_fac_gather(const XgmiFacArgs& a, hipStream_t s) {
  const int n = a.sync.nranks;
  if (n < 1 || n > xgmi::kMaxRanks || !a.sync.flags || !a.sync.epoch || !a.sync.error)
    throw std::runtime_error("xgmi_fac_gather: communicator not set up");
  for (int k = 0; k < XgmiFacArgs::kBufs; ++k)
    for (int r = 0; r < n; ++r)
      if (a.slot4[k] > 0 && !a.buf[k][r])
        throw std::runtime_error("xgmi_fac_gather: a rank's factor buffer is not mapped");
  xgmi_fac_gather_kernel<<<a.sync.lean ? 16 : 128, 256, 0, s>>>(a);
}

void launch_grad_finalize(const float* part2, int ngroups, const float* part1, int nblk1,
                          float* g_w2, float* g_b2, float* g_w1, float* g_b1, hipStream_t s) {
  if (reinterpret_cast<uintptr_t>(g_w2) % 16 || reinterpret_cast<uintptr_t>(part2) % 16)
    throw std::runtime_error("grad_finalize: dW2 / slabs must be 16-byte aligned");
  const int b2 = 51200 / 4 / 256 + 16;
  const int b1 = cdiv(832, 4);
  grad_finalize_kernel<<<b2 + b1, 256, 0, s>>>(part2, part2 + (size_t)ngroups * 51200, ngroups,
                                               part1, nblk1, g_w2, g_b2, g_w1, g_b1);
}

size_t part2_floats(int batch) { return (size_t)conv2_filter_splits(batch) * (51200 + 256); }
size_t part1_floats(int batch) { return (size_t)conv1_filter_blocks(batch) * 832; }
size_t fc1_part_floats(int batch) { return (size_t)FC1_SPLITS * batch * FC1_OUT; }

}  // namespace mnist
