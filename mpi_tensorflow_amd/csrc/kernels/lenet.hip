// Fused fp32 LeNet-5 kernel set for gfx950 (BASELINE config 4).
//
// Model (models/generic.py LeNet5, same op pattern as the reference's
// conv -> bias+ReLU -> pool -> ... -> matmul chain, /root/reference/mpipy.py:155-167):
//   x [32,32,3] -> conv5x5(3->6) valid + b, ReLU, maxpool2 -> [14,14,6]
//   -> conv5x5(6->16) valid + b, ReLU, maxpool2 -> [5,5,16] = 400 (h,w,c)
//   -> FC 400->120 + ReLU -> FC 120->84 + ReLU -> FC 84->10 -> softmax xent.
//
// At B = 64 the whole step is ~250 MFLOP: the round-1 generic path spent it
// in ~37 launches (conv engines, library GEMMs, reductions, 239 us/step).
// Here a train step is TWO launches:
//
//  image kernel  PARTS (4) 512-thread workgroups per image, everything in LDS
//                (train; eval runs one per image).  Each of the 4 runs the
//                image's forward and FC backward chain itself (cheap, redundant)
//                and then a quarter of the conv backward: conv2 filter grad of
//                4 of the 16 output channels, conv2 data grad / conv1 filter
//                grad of its share of the 6 conv1 channels ({0,1} {2,3} {4} {5}).
//                256 workgroups at B = 64 instead of 64 on a 256-CU part:
//                batch row at the device-step offset, conv1 / conv2 with the
//                pool + argmax in the epilogue (pool windows = 4 accumulators
//                of one thread, as float2 pairs -> v_pk_fma_f32), the FC chain
//                and softmax xent forward, then the whole backward pass: FC
//                dX chain, pool2/ReLU2 scatter, conv2 filter grad (sparse:
//                only the 25 argmax pixels per channel carry gradient),
//                conv2 data grad, pool1/ReLU1, conv1 filter grad (sparse
//                again).  Per image it writes the FC layer inputs / deltas and
//                its 2872 conv weight-gradient partials.
//  update kernel FC weight grads as act^T delta over the batch (LDS-staged
//                tiles), conv grads as the sum of the per-image partials (in
//                image order: deterministic), then momentum SGD with the
//                device LR, and the device-step bump.
//
// Eval is the image kernel's forward half, ending in argmax + error count.
#include <stdexcept>

#include "common.h"
#include "lenet.h"

namespace lenet {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int NT = 512;  // threads per image workgroup
constexpr int PARTS = 4;  // train: workgroups per image (blockIdx = part * batch + image)
constexpr int IH = 32, IC = 3;
constexpr int C1 = 6, P1 = 14;
constexpr int C2 = 16, O2 = 10, P2 = 5;
constexpr int F0 = 400, F1 = 120, F2 = 84, F3 = 10;
constexpr int W1N = 25 * IC * C1;  // 450
constexpr int W2N = 25 * C1 * C2;  // 2400
constexpr int DP = O2 + 8;         // zero-bordered dpre2 plane (18 x 18)
constexpr int DPS = 20;            // dpre2 pixel stride: 16 channels + 4 pad (bank spread)
constexpr int XRS = 36, XPL = IH * XRS + 20;  // input row / plane strides (bank spread)

// LDS layout (floats).  gfx950 lets one workgroup own up to 160 KiB.
constexpr int S_X = 0;                        // input planes [3][32][XRS]
constexpr int S_W1 = S_X + IC * XPL;          // conv1 HWIO weights + bias
constexpr int S_B1 = S_W1 + 456;
constexpr int S_W2 = S_B1 + 8;                // conv2 HWIO [tap][ci][co]
constexpr int S_W2T = S_W2 + W2N;             // conv2 [tap][co][ci] (data grad operand)
constexpr int S_B2 = S_W2T + W2N;
constexpr int S_P1 = S_B2 + C2;               // pooled conv1 [14][14][6]
constexpr int S_P2 = S_P1 + P1 * P1 * C1;     // pooled conv2 [5][5][16] = a2
constexpr int S_H1 = S_P2 + F0;
constexpr int S_H2 = S_H1 + 128;
constexpr int S_D3 = S_H2 + 88;               // dlogits
constexpr int S_D2 = S_D3 + 16;               // dz2
constexpr int S_D1 = S_D2 + 88;               // dz1
constexpr int S_T2 = S_D1 + 128;              // (g2, p1 offset of the argmax) per (pp, co)
constexpr int S_DPRE2 = S_T2 + 2 * F0;        // dpre2 [18][18][DPS], zero border
constexpr int S_T1 = S_DPRE2;                 // (g1, x offset of the argmax) per (p, c): after I
constexpr int S_G1 = S_DPRE2 + DP * DP * DPS; // data-grad partials of co quarters 1..3
constexpr int S_RED = S_G1 + 3 * P1 * P1 * C1; // split-K partials
constexpr int S_FB = S_RED + NT;              // FC biases [120 | 84 | 10] (loaded in A)
constexpr int S_C2P = S_FB + F1 + F2 + F3 + 2;  // conv2 partials [ci][pp][4][co] (phase C)
constexpr int S_TOTAL = S_C2P + C1 * P2 * P2 * 4 * C2;
static_assert(S_TOTAL * 4 <= 160 * 1024, "image kernel LDS budget");
static_assert(S_W2 % 4 == 0 && S_C2P % 4 == 0, "float4 LDS regions");
static_assert(2 * P1 * P1 * C1 <= DP * DP * DPS, "T1 must fit in the dpre2 region");

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// 2x2 max pool of accumulators (q order: (0,0) (0,1) (1,0) (1,1), strict >
// so the first maximum wins, like TF / torch max pooling)
__device__ __forceinline__ void pool4(f2 a01, f2 a23, float& v, int& q) {
  v = a01.x;
  q = 0;
  if (a01.y > v) { v = a01.y; q = 1; }
  if (a23.x > v) { v = a23.x; q = 2; }
  if (a23.y > v) { v = a23.y; q = 3; }
}

// (phase barriers: lds_barrier, common.h - the FC weight prefetches below stay
// in flight across them)
// one workgroup per CU (LDS): 2 waves a SIMD, up to 256 VGPRs a lane - the room
// the FC weight prefetches live in
template <bool TRAIN>
__global__ __launch_bounds__(NT, 1) void image_kernel(const ImageArgs a) {
  __shared__ float sm[S_TOTAL];
  __shared__ uint8_t q1s[P1 * P1 * C1];
  __shared__ uint8_t q2s[F0];
  const int tid = threadIdx.x;
  // train: part q of image img; the PARTS workgroups of an image are batch
  // blocks apart (same blockIdx % 8 for B % 8 == 0: one XCD, one L2)
  const int q = TRAIN ? (int)blockIdx.x / a.batch : 0;
  const int img = TRAIN ? (int)blockIdx.x % a.batch : (int)blockIdx.x;
  long long row = img;
  if (TRAIN) {
    const long long st = *a.step;
    row = (st * a.batch) % (long long)(a.n_local - a.batch) + img;
    if (img == 0 && q == 0 && tid == 0)  // reference LR schedule (mpipy.py:59-64), staircase per local epoch
      *a.lr_out = a.base_lr * powf(a.lr_decay, (float)((st * a.batch) / a.n_local));
  }
  const float* W = a.params;
  const Offsets o = a.off;

  // ---- A: every global load of the phase issued before any LDS store (one
  // memory round trip): image rows (NHWC float4 -> padded planes), conv
  // weights (+ the [tap][co][ci] copy of W2 for the data grad)
  {
    const float4* xr4 = reinterpret_cast<const float4*>(a.x + row * (IH * IH * IC));
    float4 xv[2];
    xv[0] = xr4[tid];
    if (tid < 256) xv[1] = xr4[tid + NT];
    const float w1v = tid < W1N ? W[o.c1w + tid] : 0.f;
    const float b1v = tid < C1 ? W[o.c1b + tid] : 0.f;
    const float b2v = tid < C2 ? W[o.c2b + tid] : 0.f;
    // the FC biases (read after a phase barrier, each was an exposed round trip)
    const float fbv = tid < F1 ? W[o.f1b + tid]
                      : tid < F1 + F2 ? W[o.f2b + tid - F1]
                      : tid < F1 + F2 + F3 ? W[o.f3b + tid - F1 - F2] : 0.f;
    float w2v[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int e = tid + NT * k;
      w2v[k] = e < W2N ? W[o.c2w + e] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && tid >= 256) break;
      const int e0 = 4 * (tid + NT * k);
      const float v[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = e0 + j, ci = e % IC, pix = e / IC;
        sm[S_X + ci * XPL + (pix >> 5) * XRS + (pix & 31)] = v[j];
      }
    }
    if (tid < W1N) sm[S_W1 + tid] = w1v;
    if (tid < C1) sm[S_B1 + tid] = b1v;
    if (tid < C2) sm[S_B2 + tid] = b2v;
    if (tid < F1 + F2 + F3) sm[S_FB + tid] = fbv;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int e = tid + NT * k;
      if (e < W2N) {
        sm[S_W2 + e] = w2v[k];
        const int co = e & 15, ci = (e >> 4) % C1, t = (e >> 4) / C1;
        sm[S_W2T + (t * C2 + co) * C1 + ci] = w2v[k];
      }
    }
    if (TRAIN)
#pragma unroll
      for (int k = 0; k < (DP * DP * DPS + NT - 1) / NT; ++k) {
        const int e = tid + NT * k;
        if (e < DP * DP * DPS) sm[S_DPRE2 + e] = 0.f;
      }
  }
  const int label = a.y[row];
  lds_barrier();
  if (a.stop_phase == 0) return;
  // ---- B: conv1 + bias + ReLU + pool: thread = pooled pixel, all 6 channels
  // (each input read feeds 6 channels; the weights are LDS broadcasts)
  if (tid < P1 * P1) {
    const int p = tid, py = p / P1, px = p % P1;
    f2 s01[C1], s23[C1];
#pragma unroll
    for (int c = 0; c < C1; ++c) s01[c] = s23[c] = f2{0.f, 0.f};
#pragma unroll
    for (int ci = 0; ci < IC; ++ci)
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float* xp = sm + S_X + ci * XPL + (2 * py + kh) * XRS + 2 * px + kw;
          const f2 x01 = {xp[0], xp[1]}, x23 = {xp[XRS], xp[XRS + 1]};
          const float* wp = sm + S_W1 + ((kh * 5 + kw) * IC + ci) * C1;
#pragma unroll
          for (int c = 0; c < C1; ++c) {
            const f2 w = {wp[c], wp[c]};
            s01[c] = __builtin_elementwise_fma(x01, w, s01[c]);
            s23[c] = __builtin_elementwise_fma(x23, w, s23[c]);
          }
        }
#pragma unroll
    for (int c = 0; c < C1; ++c) {
      float v;
      int q;
      pool4(s01[c], s23[c], v, q);
      sm[S_P1 + p * C1 + c] = relu(v + sm[S_B1 + c]);
      q1s[p * C1 + c] = (uint8_t)q;
    }
  }
  lds_barrier();
  if (a.stop_phase == 1) return;
  // the FC1 weights, requested now (their round trip hides under conv2) and
  // kept in registers for BOTH FC1 passes: thread t < 500 holds the 8 x 12
  // block (rows 8 rb .., columns 12 cb ..) of W1 [400][120] - forward
  // (phase D) and backward (da2 in phase G) each sum in-thread over one block
  // axis and across threads over the other, through LDS.  (With a column per
  // thread, the backward had to read W1 again by rows: a 49 MB burst over all
  // workgroups at once, ~3 us.)
  const int fj = tid & 127, fg = tid >> 7;
  const int rb = min(tid, 499) / 10, cb = min(tid, 499) % 10, i0 = 8 * rb, j0 = 12 * cb;
  float w1b[8][12];
  {
    const float4* wp = reinterpret_cast<const float4*>(W + o.f1w + i0 * F1 + j0);
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float4 v = wp[(r * F1) / 4 + c];
        w1b[r][4 * c] = v.x;
        w1b[r][4 * c + 1] = v.y;
        w1b[r][4 * c + 2] = v.z;
        w1b[r][4 * c + 3] = v.w;
      }
  }

  // ---- C: conv2 + bias + ReLU + pool, register-blocked: thread = (input
  // channel ci, output-channel octet cg, pooled pixel pp) holds the 6 x 6 input
  // patch of its pool window in registers and forms 8 channels x 4 window
  // positions from each pair of float4 weight reads - a quarter of the LDS
  // bytes of one thread per (pp, co), which made this phase LDS-bound.  The 6
  // per-channel partials are then summed in ci order by (pp, co) threads.
  if (tid < C1 * 2 * P2 * P2) {
    const int ci = tid / 50, r = tid % 50, cg = r / 25, pp = r % 25, py = pp / P2, px = pp % P2;
    float xq[6][6];
    const float* xb = sm + S_P1 + (2 * py * P1 + 2 * px) * C1 + ci;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) xq[i][j] = xb[(i * P1 + j) * C1];
    f2 acc[4][4];  // [window position (dy, dx)][output-channel pair]
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[u][c] = f2{0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const float4* wp =
            reinterpret_cast<const float4*>(sm + S_W2 + ((kh * 5 + kw) * C1 + ci) * C2 + 8 * cg);
        const float4 wa = wp[0], wb = wp[1];
        const f2 w[4] = {{wa.x, wa.y}, {wa.z, wa.w}, {wb.x, wb.y}, {wb.z, wb.w}};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float xv = xq[kh + (u >> 1)][kw + (u & 1)];
          const f2 xx = {xv, xv};
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[u][c] = __builtin_elementwise_fma(xx, w[c], acc[u][c]);
        }
      }
    // partials [ci][pp][position][co]
    float4* pp4 = reinterpret_cast<float4*>(sm + S_C2P + ((ci * 25 + pp) * 4) * C2 + 8 * cg);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      pp4[u * 4] = make_float4(acc[u][0].x, acc[u][0].y, acc[u][1].x, acc[u][1].y);
      pp4[u * 4 + 1] = make_float4(acc[u][2].x, acc[u][2].y, acc[u][3].x, acc[u][3].y);
    }
  }
  lds_barrier();
  if (tid < F0) {
    const int co = tid & 15, pp = tid >> 4;
    float v4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float s = 0.f;
#pragma unroll
      for (int ci = 0; ci < C1; ++ci) s += sm[S_C2P + ((ci * 25 + pp) * 4 + u) * C2 + co];
      v4[u] = s;
    }
    float v;
    int q;
    pool4(f2{v4[0], v4[1]}, f2{v4[2], v4[3]}, v, q);
    sm[S_P2 + tid] = relu(v + sm[S_B2 + co]);  // (h, w, c) flatten = FC1 input order
    q2s[tid] = (uint8_t)q;
  }
  lds_barrier();
  if (a.stop_phase == 2) return;

  // FC2 / FC3 weights of phases E, F
  float wv2[30], wv3[3];
  if (fj < F2) {
    const float* wp = W + o.f2w + (fg * 30) * F2 + fj;
#pragma unroll
    for (int i = 0; i < 30; ++i) wv2[i] = wp[i * F2];
  }
  {
    const int j3 = tid & 15, g3 = tid >> 4;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int i = g3 + 32 * u;
      wv3[u] = (j3 < F3 && i < F2) ? W[o.f3w + i * F3 + j3] : 0.f;
    }
  }
  // ---- D: FC1 400 -> 120 + ReLU from the register blocks: partials
  // [rb][j] in the (free) conv2 partial region, then 50 row blocks summed in
  // order per output
  if (tid < 500) {
    float xv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xv[r] = sm[S_P2 + i0 + r];
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) acc = fmaf(xv[r], w1b[r][c], acc);
      sm[S_C2P + rb * F1 + j0 + c] = acc;
    }
  }
  lds_barrier();
  if (tid < F1) {
    float z = sm[S_FB + tid];
#pragma unroll 10
    for (int r = 0; r < 50; ++r) z += sm[S_C2P + r * F1 + tid];
    sm[S_H1 + tid] = relu(z);
  }
  lds_barrier();
  if (a.stop_phase == 10) return;  // (labs: lenet_phases.py sub-phase stops)
  // the FC backward (dX chain) weights of phase G, requested now (train)
  float g3w[F3], g2w[21];
  if (TRAIN) {
    if (tid < F2) {
#pragma unroll
      for (int j = 0; j < F3; ++j) g3w[j] = W[o.f3w + tid * F3 + j];
    }
    if ((tid >> 2) < F1) {
      const float* wp = W + o.f2w + (tid >> 2) * F2 + (tid & 3) * 21;
#pragma unroll
      for (int j = 0; j < 21; ++j) g2w[j] = wp[j];
    }
  }
  // ---- E: FC2 120 -> 84 + ReLU
  {
    float acc = 0.f;
    if (fj < F2) {
      const float* xp = sm + S_H1 + fg * 30;
#pragma unroll
      for (int i = 0; i < 30; ++i) acc = fmaf(xp[i], wv2[i], acc);
    }
    sm[S_RED + tid] = acc;
  }
  lds_barrier();
  if (tid < F2) {
    const float z = sm[S_FB + F1 + tid] + sm[S_RED + tid] + sm[S_RED + 128 + tid] +
                    sm[S_RED + 256 + tid] + sm[S_RED + 384 + tid];
    sm[S_H2 + tid] = relu(z);
  }
  lds_barrier();
  if (a.stop_phase == 11) return;
  // ---- F: FC3 84 -> 10: 32 K groups of <= 3
  {
    const int j = tid & 15, g = tid >> 4;
    float acc = 0.f;
    if (j < F3)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = g + 32 * u;
        if (i < F2) acc = fmaf(sm[S_H2 + i], wv3[u], acc);
      }
    sm[S_RED + tid] = acc;
  }
  lds_barrier();
  if (a.stop_phase == 12) return;
  if (tid < 64) {  // one wave: logits, softmax xent, argmax
    float lg = -INFINITY;
    if (tid < F3) {
      float z = sm[S_FB + F1 + F2 + tid];
      for (int g = 0; g < 32; ++g) z += sm[S_RED + g * 16 + tid];
      lg = z;
    }
    const float mx = wave_max(lg);
    const unsigned long long bal = __ballot(tid < F3 && lg == mx);
    const int am = __ffsll((long long)bal) - 1;
    if (!TRAIN) {
      if (a.logits && tid < F3) a.logits[(size_t)img * F3 + tid] = lg;
      if (tid == 0 && a.errors && am != label) atomicAdd(a.errors, 1);
      return;
    }
    const float e = tid < F3 ? __expf(lg - mx) : 0.f;
    const float se = wave_sum(e);
    const float lab = wave_sum(tid == label ? lg : 0.f);
    if (tid < F3) sm[S_D3 + tid] = (e / se - (tid == label ? 1.f : 0.f)) / (float)a.batch;
    if (tid == 0 && q == 0) {
      a.loss_rows[img] = logf(se) + mx - lab;
      if (a.correct && am == label) atomicAdd(a.correct, 1);
    }
  }
  if (!TRAIN) return;
  lds_barrier();
  if (a.stop_phase == 3) return;

  // ---- G: FC backward (dX chain), ReLU masks from the stored activations
  float* act = a.acts + (size_t)img * ACT_STRIDE;
  float* del = a.deltas + (size_t)img * DELTA_STRIDE;
  if (tid < F2) {  // dz2 = relu'(h2) * W3 dz3
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < F3; ++j) s = fmaf(g3w[j], sm[S_D3 + j], s);
    sm[S_D2 + tid] = sm[S_H2 + tid] > 0.f ? s : 0.f;
  }
  lds_barrier();
  {  // dz1 = relu'(h1) * W2f dz2: 4 lanes per row, 21 columns each
    const int i = tid >> 2, part = tid & 3;
    float s = 0.f;
    if (i < F1) {
#pragma unroll
      for (int j = 0; j < 21; ++j) s = fmaf(g2w[j], sm[S_D2 + part * 21 + j], s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (i < F1 && part == 0) sm[S_D1 + i] = sm[S_H1 + i] > 0.f ? s : 0.f;
  }
  lds_barrier();
  // da2 = W1f dz1 from the register blocks: partials [cb][i], then 10 column
  // blocks summed in order per input, through ReLU2 (pooled > 0) -> g2
  if (tid < 500) {
    float dv[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) dv[c] = sm[S_D1 + j0 + c];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 12; ++c) acc = fmaf(w1b[r][c], dv[c], acc);
      sm[S_C2P + cb * F0 + i0 + r] = acc;
    }
  }
  lds_barrier();
  if (tid < F0) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) s += sm[S_C2P + c * F0 + tid];
    const float g2 = sm[S_P2 + tid] > 0.f ? s : 0.f;
    // pool2 backward: the gradient lands on the argmax pixel of the window
    const int co = tid & 15, pp = tid >> 4, py = pp / P2, px = pp % P2, q = q2s[tid];
    const int u = 2 * py + (q >> 1), v = 2 * px + (q & 1);
    sm[S_DPRE2 + ((u + 4) * DP + v + 4) * DPS + co] = g2;
    sm[S_T2 + 2 * tid] = g2;
    sm[S_T2 + 2 * tid + 1] = __int_as_float((u * P1 + v) * C1);
  }
  // FC layer inputs / deltas for the batch-level weight gradients (part 0)
  if (q == 0) {
    if (tid < F0) act[tid] = sm[S_P2 + tid];
    if (tid < F1) act[F0 + tid] = sm[S_H1 + tid];
    if (tid < F2) act[F0 + F1 + tid] = sm[S_H2 + tid];
    if (tid < F1) del[tid] = sm[S_D1 + tid];
    if (tid < F2) del[F1 + tid] = sm[S_D2 + tid];
    if (tid < F3) del[F1 + F2 + tid] = sm[S_D3 + tid];
  }
  lds_barrier();

  float* cp = a.convp + (size_t)img * CONVP_STRIDE;
  if (a.stop_phase == 4) return;
  // ---- H: conv2 filter grad, sparse over the 25 argmax pixels per channel
  // (table T2 = (g2, p1 offset of the argmax pixel) per (pp, co)):
  // dW2[kh,kw,ci,co] = sum_pp g2[pp,co] * p1[u_pp + kh, v_pp + kw, ci];
  // this part's 4 output channels co = 4q .. 4q + 3 (600 weights)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int f = tid + NT * k;
    if (f < W2N / PARTS) {
      const int co = 4 * q + (f & 3), r = f >> 2, ci = r % C1, t = r / C1, kh = t / 5, kw = t % 5;
      const int e = r * C2 + co;
      const float* p1 = sm + S_P1 + (kh * P1 + kw) * C1 + ci;
      const float2* t2 = reinterpret_cast<const float2*>(sm + S_T2) + co;
      float s = 0.f;
#pragma unroll
      for (int pp = 0; pp < P2 * P2; ++pp) {
        const float2 tv = t2[pp * C2];
        s = fmaf(tv.x, p1[__float_as_int(tv.y)], s);
      }
      cp[W1N + 8 + e] = s;
    }
  }
  if (tid < 4) {  // db2 of this part's channels
    const int co = 4 * q + tid;
    float s = 0.f;
    for (int pp = 0; pp < P2 * P2; ++pp) s += sm[S_T2 + 2 * (pp * C2 + co)];
    cp[W1N + 8 + W2N + co] = s;
  }
  if (a.stop_phase == 5) return;
  // ---- I: conv2 data grad over the zero-bordered dpre2 plane:
  // dp1[y,x,ci] = sum_{kh,kw,co} dpre2[y-kh, x-kw, co] W2[kh,kw,ci,co].
  // This part's conv1 channels as ONE packed pair (v_pk_fma_f32): pair pi =
  // {2 pi, 2 pi + 1}, parts 0 / 1 use pairs 0 / 1, parts 2 / 3 pair 2 (channel
  // 4 / 5 of it); the weights from the [tap][co][ci] copy of W2.
  const int pi = q < 2 ? q : 2;
  const int c_lo = q < 2 ? 2 * q : q + 2, c_hi = q < 2 ? 2 * q + 2 : q + 3;
  // Register-blocked: thread = (output-channel quarter grp, pair of adjacent
  // pooled1 pixels) - the two pixels' 5 x 5 dpre2 windows share 4 of their
  // 5 columns (6 float4 reads a kernel row for both) and every weight read
  // serves both pixels.  The quarters' partials are summed in grp order.
  {
    const int grp = tid >> 7, pr = tid & 127;
    const bool act = pr < P1 * P1 / 2;
    const int y = pr / (P1 / 2), x = 2 * (pr % (P1 / 2));
    f2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};  // pixels (y, x), (y, x + 1)
    if (act) {
#pragma unroll
      for (int kh = 0; kh < 5; ++kh) {
        const float4* rp =
            reinterpret_cast<const float4*>(sm + S_DPRE2 + ((y - kh + 4) * DP + x) * DPS + 4 * grp);
        float4 dr[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) dr[k] = rp[k * (DPS / 4)];
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const f2* wp =
              reinterpret_cast<const f2*>(sm + S_W2T + ((kh * 5 + kw) * C2 + 4 * grp) * C1);
          const float4 da = dr[4 - kw], db = dr[5 - kw];
          const float av[4] = {da.x, da.y, da.z, da.w}, bv[4] = {db.x, db.y, db.z, db.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const f2 w = wp[3 * c + pi];
            s0 = __builtin_elementwise_fma(f2{av[c], av[c]}, w, s0);
            s1 = __builtin_elementwise_fma(f2{bv[c], bv[c]}, w, s1);
          }
        }
      }
      if (grp > 0) {
        float* gp = sm + S_G1 + (grp - 1) * (P1 * P1 * C1) + (y * P1 + x) * C1 + 2 * pi;
        gp[0] = s0.x, gp[1] = s0.y;
        gp[C1] = s1.x, gp[C1 + 1] = s1.y;
      }
    }
    lds_barrier();  // every dpre2 read is done: the T1 table may overwrite it
    if (grp == 0 && act) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int px = x + h, p = y * P1 + px;
        const f2 sp = h ? s1 : s0;
        for (int c = c_lo; c < c_hi; ++c) {
          float g = c == 2 * pi ? sp.x : sp.y;
#pragma unroll
          for (int k = 0; k < 3; ++k) g += sm[S_G1 + k * (P1 * P1 * C1) + p * C1 + c];
          const int qq = q1s[p * C1 + c];
          const int u = 2 * y + (qq >> 1), v = 2 * px + (qq & 1);
          // ReLU1 through the pooled output; T1 = (g1, input offset of the argmax)
          sm[S_T1 + 2 * (p * C1 + c)] = sm[S_P1 + p * C1 + c] > 0.f ? g : 0.f;
          sm[S_T1 + 2 * (p * C1 + c) + 1] = __int_as_float(u * XRS + v);
        }
      }
    }
  }
  lds_barrier();
  if (a.stop_phase == 6) return;
  // ---- J: conv1 filter grad, sparse over the 196 argmax pixels per channel:
  // dW1[kh,kw,ci,c] = sum_p g1[p,c] * x[ci, u_p + kh, v_p + kw], for this
  // part's channels c in [c_lo, c_hi).  Register-blocked over kw: a thread
  // forms the 5 weights of one (c, ci, kh) row from one T1 read per pixel;
  // S threads of a row split the pixels (p = part, part + S, ...), summed by a
  // fixed xor tree.  240 threads: waves 0-3 (db1 below runs in wave 7).
  {
    const int nc = c_hi - c_lo;              // 2 (parts 0, 1) or 1 (parts 2, 3)
    const int lgS = nc == 2 ? 3 : 4, S = 1 << lgS;
    const int row = tid >> lgS, part = tid & (S - 1);
    const bool act = row < 15 * nc;          // (c, ci, kh) rows of this part
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    const int c = c_lo + row % nc, ci = (row / nc) % IC, kh = row / (nc * IC);
    if (act) {
      const float* xp = sm + S_X + ci * XPL + kh * XRS;
      const float2* t1 = reinterpret_cast<const float2*>(sm + S_T1) + c;
#pragma unroll 4
      for (int p = part; p < P1 * P1; p += S) {
        const float2 tv = t1[p * C1];
        const float* xr = xp + __float_as_int(tv.y);
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc[kw] = fmaf(tv.x, xr[kw], acc[kw]);
      }
    }
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
#pragma unroll
      for (int m = 1; m < 16; m <<= 1)
        if (m < S) acc[kw] += __shfl_xor(acc[kw], m, 64);
    }
    if (act && part == 0) {
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) cp[((kh * 5 + kw) * IC + ci) * C1 + c] = acc[kw];
    }
    if (tid >= 448) {  // db1: wave 7 (idle above), lanes over the pixels + a wave sum
      const int lane = tid - 448;
      for (int c = c_lo; c < c_hi; ++c) {
        float sb = 0.f;
        for (int p = lane; p < P1 * P1; p += 64) sb += sm[S_T1 + 2 * (p * C1 + c)];
        sb = wave_sum(sb);
        if (lane == 0) cp[W1N + c] = sb;
      }
    }
  }
}

// ------------------------------------------------------------- update ----
// Blocks: FC weight gradients as fp32-MFMA tiles, g[i][j] = sum_n act[n][i]
// delta[n][j] (M = inputs i, N = outputs j, K = the batch): one 32 x 32 tile a
// wave, four a block (f1: 13 x 4, f2: 4 x 3, f3: 3 x 1 tiles; the row-0 tiles
// also sum the bias), operands straight from L2 with every load of a 64-image
// chunk in flight; then 12 blocks of 256 conv parameters.  (The round-4
// VALU form - 16-row tiles on 39 blocks, LDS-staged deltas - was ~2/3 of the
// 10.5 us update launch.)
constexpr int FT_F1 = ((F0 + 31) / 32) * ((F1 + 31) / 32);  // 52
constexpr int FT_F2 = ((F1 + 31) / 32) * ((F2 + 31) / 32);  // 12
constexpr int FT_F3 = ((F2 + 31) / 32) * ((F3 + 31) / 32);  // 3
constexpr int FT_ALL = FT_F1 + FT_F2 + FT_F3;
constexpr int UB_FC = (FT_ALL + 3) / 4;
constexpr int CONV_N = W1N + 8 + W2N + C2;  // 2874 slots (2872 used)
constexpr int UB_CONV = (CONV_N + 255) / 256;

template <bool APPLY>
__device__ __forceinline__ void apply_one(float* w, float* g, float* m, int i, float gv, float mu,
                                          float lr) {
  if (APPLY) {
    const float mv = mu * m[i] + gv;
    m[i] = mv;
    w[i] -= lr * mv;
  } else {
    g[i] = gv;
  }
}

// FC tile ft (0 .. FT_ALL - 1) of the update launch: geometry and the lane's
// weight / bias indices
struct FcTile {
  int nin, nout, aoff, doff, woff, boff, i0, j0, ia, jb;
  bool bias_tile;
};
__device__ __forceinline__ FcTile fc_tile(int ft, const Offsets& o, int lane) {
  int layer, t;
  if (ft < FT_F1) {
    layer = 0;
    t = ft;
  } else if (ft < FT_F1 + FT_F2) {
    layer = 1;
    t = ft - FT_F1;
  } else {
    layer = 2;
    t = ft - FT_F1 - FT_F2;
  }
  FcTile f;
  f.nin = layer == 0 ? F0 : (layer == 1 ? F1 : F2);
  f.nout = layer == 0 ? F1 : (layer == 1 ? F2 : F3);
  f.aoff = layer == 0 ? 0 : (layer == 1 ? F0 : F0 + F1);
  f.doff = layer == 0 ? 0 : (layer == 1 ? F1 : F1 + F2);
  f.woff = layer == 0 ? o.f1w : (layer == 1 ? o.f2w : o.f3w);
  f.boff = layer == 0 ? o.f1b : (layer == 1 ? o.f2b : o.f3b);
  const int ntj = (f.nout + 31) / 32;
  f.i0 = (t / ntj) * 32;
  f.j0 = (t % ntj) * 32;
  f.ia = min(f.i0 + (lane & 31), f.nin - 1);
  f.jb = min(f.j0 + (lane & 31), f.nout - 1);
  f.bias_tile = f.i0 == 0;
  return f;
}

// g[i][j] = sum_n act[n][i] delta[n][j] of the tile (acc) and, on the row-0
// tiles, the bias column sum (bs, both lane halves)
__device__ __forceinline__ void fc_tile_product(const float* __restrict__ acts,
                                                const float* __restrict__ deltas, int batch,
                                                const FcTile& f, int lane, f32x16& acc, float& bs) {
  const int kh = lane >> 5;
  acc = zero16();
  bs = 0.f;
  for (int n0 = 0; n0 < batch; n0 += 64) {
    float av[32], dv[32];
#pragma unroll
    for (int st = 0; st < 32; ++st) {
      const int n = min(n0 + 2 * st + kh, batch - 1);
      av[st] = acts[(size_t)n * ACT_STRIDE + f.aoff + f.ia];
      dv[st] = deltas[(size_t)n * DELTA_STRIDE + f.doff + f.jb];
    }
    // every load of the chunk issued before the first product
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int st = 0; st < 32; ++st) {
      const bool ok = n0 + 2 * st + kh < batch;
      const float d = ok ? dv[st] : 0.f;
      acc = mfma32x32x2(av[st], d, acc);
      bs += d;
    }
  }
  bs += __shfl_xor(bs, 32, 64);
}

// conv slot e (0 .. CONV_N - 1) -> flat parameter index, or -1 (padding)
__device__ __forceinline__ int conv_dst(int e, const Offsets& o) {
  if (e >= CONV_N) return -1;
  if (e < W1N) return o.c1w + e;
  if (e < W1N + C1) return o.c1b + (e - W1N);
  if (e < W1N + 8) return -1;
  if (e < W1N + 8 + W2N) return o.c2w + (e - W1N - 8);
  return o.c2b + (e - W1N - 8 - W2N);
}

// the sum of the per-image partials of conv slot e, in image order
__device__ __forceinline__ float conv_partial_sum(const float* __restrict__ convp, int batch,
                                                  int e) {
  float s = 0.f;
  for (int n0 = 0; n0 < batch; n0 += 64) {  // 64 image partials in flight, summed in order
    float v[64];
#pragma unroll
    for (int u = 0; u < 64; ++u)
      v[u] = n0 + u < batch ? convp[(size_t)(n0 + u) * CONVP_STRIDE + e] : 0.f;
#pragma unroll
    for (int u = 0; u < 64; ++u) s += v[u];
  }
  return s;
}

template <bool APPLY>
__global__ __launch_bounds__(256) void update_kernel(const float* __restrict__ acts,
                                                     const float* __restrict__ deltas,
                                                     const float* __restrict__ convp, int batch,
                                                     const Offsets o, float* __restrict__ w,
                                                     float* __restrict__ g, float* __restrict__ m,
                                                     float mu, const float* lr_ptr,
                                                     long long* step, long long dbuf) {
  const int tid = threadIdx.x;
  const float lr = APPLY ? *lr_ptr : 0.f;
  if (!APPLY && dbuf > 0) g += ((*step) & 1) * dbuf;  // the one-shot sync's slot
  int blk = blockIdx.x;
  if (APPLY && blk == 0 && tid == 0) *step += 1;
  if (blk < UB_FC) {
    const int lane = tid & 63, ft = blk * 4 + (tid >> 6);
    if (ft >= FT_ALL) return;
    const FcTile f = fc_tile(ft, o, lane);
    const int l31 = lane & 31, kh = lane >> 5;
    // the SGD operands of this lane's 16 weights (+ its bias) first: they are
    // independent of the gradient and arrive under the products
    float wv[16], mv[16], bwv = 0.f, bmv = 0.f;
    if (APPLY) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int wi = f.woff + min(f.i0 + mfma32_row(q, lane), f.nin - 1) * f.nout + f.jb;
        wv[q] = w[wi];
        mv[q] = m[wi];
      }
      if (f.bias_tile) {
        bwv = w[f.boff + f.jb];
        bmv = m[f.boff + f.jb];
      }
    }
    f32x16 acc;
    float bs;
    fc_tile_product(acts, deltas, batch, f, lane, acc, bs);
    if (f.j0 + l31 < f.nout) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = f.i0 + mfma32_row(q, lane);
        if (i >= f.nin) continue;
        const int wi = f.woff + i * f.nout + f.j0 + l31;
        if (APPLY) {
          const float mn = mu * mv[q] + acc[q];
          m[wi] = mn;
          w[wi] = wv[q] - lr * mn;
        } else {
          g[wi] = acc[q];
        }
      }
      if (f.bias_tile && kh == 0) {
        if (APPLY) {
          const float mn = mu * bmv + bs;
          m[f.boff + f.j0 + l31] = mn;
          w[f.boff + f.j0 + l31] = bwv - lr * mn;
        } else {
          g[f.boff + f.j0 + l31] = bs;
        }
      }
    }
    return;
  }
  // conv parameters: sum of the per-image partials, in image order
  const int e = (blk - UB_FC) * 256 + tid;
  const int dst = conv_dst(e, o);
  if (dst < 0) return;
  float wd = 0.f, md = 0.f;
  if (APPLY) {  // SGD operands first (independent of the gradient)
    wd = w[dst];
    md = m[dst];
  }
  const float s = conv_partial_sum(convp, batch, e);
  if (APPLY) {
    const float mn = mu * md + s;
    m[dst] = mn;
    w[dst] = wd - lr * mn;
    return;
  }
  apply_one<APPLY>(w, g, m, dst, s, mu, lr);
}

// The update launch with the xGMI push sync (PushArgs, lenet.h).  Same blocks
// and gradient forms as update_kernel; no thread leaves before the barrier
// (every block takes part in it).  A lane's values: FC - its 16 weights of
// the tile (+ the bias on the row-0 tiles, lanes 0-31); conv - one slot.
constexpr int PUSH_VALS = 17;
__global__ __launch_bounds__(256) void update_push_kernel(
    const float* __restrict__ acts, const float* __restrict__ deltas,
    const float* __restrict__ convp, int batch, const Offsets o, float* __restrict__ w,
    float* __restrict__ m, float mu, const float* lr_ptr, long long* step, const PushArgs pa) {
  __shared__ unsigned ep;
  const xgmi::Sync& S = pa.sync;
  const int n = S.nranks, me = S.rank, tid = threadIdx.x, lane = tid & 63;
  const int blk = blockIdx.x;
  if (blk == 0 && tid == 0) *step += 1;
  float gv[PUSH_VALS];
  int wi[PUSH_VALS];  // flat index of value v, or -1
#pragma unroll
  for (int v = 0; v < PUSH_VALS; ++v) {
    gv[v] = 0.f;
    wi[v] = -1;
  }
  if (blk < UB_FC) {
    const int ft = blk * 4 + (tid >> 6);
    if (ft < FT_ALL) {
      const FcTile f = fc_tile(ft, o, lane);
      f32x16 acc;
      float bs;
      fc_tile_product(acts, deltas, batch, f, lane, acc, bs);
      if (f.j0 + (lane & 31) < f.nout) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = f.i0 + mfma32_row(q, lane);
          gv[q] = acc[q];
          wi[q] = i < f.nin ? f.woff + i * f.nout + f.j0 + (lane & 31) : -1;
        }
        if (f.bias_tile && lane < 32) {
          gv[16] = bs;
          wi[16] = f.boff + f.j0 + lane;
        }
      }
    }
  } else {
    const int e = (blk - UB_FC) * 256 + tid;
    const int dst = conv_dst(e, o);
    if (dst >= 0) {
      gv[0] = conv_partial_sum(convp, batch, e);
      wi[0] = dst;
    }
  }
  // push: slot [parity][me] of every peer's receive buffer
  const long long slot_bytes = pa.total * 4;
  const long long rbytes = 2 * (long long)n * slot_bytes;
  const unsigned e = xgmi::next_epoch(S, &ep);
  const int par = (int)(e & 1u);
  const long long t0 = xgmi::now_ticks();
#pragma unroll
  for (int r = 0; r < xgmi::kMaxRanks; ++r) {
    if (r >= n || r == me) continue;
    const xgmi::Rsrc rs = xgmi::rsrc(pa.recv[r], rbytes);
    const unsigned base = (unsigned)(((long long)par * n + me) * slot_bytes);
#pragma unroll
    for (int v = 0; v < PUSH_VALS; ++v)
      if (wi[v] >= 0) xgmi::st_sys(rs, base + 4u * (unsigned)wi[v], gv[v]);
  }
  xgmi::link_floor(S, t0, slot_bytes);
  xgmi::barrier(S, 0, e, /*release=*/false);  // the pushed values are system-scope stores
  // every rank's values of every slot in flight at once (one round trip: the
  // SGD stores of a slot would otherwise keep the next slot's loads behind
  // them), then summed in rank order and applied
  const xgmi::Rsrc mine = xgmi::rsrc(pa.recv[me], rbytes);
  const float lr = *lr_ptr;
  float x[PUSH_VALS][xgmi::kMaxRanks];
#pragma unroll
  for (int v = 0; v < PUSH_VALS; ++v)
#pragma unroll
    for (int r = 0; r < xgmi::kMaxRanks; ++r)
      if (r < n && wi[v] >= 0)
        x[v][r] = !xgmi::contributes(S, r) ? 0.f
                  : r == me ? gv[v]
                            : xgmi::ld_sys(mine, (unsigned)(((long long)par * n + r) * slot_bytes +
                                                            4LL * wi[v]));
  float wv[PUSH_VALS], mv[PUSH_VALS];
#pragma unroll
  for (int v = 0; v < PUSH_VALS; ++v)
    if (wi[v] >= 0) {
      wv[v] = w[wi[v]];
      mv[v] = m[wi[v]];
    }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int v = 0; v < PUSH_VALS; ++v) {
    if (wi[v] < 0) continue;
    float sum = x[v][0];
#pragma unroll
    for (int r = 1; r < xgmi::kMaxRanks; ++r)
      if (r < n) sum += x[v][r];
    // optim::sgd_momentum_flat_kernel's expression forms (l2 = 0)
    const float g = __builtin_fmaf(0.f, wv[v], sum * pa.gscale);
    const float mn = mu * mv[v] + g;
    m[wi[v]] = mn;
    w[wi[v]] = wv[v] - lr * mn;
  }
}

// ------------------------------------------------------------- launchers ----
void launch_image_train(const ImageArgs& a, hipStream_t s) {
  if (a.batch <= 0 || a.n_local <= a.batch)
    throw std::runtime_error("lenet: the local shard must exceed the batch");
  image_kernel<true><<<a.batch * PARTS, NT, 0, s>>>(a);
}

void launch_image_eval(const ImageArgs& a, int rows, hipStream_t s) {
  if (rows <= 0) return;
  image_kernel<false><<<rows, NT, 0, s>>>(a);
}

void launch_update(const float* acts, const float* deltas, const float* convp, int batch,
                   const Offsets& off, float* params, float* grads, float* mom, float momentum,
                   const float* lr, long long* step, bool apply, hipStream_t s, long long dbuf) {
  const int blocks = UB_FC + UB_CONV;
  if (dbuf && (apply || !step)) throw std::runtime_error("lenet update: dbuf needs grads + step");
  if (apply)
    update_kernel<true><<<blocks, 256, 0, s>>>(acts, deltas, convp, batch, off, params, grads, mom,
                                               momentum, lr, step, 0);
  else
    update_kernel<false><<<blocks, 256, 0, s>>>(acts, deltas, convp, batch, off, params, grads,
                                                mom, momentum, lr, step, dbuf);
}

void launch_update_push(const float* acts, const float* deltas, const float* convp, int batch,
                        const Offsets& off, float* params, float* mom, float momentum,
                        const float* lr, long long* step, const PushArgs& pa, hipStream_t s) {
  const int n = pa.sync.nranks;
  if (n < 1 || n > xgmi::kMaxRanks || !pa.sync.flags || !pa.sync.epoch || !pa.sync.error ||
      pa.total <= 0 || 2LL * n * pa.total * 4 >= (1LL << 32))
    throw std::runtime_error("lenet push sync: communicator / receive buffer not set up");
  for (int r = 0; r < n; ++r)
    if (!pa.recv[r]) throw std::runtime_error("lenet push sync: receive buffer of a rank unmapped");
  update_push_kernel<<<UB_FC + UB_CONV, 256, 0, s>>>(acts, deltas, convp, batch, off, params, mom,
                                                     momentum, lr, step, pa);
}

size_t acts_floats(int batch) { return (size_t)batch * ACT_STRIDE; }
size_t deltas_floats(int batch) { return (size_t)batch * DELTA_STRIDE; }
size_t convp_floats(int batch) { return (size_t)batch * CONVP_STRIDE; }

}  // namespace lenet
