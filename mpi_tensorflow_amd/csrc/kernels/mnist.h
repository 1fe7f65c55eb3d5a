// Host launchers of the MNIST kernel set (mnist.hip) and the flat SGD kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "xgmi.h"

namespace mnist {
// world-1 FC-bucket momentum SGD run as extra blocks of a conv2 bwd-data launch
// (mnist_shared.h fc_sgd_role): flat [0, n) floats, L2 on all of it, device lr
struct FcSgdArgs {
  float* w;
  const float* g;
  float* m;
  long long n;
  float l2, momentum;
  const float* lr;
  int rounds;  // FC_SGD_UNROLL-float4 rounds per thread (sets the block count)
  // bf16 engine: also write the fc1 weight's bf16 shadows (w1 = its float offset)
  uint16_t* w1b = nullptr;
  uint16_t* w1t = nullptr;
  long long w1 = 0;
  float gscale = 1.f;  // world > 1: the grads are the rank sum (1 / ranks)
  // fp32 single rank, Winograd bwd-data launch: the fc1 weight's gradient is
  // formed in the SGD itself (dW1 = a2^T dh tiles, no g round trip; fc1
  // backward then runs without its dW1 role); w1 = the fc1 weight's offset
  const float* a2 = nullptr;
  const float* dh = nullptr;
  int batch = 0;
};
// conv1 filter-grad role appended to a conv2 filter-gradient launch (its input
// dA1m must be final: the conv2 bwd-data launch ran before)
struct C1FilterArgs {
  const float* data;
  const long long* step;
  int n_local;
  const float* da1m;
  const uint8_t* idx1;
  float* part1;
};
// out_pad (optional): zero-bordered NHWC copy [batch][18][18][32] of the pooled
// output (its border is never written: allocate it zeroed)
void launch_conv1_fwd(const float* data, const long long* step, int n_local, int batch,
                      const float* w, const float* b, float* out, uint8_t* argmax, hipStream_t s,
                      float* out_pad = nullptr);
// bf16 engine: pooled conv1 output as zero-bordered bf16 images (see mnist_bf16.h);
// with w1b != nullptr the same launch also re-derives the bf16 weight shadows
// of the fp32 fc1 (w3) / conv2 (w2) weights (mnist_shared.h shadow_block)
void launch_conv1_fwd_bf16(const float* data, const long long* step, int n_local, int batch,
                           const float* w, const float* b, uint16_t* a1p, uint16_t* a1t,
                           uint8_t* argmax, int ld_batch, hipStream_t s,
                           const float* w3 = nullptr, const float* w2 = nullptr,
                           uint16_t* w1b = nullptr, uint16_t* w1t = nullptr,
                           uint16_t* w2tb = nullptr, uint16_t* w2b = nullptr);
// Train forward of conv1 + conv2 in ONE launch (fp32): every conv2 block
// computes the pooled conv1 rows of its input halo itself (~2x recompute of the
// 25-tap conv1) and writes the rows it owns to a1 / a1pf / idx1 (the layouts
// of launch_conv1_fwd); data rows at the device-step batch offset.
struct C12In {
  const float* data = nullptr;
  const long long* step = nullptr;
  int n_local = 0;
  const float* w1 = nullptr;
  const float* b1 = nullptr;
  float* a1 = nullptr;
  float* a1pf = nullptr;
  uint8_t* idx1 = nullptr;
};
void launch_conv12_fwd(const C12In& c1, int batch, const float* w2, const float* b2, float* a2,
                       uint8_t* idx2, float* w2t, hipStream_t s);
// bf16 engine: conv1 + conv2 (+bias, ReLU, pool, argmax) in one launch; conv1
// owned rows to a1p / a1t / c1.idx1, conv2 to a2p / a2t / idx2 (mnist_bf16.h
// layouts, ld_batch = batch); w2tb = the bf16 conv2 shadow [25][2][64][16],
// already current (batch % 16 == 0)
void launch_conv12_fwd_bf16(const C12In& c1, int batch, const uint16_t* w2tb, const float* b2,
                            uint16_t* a1p, uint16_t* a1t, uint16_t* a2p, uint16_t* a2t,
                            uint8_t* idx2, hipStream_t s);
// w2t (optional): also writes the transposed weights W2T[t][co][ci] for bwd-data
void launch_conv2_fwd(const float* a1, int batch, const float* w, const float* b, float* out,
                      uint8_t* argmax, float* w2t, hipStream_t s);
// Winograd F(2x2,5x5) conv2 (wino.h): transformed filters U [36][32][64] and,
// when Ud != nullptr, Ud [36][64][32] of the rotated filter (bwd-data)
void launch_conv2_wino_weights(const float* w2, float* U, float* Ud, hipStream_t s);
// prof (labs): per-wave phase stamps [blocks][8 waves][5] (s_memtime)
// a2t (optional): a2 also feature-major [3136][batch] (launch_fc1_fwd_train_t)
void launch_conv12_fwd_wino(const C12In& c1, int batch, const float* w2, const float* U,
                            const float* b2, float* a2, uint8_t* idx2, float* w2t, hipStream_t s,
                            unsigned long long* prof = nullptr, float* a2t = nullptr);
void launch_conv2_fwd_wino(const float* a1, int batch, const float* w2, const float* U,
                           const float* b, float* out, uint8_t* argmax, float* w2t, hipStream_t s);
// Winograd bwd-data: dy2 = NHWC dY2 [B][14][14][64] (launch_fc1_bwd), Ud from
// launch_conv2_wino_weights; da1m = dA1 masked by a1 > 0
// prof (labs): per-wave phase stamps [blocks][8 waves][7] (s_memtime)
void launch_conv2_bwd_data_wino(const float* dy2, const float* Ud, const float* a1, int batch,
                                float* da1m, hipStream_t s, const FcSgdArgs* fc_sgd = nullptr,
                                const C1FilterArgs* c1 = nullptr,
                                unsigned long long* prof = nullptr);
// Both Winograd conv2 backward products in one launch: bwd-data (as
// launch_conv2_bwd_data_wino, dy2 / Ud / a1 -> da1m, + the conv1 filter-grad
// partials c1; no FC SGD) and the filter gradient (as
// launch_conv2_bwd_filter_wino without its conv1 role: a1p / dy2 -> part2)
// xfc (optional, world > 1 over xGMI): the FC bucket's exchange + SGD as the
// first blocks of this launch (mnist.h XgmiStepArgs; then launch_xgmi_step
// with fc_in_bwd for the conv parameters)
struct XgmiStepArgs;
void launch_conv2_bwd_wino(const float* Ud, const float* a1, const float* a1p, const float* dy2,
                           int batch, float* da1m, float* part2, hipStream_t s,
                           const C1FilterArgs* c1 = nullptr, const XgmiStepArgs* xfc = nullptr);
int fc1_train_splits();
void launch_fc1_fwd_train(const float* a2, const float* w, int batch, float* part, hipStream_t s);
// fc1 train forward over the feature-major a2t [3136][batch] (batch % 32 ==
// 0): fc1_train_t_splits() slabs, no LDS staging (mnist.hip fc1_fwd_t_kernel)
int fc1_train_t_splits();
void launch_fc1_fwd_train_t(const float* a2t, const float* w, int batch, float* part,
                            hipStream_t s);
void launch_fc1_fwd_eval(const float* a2, const float* w, const float* b, int M, float* h,
                         uint32_t key, float keep_prob, hipStream_t s);
void launch_fc_head_train(const float* part, const float* b3, const float* w4, const float* b4,
                          const int* labels, int n_local, const long long* step, int batch,
                          float keep_prob, uint32_t seed, uint32_t rank, float base_lr,
                          float lr_decay, float* hd, float* dh, float* dlog, float* loss_rows,
                          float* lr_out, int* correct, hipStream_t s, uint16_t* dh16 = nullptr,
                          uint16_t* dht16 = nullptr, int splits = 14);  // slabs in part
void launch_fc_head_eval(const float* h, const float* w4, const float* b4, const int* labels,
                         int M, float* logits, int* errors, hipStream_t s);
// dY2 as NHWC dy2 [B][14][14][64] and (dy2t != nullptr: the direct
// bwd-data's operand) channel-major zero-bordered dy2t [B][64][18][MNIST32_T_LD]
void launch_fc1_bwd(const float* a2, const uint8_t* idx2, const float* dh, const float* hd,
                    const float* dlog, const float* w1, int batch, float* g_w3, float* g_b3,
                    float* g_w4, float* g_b4, float* dy2, float* dy2t, hipStream_t s,
                    int roles = 7);  // roles: bit 0 dX, bit 1 dW1, bit 2 small grads
                                     // (roles == 1: a dX-only grid, SCHED_FACTORS)
// FC weight / bias grads over `rows` gathered rows (rank-major a2 [rows][3136],
// dh / hd [rows][512], dlog [rows][10]); SCHED_FACTORS
void launch_fc1_bwd_weights(const float* a2, const float* dh, const float* hd, const float* dlog,
                            int rows, float* g_w3, float* g_b3, float* g_w4, float* g_b4,
                            hipStream_t s);
int conv2_filter_splits(int batch);
// a1p: the zero-bordered NHWC pooled conv1 output [batch][18][18][32]
void launch_conv2_bwd_filter(const float* a1p, const float* dy2, int batch, float* part2,
                             hipStream_t s, const C1FilterArgs* c1 = nullptr);
// Winograd conv2 filter gradient: tap slabs part2 [groups of 2 images][800][64]
// + db2 partials [4 groups][64], the layout of launch_conv2_bwd_filter with
// conv2_wino_filter_groups(B) groups.  c1: the conv1 filter grad as
// whole-image role blocks (conv1_filter_blocks(B, 1) partial rows).
int conv2_wino_filter_groups(int batch);
size_t part2_floats_wino(int batch);
void launch_conv2_bwd_filter_wino(const float* a1p, const float* dy2, int batch, float* part2,
                                  hipStream_t s, const C1FilterArgs* c1 = nullptr);
// phase timing of the above (s_memtime per wave, [blocks][waves][5]); labs only
void launch_conv2_bwd_filter_wino_prof(const float* a1p, const float* dy2, int batch,
                                       float* part2, unsigned long long* prof, hipStream_t s);
// L2-direct bwd-data (the one the executor uses): dy2t from launch_fc1_bwd,
// w2t from launch_conv2_fwd; batch % 8 == 0
void launch_conv2_bwd_data_l2(const float* dy2t, const float* w2t, const float* a1, int batch,
                              float* da1m, hipStream_t s, const FcSgdArgs* fc_sgd = nullptr);


// conv1 filter-grad units: batch * split (split 7: pooled-row pairs, the
// default; 4: the Winograd bwd-data blocks' bands of 4 a1 rows; 1: whole
// images)
int conv1_filter_blocks(int batch, int split = 7);
// labs: 6 clock stamps per block of launch_xgmi_step into p (null: off)
void set_xgmi_step_prof(unsigned long long* p);
// labs: per-block [start, end] 100 MHz clock stamps of launch_conv2_bwd_wino into
// p (2 x blocks u64; null turns them off)
void set_conv2_bwd_wino_prof(unsigned long long* p);
void launch_conv1_bwd_filter(const float* data, const long long* step, int n_local, int batch,
                             const float* da1m, const uint8_t* idx1, float* part1, hipStream_t s);
void launch_grad_finalize(const float* part2, int ngroups, const float* part1, int nblk1,
                          float* g_w2, float* g_b2, float* g_w1, float* g_b1, hipStream_t s);
// The SGD launch that ends a train step (mnist.hip sgd_finalize_kernel):
// momentum SGD of the FC bucket [0, fc_end) (optional; L2 on all of it) and
// of the conv parameters (optional), whose grads are either summed from the
// filter-gradient slabs (world 1: part2 / part1 set) or read from the flat
// buffer (world > 1, after their all-reduce: part2 == nullptr).  Grads are
// scaled by gscale (1 / ranks).  It also writes what the next step reads of
// the updated weights: the Winograd transforms (wino_u / wino_ud), the bf16
// conv2 shadows (w2tb / w2b) and, with the FC bucket, the bf16 fc1 shadows
// (w1b / w1t; off_w1fc = the fc1 weight's float offset).  step: bumped once.
struct SgdStepArgs {
  float* w = nullptr;
  const float* g = nullptr;
  float* mom = nullptr;
  float l2 = 0.f, momentum = 0.f, gscale = 1.f;
  const float* lr = nullptr;
  long long* step = nullptr;
  long long fc_end = 0;
  int fc_rounds = 2;
  uint16_t* w1b = nullptr;
  uint16_t* w1t = nullptr;
  long long off_w1fc = 0;
  // fused fc1 weight gradient in the FC role (FcSgdArgs::a2; single rank)
  const float* a2 = nullptr;
  const float* dh = nullptr;
  int batch = 0;
  bool conv = true;
  int off_w2 = 0, off_b2 = 0, off_w1 = 0, off_b1 = 0;
  const float* part2 = nullptr;
  int ngroups = 0;
  const float* part1 = nullptr;
  int nblk1 = 0;
  float* wino_u = nullptr;
  float* wino_ud = nullptr;
  uint16_t* w2tb = nullptr;
  uint16_t* w2b = nullptr;
};
void launch_sgd_step(const SgdStepArgs& a, hipStream_t s);
// lab: per-block [start, end] clock pairs of later SGD launches (nullptr: off)
void set_sgd_prof(unsigned long long* p);
// World > 1 over the xGMI peer-to-peer communicator (MnistExecutor SCHED_XGMI,
// mnist.hip xgmi_step_kernel): ONE launch on the compute stream does the whole
// gradient sync and the update.
//  * FC bucket [0, 4 * fc4): rank r sums float4s of segment r (fc4 / N of
//    them) over every rank's grads (rank order), applies the momentum SGD to
//    its own params / momentum there (sharded optimizer state), and after a
//    barrier copies the other segments' updated params from their owners;
//  * conv parameters: every rank first writes its own slab sums (the
//    grad_finalize forms) into its grads, then - after the arrival barrier -
//    sums every rank's conv grads in rank order and updates the conv
//    parameters itself (replicated; they are 3 % of the bytes), writing the
//    next step's Winograd transforms (the bf16 engine re-derives its shadows
//    in the next step's conv1 launch: fresh = false);
//  * bumps the device step.
// g[r] / w[r]: rank r's flat grads / params as mapped here (XgmiComm).
// Same sums and SGD forms as the buckets schedule over a rank-order
// all-reduce, so the replicas stay bit-identical.
struct XgmiStepArgs {
  xgmi::Sync sync;
  const float* g[xgmi::kMaxRanks] = {};
  float* w[xgmi::kMaxRanks] = {};
  float* mom = nullptr;
  long long fc4 = 0;  // FC bucket float4s (a multiple of the rank count)
  float l2 = 0.f, momentum = 0.f, gscale = 1.f;
  const float* lr = nullptr;
  long long* step = nullptr;
  int off_w2 = 0, off_b2 = 0, off_w1 = 0, off_b1 = 0;
  const float* part2 = nullptr;
  int ngroups = 0;
  const float* part1 = nullptr;
  int nblk1 = 0;
  float* wino_u = nullptr;
  float* wino_ud = nullptr;
  // the FC bucket already went through the conv2 backward launch's role
  // blocks (launch_conv2_bwd_wino with these args): the step does the conv part
  int fc_in_bwd = 0;
  // set by the launchers (xgmi_fc_plan)
  long long seg4 = 0;
  int per4 = 0, nfc = 0, ncv = 0, ngather = 0;
  // every rank's conv-grad exchange buffer (2 x cstride floats, by epoch
  // parity; xgmi_conv_floats), or null: the conv grads go through the grads
  // buffer and the conv blocks keep the closing "done reading" barrier
  float* xc[xgmi::kMaxRanks] = {};
  long long cstride = 0;
  // SCHED_XGMI_FAC: the FC grads are already the global sums (formed from the
  // gathered factors, launch_xgmi_fac_gather + launch_fc1_bwd_weights): the FC
  // blocks apply the momentum SGD to the whole bucket locally - no FC exchange,
  // no FC barrier, replicated FC momentum
  int fc_local = 0;
  // fc_local: the FC factors of every rank (rank-major, frows = N x B rows):
  // the fc1 weight's gradient tiles are formed and applied in the step launch
  // (fc1_dw_sgd, K = frows); the small FC grads come from launch_fc1_small_grads
  const float* fa2 = nullptr;
  const float* fdh = nullptr;
  int frows = 0, off_w3 = 0;
  // labs: per block 6 clock stamps (100 MHz) of xgmi_step_kernel, or null
  unsigned long long* prof = nullptr;
};
void launch_xgmi_step(const XgmiStepArgs& a, hipStream_t s);
// SCHED_XGMI_FAC factor gather: nbuf rank-major gathered buffers (slot r =
// rank r's rows, slot4[k] float4s a slot); every rank copies each peer's own
// slot out of that peer's buffer (buf[k][r]: rank r's buffer k) over its link,
// after an arrival barrier (the peers' forward / head kernels wrote them)
struct XgmiFacArgs {
  xgmi::Sync sync;
  static constexpr int kBufs = 4;
  float* buf[kBufs][xgmi::kMaxRanks] = {};
  long long slot4[kBufs] = {};
};
void launch_xgmi_fac_gather(const XgmiFacArgs& a, hipStream_t s);
// fc1 backward dX (roles == 1 grid of launch_fc1_bwd) with the SCHED_XGMI_FAC
// factor gather as extra role blocks (the factors are final after the head)
void launch_fc1_bwd_dx_fac_gather(const float* a2, const uint8_t* idx2, const float* dh,
                                  const float* w1, int batch, float* dy2, float* dy2t,
                                  const XgmiFacArgs& f, hipStream_t s);
// fc2 / bias grads (dW2, db2, db1) over `rows` gathered rows (the small role of
// launch_fc1_bwd_weights alone)
void launch_fc1_small_grads(const float* dh, const float* hd, const float* dlog, int rows,
                            float* g_b3, float* g_w4, float* g_b4, hipStream_t s);
// FC role geometry for `threads`-thread blocks (<= max_blocks, rounded up to 8)
void xgmi_fc_plan(XgmiStepArgs& a, int threads, int max_blocks);
// floats of one parity half of the conv-grad exchange buffer (off_b1: the
// conv1 bias offset, the conv params being the flat buffer's prefix)
long long xgmi_conv_floats(long long off_b1);
size_t part2_floats(int batch);
size_t part1_floats(int batch);
size_t fc1_part_floats(int batch);
}  // namespace mnist

namespace optim {
// w, g, mom: flat fp32 buffers of n floats (n % 4 == 0, 16-B aligned).
// g_eff = g * gscale (+ l2 * w for i < l2_end); mom = momentum * mom + g_eff;
// w -= lr * mom.  lr is read from lr_ptr when non-null (device-computed
// schedule), else lr_const.  step_ptr (optional) is incremented once.
void launch_sgd_momentum(float* w, const float* g, float* mom, long long n, long long l2_end,
                         float l2, float momentum, float gscale, const float* lr_ptr,
                         float lr_const, long long* step_ptr, hipStream_t s);
void launch_scale(float* x, long long n, float a, hipStream_t s);
// bf16 gradient wire: bucket copies around a collective (n % 4 == 0, 16-B aligned)
void launch_to_bf16(const float* x, uint16_t* y, long long n, hipStream_t s);
void launch_from_bf16(const uint16_t* x, float* y, long long n, hipStream_t s);
// *out = replica fingerprint of n raw 32-bit words (sgd.hip hash_words_kernel)
void launch_hash_words(const uint32_t* x, long long n, unsigned long long* out, hipStream_t s);
}  // namespace optim
