#include "mnist_executor.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels/common.h"
#include "kernels/mnist.h"
#include "kernels/mnist_bf16.h"

// FC factor row widths (models/mnist_cnn.py: 7*7*64 -> 512 -> 10)
constexpr size_t kFc1In = 3136, kFc1Out = 512, kNcls = 10;

template <class T>
static inline T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}

MnistExecutor::MnistExecutor(const MnistPtrs& p) : p_(p) {
  if (p_.batch <= 0 || p_.batch % 32 != 0)
    throw std::runtime_error("MnistExecutor: batch must be a positive multiple of 32");
  if (p_.n_local <= p_.batch)
    throw std::runtime_error("MnistExecutor: local shard must exceed the batch");
  if (p_.total % 4 != 0 || p_.l2_end % 4 != 0 || p_.bucket1 % 4 != 0 || p_.l2_end > p_.bucket1)
    throw std::runtime_error(
        "MnistExecutor: flat segments must be multiples of 4 floats with the L2 prefix in bucket 1");
  // (hipEventDisableSystemFence / hipEventReleaseToDevice on these events
  // changed nothing in graph replay: captured edges do not use the flags)
  for (hipEvent_t* e : {&ev_dw_, &ev_b1_, &ev_fin_, &ev_done_, &ev_fac_})
    HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
}

MnistExecutor::~MnistExecutor() {
  for (hipEvent_t e : {ev_dw_, ev_b1_, ev_fin_, ev_done_, ev_fac_})
    if (e) (void)hipEventDestroy(e);
}

// forward + backward into the flat grad buffer, all on ONE stream: in hipGraph
// replay a same-stream kernel boundary costs ~0.1 us while every cross-stream
// event dependency was measured at 5-18 us of idle gap (rocprofv3 timeline,
// profiles/), and the two MFMA-bound conv2 backward kernels gain nothing from
// running concurrently.  Independent work is therefore merged into single
// launches instead (fc1 backward: dX + dW1 + fc2 grads in one grid).
// ev_dw_ is recorded when the FC bucket (bucket 1) of the grads is final.
void MnistExecutor::enqueue_fwd_bwd(hipStream_t s, bool finalize,
                                    const mnist::FcSgdArgs* fc_sgd, bool factors, bool fresh,
                                    bool fc1_dw_fused, const mnist::XgmiStepArgs* xfc,
                                    const mnist::XgmiFacArgs* xfac) {
  if (p_.bf16) {
    if (factors) throw std::runtime_error("MnistExecutor: SCHED_FACTORS is fp32 only");
    return enqueue_fwd_bwd_bf16(s, finalize, fc_sgd, fresh);
  }
  const MnistPtrs& p = p_;
  float* W = P<float>(p.params);
  float* G = P<float>(p.grads);
  const long long* step = P<const long long>(p.step);
  const int B = p.batch;
  // forward
  // conv1 is recomputed inside the conv2 blocks (one launch, ~3 us less than a
  // separate conv1 launch staging a1 through memory: 108.2 -> 105.0 us/step)
  mnist::C12In cf;
  cf.data = P<const float>(p.train_x);
  cf.step = step;
  cf.n_local = p.n_local;
  cf.w1 = W + p.off_w1;
  cf.b1 = W + p.off_b1;
  cf.a1 = P<float>(p.a1);
  cf.a1pf = P<float>(p.a1pf);
  cf.idx1 = P<uint8_t>(p.idx1);
  if (p.wino) {
    // transformed filters of this step's weights (forward U, bwd-data Ud);
    // the previous step's SGD launch already wrote them (fresh)
    if (!fresh)
      mnist::launch_conv2_wino_weights(W + p.off_w2, P<float>(p.wino_u), P<float>(p.wino_ud), s);
    mnist::launch_conv12_fwd_wino(cf, B, W + p.off_w2, P<const float>(p.wino_u), W + p.off_b2,
                                  P<float>(p.a2), P<uint8_t>(p.idx2), nullptr, s, nullptr,
                                  P<float>(p.a2ft));
  } else {
    mnist::launch_conv12_fwd(cf, B, W + p.off_w2, W + p.off_b2, P<float>(p.a2),
                             P<uint8_t>(p.idx2), P<float>(p.w2t), s);
  }
  wait_fc_params(s);  // sharded FC update of the previous step (all-gather in flight)
  const bool fc1_t = p.wino && p.a2ft != 0;
  if (fc1_t)
    mnist::launch_fc1_fwd_train_t(P<const float>(p.a2ft), W + p.off_w3, B, P<float>(p.fc1_part), s);
  else
    mnist::launch_fc1_fwd_train(P<const float>(p.a2), W + p.off_w3, B, P<float>(p.fc1_part), s);
  mnist::launch_fc_head_train(P<const float>(p.fc1_part), W + p.off_b3, W + p.off_w4,
                              W + p.off_b4, P<const int>(p.train_y), p.n_local, step, B,
                              p.keep_prob, p.seed, p.rank, p.base_lr, p.lr_decay, P<float>(p.hd),
                              P<float>(p.dh), P<float>(p.dlog), P<float>(p.loss_rows),
                              P<float>(p.lr), P<int>(p.correct), s, nullptr, nullptr,
                              fc1_t ? mnist::fc1_train_t_splits() : mnist::fc1_train_splits());
  if (factors && sched_ == SCHED_FACTORS) HIP_CHECK(hipEventRecord(ev_fac_, s));
  // backward: fc1 dX (+pool2/ReLU2 scatter) | dW1 | fc2 grads, one launch
  // (SCHED_XGMI_FAC: dX | the peers' factor rows over the links)
  if (xfac)
    mnist::launch_fc1_bwd_dx_fac_gather(P<const float>(p.a2), P<const uint8_t>(p.idx2),
                                        P<const float>(p.dh), W + p.off_w3, B, P<float>(p.dy2),
                                        p.wino ? nullptr : P<float>(p.dy2t), *xfac, s);
  else
    mnist::launch_fc1_bwd(P<const float>(p.a2), P<const uint8_t>(p.idx2), P<const float>(p.dh),
                          P<const float>(p.hd), P<const float>(p.dlog), W + p.off_w3, B,
                          G + p.off_w3, G + p.off_b3, G + p.off_w4, G + p.off_b4,
                          P<float>(p.dy2), p.wino ? nullptr : P<float>(p.dy2t), s,
                          factors ? 1 : (fc1_dw_fused ? 5 : 7));
  HIP_CHECK(hipEventRecord(ev_dw_, s));
  // conv1 filter grad: Winograd - in the bwd-data blocks' epilogue, from the
  // dA1 values they produce; direct - role blocks of the filter-grad launch
  const mnist::C1FilterArgs c1{P<const float>(p.train_x), step, p.n_local,
                               P<const float>(p.da1m), P<const uint8_t>(p.idx1),
                               P<float>(p.part1)};
  if (p.wino && fc_sgd == nullptr) {  // bwd-data (+ conv1 filter grad) and filter grad: one launch
    mnist::launch_conv2_bwd_wino(P<const float>(p.wino_ud), P<const float>(p.a1),
                                 P<const float>(p.a1pf), P<const float>(p.dy2), B,
                                 P<float>(p.da1m), P<float>(p.part2), s, &c1, xfc);
  } else if (p.wino) {  // the FC SGD rides in the bwd-data launch
    mnist::launch_conv2_bwd_data_wino(P<const float>(p.dy2), P<const float>(p.wino_ud),
                                      P<const float>(p.a1), B, P<float>(p.da1m), s, fc_sgd, &c1);
    mnist::launch_conv2_bwd_filter_wino(P<const float>(p.a1pf), P<const float>(p.dy2), B,
                                        P<float>(p.part2), s);
  } else {
    mnist::launch_conv2_bwd_data_l2(P<const float>(p.dy2t), P<const float>(p.w2t),
                                    P<const float>(p.a1), B, P<float>(p.da1m), s, fc_sgd);
    mnist::launch_conv2_bwd_filter(P<const float>(p.a1pf), P<const float>(p.dy2), B,
                                   P<float>(p.part2), s, &c1);
  }
  if (finalize)
    mnist::launch_grad_finalize(P<const float>(p.part2), conv2_groups(), P<const float>(p.part1),
                                conv1_blocks(), G + p.off_w2, G + p.off_b2, G + p.off_w1,
                                G + p.off_b1, s);
}

// bf16 step: same kernel boundaries; the first launch re-derives the bf16
// weight shadows from the fp32 master weights, conv1 (K = 25, tiny) stays on
// fp32 MFMA and writes bf16 images, the conv1 filter grad / fc2 head / slab
// reductions / SGD stay fp32.
void MnistExecutor::enqueue_fwd_bwd_bf16(hipStream_t s, bool finalize,
                                         const mnist::FcSgdArgs* fc_sgd, bool shadows_fresh) {
  const MnistPtrs& p = p_;
  float* W = P<float>(p.params);
  float* G = P<float>(p.grads);
  const long long* step = P<const long long>(p.step);
  const int B = p.batch;
  using U16 = uint16_t;
  if (shadows_fresh && B % 16 == 0) {
    // every shadow is current (the previous step's SGD launch, or
    // refresh_shadows), so conv1 runs inside the conv2 blocks (one launch);
    // the FC weights are first read by fc1 forward
    mnist::C12In cf;
    cf.data = P<const float>(p.train_x);
    cf.step = step;
    cf.n_local = p.n_local;
    cf.w1 = W + p.off_w1;
    cf.b1 = W + p.off_b1;
    cf.idx1 = P<uint8_t>(p.idx1);
    mnist::launch_conv12_fwd_bf16(cf, B, P<const U16>(p.w2tb), W + p.off_b2, P<U16>(p.a1p),
                                  P<U16>(p.a1t), P<U16>(p.a2h), P<U16>(p.a2t), P<uint8_t>(p.idx2),
                                  s);
    wait_fc_params(s);  // sharded FC update of the previous step (all-gather in flight)
  } else {
    // the conv1 launch re-derives the bf16 weight shadows (block role) from the
    // fp32 master weights, the FC ones included: wait for those first
    wait_fc_params(s);
    const bool w1_done = fc_sgd != nullptr && fc_sgd->w1b != nullptr;
    mnist::launch_conv1_fwd_bf16(P<const float>(p.train_x), step, p.n_local, B, W + p.off_w1,
                                 W + p.off_b1, P<U16>(p.a1p), P<U16>(p.a1t), P<uint8_t>(p.idx1),
                                 B, s, W + p.off_w3, W + p.off_w2,
                                 w1_done ? nullptr : P<U16>(p.w1b), P<U16>(p.w1t), P<U16>(p.w2tb),
                                 P<U16>(p.w2b));
    mnist16::launch_conv2_fwd(P<const U16>(p.a1p), B, P<const U16>(p.w2tb), W + p.off_b2,
                              P<U16>(p.a2h), P<U16>(p.a2t), P<uint8_t>(p.idx2), s);
  }
  mnist16::launch_fc1_fwd_train(P<const U16>(p.a2h), P<const U16>(p.w1t), B, P<float>(p.fc1_part),
                                s);
  mnist::launch_fc_head_train(P<const float>(p.fc1_part), W + p.off_b3, W + p.off_w4,
                              W + p.off_b4, P<const int>(p.train_y), p.n_local, step, B,
                              p.keep_prob, p.seed, p.rank, p.base_lr, p.lr_decay, P<float>(p.hd),
                              P<float>(p.dh), P<float>(p.dlog), P<float>(p.loss_rows),
                              P<float>(p.lr), P<int>(p.correct), s, P<U16>(p.dh16),
                              P<U16>(p.dht16));
  mnist16::launch_fc1_bwd(P<const U16>(p.a2h), P<const U16>(p.a2t), P<const uint8_t>(p.idx2),
                          P<const U16>(p.dh16), P<const U16>(p.dht16), P<const float>(p.hd),
                          P<const float>(p.dh), P<const float>(p.dlog), P<const U16>(p.w1b), B,
                          G + p.off_w3, G + p.off_b3, G + p.off_w4, G + p.off_b4, P<U16>(p.dy2p),
                          P<U16>(p.dy2t), s);
  HIP_CHECK(hipEventRecord(ev_dw_, s));
  // conv2 bwd-data (+ conv1 filter grad) | conv2 filter grad | FC SGD: one launch
  const mnist::C1FilterArgs c1{P<const float>(p.train_x), step, p.n_local,
                               P<const float>(p.da1m), P<const uint8_t>(p.idx1),
                               P<float>(p.part1)};
  static const bool lab_split = [] {  // lab (MTA_C2B_LAB=3): the two-launch form
    const char* e = getenv("MTA_C2B_LAB");
    return e && atoi(e) == 3;
  }();
  if (lab_split) {
    mnist16::launch_conv2_bwd_data(P<const U16>(p.dy2p), P<const U16>(p.w2b), P<const U16>(p.a1p),
                                   B, P<float>(p.da1m), s, fc_sgd);
    mnist16::launch_conv2_bwd_filter(P<const U16>(p.a1t), P<const U16>(p.dy2t), B,
                                     P<float>(p.part2), s, &c1);
  } else {
    mnist16::launch_conv2_bwd(P<const U16>(p.dy2p), P<const U16>(p.w2b), P<const U16>(p.a1p),
                              P<const U16>(p.a1t), P<const U16>(p.dy2t), B, P<float>(p.da1m),
                              P<float>(p.part2), s, fc_sgd, &c1);
  }
  if (finalize)
    mnist::launch_grad_finalize(P<const float>(p.part2), mnist16::conv2_filter_groups(B),
                                P<const float>(p.part1), conv1_blocks(),
                                G + p.off_w2, G + p.off_b2, G + p.off_w1, G + p.off_b1, s);
}

int MnistExecutor::conv2_groups() const {
  if (p_.bf16) return mnist16::conv2_filter_groups(p_.batch);
  return p_.wino ? mnist::conv2_wino_filter_groups(p_.batch)
                 : mnist::conv2_filter_splits(p_.batch);
}

// the Winograd bwd-data blocks produce one conv1 partial per band of 4 a1 rows,
// the bf16 merged conv2 backward one per 128 pooled pixels
int MnistExecutor::conv1_blocks() const {
  if (p_.bf16) {
    const char* e = getenv("MTA_C2B_LAB");
    if (e && atoi(e) == 3) return mnist::conv1_filter_blocks(p_.batch, 7);
    return mnist16::conv2_bwd_conv1_rows(p_.batch);
  }
  return mnist::conv1_filter_blocks(p_.batch, p_.wino ? 4 : 7);
}

void MnistExecutor::forward_backward(hipStream_t s) {
  wait_fc_params(s);
  enqueue_fwd_bwd(s);
}

void MnistExecutor::sgd(hipStream_t s, float gscale) {
  wait_fc_params(s);
  sgd_range(s, 0, p_.total, gscale, true);
}

// momentum SGD over flat floats [lo, hi) (lo, hi multiples of 4); the L2
// prefix [0, l2_end) is clipped to the range; bump_step increments the
// device step once (the last segment of a step)
void MnistExecutor::sgd_range(hipStream_t s, long long lo, long long hi, float gscale,
                              bool bump_step) {
  const MnistPtrs& p = p_;
  const long long l2 = p.l2_end > lo ? (p.l2_end < hi ? p.l2_end : hi) - lo : 0;
  optim::launch_sgd_momentum(P<float>(p.params) + lo, P<const float>(p.grads) + lo,
                             P<float>(p.mom) + lo, hi - lo, l2, p.l2, p.momentum, gscale,
                             P<const float>(p.lr), 0.f,
                             bump_step ? P<long long>(p.step) : nullptr, s);
}

// The fused SGD launch (kernels/mnist.h launch_sgd_step) over the flat grads
// at world > 1 (rank sums, x gscale): fc - the FC bucket, conv - the conv
// parameters (then it also bumps the step).  It writes the derived weights of
// what it updates - Winograd transforms, bf16 conv2 shadows, with the FC
// bucket the bf16 fc1 shadows - so the next step's forward takes them as
// current instead of re-deriving them in a launch of its own.
void MnistExecutor::sgd_step(hipStream_t s, float gscale, bool fc, bool conv,
                             long long fc_end) {
  const MnistPtrs& p = p_;
  mnist::SgdStepArgs a;
  a.w = P<float>(p.params);
  a.g = P<const float>(p.grads);
  a.mom = P<float>(p.mom);
  a.l2 = p.l2;
  a.momentum = p.momentum;
  a.gscale = gscale;
  a.lr = P<const float>(p.lr);
  a.step = conv ? P<long long>(p.step) : nullptr;
  if (fc) {
    a.fc_end = fc_end >= 0 ? fc_end : p.bucket1;
    a.fc_rounds = 1;  // a launch of its own: twice the blocks of the in-launch role
    if (p.bf16) {
      a.w1b = P<uint16_t>(p.w1b);
      a.w1t = P<uint16_t>(p.w1t);
      a.off_w1fc = p.off_w3;
    }
  }
  a.conv = conv;
  a.off_w2 = (int)p.off_w2;
  a.off_b2 = (int)p.off_b2;
  a.off_w1 = (int)p.off_w1;
  a.off_b1 = (int)p.off_b1;
  if (conv && p.wino) {
    a.wino_u = P<float>(p.wino_u);
    a.wino_ud = P<float>(p.wino_ud);
  }
  if (conv && p.bf16) {
    a.w2tb = P<uint16_t>(p.w2tb);
    a.w2b = P<uint16_t>(p.w2b);
  }
  mnist::launch_sgd_step(a, s);
}

void MnistExecutor::reduce_bucket(Collective* comm, long long lo, long long n, hipStream_t cs) {
  float* G = P<float>(p_.grads) + lo;
  if (!p_.grad_bf16) {
    comm->all_reduce(G, G, (size_t)n, ncclFloat32, ncclSum, cs);
    return;
  }
  uint16_t* B = P<uint16_t>(p_.gb16) + lo;
  optim::launch_to_bf16(G, B, n, cs);
  comm->all_reduce(B, B, (size_t)n, ncclBfloat16, ncclSum, cs);
  optim::launch_from_bf16(B, G, n, cs);
}

void MnistExecutor::refresh_shadows(hipStream_t s) {
  shadows_stale_ = false;
  if (p_.wino) {
    const float* W = P<const float>(p_.params);
    mnist::launch_conv2_wino_weights(W + p_.off_w2, P<float>(p_.wino_u), P<float>(p_.wino_ud), s);
  }
  if (!p_.bf16) return;
  const float* W = P<const float>(p_.params);
  mnist16::launch_shadows(W + p_.off_w3, W + p_.off_w2, P<uint16_t>(p_.w1b), P<uint16_t>(p_.w1t),
                          P<uint16_t>(p_.w2tb), P<uint16_t>(p_.w2b), s);
}

void MnistExecutor::set_schedule(int sched) {
  if (sched != SCHED_BUCKETS && sched != SCHED_SHARDED_FC && sched != SCHED_SPLIT &&
      sched != SCHED_FACTORS && sched != SCHED_SERIAL && sched != SCHED_DEFER &&
      sched != SCHED_XGMI && sched != SCHED_XGMI_STEP && sched != SCHED_XGMI_FAC)
    throw std::runtime_error("MnistExecutor: unknown sync schedule");
  if (fc_pending_)
    throw std::runtime_error("MnistExecutor: join() the stream before changing the schedule");
  sched_ = sched;
}

// bf16: the sharded schedule's FC shard update leaves the fc1 bf16 shadows
// (w1b / w1t) one update behind (its next step re-derives them in the conv1
// launch, fresh = false); a step of any other schedule that would take the
// shadows as current re-derives them first instead (fresh = false once).
bool MnistExecutor::take_fresh(bool want) {
  const bool stale = shadows_stale_;
  shadows_stale_ = false;
  return want && !stale;
}

bool MnistExecutor::sharded_ok(int nranks) const {
  return nranks > 1 && p_.bucket1 % (4LL * nranks) == 0;
}

bool MnistExecutor::factors_ok(int nranks) const {
  return nranks > 1 && nranks == p_.fac_ranks && !p_.bf16 && p_.a2_all && p_.dh_all &&
         p_.hd_all && p_.dlog_all;
}

bool MnistExecutor::defer_ok() const { return !p_.bf16 && fused_sgd_ok(); }

bool MnistExecutor::xgmi_ok() const {
  if (xgmi_ == nullptr || !xgmi_->ready() || !fused_sgd_ok()) return false;
  const int n = xgmi_->size();
  const size_t fb = (size_t)p_.total * sizeof(float);
  return p_.bucket1 % (4LL * n) == 0 && xgmi_->registered(P<const void>(p_.grads), fb) &&
         xgmi_->registered(P<const void>(p_.params), fb);
}

// the factor schedule over xGMI: fp32 Winograd, the rank-major factor
// buffers sized for this communicator and mapped on every rank
bool MnistExecutor::xgmi_fac_ok() const {
  if (!xgmi_ok() || p_.bf16 || !p_.wino) return false;
  const int n = xgmi_->size();
  if (n < 2 || n != p_.fac_ranks || !p_.a2_all || !p_.dh_all || !p_.hd_all || !p_.dlog_all)
    return false;
  const size_t B = (size_t)p_.batch;
  return xgmi_->registered(P<const void>(p_.a2_all), n * B * kFc1In * sizeof(float)) &&
         xgmi_->registered(P<const void>(p_.dh_all), n * B * kFc1Out * sizeof(float)) &&
         xgmi_->registered(P<const void>(p_.hd_all), n * B * kFc1Out * sizeof(float)) &&
         xgmi_->registered(P<const void>(p_.dlog_all), n * B * kNcls * sizeof(float));
}

void MnistExecutor::set_defer_split(float f) {
  if (!(f > 0.f && f < 1.f)) throw std::runtime_error("MnistExecutor: defer split must be in (0, 1)");
  defer_split_ = f;
}

void MnistExecutor::wait_fc_params(hipStream_t s) {
  if (fc_pending_) {
    HIP_CHECK(hipStreamWaitEvent(s, ev_b1_, 0));
    fc_pending_ = false;
  }
}

void MnistExecutor::join(hipStream_t s) { wait_fc_params(s); }

bool MnistExecutor::fused_sgd_ok() const { return p_.l2_end == p_.bucket1; }

void MnistExecutor::train_step(hipStream_t s, Collective* comm, hipStream_t cs,
                               Collective* comm2) {
  if ((sched_ == SCHED_XGMI || sched_ == SCHED_XGMI_STEP) && xgmi_ok()) {  // no comm stream
    train_step_xgmi(s);
    return;
  }
  if (sched_ == SCHED_XGMI_FAC && xgmi_fac_ok()) {
    train_step_xgmi_fac(s);
    return;
  }
  if (comm == nullptr) {  // single rank (or caller-driven parameter averaging)
    const MnistPtrs& p = p_;
    wait_fc_params(s);
    if (!fused_sgd_ok()) {  // (not the reference layout) plain launches
      enqueue_fwd_bwd(s);
      sgd_range(s, 0, p.total, 1.f, true);
      return;
    }
    // the FC bucket's SGD rides in the conv2 bwd-data launch (its grads are final
    // after fc1 backward); the slab sums + conv SGD run in the last launch
    mnist::FcSgdArgs fc{P<float>(p.params), P<const float>(p.grads), P<float>(p.mom),
                        p.bucket1, p.l2, p.momentum, P<const float>(p.lr),
                        fc_sgd_rounds_ >= 0 ? fc_sgd_rounds_ : (p.bf16 ? 2 : 0)};
    if (p.bf16) {  // the SGD also writes the fc1 bf16 shadows (see refresh_shadows)
      fc.w1b = P<uint16_t>(p.w1b);
      fc.w1t = P<uint16_t>(p.w1t);
      fc.w1 = p.off_w3;
    }
    // fp32 Winograd: dW1 is formed inside the FC SGD (fc1 backward skips it)
    const bool fuse_dw1 = p.wino && !p.bf16;
    if (fuse_dw1) {
      fc.a2 = P<const float>(p.a2);
      fc.dh = P<const float>(p.dh);
      fc.batch = p.batch;
      fc.w1 = p.off_w3;
    }
    const bool role = fc.rounds > 0;
    // the derived weights (Winograd transforms, bf16 shadows) come from the
    // previous step's SGD (or refresh_shadows() before the first step of a
    // run) and are rewritten by this step's SGD for the next one
    enqueue_fwd_bwd(s, /*finalize=*/false, role ? &fc : nullptr, false, take_fresh(true), fuse_dw1);
    mnist::SgdStepArgs a;
    a.w = P<float>(p.params);
    a.g = P<const float>(p.grads);
    a.mom = P<float>(p.mom);
    a.l2 = p.l2;
    a.momentum = p.momentum;
    a.lr = P<const float>(p.lr);
    a.step = P<long long>(p.step);
    if (!role) {  // the FC bucket in this launch (fc_sgd_rounds 0)
      a.fc_end = p.bucket1;
      a.w1b = fc.w1b;
      a.w1t = fc.w1t;
      a.off_w1fc = fc.w1;
      a.a2 = fc.a2;
      a.dh = fc.dh;
      a.batch = fc.batch;
    }
    a.off_w2 = (int)p.off_w2;
    a.off_b2 = (int)p.off_b2;
    a.off_w1 = (int)p.off_w1;
    a.off_b1 = (int)p.off_b1;
    a.part2 = P<const float>(p.part2);
    a.ngroups = conv2_groups();
    a.part1 = P<const float>(p.part1);
    a.nblk1 = conv1_blocks();
    if (p.wino) {
      a.wino_u = P<float>(p.wino_u);
      a.wino_ud = P<float>(p.wino_ud);
    }
    if (p.bf16) {
      a.w2tb = P<uint16_t>(p.w2tb);
      a.w2b = P<uint16_t>(p.w2b);
    }
    mnist::launch_sgd_step(a, s);
    return;
  }
  if (sched_ == SCHED_SHARDED_FC && sharded_ok(comm->size())) {
    train_step_sharded(s, comm, cs);
    return;
  }
  if (sched_ == SCHED_SERIAL) {
    train_step_serial(s, comm);
    return;
  }
  if (sched_ == SCHED_DEFER && defer_ok()) {
    train_step_defer(s, comm, cs);
    return;
  }
  if (sched_ == SCHED_FACTORS && factors_ok(comm->size())) {
    train_step_factors(s, comm, cs);
    return;
  }
  if (sched_ == SCHED_SPLIT && comm2 != nullptr && comm2->size() == comm->size()) {
    train_step_split(s, comm, cs, comm2);
    return;
  }
  const MnistPtrs& p = p_;
  const bool fused = fused_sgd_ok();
  // fused: this step's single SGD launch writes the next step's derived
  // weights, so the forward reads them as they are (one launch fewer)
  enqueue_fwd_bwd(s, true, nullptr, false, take_fresh(fused));
  // size-1 comms are allowed (they exercise the capture path on one GPU)
  const float gscale = 1.0f / (float)comm->size();
  // bucket 1 (FC grads, 97 % of the bytes) as soon as fc1 backward is done;
  // it overlaps the conv backward still running on the compute stream
  HIP_CHECK(hipStreamWaitEvent(cs, ev_dw_, 0));
  reduce_bucket(comm, 0, p.bucket1, cs);
  HIP_CHECK(hipEventRecord(ev_b1_, cs));
  // bucket 2 (conv grads) after the slab reduction, same ordered stream
  HIP_CHECK(hipEventRecord(ev_fin_, s));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fin_, 0));
  reduce_bucket(comm, p.bucket1, p.total - p.bucket1, cs);
  HIP_CHECK(hipEventRecord(ev_done_, cs));
  if (fused) {
    // ONE join: bucket 2 completes after bucket 1 on the ordered comm stream,
    // and one SGD launch updates every parameter (a cross-queue wait costs
    // ~10 us of idle queue in graph replay whether or not its event is done)
    HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
    sgd_step(s, gscale, true, true);
    return;
  }
  // FC update while bucket 2 is in flight, then the conv update
  HIP_CHECK(hipStreamWaitEvent(s, ev_b1_, 0));
  sgd_range(s, 0, p.bucket1, gscale, false);
  HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
  sgd_range(s, p.bucket1, p.total, gscale, true);
}

// Sharded FC update (ZeRO-1 style for bucket 1).  Comm stream, per step:
//   reduce-scatter(FC grads) -> momentum SGD of this rank's 1/N shard ->
//   [conv grads final] all-reduce(conv grads) -> all-gather(FC params)
// Compute stream: conv SGD after the conv all-reduce, then the NEXT step's
// conv forward runs while the FC all-gather is still in flight; only its fc1
// forward waits for the gathered FC params (wait_fc_params).  Same bytes on
// the wire as the all-reduce (RS + AG is how the ring all-reduce moves them),
// but the FC momentum / SGD traffic drops by N and the all-gather half of the
// FC collective overlaps the next forward instead of extending this step.
// The FC momentum is sharded: gather_optimizer_state() before reading it.
// bf16: the shard update cannot write the fc1 shadows (64 x 64 tiles), so the
// next step's conv1 launch re-derives the shadows (fresh = false).
void MnistExecutor::train_step_sharded(hipStream_t s, Collective* comm, hipStream_t cs) {
  const MnistPtrs& p = p_;
  float* G = P<float>(p.grads);
  float* W = P<float>(p.params);
  const int n = comm->size();
  const float gscale = 1.0f / (float)n;
  const long long chunk = p.bucket1 / n, lo = chunk * comm->rank();
  const bool fused = fused_sgd_ok();
  enqueue_fwd_bwd(s, true, nullptr, false, take_fresh(fused && !p.bf16));
  if (p.bf16) shadows_stale_ = true;  // the FC shard update writes no fc1 shadows
  HIP_CHECK(hipStreamWaitEvent(cs, ev_dw_, 0));
  if (p.grad_bf16) {  // bf16 wire: the shard comes back to fp32 before its SGD
    uint16_t* Gb = P<uint16_t>(p.gb16);
    optim::launch_to_bf16(G, Gb, p.bucket1, cs);
    comm->reduce_scatter(Gb, Gb + lo, (size_t)chunk, ncclBfloat16, ncclSum, cs);
    optim::launch_from_bf16(Gb + lo, G + lo, chunk, cs);
  } else {
    comm->reduce_scatter(G, G + lo, (size_t)chunk, ncclFloat32, ncclSum, cs);
  }
  sgd_range(cs, lo, lo + chunk, gscale, false);
  HIP_CHECK(hipEventRecord(ev_fin_, s));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fin_, 0));
  reduce_bucket(comm, p.bucket1, p.total - p.bucket1, cs);
  HIP_CHECK(hipEventRecord(ev_done_, cs));
  comm->all_gather(W + lo, W, (size_t)chunk, ncclFloat32, cs);
  HIP_CHECK(hipEventRecord(ev_b1_, cs));
  fc_pending_ = true;
  HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
  if (fused)
    sgd_step(s, gscale, false, true);
  else
    sgd_range(s, p.bucket1, p.total, gscale, true);
}

// Split schedule: ONE fork and ONE join per step.  The FC all-reduce and the
// FC momentum SGD run on the comm stream; the conv all-reduce (0.2 MB,
// latency-bound) runs on the compute stream itself through a second
// communicator (two ops on one communicator must not run concurrently), so it
// costs a same-queue kernel boundary instead of two cross-queue hops; the
// join sits in front of the NEXT step's fc1 forward, behind its conv forward.
void MnistExecutor::train_step_split(hipStream_t s, Collective* comm, hipStream_t cs,
                                     Collective* comm2) {
  const MnistPtrs& p = p_;
  const float gscale = 1.0f / (float)comm->size();
  const bool fused = fused_sgd_ok();
  enqueue_fwd_bwd(s, true, nullptr, false, take_fresh(fused));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_dw_, 0));
  reduce_bucket(comm, 0, p.bucket1, cs);
  if (fused)
    sgd_step(cs, gscale, true, false);  // + the bf16 fc1 shadows
  else
    sgd_range(cs, 0, p.bucket1, gscale, false);
  HIP_CHECK(hipEventRecord(ev_b1_, cs));
  fc_pending_ = true;
  // host-progress communicators block a runtime thread per exchange: every
  // rank must reach the FC exchange before the conv exchange (collective.h)
  if (comm->host_progress() || comm2->host_progress()) wait_fc_params(s);
  reduce_bucket(comm2, p.bucket1, p.total - p.bucket1, s);
  if (fused)
    sgd_step(s, gscale, false, true);
  else
    sgd_range(s, p.bucket1, p.total, gscale, true);
}

// Factor schedule (sufficient-factor exchange).  The FC gradients of a batch
// are products of per-row factors: dW1 = a2^T dh (rank B), dW2 = hd^T dlog,
// db1 = sum dh, db2 = sum dlog.  Instead of all-reducing the 6.45 MB FC
// gradient (ring: 2 (N-1)/N x 6.45 MB sent per rank), every rank all-gathers
// the factors of all ranks (B x 4170 floats = 1.07 MB per rank at B = 64;
// (N-1)/N x N x 1.07 MB sent per rank: 6x fewer bytes at N = 2, 3.4x at 4,
// 1.7x at 8) and forms the global FC gradients itself with K = N x B.  All
// ranks compute the same sums in the same order, so the replicas stay
// bit-identical.
//   compute stream: fwd, head (-> ev_fac_), fc1 dX, conv bwd, slab reduction
//                   (-> ev_fin_), wait ev_b1_ -> FC weight grads over the
//                   gathered rows, wait ev_done_ -> SGD of every parameter
//   comm stream:    wait ev_fac_ -> grouped all-gather of the factors
//                   (-> ev_b1_), wait ev_fin_ -> all-reduce conv grads
//                   (-> ev_done_)
// The gather runs under the whole conv backward; the latency-bound conv
// all-reduce runs under the FC weight-gradient GEMM.  The factor slots are
// rewritten only by the next step's forward / head, after this step's GEMM.
void MnistExecutor::train_step_factors(hipStream_t s, Collective* comm, hipStream_t cs) {
  const MnistPtrs& p = p_;
  float* G = P<float>(p.grads);
  const int n = comm->size(), r = comm->rank();
  const size_t B = (size_t)p.batch;
  const float gscale = 1.0f / (float)n;
  const bool fused = fused_sgd_ok();
  enqueue_fwd_bwd(s, /*finalize=*/true, nullptr, /*factors=*/true, take_fresh(fused));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fac_, 0));
  float* a2 = P<float>(p.a2_all);
  float* dh = P<float>(p.dh_all);
  float* hd = P<float>(p.hd_all);
  float* dl = P<float>(p.dlog_all);
  comm->group_start();
  comm->all_gather(a2 + r * B * kFc1In, a2, B * kFc1In, ncclFloat32, cs);
  comm->all_gather(dh + r * B * kFc1Out, dh, B * kFc1Out, ncclFloat32, cs);
  comm->all_gather(hd + r * B * kFc1Out, hd, B * kFc1Out, ncclFloat32, cs);
  comm->all_gather(dl + r * B * kNcls, dl, B * kNcls, ncclFloat32, cs);
  comm->group_end();
  HIP_CHECK(hipEventRecord(ev_b1_, cs));
  HIP_CHECK(hipEventRecord(ev_fin_, s));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fin_, 0));
  reduce_bucket(comm, p.bucket1, p.total - p.bucket1, cs);
  HIP_CHECK(hipEventRecord(ev_done_, cs));
  // (an FC momentum SGD applied in the GEMM epilogue instead of this SGD pass
  // measured slower with per-element update chains and neutral with all
  // loads batched first, docs/PERF_NOTES.md)
  HIP_CHECK(hipStreamWaitEvent(s, ev_b1_, 0));
  mnist::launch_fc1_bwd_weights(a2, dh, hd, dl, n * p.batch, G + p.off_w3, G + p.off_b3,
                                G + p.off_w4, G + p.off_b4, s);
  HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
  if (fused)
    sgd_step(s, gscale, true, true);
  else
    sgd_range(s, 0, p.total, gscale, true);
}

// Serial schedule: the whole step on ONE queue.  In graph replay every
// cross-queue event edge costs 5-18 us of idle queue (docs/PERF_NOTES.md)
// whether or not its event is done; the overlapped schedules pay 3 of them per
// step.  Here the collective simply runs in stream order after the slab
// reduction - one all-reduce of the whole 6.65 MB flat gradient (fp32 or the
// bf16 wire) - followed by the one SGD launch: no fork, no join, no overlap.
// It wins where the fabric makes the all-reduce shorter than the edges it
// saves (the startup autotune decides, on the real communicator).
void MnistExecutor::train_step_serial(hipStream_t s, Collective* comm) {
  const MnistPtrs& p = p_;
  const float gscale = 1.0f / (float)comm->size();
  const bool fused = fused_sgd_ok();
  wait_fc_params(s);
  enqueue_fwd_bwd(s, true, nullptr, false, take_fresh(fused));
  reduce_bucket(comm, 0, p.total, s);
  if (fused)
    sgd_step(s, gscale, true, true);
  else
    sgd_range(s, 0, p.total, gscale, true);
}

// Deferred-FC schedule (fp32, one communicator).  The FC all-reduce is cut in
// two parts; the comm stream runs, in order:
//   FC part A [0, A)          from fc1 backward, under the conv backward
//   conv bucket               once the slab reduction is done (-> ev_done_)
//   FC part B [A, bucket1)    + its momentum SGD (-> ev_b1_)
// The compute stream joins after the conv bucket and runs ONE SGD launch over
// FC part A and the conv parameters (writing the next step's Winograd
// filters); the NEXT step's conv forward then runs while part B is still in
// flight, and only its fc1 forward waits for it (wait_fc_params).  This is
// the split schedule's overlap without a second communicator: collectives of
// two RCCL communicators running at once rely on both staying resident.
// Same sums and SGD forms as buckets (bit-identical).
void MnistExecutor::train_step_defer(hipStream_t s, Collective* comm, hipStream_t cs) {
  const MnistPtrs& p = p_;
  const float gscale = 1.0f / (float)comm->size();
  const long long A = std::max(4LL, (long long)(defer_split_ * (double)p.bucket1) / 4 * 4);
  enqueue_fwd_bwd(s, true, nullptr, false, take_fresh(true));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_dw_, 0));
  reduce_bucket(comm, 0, A, cs);
  HIP_CHECK(hipEventRecord(ev_fin_, s));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fin_, 0));
  reduce_bucket(comm, p.bucket1, p.total - p.bucket1, cs);
  HIP_CHECK(hipEventRecord(ev_done_, cs));
  reduce_bucket(comm, A, p.bucket1 - A, cs);
  sgd_range(cs, A, p.bucket1, gscale, false);
  HIP_CHECK(hipEventRecord(ev_b1_, cs));
  fc_pending_ = true;
  HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
  sgd_step(s, gscale, true, true, A);
}

// xGMI peer-to-peer schedule: forward + backward as at world 1 but with the
// conv filter grads left as slabs and dW1 formed by fc1 backward, then ONE
// launch (mnist.h XgmiStepArgs) that syncs and updates everything.  The FC
// momentum is sharded (each rank keeps its own segment current):
// gather_optimizer_state() before reading it.  bf16: the FC update writes no
// fc1 shadows, so the next step re-derives them (fresh = false).
mnist::XgmiStepArgs MnistExecutor::xgmi_step_args() const {
  const MnistPtrs& p = p_;
  XgmiComm* x = xgmi_;
  const int n = x->size();
  mnist::XgmiStepArgs a;
  a.sync = x->sync();
  for (int r = 0; r < n; ++r) {
    a.g[r] = static_cast<const float*>(x->peer_ptr(P<const void>(p.grads), r));
    a.w[r] = static_cast<float*>(x->peer_ptr(P<const void>(p.params), r));
  }
  const long long cf = mnist::xgmi_conv_floats(p.off_b1);
  if (xconv_ && x->registered(reinterpret_cast<const void*>(xconv_), 2 * cf * sizeof(float))) {
    for (int r = 0; r < n; ++r)
      a.xc[r] = static_cast<float*>(x->peer_ptr(reinterpret_cast<const void*>(xconv_), r));
    a.cstride = cf;
  }
  a.mom = P<float>(p.mom);
  a.fc4 = p.bucket1 / 4;
  a.l2 = p.l2;
  a.momentum = p.momentum;
  a.gscale = 1.0f / (float)n;
  a.lr = P<const float>(p.lr);
  a.step = P<long long>(p.step);
  a.off_w2 = (int)p.off_w2;
  a.off_b2 = (int)p.off_b2;
  a.off_w1 = (int)p.off_w1;
  a.off_b1 = (int)p.off_b1;
  a.part2 = P<const float>(p.part2);
  a.ngroups = conv2_groups();
  a.part1 = P<const float>(p.part1);
  a.nblk1 = conv1_blocks();
  if (p.wino) {
    a.wino_u = P<float>(p.wino_u);
    a.wino_ud = P<float>(p.wino_ud);
  }
  return a;
}

void MnistExecutor::train_step_xgmi(hipStream_t s) {
  const MnistPtrs& p = p_;
  wait_fc_params(s);
  mnist::XgmiStepArgs a = xgmi_step_args();
  // fp32 Winograd: the FC exchange + SGD ride as the first blocks of the
  // merged conv2 backward launch (its grads are final after fc1 backward), so
  // the link time overlaps the conv backward; the step launch then syncs the
  // conv parameters only
  const bool fc_in_bwd = p.wino && !p.bf16 && xgmi_fc_in_bwd_ && sched_ == SCHED_XGMI;
  a.fc_in_bwd = fc_in_bwd ? 1 : 0;
  enqueue_fwd_bwd(s, /*finalize=*/false, nullptr, false, take_fresh(!p.bf16), false,
                  fc_in_bwd ? &a : nullptr);
  mnist::launch_xgmi_step(a, s);
  if (p.bf16) shadows_stale_ = true;
}

// SCHED_XGMI_FAC: forward (the factor rows land in this rank's slots of the
// rank-major buffers) | fc1 dX only | conv2 backward; the peers' factor rows
// over the links; the FC gradients over all N x B rows (the exact global
// sums, formed in one fixed order on every rank); the step launch: local FC
// SGD + the conv sync.  No FC exchange, no FC momentum shard.
void MnistExecutor::train_step_xgmi_fac(hipStream_t s) {
  const MnistPtrs& p = p_;
  XgmiComm* x = xgmi_;
  const int n = x->size();
  wait_fc_params(s);
  mnist::XgmiFacArgs f;
  f.sync = x->sync();
  const size_t B = (size_t)p.batch;
  const uintptr_t bufs[4] = {p.a2_all, p.dh_all, p.hd_all, p.dlog_all};
  const size_t rows[4] = {B * kFc1In, B * kFc1Out, B * kFc1Out, B * kNcls};
  for (int k = 0; k < 4; ++k) {
    if (rows[k] % 4) throw std::runtime_error("xgmi_fac: factor slot not a multiple of 4 floats");
    f.slot4[k] = (long long)(rows[k] / 4);
    for (int r = 0; r < n; ++r)
      f.buf[k][r] = static_cast<float*>(x->peer_ptr(reinterpret_cast<const void*>(bufs[k]), r));
  }
  // forward; fc1 dX | the factor gather; conv2 backward
  enqueue_fwd_bwd(s, /*finalize=*/false, nullptr, /*factors=*/true, take_fresh(true), false,
                  nullptr, &f);
  // the fc2 / bias grads over every rank's rows; the fc1 weight's are formed
  // and applied by the step launch's FC tiles
  float* G = P<float>(p.grads);
  mnist::launch_fc1_small_grads(P<const float>(p.dh_all), P<const float>(p.hd_all),
                                P<const float>(p.dlog_all), n * p.batch, G + p.off_b3,
                                G + p.off_w4, G + p.off_b4, s);
  mnist::XgmiStepArgs a = xgmi_step_args();
  a.fc_local = 1;
  a.fa2 = P<const float>(p.a2_all);
  a.fdh = P<const float>(p.dh_all);
  a.frows = n * p.batch;
  a.off_w3 = (int)p.off_w3;
  mnist::launch_xgmi_step(a, s);
}

void MnistExecutor::gather_optimizer_state(hipStream_t s, Collective* comm, hipStream_t cs) {
  wait_fc_params(s);
  if (sched_ == SCHED_XGMI_FAC) return;  // every FC / conv momentum is replicated
  if ((sched_ == SCHED_XGMI || sched_ == SCHED_XGMI_STEP) && xgmi_ok()) {  // FC momentum segments
    xgmi_->gather_segments(P<float>(p_.mom), (size_t)p_.bucket1, s);
    return;
  }
  if (comm == nullptr || sched_ != SCHED_SHARDED_FC || !sharded_ok(comm->size())) return;
  float* Mo = P<float>(p_.mom);
  const long long chunk = p_.bucket1 / comm->size(), lo = chunk * comm->rank();
  HIP_CHECK(hipEventRecord(ev_fin_, s));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_fin_, 0));
  comm->all_gather(Mo + lo, Mo, (size_t)chunk, ncclFloat32, cs);
  HIP_CHECK(hipEventRecord(ev_done_, cs));
  HIP_CHECK(hipStreamWaitEvent(s, ev_done_, 0));
}

void MnistExecutor::eval_chunk(const MnistPtrs& p, uintptr_t x, uintptr_t y, int M,
                               uintptr_t ws_a1, uintptr_t ws_a2, uintptr_t ws_h, uintptr_t logits,
                               uintptr_t errors, float keep_prob, uint32_t drop_key,
                               hipStream_t s) {
  const float* W = P<const float>(p.params);
  if (p.bf16) {
    using U16 = uint16_t;
    const int Mp = (M + 7) / 8 * 8;  // conv2 tiles cover whole groups of 8 images
    mnist::launch_conv1_fwd_bf16(P<const float>(x), nullptr, 0, M, W + p.off_w1, W + p.off_b1,
                                 P<U16>(ws_a1), nullptr, nullptr, Mp, s, W + p.off_w3,
                                 W + p.off_w2, P<U16>(p.w1b), P<U16>(p.w1t), P<U16>(p.w2tb),
                                 P<U16>(p.w2b));
    mnist16::launch_conv2_fwd(P<const U16>(ws_a1), Mp, P<const U16>(p.w2tb), W + p.off_b2,
                              P<U16>(ws_a2), nullptr, nullptr, s);
    mnist16::launch_fc1_fwd_eval(P<const U16>(ws_a2), Mp, P<const U16>(p.w1t), W + p.off_b3, M,
                                 P<float>(ws_h), drop_key, keep_prob, s);
    mnist::launch_fc_head_eval(P<const float>(ws_h), W + p.off_w4, W + p.off_b4, P<const int>(y),
                               M, P<float>(logits), P<int>(errors), s);
    return;
  }
  mnist::launch_conv1_fwd(P<const float>(x), nullptr, 0, M, W + p.off_w1, W + p.off_b1,
                          P<float>(ws_a1), nullptr, s);
  mnist::launch_conv2_fwd(P<const float>(ws_a1), M, W + p.off_w2, W + p.off_b2, P<float>(ws_a2),
                          nullptr, nullptr, s);
  mnist::launch_fc1_fwd_eval(P<const float>(ws_a2), W + p.off_w3, W + p.off_b3, M, P<float>(ws_h),
                             drop_key, keep_prob, s);
  mnist::launch_fc_head_eval(P<const float>(ws_h), W + p.off_w4, W + p.off_b4, P<const int>(y), M,
                             P<float>(logits), P<int>(errors), s);
}
