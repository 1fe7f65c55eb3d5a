// Native training-step executor for the MNIST CNN.
//
// Replaces TF's Session.run(optimizer) step (/root/reference/mpipy.py:83-85)
// plus the DP sync (:91, :95-153).  One call enqueues the whole step on a HIP
// stream — fused forward, backward, all-reduce buckets, SGD — with no host
// synchronisation, no allocation and no host-side step state: the batch
// offset, dropout stream and LR are derived on the device from the device
// step counter.  The call is therefore capturable into a hipGraph and the
// Python trainer replays the captured graph.
//
// Compute runs on ONE stream (cross-stream event hops cost 5-18 us each in
// graph replay); independent work is merged into single launches instead.
// Gradient all-reduce (when a communicator is attached) runs in two buckets
// on a dedicated comm stream:
//   bucket 1 = FC params (97 % of the bytes), launched as soon as the fc1
//              backward kernel has written them, overlapping the conv
//              backward kernels on the compute stream;
//   bucket 2 = conv params, after the final slab reduction.
// The SGD runs in two parts: the FC segment (97 % of the update traffic)
// as soon as bucket 1 is reduced - overlapping bucket 2's all-reduce - and
// the conv segment after bucket 2; both divide by the world size.
// The alternative SCHED_SHARDED_FC schedule (train_step_sharded) splits the
// FC collective into reduce-scatter + all-gather around a 1/N-shard update so
// the all-gather overlaps the next step's conv forward.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "collective.h"
#include "rccl_comm.h"
#include "xgmi_comm.h"

struct MnistPtrs {
  // dataset (device resident)
  uintptr_t train_x = 0, train_y = 0;
  int n_local = 0, batch = 64;
  // flat buffers
  uintptr_t params = 0, grads = 0, mom = 0;
  long long total = 0, l2_end = 0, bucket1 = 0;  // floats
  long long off_w4 = 0, off_b4 = 0, off_w3 = 0, off_b3 = 0, off_w2 = 0, off_b2 = 0, off_w1 = 0,
            off_b1 = 0;
  // device scalars
  uintptr_t step = 0, lr = 0, correct = 0;
  // activations / workspaces
  uintptr_t a1 = 0, idx1 = 0, a2 = 0, idx2 = 0, fc1_part = 0, hd = 0, dh = 0, dlog = 0,
            loss_rows = 0, dy2 = 0, da1m = 0, part2 = 0, part1 = 0, w2t = 0, a1pf = 0;
  // fp32: dy2t = channel-major zero-bordered dY2 (direct bwd-data operand); a1pf =
  // zero-bordered NHWC a1 [B][18][18][32] (filter-grad operand).
  // bf16 engine (bf16 != 0): bf16 activation images and weight shadows
  // (layouts: kernels/mnist_bf16.h); a1 / a2 / dy2 / w2t above are unused
  int bf16 = 0;
  uintptr_t a1p = 0, a1t = 0, a2h = 0, a2t = 0, dy2p = 0, dy2t = 0, dh16 = 0, dht16 = 0,
            w1b = 0, w1t = 0, w2tb = 0, w2b = 0;
  // hyper-parameters
  float keep_prob = 0.5f, base_lr = 0.01f, lr_decay = 0.95f, l2 = 5e-4f, momentum = 0.9f;
  uint32_t seed = 1, rank = 0;
  int world = 1;
  // gradient wire dtype of the collectives (--grad-comm-dtype): 0 = fp32 (the
  // reference's), 1 = bf16 (half the bytes over xGMI; gb16 = a bf16 staging
  // buffer of `total` elements)
  int grad_bf16 = 0;
  uintptr_t gb16 = 0;
  // SCHED_FACTORS (fp32, world > 1): rank-major gathered FC factors of all
  // ranks, [world * batch] rows each (a2 [.][3136], dh / hd [.][512], dlog
  // [.][10]); a2 / dh / hd / dlog above point at this rank's slot in them
  uintptr_t a2_all = 0, dh_all = 0, hd_all = 0, dlog_all = 0;
  int fac_ranks = 0;  // communicator size the factor buffers were sized for
  // fp32 conv2 by Winograd F(2x2,5x5) (kernels/wino.h): transformed filters
  // wino_u [36][32][64] (forward) and wino_ud [36][64][32] (bwd-data)
  int wino = 0;
  uintptr_t wino_u = 0, wino_ud = 0;
  // fp32 Winograd step (optional): a2 also feature-major [3136][batch], written
  // by the conv2 forward for the LDS-free fc1 forward (0: the LDS-staged one)
  uintptr_t a2ft = 0;
};

namespace mnist {
struct FcSgdArgs;
struct XgmiStepArgs;
struct XgmiFacArgs;
}

class MnistExecutor {
 public:
  explicit MnistExecutor(const MnistPtrs& p);
  ~MnistExecutor();

  // Full training step.  comm may be null (single rank, or periodic
  // parameter averaging done by the caller); comm_stream is used only when
  // comm is attached.
  // comm2 (optional): second communicator of the same ranks, used by
  // SCHED_SPLIT for the conv bucket on the compute stream.
  void train_step(hipStream_t s, Collective* comm, hipStream_t comm_stream,
                  Collective* comm2 = nullptr);
  // Gradient-sync schedule used when a communicator of size > 1 is attached:
  //   SCHED_BUCKETS    - all-reduce of bucket 1 (FC) then bucket 2 (conv);
  //   SCHED_SHARDED_FC - reduce-scatter FC grads, SGD on the local 1/N shard,
  //                      all-gather FC params overlapped with the next
  //                      step's conv forward (see train_step_sharded);
  //   SCHED_SPLIT      - FC all-reduce + FC SGD on the comm stream, conv
  //                      all-reduce on the compute stream via comm2 (one
  //                      fork + one join per step, see train_step_split).
  //   SCHED_FACTORS    - all-gather the FC layers' gradient FACTORS (a2, dh,
  //                      hd, dlog: 1.07 MB per rank at B = 64) instead of
  //                      all-reducing the 6.45 MB FC gradient, then form the
  //                      global FC gradients on every rank (see
  //                      train_step_factors).
  //   SCHED_SERIAL     - no second queue at all: one all-reduce of the whole
  //                      flat gradient on the compute stream after the slab
  //                      reduction, then the SGD (no cross-queue edges, no
  //                      overlap; see train_step_serial).
  //   SCHED_DEFER      - (fp32) one communicator: FC part A, conv bucket, FC
  //                      part B + its SGD in order on the comm stream; the
  //                      next step's conv forward overlaps part B (see
  //                      train_step_defer).
  //   SCHED_XGMI       - the xGMI peer-to-peer communicator (set_xgmi): no
  //                      collective library and no second stream; after the
  //                      backward ONE launch on the compute stream reduces this
  //                      rank's 1/N of the FC gradients straight out of every
  //                      peer's memory, updates those parameters, gathers the
  //                      other segments back, and updates the (replicated)
  //                      conv parameters from the summed slab reductions (see
  //                      train_step_xgmi, mnist.h XgmiStepArgs).  fp32: the
  //                      FC exchange + SGD ride as role blocks of the conv2
  //                      backward launch (overlapping its link time with the
  //                      conv backward);
  //   SCHED_XGMI_FAC   - fp32: the FC factors (a2, dh, hd, dlog: 1.07 MB a
  //                      rank at B = 64, against a 6.4 MB FC gradient) copied
  //                      from every peer over its link (train_step_xgmi_fac),
  //                      the FC gradients formed from them with K = N x B
  //                      (the global sums, the same on every rank) and applied
  //                      locally; the conv sync as SCHED_XGMI_STEP.  Few
  //                      ranks: one link per peer carries 1/6 of the bytes.
  //   SCHED_XGMI_STEP  - the same with the whole FC exchange in the step
  //                      launch (no CUs taken from the conv backward: its 512
  //                      blocks are 2 exact rounds on 256 CUs, role blocks add a
  //                      third; the auto-tune picks by the real link speed).
  static constexpr int SCHED_BUCKETS = 0, SCHED_SHARDED_FC = 1, SCHED_SPLIT = 2,
                       SCHED_FACTORS = 3, SCHED_SERIAL = 4, SCHED_DEFER = 5, SCHED_XGMI = 6,
                       SCHED_XGMI_STEP = 7, SCHED_XGMI_FAC = 8;
  // the peer-to-peer communicator of SCHED_XGMI: the flat grads and params must
  // be registered with it (XgmiComm::open_buffer / emulate_buffer)
  void set_xgmi(XgmiComm* x) { xgmi_ = x; }
  // the conv-grad exchange buffer of the step launch (2 x
  // mnist::xgmi_conv_floats(off_b1) floats, registered with the communicator;
  // 0: the conv grads go through the grads buffer)
  void set_xgmi_xconv(uintptr_t p) { xconv_ = p; }
  // fp32 SCHED_XGMI: the FC exchange inside the conv2 backward launch
  // (default) or in the step launch (= SCHED_XGMI_STEP; labs)
  void set_xgmi_fc_in_bwd(bool on) { xgmi_fc_in_bwd_ = on; }
  bool xgmi_ok() const;
  bool xgmi_fac_ok() const;
  void set_schedule(int sched);
  int schedule() const { return sched_; }
  bool sharded_ok(int nranks) const;
  bool factors_ok(int nranks) const;
  bool defer_ok() const;
  // SCHED_DEFER: the fraction of the FC bucket in part A (reduced under the
  // conv backward; the rest overlaps the next step's conv forward)
  void set_defer_split(float f);
  float defer_split() const { return defer_split_; }
  // Makes stream s wait for any collective still in flight from the last
  // step (call at the end of every captured / eager run of steps).
  void join(hipStream_t s);
  // Sharded schedule: all-gathers the FC momentum shards so the whole
  // momentum buffer is valid (before checkpointing).  No-op otherwise.
  void gather_optimizer_state(hipStream_t s, Collective* comm, hipStream_t comm_stream);
  // Forward+backward only (grads in the flat grad buffer; no sync, no SGD).
  void forward_backward(hipStream_t s);
  void sgd(hipStream_t s, float gscale);

  // Evaluation of M rows starting at x (NHWC [M,28,28,1]): writes logits
  // [M,10] when logits != 0 and adds the error count to *errors.  ws_* are
  // caller-provided work buffers sized for `chunk` rows (bf16 engine: ws_a1
  // = zero-bordered bf16 a1p image of round_up(chunk, 8) rows, ws_a2 = bf16
  // a2 of as many rows).
  static void eval_chunk(const MnistPtrs& p, uintptr_t x, uintptr_t y, int M, uintptr_t ws_a1,
                         uintptr_t ws_a2, uintptr_t ws_h, uintptr_t logits, uintptr_t errors,
                         float keep_prob, uint32_t drop_key, hipStream_t s);

  const MnistPtrs& ptrs() const { return p_; }
  // single-rank step: where the FC-bucket SGD runs.  r > 0: in the conv2
  // bwd-data launch (r rounds of FC_SGD_UNROLL float4s per thread of the
  // appended role; the Winograd launch spreads it over its own blocks); 0: in
  // the final SGD launch, beside the latency-bound conv SGD blocks; r < 0: the
  // measured default per engine - fp32 0 (89.8 vs 94.2 us per step with the
  // fused dW1 tiles), bf16 2
  void set_fc_sgd_rounds(int r) { fc_sgd_rounds_ = r < 0 ? -1 : r; }
  // Re-derives every weight copy the step kernels read from the fp32 master
  // weights: the Winograd filter transforms (fp32, wino) and the bf16
  // shadows (bf16 engine).  A single-rank bf16 step writes the fc1 shadows from its SGD and
  // the next step relies on them, so the caller refreshes them once before a
  // run of steps (the engine does so at the start of every train() call):
  // any change to the weights between runs (init, checkpoint load, ...) is
  // picked up there.
  void refresh_shadows(hipStream_t s);

 private:
  // finalize = false: leave the conv filter grads as slabs (the world-1 SGD
  // launch reduces them itself)
  // fc_sgd (single rank): FC-bucket SGD appended to the conv2 bwd-data launch
  // factors: record ev_fac_ once the FC factors are written (after the head)
  // and compute only dX in fc1 backward (the FC weight grads come from the
  // gathered factors)
  // fresh: the derived weights (Winograd filter transforms; bf16 shadows) are
  // already current - the previous step's SGD launch wrote them (sgd_step,
  // launch_sgd_step); otherwise the step derives them from the weights first
  // fc1_dw_fused: the fc1 weight gradient is formed inside this step's SGD
  // (single rank, fp32 Winograd): fc1 backward skips its dW1 role
  // xfc (fp32 Winograd, SCHED_XGMI): the FC bucket's peer-to-peer exchange +
  // SGD as role blocks of the merged conv2 backward launch
  void enqueue_fwd_bwd(hipStream_t s, bool finalize = true,
                       const mnist::FcSgdArgs* fc_sgd = nullptr, bool factors = false,
                       bool fresh = false, bool fc1_dw_fused = false,
                       const mnist::XgmiStepArgs* xfc = nullptr,
                       const mnist::XgmiFacArgs* xfac = nullptr);
  // the fused SGD launch applies (L2 prefix == the FC bucket, as in the
  // reference layout)
  bool fused_sgd_ok() const;
  // world > 1: the fused SGD launch over the all-reduced flat grads (FC
  // bucket and / or conv parameters), writing the next step's derived weights
  // fc_end >= 0: the FC part is [0, fc_end) instead of the whole bucket
  void sgd_step(hipStream_t s, float gscale, bool fc, bool conv, long long fc_end = -1);
  int conv1_blocks() const;
  int conv2_groups() const;
  void train_step_sharded(hipStream_t s, Collective* comm, hipStream_t cs);
  void train_step_split(hipStream_t s, Collective* comm, hipStream_t cs, Collective* comm2);
  void train_step_factors(hipStream_t s, Collective* comm, hipStream_t cs);
  void train_step_serial(hipStream_t s, Collective* comm);
  void train_step_defer(hipStream_t s, Collective* comm, hipStream_t cs);
  void train_step_xgmi(hipStream_t s);
  void train_step_xgmi_fac(hipStream_t s);
  mnist::XgmiStepArgs xgmi_step_args() const;
  XgmiComm* xgmi_ = nullptr;
  uintptr_t xconv_ = 0;
  bool xgmi_fc_in_bwd_ = true;
  float defer_split_ = 0.5f;
  void wait_fc_params(hipStream_t s);
  // all-reduce (sum) of grads [lo, lo + n) on cs, over the bf16 wire if set
  void reduce_bucket(Collective* comm, long long lo, long long n, hipStream_t cs);
  int sched_ = SCHED_BUCKETS;
  bool fc_pending_ = false;  // an FC all-gather was enqueued and not yet waited on
  // shadows_fresh: every bf16 weight shadow is current (single-rank step)
  void enqueue_fwd_bwd_bf16(hipStream_t s, bool finalize = true,
                            const mnist::FcSgdArgs* fc_sgd = nullptr, bool shadows_fresh = false);
  int fc_sgd_rounds_ = -1;
  // bf16: the fc1 shadows are one FC update behind (after a sharded step)
  bool shadows_stale_ = false;
  bool take_fresh(bool want);
  MnistPtrs p_;
  void sgd_range(hipStream_t s, long long lo, long long hi, float gscale, bool bump_step);
  // ev_dw_: FC grads final (bucket 1 may start); ev_b1_: bucket 1 reduced;
  // ev_fin_: conv grads final (bucket 2 may start); ev_done_: bucket 2 reduced.
  // Sharded schedule: ev_b1_ = FC params gathered
  // ev_fac_: FC factors written (SCHED_FACTORS all-gather may start)
  hipEvent_t ev_dw_ = nullptr, ev_b1_ = nullptr, ev_fin_ = nullptr, ev_done_ = nullptr,
             ev_fac_ = nullptr;
};
