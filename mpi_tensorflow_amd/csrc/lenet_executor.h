// Native training-step executor for LeNet-5 (BASELINE config 4).
//
// Same contract as MnistExecutor (mnist_executor.h): one call enqueues a whole
// training step on a HIP stream with no host synchronisation, no allocation
// and no host-side step state (batch offset and LR come from the device step
// counter), so the Python engine captures G steps into one hipGraph.
//   world 1:  image kernel -> update kernel (grads + momentum SGD)   2 launches
//   world N, xGMI communicator, mode push: image kernel -> update kernel
//             with the push sync fused (lenet.h PushArgs)           2 launches
//   world N, xGMI communicator, mode pull: image kernel -> update kernel
//             (grads into slot step & 1 of xgrads2) -> one-shot sum of every
//             rank's slot + replicated SGD (xgmi.h OneShotArgs)     3 launches
//   world N, xGMI communicator, mode two-phase: image -> update (grads) ->
//             all_reduce_sgd (segment sum + SGD, gather)           3 launches
//   world N:  image kernel -> update kernel (grads into the flat buffer)
//             -> in-place all-reduce of the whole 250 KB flat gradient on
//             the compute stream (one latency-bound bucket: a cross-stream
//             fork/join would cost more than it hides) -> flat SGD with
//             gscale 1/N                                    3 launches + 1 collective
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "collective.h"
#include "kernels/lenet.h"

struct LenetPtrs {
  uintptr_t train_x = 0, train_y = 0;
  int n_local = 0, batch = 64;
  uintptr_t params = 0, grads = 0, mom = 0;
  long long total = 0;
  lenet::Offsets off{};
  uintptr_t step = 0, lr = 0, correct = 0;
  uintptr_t acts = 0, deltas = 0, convp = 0, loss_rows = 0;
  float base_lr = 0.01f, lr_decay = 0.95f, momentum = 0.9f;
  // --grad-comm-dtype bf16: the all-reduce runs on a bf16 copy (gb16, total
  // elements) of the grads
  int grad_bf16 = 0;
  uintptr_t gb16 = 0;
  // xGMI push sync (lenet.h PushArgs): the registered receive buffer
  // [2][N][total] floats; 0 = the two-phase all_reduce_sgd instead
  uintptr_t xrecv = 0;
  // xGMI one-shot (pull) sync: the registered double-buffered gradient
  // [2][total] floats and a zeroed device word (the launch's completion count)
  uintptr_t xgrads2 = 0, xdone = 0;
};

class LenetExecutor {
 public:
  explicit LenetExecutor(const LenetPtrs& p);
  void train_step(hipStream_t s, Collective* comm);
  // the sync over an XgmiComm: XGMI_TWO_PHASE (all_reduce_sgd), XGMI_PUSH
  // (needs xrecv) or XGMI_PULL (needs xgrads2 + xdone)
  enum { XGMI_TWO_PHASE = 0, XGMI_PUSH = 1, XGMI_PULL = 2 };
  void set_xgmi_mode(int m);
  int xgmi_mode() const { return mode_; }
  // forward + backward with the weight grads in the flat grad buffer (no
  // sync, no SGD, no step bump): numerics tests
  void forward_backward(hipStream_t s);
  // forward of rows [x, x + M) (device), argmax vs labels -> *errors (+ logits)
  static void eval_chunk(const LenetPtrs& p, uintptr_t x, uintptr_t y, int M, uintptr_t logits,
                         uintptr_t errors, hipStream_t s);

 private:
  lenet::ImageArgs image_args() const;
  LenetPtrs p_;
  int mode_ = XGMI_TWO_PHASE;
};
