// Host launchers of the fused LeNet-5 kernel set (lenet.hip), BASELINE
// config 4 ("LeNet-5 on synthetic 32x32x3 (CIFAR-shape)").
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "xgmi.h"

namespace lenet {

// per-image buffers written by the image kernel (floats per image)
constexpr int ACT_STRIDE = 608;    // a2 (400) | h1 (120) | h2 (84)   (pooled2 flatten = FC1 input)
constexpr int DELTA_STRIDE = 216;  // dz1 (120) | dz2 (84) | dz3 (10)  (pre-activation grads)
constexpr int CONVP_STRIDE = 2880; // dW1 (450) | db1 (6) | dW2 (2400) | db2 (16)
constexpr int NPARAM_TENSORS = 10;

// flat-buffer offsets of the ten LeNet-5 tensors (parallel/flat.py layout)
struct Offsets {
  int c1w, c1b, c2w, c2b, f1w, f1b, f2w, f2b, f3w, f3b;
};

struct ImageArgs {
  const float* x;       // dataset rows [N][32][32][3] (NHWC)
  const int* y;         // labels [N]
  int n_local, batch;   // train: row = (step * batch) % (n_local - batch) + image
  const long long* step;  // device step (train); nullptr: row = image (eval)
  const float* params;
  Offsets off;
  // train outputs
  float* acts;      // [batch][ACT_STRIDE]
  float* deltas;    // [batch][DELTA_STRIDE]
  float* convp;     // [batch][CONVP_STRIDE]
  float* loss_rows; // [batch]
  float* lr_out;    // device LR of this step (image 0 writes it)
  float base_lr, lr_decay;
  int* correct;     // optional train-accuracy counter
  // eval outputs
  int* errors;      // wrong-prediction counter
  float* logits;    // optional [rows][10]
  int stop_phase = 99;  // profiling: return after this phase
};

// one workgroup per image: forward (conv1+ReLU+pool, conv2+ReLU+pool, FC chain,
// softmax xent) and, for train, the whole backward pass up to the per-image
// conv weight-gradient partials
void launch_image_train(const ImageArgs& a, hipStream_t s);
void launch_image_eval(const ImageArgs& a, int rows, hipStream_t s);

// batch-level weight gradients (FC: act^T delta over the batch; conv: sum of
// the per-image partials) then, when `apply`, momentum SGD with the device LR
// and the device-step bump; otherwise the grads go to `grads` (all-reduce
// follows, then the flat SGD kernel)
void launch_update(const float* acts, const float* deltas, const float* convp, int batch,
                   const Offsets& off, float* params, float* grads, float* mom, float momentum,
                   const float* lr, long long* step, bool apply, hipStream_t s, long long dbuf = 0);
// dbuf > 0 (apply = false): the grads go to slot (*step) & 1 of a double-
// buffered [2][dbuf] buffer at `grads` (the xGMI one-shot sync reads it)

// xGMI "push" sync fused into the update launch (LenetExecutor with an
// XgmiComm and a registered receive buffer): every block pushes its freshly
// formed gradient values into slot [parity][me] of every peer's receive
// buffer (system-scope remote stores), meets the peers' same block at ONE
// barrier, sums the N slots of its values in rank order and applies the
// replicated momentum SGD (gscale 1/N) - one launch, one barrier, no gather
// phase and no sharded momentum.  For a 62 K-parameter model each link carries
// the whole gradient once (250 KB, ~1.7 us at 150 GB/s), less than the two
// barriers of the two-phase all-reduce cost.  The parity comes from the
// block's barrier epoch, so a peer still reading step t's slots is never
// overwritten by step t + 1 (same argument as the MNIST conv exchange).
struct PushArgs {
  xgmi::Sync sync;
  float* recv[xgmi::kMaxRanks] = {};  // every rank's receive buffer [2][N][total], mapped here
  long long total = 0;                // floats per slot (the flat gradient)
  float gscale = 1.f;
};
void launch_update_push(const float* acts, const float* deltas, const float* convp, int batch,
                        const Offsets& off, float* params, float* mom, float momentum,
                        const float* lr, long long* step, const PushArgs& pa, hipStream_t s);

size_t acts_floats(int batch);
size_t deltas_floats(int batch);
size_t convp_floats(int batch);

}  // namespace lenet
