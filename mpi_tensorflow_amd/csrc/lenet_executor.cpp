#include "lenet_executor.h"

#include <stdexcept>

#include "kernels/mnist.h"  // optim::launch_sgd_momentum
#include "xgmi_comm.h"

template <class T>
static inline T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}

LenetExecutor::LenetExecutor(const LenetPtrs& p) : p_(p) {
  if (p_.batch <= 0 || p_.n_local <= p_.batch)
    throw std::runtime_error("LenetExecutor: the local shard must exceed the batch");
  if (p_.total % 4 != 0) throw std::runtime_error("LenetExecutor: flat buffer not float4-sized");
}

void LenetExecutor::set_xgmi_mode(int m) {
  if (m == XGMI_PUSH && !p_.xrecv) throw std::runtime_error("LenetExecutor: push needs xrecv");
  if (m == XGMI_PULL && (!p_.xgrads2 || !p_.xdone))
    throw std::runtime_error("LenetExecutor: pull needs xgrads2 and xdone");
  if (m < XGMI_TWO_PHASE || m > XGMI_PULL) throw std::runtime_error("LenetExecutor: xgmi mode");
  mode_ = m;
}

lenet::ImageArgs LenetExecutor::image_args() const {
  lenet::ImageArgs a{};
  a.x = P<const float>(p_.train_x);
  a.y = P<const int>(p_.train_y);
  a.n_local = p_.n_local;
  a.batch = p_.batch;
  a.step = P<const long long>(p_.step);
  a.params = P<const float>(p_.params);
  a.off = p_.off;
  a.acts = P<float>(p_.acts);
  a.deltas = P<float>(p_.deltas);
  a.convp = P<float>(p_.convp);
  a.loss_rows = P<float>(p_.loss_rows);
  a.lr_out = P<float>(p_.lr);
  a.base_lr = p_.base_lr;
  a.lr_decay = p_.lr_decay;
  a.correct = P<int>(p_.correct);
  return a;
}

void LenetExecutor::forward_backward(hipStream_t s) {
  lenet::launch_image_train(image_args(), s);
  lenet::launch_update(P<const float>(p_.acts), P<const float>(p_.deltas), P<const float>(p_.convp),
                       p_.batch, p_.off, P<float>(p_.params), P<float>(p_.grads), P<float>(p_.mom),
                       p_.momentum, P<const float>(p_.lr), P<long long>(p_.step), false, s);
}

void LenetExecutor::train_step(hipStream_t s, Collective* comm) {
  lenet::launch_image_train(image_args(), s);
  if (auto* x = dynamic_cast<XgmiComm*>(comm); x != nullptr && mode_ == XGMI_PULL) {
    float* G2 = P<float>(p_.xgrads2);
    lenet::launch_update(P<const float>(p_.acts), P<const float>(p_.deltas),
                         P<const float>(p_.convp), p_.batch, p_.off, P<float>(p_.params), G2,
                         P<float>(p_.mom), p_.momentum, P<const float>(p_.lr),
                         P<long long>(p_.step), false, s, p_.total);
    x->all_reduce_sgd_oneshot(G2, P<float>(p_.params), P<float>(p_.mom), (size_t)p_.total,
                              p_.momentum, 1.0f / (float)x->size(), P<const float>(p_.lr),
                              P<long long>(p_.step), P<unsigned>(p_.xdone), s);
    return;
  }
  if (auto* x = dynamic_cast<XgmiComm*>(comm); x != nullptr && mode_ == XGMI_PUSH) {
    lenet::PushArgs pa;
    pa.sync = x->sync();
    for (int r = 0; r < x->size(); ++r)
      pa.recv[r] = static_cast<float*>(x->peer_ptr(reinterpret_cast<const void*>(p_.xrecv), r));
    pa.total = p_.total;
    pa.gscale = 1.0f / (float)x->size();
    lenet::launch_update_push(P<const float>(p_.acts), P<const float>(p_.deltas),
                              P<const float>(p_.convp), p_.batch, p_.off, P<float>(p_.params),
                              P<float>(p_.mom), p_.momentum, P<const float>(p_.lr),
                              P<long long>(p_.step), pa, s);
    return;
  }
  const bool apply = comm == nullptr;
  lenet::launch_update(P<const float>(p_.acts), P<const float>(p_.deltas), P<const float>(p_.convp),
                       p_.batch, p_.off, P<float>(p_.params), P<float>(p_.grads), P<float>(p_.mom),
                       p_.momentum, P<const float>(p_.lr), P<long long>(p_.step), apply, s);
  if (apply) return;
  float* G = P<float>(p_.grads);
  if (auto* x = dynamic_cast<XgmiComm*>(comm); x != nullptr && !p_.grad_bf16) {
    // xGMI peer to peer: the sum of this rank's segment and its SGD in one
    // launch on this stream, then the updated segments gathered (sharded momentum)
    x->all_reduce_sgd(G, P<float>(p_.params), P<float>(p_.mom), (size_t)p_.total, 0, 0.f,
                      p_.momentum, 1.0f / (float)comm->size(), P<const float>(p_.lr),
                      P<long long>(p_.step), s);
    return;
  }
  if (p_.grad_bf16) {
    uint16_t* B = P<uint16_t>(p_.gb16);
    optim::launch_to_bf16(G, B, p_.total, s);
    comm->all_reduce(B, B, (size_t)p_.total, 9 /*ncclBfloat16*/, 0 /*ncclSum*/, s);
    optim::launch_from_bf16(B, G, p_.total, s);
  } else {
    comm->all_reduce(G, G, (size_t)p_.total, 7 /*ncclFloat32*/, 0 /*ncclSum*/, s);
  }
  optim::launch_sgd_momentum(P<float>(p_.params), G, P<float>(p_.mom), p_.total, 0, 0.f,
                             p_.momentum, 1.0f / (float)comm->size(), P<const float>(p_.lr), 0.f,
                             P<long long>(p_.step), s);
}

void LenetExecutor::eval_chunk(const LenetPtrs& p, uintptr_t x, uintptr_t y, int M,
                               uintptr_t logits, uintptr_t errors, hipStream_t s) {
  lenet::ImageArgs a{};
  a.x = P<const float>(x);
  a.y = P<const int>(y);
  a.n_local = M;
  a.batch = M;
  a.step = nullptr;
  a.params = P<const float>(p.params);
  a.off = p.off;
  a.errors = P<int>(errors);
  a.logits = P<float>(logits);
  lenet::launch_image_eval(a, M, s);
}
