// pybind11 module `mpi_tensorflow_amd._C`: the native runtime of the
// framework (HIP kernels, step executor, RCCL communicator, IDX loader).
//
// Device buffers cross the boundary as raw addresses (torch tensors'
// data_ptr()) and streams as hipStream_t handles (torch's
// current_stream().cuda_stream); the Python layer (ops/, runtime/) validates
// shapes, dtypes, devices and contiguity BEFORE calling in, because the
// kernels assume the geometry they were compiled for.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "idx_loader.h"
#include "kernels/mnist.h"
#include "kernels/mnist_bf16.h"
#include "kernels/ops_generic.h"
#include "lenet_executor.h"
#include "mnist_executor.h"
#include "rccl_comm.h"
#include "shm_comm.h"
#include "xgmi_comm.h"

namespace py = pybind11;

template <class T>
static inline T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}
static inline hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("kernel launch failed: ") + hipGetErrorString(e));
}

// Host-callback communicator (tests only): every collective calls a Python
// function (op, send, recv, count, dtype) that stages the data through the
// host and a gloo group.  Lets several ranks share ONE GPU and drive the
// native executors' sync schedules eagerly (not capturable).
class PyComm : public Collective {
 public:
  PyComm(int nranks, int rank, py::function fn) : n_(nranks), r_(rank), fn_(std::move(fn)) {}
  int rank() const override { return r_; }
  int size() const override { return n_; }
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int,
                  hipStream_t) override {
    fn_("all_reduce", (uintptr_t)send, (uintptr_t)recv, count, dtype);
  }
  void all_gather(const void* send, void* recv, size_t send_count, int dtype,
                  hipStream_t) override {
    fn_("all_gather", (uintptr_t)send, (uintptr_t)recv, send_count, dtype);
  }
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int,
                      hipStream_t) override {
    fn_("reduce_scatter", (uintptr_t)send, (uintptr_t)recv, recv_count, dtype);
  }

 private:
  int n_, r_;
  py::function fn_;
};

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native runtime for mpi_tensorflow_amd (gfx950 HIP kernels, RCCL, IDX)";
  m.attr("ARCH") = "gfx950";

  // ------------------------------------------------------------- kernels
  auto k = m.def_submodule("mnist", "fused fp32 MNIST CNN kernels (gfx950 MFMA)");
  k.def("conv1_fwd", [](uintptr_t data, uintptr_t step, int n_local, int batch, uintptr_t w,
                        uintptr_t b, uintptr_t out, uintptr_t argmax, uintptr_t s, uintptr_t out_pad) {
    mnist::launch_conv1_fwd(P<const float>(data), P<const long long>(step), n_local, batch,
                            P<const float>(w), P<const float>(b), P<float>(out), P<uint8_t>(argmax),
                            S(s), P<float>(out_pad));
    check_launch();
  }, py::arg("data"), py::arg("step"), py::arg("n_local"), py::arg("batch"), py::arg("w"),
     py::arg("b"), py::arg("out"), py::arg("argmax"), py::arg("stream"), py::arg("out_pad") = 0);
  k.def("conv12_fwd", [](uintptr_t data, uintptr_t step, int n_local, int batch, uintptr_t w1,
                         uintptr_t b1, uintptr_t a1, uintptr_t a1pf, uintptr_t idx1, uintptr_t w2,
                         uintptr_t b2, uintptr_t a2, uintptr_t idx2, uintptr_t w2t, uintptr_t s) {
    mnist::C12In c;
    c.data = P<const float>(data);
    c.step = P<const long long>(step);
    c.n_local = n_local;
    c.w1 = P<const float>(w1);
    c.b1 = P<const float>(b1);
    c.a1 = P<float>(a1);
    c.a1pf = P<float>(a1pf);
    c.idx1 = P<uint8_t>(idx1);
    mnist::launch_conv12_fwd(c, batch, P<const float>(w2), P<const float>(b2), P<float>(a2),
                             P<uint8_t>(idx2), P<float>(w2t), S(s));
    check_launch();
  });
  k.def("conv12_fwd_wino", [](uintptr_t data, uintptr_t step, int n_local, int batch, uintptr_t w1,
                              uintptr_t b1, uintptr_t a1, uintptr_t a1pf, uintptr_t idx1,
                              uintptr_t w2, uintptr_t U, uintptr_t b2, uintptr_t a2, uintptr_t idx2,
                              uintptr_t w2t, uintptr_t s, uintptr_t prof, uintptr_t a2t) {
    mnist::C12In c;
    c.data = P<const float>(data);
    c.step = P<const long long>(step);
    c.n_local = n_local;
    c.w1 = P<const float>(w1);
    c.b1 = P<const float>(b1);
    c.a1 = P<float>(a1);
    c.a1pf = P<float>(a1pf);
    c.idx1 = P<uint8_t>(idx1);
    mnist::launch_conv12_fwd_wino(c, batch, P<const float>(w2), P<const float>(U),
                                  P<const float>(b2), P<float>(a2), P<uint8_t>(idx2),
                                  P<float>(w2t), S(s), P<unsigned long long>(prof), P<float>(a2t));
    check_launch();
  }, py::arg("data"), py::arg("step"), py::arg("n_local"), py::arg("batch"), py::arg("w1"), py::arg("b1"), py::arg("a1"), py::arg("a1pf"), py::arg("idx1"), py::arg("w2"), py::arg("U"), py::arg("b2"), py::arg("a2"), py::arg("idx2"), py::arg("w2t"), py::arg("s"), py::arg("prof") = 0, py::arg("a2t") = 0);
  // bf16 engine forward pieces (tests): two-launch conv1 -> conv2 and the fused launch
  k.def("conv1_fwd_bf16", [](uintptr_t data, uintptr_t step, int n_local, int batch, uintptr_t w1,
                             uintptr_t b1, uintptr_t a1p, uintptr_t a1t, uintptr_t idx1,
                             uintptr_t s) {
    mnist::launch_conv1_fwd_bf16(P<const float>(data), P<const long long>(step), n_local, batch,
                                 P<const float>(w1), P<const float>(b1), P<uint16_t>(a1p),
                                 P<uint16_t>(a1t), P<uint8_t>(idx1), batch, S(s));
    check_launch();
  });
  k.def("conv2_fwd_bf16", [](uintptr_t a1p, int batch, uintptr_t w2tb, uintptr_t b2, uintptr_t a2p,
                             uintptr_t a2t, uintptr_t idx2, uintptr_t s) {
    mnist16::launch_conv2_fwd(P<const uint16_t>(a1p), batch, P<const uint16_t>(w2tb),
                              P<const float>(b2), P<uint16_t>(a2p), P<uint16_t>(a2t),
                              P<uint8_t>(idx2), S(s));
    check_launch();
  });
  k.def("conv12_fwd_bf16", [](uintptr_t data, uintptr_t step, int n_local, int batch, uintptr_t w1,
                              uintptr_t b1, uintptr_t idx1, uintptr_t w2tb, uintptr_t b2,
                              uintptr_t a1p, uintptr_t a1t, uintptr_t a2p, uintptr_t a2t,
                              uintptr_t idx2, uintptr_t s) {
    mnist::C12In c;
    c.data = P<const float>(data);
    c.step = P<const long long>(step);
    c.n_local = n_local;
    c.w1 = P<const float>(w1);
    c.b1 = P<const float>(b1);
    c.idx1 = P<uint8_t>(idx1);
    mnist::launch_conv12_fwd_bf16(c, batch, P<const uint16_t>(w2tb), P<const float>(b2),
                                  P<uint16_t>(a1p), P<uint16_t>(a1t), P<uint16_t>(a2p),
                                  P<uint16_t>(a2t), P<uint8_t>(idx2), S(s));
    check_launch();
  });
  k.def("shadows_bf16", [](uintptr_t w1, uintptr_t w2, uintptr_t w1b, uintptr_t w1t,
                           uintptr_t w2tb, uintptr_t w2b, uintptr_t s) {
    mnist16::launch_shadows(P<const float>(w1), P<const float>(w2), P<uint16_t>(w1b),
                            P<uint16_t>(w1t), P<uint16_t>(w2tb), P<uint16_t>(w2b), S(s));
    check_launch();
  });
  k.def("conv2_fwd", [](uintptr_t a1, int batch, uintptr_t w, uintptr_t b, uintptr_t out,
                        uintptr_t argmax, uintptr_t w2t, uintptr_t s) {
    mnist::launch_conv2_fwd(P<const float>(a1), batch, P<const float>(w), P<const float>(b),
                            P<float>(out), P<uint8_t>(argmax), P<float>(w2t), S(s));
    check_launch();
  });
  k.def("conv2_wino_weights", [](uintptr_t w2, uintptr_t U, uintptr_t Ud, uintptr_t s) {
    mnist::launch_conv2_wino_weights(P<const float>(w2), P<float>(U), P<float>(Ud), S(s));
    check_launch();
  });
  k.def("conv2_fwd_wino", [](uintptr_t a1, int batch, uintptr_t w, uintptr_t U, uintptr_t b,
                             uintptr_t out, uintptr_t argmax, uintptr_t w2t, uintptr_t s) {
    mnist::launch_conv2_fwd_wino(P<const float>(a1), batch, P<const float>(w), P<const float>(U),
                                 P<const float>(b), P<float>(out), P<uint8_t>(argmax),
                                 P<float>(w2t), S(s));
    check_launch();
  });
  k.def("conv2_bwd_data_wino", [](uintptr_t dy2, uintptr_t Ud, uintptr_t a1, int batch,
                                  uintptr_t da1m, uintptr_t s) {
    mnist::launch_conv2_bwd_data_wino(P<const float>(dy2), P<const float>(Ud), P<const float>(a1),
                                      batch, P<float>(da1m), S(s));
    check_launch();
  });
  // labs: with the conv1 filter-gradient epilogue and per-wave phase stamps
  k.def("conv2_bwd_data_wino_prof", [](uintptr_t dy2, uintptr_t Ud, uintptr_t a1, int batch,
                                       uintptr_t da1m, uintptr_t data, uintptr_t step, int n_local,
                                       uintptr_t idx1, uintptr_t part1, uintptr_t prof,
                                       uintptr_t s) {
    const mnist::C1FilterArgs c1{P<const float>(data), P<const long long>(step), n_local,
                                 P<const float>(da1m), P<const uint8_t>(idx1), P<float>(part1)};
    mnist::launch_conv2_bwd_data_wino(P<const float>(dy2), P<const float>(Ud), P<const float>(a1),
                                      batch, P<float>(da1m), S(s), nullptr, &c1,
                                      P<unsigned long long>(prof));
    check_launch();
  });
  k.def("fc1_train_splits", &mnist::fc1_train_splits);
  k.def("conv2_filter_splits", &mnist::conv2_filter_splits);
  k.def("conv1_filter_blocks", [](int batch, int split) {
    return mnist::conv1_filter_blocks(batch, split);
  }, py::arg("batch"), py::arg("split") = 7);

  k.def("part2_floats", &mnist::part2_floats);
  k.def("part2_floats_wino", &mnist::part2_floats_wino);
  k.def("part1_floats", &mnist::part1_floats);
  k.def("fc1_part_floats", &mnist::fc1_part_floats);
  k.def("part2_floats_bf16", &mnist16::part2_floats);
  k.def("conv2_filter_groups_bf16", &mnist16::conv2_filter_groups);
  k.def("conv2_bwd_conv1_rows_bf16", &mnist16::conv2_bwd_conv1_rows);
  k.def("xgmi_conv_floats", &mnist::xgmi_conv_floats);
  k.def("xgmi_dispatch_probe", [](uintptr_t ctr, uintptr_t out, int blocks, long long spin,
                                   uintptr_t s) {
    xgmi::launch_dispatch_probe(reinterpret_cast<unsigned*>(ctr),
                                reinterpret_cast<unsigned long long*>(out), blocks, spin, S(s));
    check_launch();
  });
  k.def("set_xgmi_step_prof", [](uintptr_t p) {
    mnist::set_xgmi_step_prof(reinterpret_cast<unsigned long long*>(p));
  });
  k.def("set_conv2_bwd_wino_prof", [](uintptr_t p) {
    mnist::set_conv2_bwd_wino_prof(reinterpret_cast<unsigned long long*>(p));
  });
  k.def("conv2_wino_filter_groups", &mnist::conv2_wino_filter_groups);
  k.def("set_sgd_prof", [](uintptr_t p) {
    mnist::set_sgd_prof(reinterpret_cast<unsigned long long*>(p));
  });
  k.def("set_conv2_bwd_prof_bf16", [](uintptr_t p) {
    mnist16::set_conv2_bwd_prof(reinterpret_cast<unsigned long long*>(p));
  });
  k.def("fc1_fwd_train", [](uintptr_t a2, uintptr_t w, int batch, uintptr_t part, uintptr_t s) {
    mnist::launch_fc1_fwd_train(P<const float>(a2), P<const float>(w), batch, P<float>(part), S(s));
    check_launch();
  });
  k.def("fc1_fwd_train_t", [](uintptr_t a2t, uintptr_t w, int batch, uintptr_t part,
                              uintptr_t s) {
    mnist::launch_fc1_fwd_train_t(P<const float>(a2t), P<const float>(w), batch, P<float>(part),
                                  S(s));
    check_launch();
  });
  k.def("fc1_train_t_splits", &mnist::fc1_train_t_splits);
  k.def("fc1_fwd_eval", [](uintptr_t a2, uintptr_t w, uintptr_t b, int M, uintptr_t h,
                           uint32_t key, float keep, uintptr_t s) {
    mnist::launch_fc1_fwd_eval(P<const float>(a2), P<const float>(w), P<const float>(b), M,
                               P<float>(h), key, keep, S(s));
    check_launch();
  });
  k.def("fc_head_train",
        [](uintptr_t part, uintptr_t b3, uintptr_t w4, uintptr_t b4, uintptr_t labels, int n_local,
           uintptr_t step, int batch, float keep, uint32_t seed, uint32_t rank, float base_lr,
           float decay, uintptr_t hd, uintptr_t dh, uintptr_t dlog, uintptr_t loss_rows,
           uintptr_t lr_out, uintptr_t correct, uintptr_t s, int splits) {
          mnist::launch_fc_head_train(P<const float>(part), P<const float>(b3), P<const float>(w4),
                                      P<const float>(b4), P<const int>(labels), n_local,
                                      P<const long long>(step), batch, keep, seed, rank, base_lr,
                                      decay, P<float>(hd), P<float>(dh), P<float>(dlog),
                                      P<float>(loss_rows), P<float>(lr_out), P<int>(correct), S(s),
                                      nullptr, nullptr, splits);
          check_launch();
        },
        py::arg("part"), py::arg("b3"), py::arg("w4"), py::arg("b4"), py::arg("labels"),
        py::arg("n_local"), py::arg("step"), py::arg("batch"), py::arg("keep"), py::arg("seed"),
        py::arg("rank"), py::arg("base_lr"), py::arg("decay"), py::arg("hd"), py::arg("dh"),
        py::arg("dlog"), py::arg("loss_rows"), py::arg("lr_out"), py::arg("correct"), py::arg("s"),
        py::arg("splits") = 14);
  k.def("fc_head_eval", [](uintptr_t h, uintptr_t w4, uintptr_t b4, uintptr_t labels, int M,
                           uintptr_t logits, uintptr_t errors, uintptr_t s) {
    mnist::launch_fc_head_eval(P<const float>(h), P<const float>(w4), P<const float>(b4),
                               P<const int>(labels), M, P<float>(logits), P<int>(errors), S(s));
    check_launch();
  });
  k.def("fc1_bwd", [](uintptr_t a2, uintptr_t idx2, uintptr_t dh, uintptr_t hd, uintptr_t dlog,
                      uintptr_t w1, int batch, uintptr_t g_w3, uintptr_t g_b3, uintptr_t g_w4,
                      uintptr_t g_b4, uintptr_t dy2, uintptr_t dy2t, uintptr_t s, int roles) {
    mnist::launch_fc1_bwd(P<const float>(a2), P<const uint8_t>(idx2), P<const float>(dh),
                          P<const float>(hd), P<const float>(dlog), P<const float>(w1), batch,
                          P<float>(g_w3), P<float>(g_b3), P<float>(g_w4), P<float>(g_b4),
                          P<float>(dy2), P<float>(dy2t), S(s), roles);
    check_launch();
  }, py::arg("a2"), py::arg("idx2"), py::arg("dh"), py::arg("hd"), py::arg("dlog"), py::arg("w1"),
     py::arg("batch"), py::arg("g_w3"), py::arg("g_b3"), py::arg("g_w4"), py::arg("g_b4"),
     py::arg("dy2"), py::arg("dy2t"), py::arg("stream"), py::arg("roles") = 7);
  k.def("conv2_bwd_data_l2", [](uintptr_t dy2t, uintptr_t w2t, uintptr_t a1, int batch,
                                uintptr_t da1m, uintptr_t s) {
    mnist::launch_conv2_bwd_data_l2(P<const float>(dy2t), P<const float>(w2t), P<const float>(a1),
                                    batch, P<float>(da1m), S(s));
    check_launch();
  });
  k.def("conv2_bwd_filter", [](uintptr_t a1p, uintptr_t dy2, int batch, uintptr_t part2, uintptr_t s) {
    mnist::launch_conv2_bwd_filter(P<const float>(a1p), P<const float>(dy2), batch, P<float>(part2),
                                   S(s));
    check_launch();
  });
  k.def("conv2_bwd_filter_wino", [](uintptr_t a1p, uintptr_t dy2, int batch, uintptr_t part2,
                                    uintptr_t s) {
    mnist::launch_conv2_bwd_filter_wino(P<const float>(a1p), P<const float>(dy2), batch,
                                        P<float>(part2), S(s));
    check_launch();
  });
  k.def("conv2_bwd_filter_wino_prof", [](uintptr_t a1p, uintptr_t dy2, int batch, uintptr_t part2,
                                         uintptr_t prof, uintptr_t s) {
    mnist::launch_conv2_bwd_filter_wino_prof(P<const float>(a1p), P<const float>(dy2), batch,
                                             P<float>(part2), P<unsigned long long>(prof), S(s));
    check_launch();
  });
  k.def("conv1_bwd_filter", [](uintptr_t data, uintptr_t step, int n_local, int batch,
                               uintptr_t da1m, uintptr_t idx1, uintptr_t part1, uintptr_t s) {
    mnist::launch_conv1_bwd_filter(P<const float>(data), P<const long long>(step), n_local, batch,
                                   P<const float>(da1m), P<const uint8_t>(idx1), P<float>(part1),
                                   S(s));
    check_launch();
  });
  k.def("grad_finalize", [](uintptr_t part2, int ns2, uintptr_t part1, int nb1, uintptr_t g_w2,
                            uintptr_t g_b2, uintptr_t g_w1, uintptr_t g_b1, uintptr_t s) {
    mnist::launch_grad_finalize(P<const float>(part2), ns2, P<const float>(part1), nb1,
                                P<float>(g_w2), P<float>(g_b2), P<float>(g_w1), P<float>(g_b1),
                                S(s));
    check_launch();
  });

  auto o = m.def_submodule("optim", "flat-buffer optimizer kernels");
  o.def("sgd_momentum", [](uintptr_t w, uintptr_t g, uintptr_t mom, long long n, long long l2_end,
                           float l2, float momentum, float gscale, uintptr_t lr_ptr,
                           float lr_const, uintptr_t step_ptr, uintptr_t s) {
    optim::launch_sgd_momentum(P<float>(w), P<const float>(g), P<float>(mom), n, l2_end, l2,
                               momentum, gscale, P<const float>(lr_ptr), lr_const,
                               P<long long>(step_ptr), S(s));
    check_launch();
  });
  o.def("to_bf16", [](uintptr_t x, uintptr_t y, long long n, uintptr_t s) {
    optim::launch_to_bf16(P<const float>(x), P<uint16_t>(y), n, S(s));
    check_launch();
  });
  o.def("from_bf16", [](uintptr_t x, uintptr_t y, long long n, uintptr_t s) {
    optim::launch_from_bf16(P<const uint16_t>(x), P<float>(y), n, S(s));
    check_launch();
  });
  o.def("hash_words", [](uintptr_t x, long long n, uintptr_t out, uintptr_t s) {
    optim::launch_hash_words(P<const uint32_t>(x), n, P<unsigned long long>(out), S(s));
    check_launch();
  });
  o.def("scale", [](uintptr_t x, long long n, float a, uintptr_t s) {
    optim::launch_scale(P<float>(x), n, a, S(s));
    check_launch();
  });

  // ------------------------------------------------------- generic ops
  auto g = m.def_submodule("ops", "generic NHWC layer kernels (conv/bn/pool/xent)");
  py::class_<gops::ConvShape>(g, "ConvShape")
      .def(py::init([](int N, int H, int W, int C, int K, int R, int S, int stride, int pad) {
             gops::ConvShape s{N, H, W, C, K, R, S, stride, pad, (H + 2 * pad - R) / stride + 1,
                               (W + 2 * pad - S) / stride + 1};
             return s;
           }))
      .def_readonly("N", &gops::ConvShape::N).def_readonly("H", &gops::ConvShape::H)
      .def_readonly("W", &gops::ConvShape::W).def_readonly("C", &gops::ConvShape::C)
      .def_readonly("K", &gops::ConvShape::K).def_readonly("R", &gops::ConvShape::R)
      .def_readonly("S", &gops::ConvShape::S).def_readonly("stride", &gops::ConvShape::stride)
      .def_readonly("pad", &gops::ConvShape::pad).def_readonly("OH", &gops::ConvShape::OH)
      .def_readonly("OW", &gops::ConvShape::OW);
  py::class_<gops::PoolShape>(g, "PoolShape")
      .def(py::init([](int N, int H, int W, int C, int k, int stride, int pad) {
        gops::PoolShape p{N, H, W, C, k, stride, pad, (H + 2 * pad - k) / stride + 1,
                          (W + 2 * pad - k) / stride + 1};
        return p;
      }))
      .def_readonly("OH", &gops::PoolShape::OH).def_readonly("OW", &gops::PoolShape::OW);
  g.def("conv_bf16_ok", &gops::conv_fwd_bf16_ok);
  // the fp32 tiled forward (its epilogue can write BatchNorm statistics)
  g.def("conv_fwd_tiled_ok", [](const gops::ConvShape& s) {
    return gops::conv_fwd_tiled_ok(s) || gops::conv_fwd_tiled_gather_ok(s);
  });
  g.def("conv_bwd_data_join_ok", &gops::conv_bwd_data_join_ok);
  // tiled-family tile / split plan (labs only; production runs the defaults)
  py::class_<gops::TiledPlan>(g, "TiledPlan")
      .def(py::init<>())
      .def_readwrite("m128_min_bf16", &gops::TiledPlan::m128_min_bf16)
      .def_readwrite("m128_min_f32", &gops::TiledPlan::m128_min_f32)
      .def_readwrite("ksplit_target", &gops::TiledPlan::ksplit_target)
      .def_readwrite("wgsplit_target", &gops::TiledPlan::wgsplit_target)
      .def_readwrite("gcap", &gops::TiledPlan::gcap)
      .def_readwrite("vcap", &gops::TiledPlan::vcap)
      .def_readwrite("wg_xcd", &gops::TiledPlan::wg_xcd)
      .def_readwrite("wg_n64", &gops::TiledPlan::wg_n64)
      .def_readwrite("wg_bk16", &gops::TiledPlan::wg_bk16)
      .def_readwrite("wg_bk16_64", &gops::TiledPlan::wg_bk16_64)
      .def_readwrite("dgrad_fwd", &gops::TiledPlan::dgrad_fwd)
      .def_readwrite("wg64", &gops::TiledPlan::wg64)
      .def_readwrite("halo_f32", &gops::TiledPlan::halo_f32)
      .def_readwrite("halo_f32_wide", &gops::TiledPlan::halo_f32_wide)
      .def_readwrite("halo_f32_bm", &gops::TiledPlan::halo_f32_bm)
      .def_readwrite("halo_f32_ch", &gops::TiledPlan::halo_f32_ch)
      .def_readwrite("halo_f32_small", &gops::TiledPlan::halo_f32_small)
      .def_readwrite("halo_f32_s2", &gops::TiledPlan::halo_f32_s2)
      .def_readwrite("ksplit_s2", &gops::TiledPlan::ksplit_s2);
  g.def("conv3f_ok", &gops::conv3f_ok);
  g.def("get_tiled_plan", []() { return gops::tiled_plan(); });
  g.def("set_tiled_plan", [](const gops::TiledPlan& p) { gops::tiled_plan() = p; });
  g.def("im2col_bf16", [](const gops::ConvShape& s, uintptr_t x, int kp, uintptr_t col,
                          uintptr_t st) {
    gops::im2col_bf16(s, P<const float>(x), kp, P<void>(col), S(st));
    check_launch();
  });
  g.def("conv_fwd_stem_bf16", [](const gops::ConvShape& s1, const gops::ConvShape& si,
                                 uintptr_t x, uintptr_t wtb, uintptr_t yb, uintptr_t st,
                                 uintptr_t stats_part, int stats_rows, uintptr_t stats_shift) {
    const gops::ConvStats cs{P<float>(stats_part), stats_rows, P<const float>(stats_shift)};
    gops::conv_fwd_stem_bf16(s1, si, P<const float>(x), P<const void>(wtb), P<void>(yb), S(st),
                             &cs);
    check_launch();
  }, py::arg("s1"), py::arg("si"), py::arg("x"), py::arg("wtb"), py::arg("yb"), py::arg("st"),
     py::arg("stats_part") = 0, py::arg("stats_rows") = 0, py::arg("stats_shift") = 0);
  g.def("conv_fwd_stats_rows", &gops::conv_fwd_stats_rows, py::arg("shape"),
        py::arg("bf16") = true);
  g.def("conv_fwd_stem_stats_rows", &gops::conv_fwd_stem_stats_rows);
  g.def("conv_bwd_filter_stem_bf16",
        [](const gops::ConvShape& s1, const gops::ConvShape& si, uintptr_t x, uintptr_t dyb,
           uintptr_t ws, uintptr_t dw, uintptr_t st) {
          gops::conv_bwd_filter_stem_bf16(s1, si, P<const float>(x), P<const void>(dyb),
                                          P<float>(ws), P<float>(dw), S(st));
          check_launch();
        });
  g.def("s2d_stem_set_preload", &gops::s2d_stem_set_preload);
  g.def("conv_fwd_s2d_stem_bf16", [](const gops::ConvShape& si, uintptr_t xs, uintptr_t wt8,
                                     uintptr_t yb, uintptr_t st, uintptr_t stats_part,
                                     int stats_rows, uintptr_t stats_shift) {
    const gops::ConvStats cs{P<float>(stats_part), stats_rows, P<const float>(stats_shift)};
    gops::conv_fwd_s2d_stem_bf16(si, P<const void>(xs), P<const void>(wt8), P<void>(yb), S(st),
                                 &cs);
    check_launch();
  }, py::arg("si"), py::arg("xs"), py::arg("wt8"), py::arg("yb"), py::arg("st"),
     py::arg("stats_part") = 0, py::arg("stats_rows") = 0, py::arg("stats_shift") = 0);
  g.def("conv_bwd_filter_s2d_stem_bf16",
        [](const gops::ConvShape& si, uintptr_t xs, uintptr_t dyb, uintptr_t ws, uintptr_t dw8,
           uintptr_t st) {
          gops::conv_bwd_filter_s2d_stem_bf16(si, P<const void>(xs), P<const void>(dyb),
                                              P<float>(ws), P<float>(dw8), S(st));
          check_launch();
        });
  g.def("s2d_stem_ws_floats", &gops::s2d_stem_ws_floats);
  g.def("s2d_stem_input", [](uintptr_t x, int N, int H, int W, int OH, int OW, uintptr_t xs,
                             uintptr_t st) {
    gops::s2d_stem_input(P<const float>(x), N, H, W, OH, OW, P<void>(xs), S(st));
    check_launch();
  });
  g.def("s2d_stem_weight", [](uintptr_t w, int K, uintptr_t wt8, uintptr_t st) {
    gops::s2d_stem_weight(P<const float>(w), K, P<void>(wt8), S(st));
    check_launch();
  });
  g.def("s2d_stem_wgrad", [](uintptr_t dw8, int K, uintptr_t gw, uintptr_t st) {
    gops::s2d_stem_wgrad(P<const float>(dw8), K, P<float>(gw), S(st));
    check_launch();
  });
  g.def("to_bf16", [](uintptr_t x, uintptr_t y, long long n, uintptr_t st) {
    gops::to_bf16(P<const float>(x), P<void>(y), n, S(st));
    check_launch();
  });
  g.def("conv_fwd", [](const gops::ConvShape& s, uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y,
                       bool relu, uintptr_t ws, uintptr_t st, bool bf16, uintptr_t xb,
                       uintptr_t wtb, uintptr_t yb, uintptr_t stats_part, int stats_rows,
                       uintptr_t stats_shift) {
    const gops::ConvStats cs{P<float>(stats_part), stats_rows, P<const float>(stats_shift)};
    gops::conv_fwd(s, P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), relu,
                   P<float>(ws), S(st), bf16, P<const void>(xb), P<const void>(wtb), P<void>(yb),
                   &cs);
    check_launch();
  }, py::arg("s"), py::arg("x"), py::arg("w"), py::arg("b"), py::arg("y"), py::arg("relu"),
     py::arg("ws"), py::arg("st"), py::arg("bf16") = false, py::arg("xb") = 0, py::arg("wtb") = 0,
     py::arg("yb") = 0, py::arg("stats_part") = 0, py::arg("stats_rows") = 0,
     py::arg("stats_shift") = 0);
  g.def("conv_bwd_data_stats_rows", &gops::conv_bwd_data_stats_rows);
  g.def("conv_bwd_data", [](const gops::ConvShape& s, uintptr_t dy, uintptr_t w, uintptr_t dx,
                            uintptr_t ws, uintptr_t st, bool bf16, uintptr_t dyb, uintptr_t addend,
                            uintptr_t wtb, uintptr_t bstats_part, int bstats_rows, uintptr_t bn_x,
                            uintptr_t bn_y, uintptr_t bn_mean, uintptr_t bn_rstd, bool bn_relu) {
    const gops::BnBwdStats bb{P<float>(bstats_part), bstats_rows, P<const void>(bn_x),
                              P<const void>(bn_y), P<const float>(bn_mean),
                              P<const float>(bn_rstd), bn_relu ? 1 : 0};
    gops::conv_bwd_data(s, P<const float>(dy), P<const float>(w), P<float>(dx), P<float>(ws), S(st),
                        bf16, P<const void>(dyb), P<const float>(addend), P<const void>(wtb), &bb);
    check_launch();
  }, py::arg("s"), py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("ws"), py::arg("st"),
     py::arg("bf16") = false, py::arg("dyb") = 0, py::arg("addend") = 0, py::arg("wtb") = 0,
     py::arg("bstats_part") = 0, py::arg("bstats_rows") = 0, py::arg("bn_x") = 0,
     py::arg("bn_y") = 0, py::arg("bn_mean") = 0, py::arg("bn_rstd") = 0,
     py::arg("bn_relu") = false);
  g.def("stem_weight_bf16", [](uintptr_t w, int R, int sc, int seg, int kp, int K, uintptr_t out,
                               uintptr_t st) {
    gops::stem_weight_bf16(P<const float>(w), R, sc, seg, kp, K, P<void>(out), S(st));
    check_launch();
  });
  g.def("stem_wgrad", [](uintptr_t gpad, int R, int sc, int seg, int K, uintptr_t gw, uintptr_t st) {
    gops::stem_wgrad(P<const float>(gpad), R, sc, seg, K, P<float>(gw), S(st));
    check_launch();
  });
  g.def("softmax_rows", [](uintptr_t x, uintptr_t y, int M, int N, uintptr_t st) {
    gops::softmax_rows(P<const float>(x), P<float>(y), M, N, S(st));
    check_launch();
  });
  g.def("wcvt_blocks", &gops::wcvt_blocks);
  g.def("sgd_wcvt", [](uintptr_t w, uintptr_t gr, uintptr_t mom, float momentum, float gscale,
                       float l2, uintptr_t lr, uintptr_t step, uintptr_t jobs, int njobs,
                       long long conv_blocks, uintptr_t ranges, int nranges,
                       long long range_blocks, uintptr_t st) {
    gops::sgd_wcvt(P<float>(w), P<const float>(gr), P<float>(mom), momentum, gscale, l2,
                   P<const float>(lr), P<long long>(step), P<const long long>(jobs), njobs,
                   conv_blocks, P<const long long>(ranges), nranges, range_blocks, S(st));
    check_launch();
  });
  g.def("wcvt_batch", [](uintptr_t jobs, int njobs, long long nblocks, uintptr_t st) {
    gops::wcvt_batch(P<const long long>(jobs), njobs, nblocks, S(st));
    check_launch();
  });
  g.def("conv_ws_floats", &gops::conv_ws_floats);
  g.def("conv_filter_splits", &gops::conv_filter_splits);
  g.def("conv_bwd_filter", [](const gops::ConvShape& s, uintptr_t x, uintptr_t dy, uintptr_t part,
                              uintptr_t dw, uintptr_t st, bool bf16, uintptr_t xb, uintptr_t dyb) {
    gops::conv_bwd_filter(s, P<const float>(x), P<const float>(dy), P<float>(part), P<float>(dw),
                          S(st), bf16, P<const void>(xb), P<const void>(dyb));
    check_launch();
  }, py::arg("s"), py::arg("x"), py::arg("dy"), py::arg("part"), py::arg("dw"), py::arg("st"),
     py::arg("bf16") = false, py::arg("xb") = 0, py::arg("dyb") = 0);
  g.def("colsum2", [](uintptr_t a, uintptr_t b, long long rows, int C, uintptr_t s1, uintptr_t s2,
                      int mode, uintptr_t ws, uintptr_t st) {
    gops::colsum2(P<const float>(a), P<const float>(b), rows, C, P<float>(s1), P<float>(s2), mode,
                  P<float>(ws), S(st));
    check_launch();
  });
  g.def("bn_set_fused", &gops::bn_set_fused);
  g.def("bn_fused_error", &gops::bn_fused_error);
  g.def("bn_set_fused_blocks_per_cu", &gops::bn_set_fused_blocks_per_cu);
  g.def("gsync_barrier_us", &gops::gsync_barrier_us);
  g.def("bn_fused_grid_cap", &gops::bn_fused_grid_cap);
  g.def("bn_fwd_partials", [](uintptr_t part, int nrows, uintptr_t shift, uintptr_t x, long long rows,
                              int C, uintptr_t gm, uintptr_t bt, uintptr_t res, uintptr_t y,
                              uintptr_t mean, uintptr_t rstd, float eps, float momentum, bool relu,
                              uintptr_t rmean, uintptr_t rvar, uintptr_t st, uintptr_t yb,
                              bool x_bf16) {
    gops::bn_fwd_partials(P<const float>(part), nrows, P<const float>(shift), P<const void>(x), rows, C,
                          P<const float>(gm), P<const float>(bt), P<const float>(res), P<float>(y),
                          P<float>(mean), P<float>(rstd), eps, momentum, relu, P<float>(rmean),
                          P<float>(rvar), S(st), P<void>(yb), x_bf16);
    check_launch();
  });
  g.def("chan_reduce_ok", &gops::chan_reduce_ok);
  g.def("chan_reduce_ws_floats", &gops::chan_reduce_ws_floats);
  g.def("bn_fwd", [](uintptr_t x, long long rows, int C, uintptr_t gm, uintptr_t bt, uintptr_t res,
                     uintptr_t y, uintptr_t mean, uintptr_t rstd, uintptr_t ws, float eps,
                     float momentum, bool relu, bool training, uintptr_t rmean, uintptr_t rvar,
                     uintptr_t st, uintptr_t yb, bool x_bf16) {
    gops::bn_fwd(P<const void>(x), rows, C, P<const float>(gm), P<const float>(bt),
                 P<const float>(res), P<float>(y), P<float>(mean), P<float>(rstd), P<float>(ws), eps,
                 momentum, relu, training, P<float>(rmean), P<float>(rvar), S(st), P<void>(yb),
                 x_bf16);
    check_launch();
  }, py::arg("x"), py::arg("rows"), py::arg("C"), py::arg("g"), py::arg("b"), py::arg("res"),
     py::arg("y"), py::arg("mean"), py::arg("rstd"), py::arg("ws"), py::arg("eps"),
     py::arg("momentum"), py::arg("relu"), py::arg("training"), py::arg("rmean"), py::arg("rvar"),
     py::arg("st"), py::arg("yb") = 0, py::arg("x_bf16") = false);
  g.def("bn_bwd", [](uintptr_t x, uintptr_t dy, uintptr_t y, uintptr_t mean, uintptr_t rstd,
                     uintptr_t gm, long long rows, int C, bool relu, uintptr_t ws, uintptr_t dg,
                     uintptr_t db, uintptr_t dx, uintptr_t dres, uintptr_t st, uintptr_t dxb,
                     bool x_bf16, bool y_bf16) {
    gops::bn_bwd(P<const void>(x), P<const float>(dy), P<const void>(y), P<const float>(mean),
                 P<const float>(rstd), P<const float>(gm), rows, C, relu, P<float>(ws), P<float>(dg),
                 P<float>(db), P<float>(dx), P<float>(dres), S(st), P<void>(dxb), x_bf16, y_bf16);
    check_launch();
  }, py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("mean"), py::arg("rstd"), py::arg("g"),
     py::arg("rows"), py::arg("C"), py::arg("relu"), py::arg("ws"), py::arg("dg"), py::arg("db"),
     py::arg("dx"), py::arg("dres"), py::arg("st"), py::arg("dxb") = 0, py::arg("x_bf16") = false,
     py::arg("y_bf16") = false);
  g.def("bn_bwd_partials", [](uintptr_t part, int nrows, uintptr_t x, uintptr_t dy, uintptr_t y,
                              uintptr_t mean, uintptr_t rstd, uintptr_t gm, long long rows, int C,
                              bool relu, uintptr_t dg, uintptr_t db, uintptr_t dx, uintptr_t dres,
                              uintptr_t st, uintptr_t dxb) {
    gops::bn_bwd_partials(P<const float>(part), nrows, P<const void>(x), P<const float>(dy),
                          P<const void>(y), P<const float>(mean), P<const float>(rstd),
                          P<const float>(gm), rows, C, relu, P<float>(dg), P<float>(db), P<float>(dx),
                          P<float>(dres), S(st), P<void>(dxb));
    check_launch();
  });
  g.def("maxpool_fwd", [](const gops::PoolShape& p, uintptr_t x, uintptr_t y, uintptr_t arg, uintptr_t st) {
    gops::maxpool_fwd(p, P<const float>(x), P<float>(y), P<int>(arg), S(st));
    check_launch();
  });
  g.def("maxpool_b16_ok", &gops::maxpool_b16_ok);
  g.def("maxpool_fwd_u8", [](const gops::PoolShape& p, uintptr_t x, uintptr_t y, uintptr_t arg,
                             uintptr_t st) {
    gops::maxpool_fwd_u8(p, P<const float>(x), P<float>(y), P<uint8_t>(arg), S(st));
    check_launch();
  });
  g.def("maxpool_fwd_b16", [](const gops::PoolShape& p, uintptr_t xb, uintptr_t y, uintptr_t yb,
                              uintptr_t arg, uintptr_t st) {
    gops::maxpool_fwd_b16(p, P<const void>(xb), P<float>(y), P<void>(yb), P<uint8_t>(arg), S(st));
    check_launch();
  });
  g.def("maxpool_bwd_b8", [](const gops::PoolShape& p, uintptr_t dy, uintptr_t arg, uintptr_t dx,
                             uintptr_t st) {
    gops::maxpool_bwd_b8(p, P<const float>(dy), P<const uint8_t>(arg), P<float>(dx), S(st));
    check_launch();
  });
  g.def("maxpool_bwd", [](const gops::PoolShape& p, uintptr_t dy, uintptr_t arg, uintptr_t dx, uintptr_t st) {
    gops::maxpool_bwd(p, P<const float>(dy), P<const int>(arg), P<float>(dx), S(st));
    check_launch();
  });
  g.def("avgpool_fwd", [](uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t st) {
    gops::avgpool_fwd(P<const float>(x), P<float>(y), N, HW, C, S(st));
    check_launch();
  });
  g.def("avgpool_bwd", [](uintptr_t dy, uintptr_t dx, int N, int HW, int C, uintptr_t st) {
    gops::avgpool_bwd(P<const float>(dy), P<float>(dx), N, HW, C, S(st));
    check_launch();
  });
  g.def("xent", [](uintptr_t logits, uintptr_t labels, int B, int C, uintptr_t loss_rows,
                   uintptr_t dlogits, uintptr_t correct, uintptr_t st) {
    gops::xent(P<const float>(logits), P<const int>(labels), B, C, P<float>(loss_rows),
               P<float>(dlogits), P<int>(correct), S(st));
    check_launch();
  });
  g.def("xent_mean", [](uintptr_t logits, uintptr_t labels, int B, int C, uintptr_t loss_rows,
                        uintptr_t dlogits, uintptr_t mean, uintptr_t correct, uintptr_t st) {
    gops::xent_mean(P<const float>(logits), P<const int>(labels), B, C, P<float>(loss_rows),
                    P<float>(dlogits), P<float>(mean), P<int>(correct), S(st));
    check_launch();
  });
  g.def("linear_fwd", [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y, int M, int K, int N,
                         bool relu, uintptr_t st) {
    gops::linear_fwd(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), M, K, N,
                     relu, S(st));
    check_launch();
  });
  g.def("linear_bwd", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t dy, uintptr_t dw,
                         uintptr_t db, uintptr_t dx, int M, int K, int N, bool relu, uintptr_t st) {
    gops::linear_bwd(P<const float>(x), P<const float>(w), P<const float>(y), P<const float>(dy),
                     P<float>(dw), P<float>(db), P<float>(dx), M, K, N, relu, S(st));
    check_launch();
  });
  g.def("relu_bwd", [](uintptr_t dy, uintptr_t y, uintptr_t dx, long long n, uintptr_t st) {
    gops::relu_bwd(P<const float>(dy), P<const float>(y), P<float>(dx), n, S(st));
    check_launch();
  });
  g.def("lr_from_step", [](uintptr_t step, int n_local, int batch, float base, float decay,
                           uintptr_t lr, uintptr_t st) {
    gops::lr_from_step(P<const long long>(step), n_local, batch, base, decay, P<float>(lr), S(st));
    check_launch();
  });
  g.def("gather_batch", [](uintptr_t data, uintptr_t labels, uintptr_t step, int n_local, int batch,
                           long long row_elems, uintptr_t xb, uintptr_t yb, uintptr_t st,
                           float lr_base, float lr_decay, uintptr_t lr_out) {
    gops::gather_batch(P<const float>(data), P<const int>(labels), P<const long long>(step), n_local,
                       batch, row_elems, P<float>(xb), P<int>(yb), S(st), lr_base, lr_decay,
                       P<float>(lr_out));
    check_launch();
  }, py::arg("data"), py::arg("labels"), py::arg("step"), py::arg("n_local"), py::arg("batch"),
     py::arg("row_elems"), py::arg("xb"), py::arg("yb"), py::arg("st"), py::arg("lr_base") = 0.f,
     py::arg("lr_decay") = 1.f, py::arg("lr_out") = 0);

  // ------------------------------------------------------------ executor
  py::class_<MnistPtrs>(m, "MnistPtrs")
      .def(py::init<>())
#define RW(f) .def_readwrite(#f, &MnistPtrs::f)
          RW(train_x) RW(train_y) RW(n_local) RW(batch) RW(params) RW(grads) RW(mom) RW(total)
              RW(l2_end) RW(bucket1) RW(off_w4) RW(off_b4) RW(off_w3) RW(off_b3) RW(off_w2)
                  RW(off_b2) RW(off_w1) RW(off_b1) RW(step) RW(lr) RW(correct) RW(a1) RW(idx1)
                      RW(a2) RW(idx2) RW(fc1_part) RW(hd) RW(dh) RW(dlog) RW(loss_rows) RW(dy2)
                          RW(da1m) RW(part2) RW(part1) RW(w2t) RW(a1pf) RW(keep_prob) RW(base_lr) RW(lr_decay)
                              RW(l2) RW(momentum) RW(seed) RW(rank) RW(world) RW(bf16) RW(grad_bf16) RW(gb16)
                                  RW(a1p) RW(a1t) RW(a2h) RW(a2t) RW(dy2p) RW(dy2t) RW(dh16)
                                      RW(dht16) RW(w1b) RW(w1t) RW(w2tb) RW(w2b) RW(a2_all)
                                          RW(dh_all) RW(hd_all) RW(dlog_all) RW(fac_ranks)
                                              RW(wino) RW(wino_u) RW(wino_ud) RW(a2ft);
#undef RW

  py::class_<Collective>(m, "Collective")
      .def_property_readonly("rank", &Collective::rank)
      .def_property_readonly("size", &Collective::size)
      .def("all_reduce",
           [](Collective& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
              uintptr_t s) { c.all_reduce(P<void>(send), P<void>(recv), count, dtype, op, S(s)); })
      .def("all_gather",
           [](Collective& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t s) {
             c.all_gather(P<void>(send), P<void>(recv), count, dtype, S(s));
           })
      .def("reduce_scatter",
           [](Collective& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
              uintptr_t s) { c.reduce_scatter(P<void>(send), P<void>(recv), count, dtype, op, S(s)); });

  py::class_<EmuComm, Collective>(m, "EmuComm")
      .def(py::init<int, int, double, double, int>(), py::arg("nranks"), py::arg("rank"),
           py::arg("lat_us"), py::arg("busbw_gbps"), py::arg("blocks"))
      .def("all_reduce_us", &EmuComm::all_reduce_us)
      .def("gather_us", &EmuComm::gather_us);

  py::class_<PyComm, Collective>(m, "PyComm")
      .def(py::init<int, int, py::function>(), py::arg("nranks"), py::arg("rank"), py::arg("fn"));

  py::class_<ShmComm, Collective>(m, "ShmComm")
      .def(py::init<const std::string&, bool, int, int, size_t, double, bool>(), py::arg("path"),
           py::arg("create"), py::arg("nranks"), py::arg("rank"), py::arg("capacity"),
           py::arg("timeout_s"), py::arg("pinned") = true)
      .def("run_host",
           [](ShmComm& c, int kind, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
              int root) { c.run_host(kind, P<void>(send), P<void>(recv), count, dtype, op, root); },
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast",
           [](ShmComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int root,
              uintptr_t s) { c.broadcast(P<void>(send), P<void>(recv), count, dtype, root, S(s)); })
      .def("reduce",
           [](ShmComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
              int root, uintptr_t s) {
             c.reduce(P<void>(send), P<void>(recv), count, dtype, op, root, S(s));
           })
      .def("async_error", &ShmComm::async_error)
      .def("error_message", &ShmComm::error_message)
      .def("abort", &ShmComm::abort)
      .def("unlink_path", &ShmComm::unlink_path)
      .def_property_readonly("capacity", &ShmComm::capacity)
      .def_property_readonly("completed", &ShmComm::completed)
      .def_property_readonly("host_progress", &ShmComm::host_progress);
  m.attr("ShmComm").attr("AR") = (int)ShmComm::AR;
  m.attr("ShmComm").attr("AG") = (int)ShmComm::AG;
  m.attr("ShmComm").attr("RS") = (int)ShmComm::RS;
  m.attr("ShmComm").attr("BC") = (int)ShmComm::BC;
  m.attr("ShmComm").attr("RD") = (int)ShmComm::RD;

  py::class_<XgmiComm, Collective>(m, "XgmiComm")
      .def(py::init<int, int, bool, double, double, double>(), py::arg("nranks"), py::arg("rank"),
           py::arg("emulate") = false, py::arg("lat_us") = 0.0, py::arg("link_gbps") = 0.0,
           py::arg("timeout_s") = 10.0)
      .def("flags_handle", [](const XgmiComm& c) { return py::bytes(c.flags_handle()); })
      .def("open_flags", [](XgmiComm& c, int r, py::bytes h) { c.open_flags(r, std::string(h)); })
      .def("export_buffer",
           [](const XgmiComm& c, uintptr_t p, size_t bytes) {
             auto hb = c.export_buffer(p, bytes);
             return py::make_tuple(py::bytes(hb.first), hb.second);
           })
      .def("open_buffer",
           [](XgmiComm& c, uintptr_t local, size_t bytes, int r, py::bytes h, size_t off) {
             c.open_buffer(local, bytes, r, std::string(h), off);
           })
      .def("emulate_buffer", &XgmiComm::emulate_buffer)
      .def("ready", &XgmiComm::ready)
      .def("set_lean", &XgmiComm::set_lean)
      .def("emulate_dead_rank", &XgmiComm::emulate_dead_rank)
      .def("inject_skip_peer", &XgmiComm::inject_skip_peer)
      .def_property_readonly("skip_peer", &XgmiComm::skip_peer)
      .def_property_readonly("link_ticks_per_mib", &XgmiComm::link_ticks_per_mib)
      .def("emulate_fill_peer", &XgmiComm::emulate_fill_peer)
      .def_property_readonly("lean", &XgmiComm::lean)
      .def("registered", [](const XgmiComm& c, uintptr_t p, size_t bytes) {
        return c.registered(reinterpret_cast<const void*>(p), bytes);
      })
      .def("peer_ptr", [](const XgmiComm& c, uintptr_t p, int r) {
        return reinterpret_cast<uintptr_t>(c.peer_ptr(reinterpret_cast<const void*>(p), r));
      })
      .def("error", &XgmiComm::error)
      .def("clear_error", &XgmiComm::clear_error)
      .def("gather_segments",
           [](XgmiComm& c, uintptr_t p, size_t count, uintptr_t s) {
             c.gather_segments(reinterpret_cast<void*>(p), count, S(s));
             check_launch();
           })
      .def_property_readonly("emulated", &XgmiComm::emulated);

  py::class_<RcclComm, Collective>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int nranks, int rank) {
             std::string s = uid;
             return new RcclComm(std::vector<char>(s.begin(), s.end()), nranks, rank);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"))
      .def_static("load", &RcclComm::load)
      .def_static("loaded", &RcclComm::loaded)
      .def_static("version", &RcclComm::version)
      .def_static("unique_id",
                  []() {
                    auto v = RcclComm::unique_id();
                    return py::bytes(v.data(), v.size());
                  })
      .def("broadcast",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int root,
              uintptr_t s) { c.broadcast(P<void>(send), P<void>(recv), count, dtype, root, S(s)); })
      .def("reduce",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op,
              int root, uintptr_t s) {
             c.reduce(P<void>(send), P<void>(recv), count, dtype, op, root, S(s));
           })
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("destroy", &RcclComm::destroy)
      .def("async_error", &RcclComm::async_error, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("comm_count", &RcclComm::comm_count)
      .def_static("error_string", &RcclComm::error_string);

  // ------------------------------------------------------------ LeNet-5
  py::class_<lenet::Offsets>(m, "LenetOffsets")
      .def(py::init<>())
#define RWO(f) .def_readwrite(#f, &lenet::Offsets::f)
          RWO(c1w) RWO(c1b) RWO(c2w) RWO(c2b) RWO(f1w) RWO(f1b) RWO(f2w) RWO(f2b) RWO(f3w) RWO(f3b);
#undef RWO
  py::class_<LenetPtrs>(m, "LenetPtrs")
      .def(py::init<>())
#define RWL(f) .def_readwrite(#f, &LenetPtrs::f)
          RWL(train_x) RWL(train_y) RWL(n_local) RWL(batch) RWL(params) RWL(grads) RWL(mom)
              RWL(total) RWL(off) RWL(step) RWL(lr) RWL(correct) RWL(acts) RWL(deltas) RWL(convp)
                  RWL(loss_rows) RWL(base_lr) RWL(lr_decay) RWL(momentum) RWL(grad_bf16) RWL(gb16)
                  RWL(xrecv) RWL(xgrads2) RWL(xdone);
#undef RWL
  m.def("lenet_buffer_floats", [](int batch) {
    return py::make_tuple(lenet::acts_floats(batch), lenet::deltas_floats(batch),
                          lenet::convp_floats(batch));
  });
  m.def("lenet_image_phase", [](const LenetPtrs& p, int stop, uintptr_t s) {
    lenet::ImageArgs a{};
    a.x = P<const float>(p.train_x);
    a.y = P<const int>(p.train_y);
    a.n_local = p.n_local;
    a.batch = p.batch;
    a.step = P<const long long>(p.step);
    a.params = P<const float>(p.params);
    a.off = p.off;
    a.acts = P<float>(p.acts);
    a.deltas = P<float>(p.deltas);
    a.convp = P<float>(p.convp);
    a.loss_rows = P<float>(p.loss_rows);
    a.lr_out = P<float>(p.lr);
    a.stop_phase = stop;
    lenet::launch_image_train(a, S(s));
    check_launch();
  });
  py::class_<LenetExecutor>(m, "LenetExecutor")
      .def(py::init<const LenetPtrs&>())
      .def("set_xgmi_mode", &LenetExecutor::set_xgmi_mode)
      .def_property_readonly("xgmi_mode", &LenetExecutor::xgmi_mode)
      .def("train_step",
           [](LenetExecutor& e, uintptr_t s, Collective* comm) {
             e.train_step(S(s), comm);
             check_launch();
           },
           py::arg("stream"), py::arg("comm") = nullptr)
      .def("forward_backward",
           [](LenetExecutor& e, uintptr_t s) {
             e.forward_backward(S(s));
             check_launch();
           })
      .def_static("eval_chunk", [](const LenetPtrs& p, uintptr_t x, uintptr_t y, int M,
                                   uintptr_t logits, uintptr_t errors, uintptr_t s) {
        LenetExecutor::eval_chunk(p, x, y, M, logits, errors, S(s));
        check_launch();
      });

  py::class_<MnistExecutor>(m, "MnistExecutor")
      .def(py::init<const MnistPtrs&>())
      .def("train_step",
           [](MnistExecutor& e, uintptr_t s, Collective* comm, uintptr_t cs, Collective* comm2) {
             e.train_step(S(s), comm, S(cs), comm2);
             check_launch();
           },
           py::arg("stream"), py::arg("comm") = nullptr, py::arg("comm_stream") = 0,
           py::arg("comm2") = nullptr)
      .def("set_schedule", &MnistExecutor::set_schedule)
      .def("set_fc_sgd_rounds", &MnistExecutor::set_fc_sgd_rounds)
      .def("refresh_shadows", [](MnistExecutor& e, uintptr_t s) { e.refresh_shadows(S(s)); })
      .def_property_readonly("schedule", &MnistExecutor::schedule)
      .def("sharded_ok", &MnistExecutor::sharded_ok)
      .def("factors_ok", &MnistExecutor::factors_ok)
      .def("defer_ok", &MnistExecutor::defer_ok)
      .def("set_defer_split", &MnistExecutor::set_defer_split)
      .def("set_xgmi", &MnistExecutor::set_xgmi, py::keep_alive<1, 2>())
      .def("xgmi_ok", &MnistExecutor::xgmi_ok)
      .def("xgmi_fac_ok", &MnistExecutor::xgmi_fac_ok)
      .def("set_xgmi_fc_in_bwd", &MnistExecutor::set_xgmi_fc_in_bwd)
      .def("set_xgmi_xconv", &MnistExecutor::set_xgmi_xconv)
      .def_property_readonly("defer_split", &MnistExecutor::defer_split)
      .def("join", [](MnistExecutor& e, uintptr_t s) { e.join(S(s)); })
      .def("gather_optimizer_state",
           [](MnistExecutor& e, uintptr_t s, Collective* comm, uintptr_t cs) {
             e.gather_optimizer_state(S(s), comm, S(cs));
             check_launch();
           })
      .def("forward_backward",
           [](MnistExecutor& e, uintptr_t s) {
             e.forward_backward(S(s));
             check_launch();
           })
      .def("sgd",
           [](MnistExecutor& e, uintptr_t s, float gscale) {
             e.sgd(S(s), gscale);
             check_launch();
           })
      .def_static("eval_chunk",
                  [](const MnistPtrs& p, uintptr_t x, uintptr_t y, int M, uintptr_t a1,
                     uintptr_t a2, uintptr_t h, uintptr_t logits, uintptr_t errors, float keep,
                     uint32_t key, uintptr_t s) {
                    MnistExecutor::eval_chunk(p, x, y, M, a1, a2, h, logits, errors, keep, key,
                                              S(s));
                    check_launch();
                  });

  m.attr("MnistExecutor").attr("SCHED_BUCKETS") = (int)MnistExecutor::SCHED_BUCKETS;
  m.attr("MnistExecutor").attr("SCHED_SHARDED_FC") = (int)MnistExecutor::SCHED_SHARDED_FC;
  m.attr("MnistExecutor").attr("SCHED_SPLIT") = (int)MnistExecutor::SCHED_SPLIT;
  m.attr("MnistExecutor").attr("SCHED_FACTORS") = (int)MnistExecutor::SCHED_FACTORS;
  m.attr("MnistExecutor").attr("SCHED_SERIAL") = (int)MnistExecutor::SCHED_SERIAL;
  m.attr("MnistExecutor").attr("SCHED_DEFER") = (int)MnistExecutor::SCHED_DEFER;
  m.attr("MnistExecutor").attr("SCHED_XGMI") = (int)MnistExecutor::SCHED_XGMI;
  m.attr("MnistExecutor").attr("SCHED_XGMI_STEP") = (int)MnistExecutor::SCHED_XGMI_STEP;
  m.attr("MnistExecutor").attr("SCHED_XGMI_FAC") = (int)MnistExecutor::SCHED_XGMI_FAC;

  // ----------------------------------------------------------------- IDX
  // pre-uploads an instantiated graph (torch CUDAGraph.raw_cuda_graph_exec())
  // so its first replay does not pay the upload inside a timed region
  m.def("graph_upload", [](uintptr_t exec, uintptr_t s) {
    const hipError_t e = hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), S(s));
    if (e != hipSuccess) throw std::runtime_error(std::string("hipGraphUpload: ") + hipGetErrorString(e));
  });
  // stream-ordering events between two streams of this device: no timing and a
  // device-scope release (a default event's system-scope fence writes back and
  // invalidates the caches under the work that follows it)
  m.def("event_create", []() -> uintptr_t {
    hipEvent_t e = nullptr;
    hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice),
           "hipEventCreateWithFlags");
    return reinterpret_cast<uintptr_t>(e);
  });
  m.def("event_destroy", [](uintptr_t e) {
    hip_ok(hipEventDestroy(reinterpret_cast<hipEvent_t>(e)), "hipEventDestroy");
  });
  m.def("event_record", [](uintptr_t e, uintptr_t s) {
    hip_ok(hipEventRecord(reinterpret_cast<hipEvent_t>(e), S(s)), "hipEventRecord");
  });
  m.def("stream_wait_event", [](uintptr_t s, uintptr_t e) {
    hip_ok(hipStreamWaitEvent(S(s), reinterpret_cast<hipEvent_t>(e), 0), "hipStreamWaitEvent");
  });
  // nodes captured so far on a capturing stream (-1: not capturing); the
  // segmented step capture (runtime/generic_engine.py) never ends an empty segment
  m.def("capture_node_count", [](uintptr_t s) -> long long {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    hipError_t e = hipStreamGetCaptureInfo_v2(S(s), &st, &id, &g, &deps, &nd);
    if (e != hipSuccess)
      throw std::runtime_error(std::string("hipStreamGetCaptureInfo_v2: ") + hipGetErrorString(e));
    if (st != hipStreamCaptureStatusActive || g == nullptr) return -1;
    size_t n = 0;
    e = hipGraphGetNodes(g, nullptr, &n);
    if (e != hipSuccess) throw std::runtime_error(std::string("hipGraphGetNodes: ") + hipGetErrorString(e));
    return (long long)n;
  });
  // uploads an instantiated graph's executable to the device ahead of its
  // first launch (bench.py: out of the timed window)
  m.def("graph_upload", [](uintptr_t exec, uintptr_t s) {
    hip_ok(hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), S(s)), "hipGraphUpload");
  });
  m.def("idx_header", [](const std::string& path) {
    IdxHeader h = idx_header(path);
    return py::make_tuple(h.magic, h.dims);
  });
  m.def("idx_read_u8", [](const std::string& path, long long start, long long stop) {
    IdxHeader h;
    std::vector<uint8_t> v = idx_read_u8(path, start, stop, &h);
    std::vector<py::ssize_t> shape{(py::ssize_t)(stop - start)};
    for (size_t i = 1; i < h.dims.size(); ++i) shape.push_back(h.dims[i]);
    py::array_t<uint8_t> a(shape);
    std::memcpy(a.mutable_data(), v.data(), v.size());
    return a;
  });
  m.def("idx_read_images_f32",
        [](const std::string& path, long long start, long long stop, float depth) {
          IdxHeader h = idx_header(path);
          std::vector<float> v = idx_read_images_f32(path, start, stop, depth);
          std::vector<py::ssize_t> shape{(py::ssize_t)(stop - start)};
          for (size_t i = 1; i < h.dims.size(); ++i) shape.push_back(h.dims[i]);
          shape.push_back(1);  // NHWC channel dim, like extract_data
          py::array_t<float> a(shape);
          std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(float));
          return a;
        });
}
