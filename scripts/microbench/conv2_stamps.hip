// In-kernel phase stamps for conv2_fwd_v3 (diagnostic build only; the shipped
// kernel compiles the stamps out).  Reports per-wave cycles in staging, MFMA
// loop and reduction, the block start skew, and the shader clock.
#define MNIST_STAMPS 1
#include "../../mpi_tensorflow_amd/csrc/kernels/mnist.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

int main() {
  const int B = 64, NB = B * 4, NW = NB * 4;
  float *a1, *w2, *b2, *out, *w2t;
  uint8_t* am;
  unsigned long long* st;
  (void)hipMalloc(&a1, B * 196 * 32 * 4);
  (void)hipMalloc(&w2, 51200 * 4);
  (void)hipMalloc(&b2, 64 * 4);
  (void)hipMalloc(&out, B * 3136 * 4);
  (void)hipMalloc(&w2t, 51200 * 4);
  (void)hipMalloc(&am, B * 3136);
  (void)hipMalloc(&st, NW * 8 * 8);
  std::vector<float> h(B * 196 * 32);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) >> 8) * 5.96e-8f;
  (void)hipMemcpy(a1, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(w2, h.data(), 51200 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(mnist::g_stamps), &st, sizeof(st));
  for (int it = 0; it < 20; ++it)
    mnist::conv2_fwd_v3_kernel<<<NB, 256>>>(a1, B, w2, b2, out, am, w2t);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> s(NW * 8);
  (void)hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
  double stage = 0, mf = 0, red = 0, clk = 0;
  unsigned long long t0 = ~0ull, t1 = 0;
  int n = 0, nk = 0;
  for (int w = 0; w < NW; ++w) {
    unsigned long long* r = &s[w * 8];
    stage += r[1] - r[0];
    mf += r[2] - r[1];
    red += r[3] - r[2];
    if (r[6] > r[5]) {
      clk += (double)(r[3] - r[0]) / (double)(r[6] - r[5]) * 0.1;
      ++nk;
    }
    t0 = std::min(t0, r[0]);
    t1 = std::max(t1, r[0]);
    ++n;
  }
  printf("per wave (cycles): staging %.0f  mfma-loop %.0f  reduce %.0f  | clock %.2f GHz | block start skew %llu cycles\n",
         stage / n, mf / n, red / n, clk / nk, t1 - t0);
  return 0;
}
