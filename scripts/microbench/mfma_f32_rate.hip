// Calibration microbenchmark: achievable v_mfma_f32_32x32x2_f32 rate on gfx950
// for the dependency / occupancy shapes the MNIST conv kernels use.
//   hipcc --offload-arch=gfx950 -O3 mfma_f32_rate.hip -o mfma_f32_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC, bool LDS, bool GLOB = false, bool RND = false>
__global__ void k(float* out, int iters, const float* __restrict__ gb) {
  __shared__ float s[4096];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += blockDim.x)
    s[i] = RND ? (float)((i * 2654435761u) >> 8) * 5.96e-8f - 0.5f : (float)(i % 7) * 0.01f;
  __syncthreads();
  f32x16 acc[NACC];
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float a = lane * 0.001f, b = lane * 0.002f;
  int off = (threadIdx.x * 33) & 4095;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int j = 0; j < NACC; ++j) {
        float aa = LDS ? s[(off + u * 2 + j * 64) & 4095] : a;
        float bb = GLOB ? gb[((it * 8 + u) * 64 + lane) & 65535] : b;
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(aa, bb, acc[j], 0, 0, 0);
      }
    }
  }
  float t = 0.f;
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) t += acc[j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int NACC, bool LDS, bool GLOB = false, bool RND = false>
void run(const char* name, int threads, float* out, const float* gb) {
  const int blocks = 256, iters = 200;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) k<NACC, LDS, GLOB, RND><<<blocks, threads>>>(out, iters, gb);
  hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) k<NACC, LDS, GLOB, RND><<<blocks, threads>>>(out, iters, gb);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double mfmas = (double)blocks * (threads / 64) * iters * 8 * NACC * reps;
  double tf = mfmas * 4096.0 / (ms * 1e-3) / 1e12;
  double cyc_per = (ms * 1e-3) * 2.4e9 / (mfmas / 1024.0);
  printf("%-34s waves/SIMD=%d  %8.1f TFLOP/s  (%.1f cyc/MFMA/SIMD @2.4GHz)\n", name, threads / 256, tf,
         cyc_per);
}

int main() {
  float *out, *gb;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  hipMalloc(&gb, 65536 * sizeof(float));
  {
    float* h = (float*)malloc(65536 * 4);
    for (int i = 0; i < 65536; ++i) h[i] = (float)((i * 2654435761u) >> 8) * 5.96e-8f - 0.5f;
    hipMemcpy(gb, h, 65536 * 4, hipMemcpyHostToDevice);
    free(h);
  }
  run<1, false>("1 acc chain, regs", 256, out, gb);
  run<1, false>("1 acc chain, regs", 512, out, gb);
  run<4, false>("4 acc chains, regs", 256, out, gb);
  run<1, true>("1 acc chain, LDS operand", 512, out, gb);
  run<1, true, false, true>("1 chain, LDS operand, random", 512, out, gb);
  run<1, true, true, true>("1 chain, LDS A + L2 B, random", 512, out, gb);
  run<1, true, true, true>("1 chain, LDS A + L2 B, random", 768, out, gb);
  run<2, true, true, true>("2 chains, LDS A + L2 B, random", 512, out, gb);
  hipFree(out);
  return 0;
}
