// Does a 16-byte global load from a 2-byte-aligned address return the right
// bytes on gfx950, and what does it cost vs aligned?  (bf16 conv filter-grad
// operand fetch with a tap shift along the contiguous axis.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef short s8 __attribute__((ext_vector_type(8)));
__global__ void rd(const short* p, int shift, int n, int iters, long long* out) {
  long long acc = 0;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    const s8 v = *(const s8*)(p + (size_t)((i * 8 + it * 7919 * 8) % n) + shift);
    for (int j = 0; j < 8; ++j) acc += v[j] * (j + 1);
  }
  out[i] = acc;
}
__global__ void one(const short* p, int shift, s8* o) { o[threadIdx.x] = *(const s8*)(p + threadIdx.x * 8 + shift); }
int main() {
  const int n = 1 << 24;
  std::vector<short> h(n + 64);
  for (int i = 0; i < n + 64; ++i) h[i] = (short)(i * 31 + 7);
  short* d; s8* o; long long* out;
  hipMalloc(&d, (n + 64) * 2); hipMalloc(&o, 64 * 16); hipMalloc(&out, 1 << 24);
  hipMemcpy(d, h.data(), (n + 64) * 2, hipMemcpyHostToDevice);
  int bad = 0;
  for (int sh = 0; sh < 8; ++sh) {
    one<<<1, 64>>>(d, sh, o);
    std::vector<short> r(64 * 8);
    hipMemcpy(r.data(), o, 64 * 16, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 8; ++j) if (r[l * 8 + j] != h[l * 8 + sh + j]) bad++;
  }
  printf("unaligned b128 correctness: %s (%d bad)\n", bad ? "WRONG" : "OK", bad);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int sh : {0, 1, 2, 4}) {
    rd<<<2048, 256>>>(d, sh, n - 64, 16, out);
    hipEventRecord(a);
    for (int k = 0; k < 10; ++k) rd<<<2048, 256>>>(d, sh, n - 64, 64, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("shift %d: %.3f ms (%.1f GB/s)\n", sh, ms / 10, 2048.0 * 256 * 64 * 16 / (ms / 10 * 1e6));
  }
  return 0;
}
