// Flat-buffer momentum SGD (replaces TF ApplyMomentum x8 + AssignAdd + the
// LR scalar ops of /root/reference/mpipy.py:59-66).
//
// One memory-bound pass over the whole flat parameter buffer, 16 B per lane:
//   g   = grad * gscale (+ l2 * w on the L2-regularised FC prefix, mpipy.py:57)
//   acc = momentum * acc + g            (TF1 ApplyMomentum, non-Nesterov)
//   w  -= lr * acc
// lr comes from the device (written by the fc head from the device step
// counter), so the kernel is graph-replayable; one thread bumps the step.
#include <stdexcept>

#include "common.h"
#include "mnist.h"

namespace optim {

__global__ __launch_bounds__(256) void sgd_momentum_flat_kernel(
    float4* __restrict__ w, const float4* __restrict__ g, float4* __restrict__ mom, long long n4,
    long long l2_end4, float l2, float momentum, float gscale, const float* lr_ptr,
    float lr_const, long long* step_ptr) {
  const float lr = lr_ptr ? *lr_ptr : lr_const;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 wv = w[i], gv = g[i], mv = mom[i];
    const float lc = i < l2_end4 ? l2 : 0.f;
    // explicit fma (mnist_shared.h sgd4 rounds identically)
    gv.x = __builtin_fmaf(lc, wv.x, gv.x * gscale);
    gv.y = __builtin_fmaf(lc, wv.y, gv.y * gscale);
    gv.z = __builtin_fmaf(lc, wv.z, gv.z * gscale);
    gv.w = __builtin_fmaf(lc, wv.w, gv.w * gscale);
    mv.x = momentum * mv.x + gv.x;
    mv.y = momentum * mv.y + gv.y;
    mv.z = momentum * mv.z + gv.z;
    mv.w = momentum * mv.w + gv.w;
    wv.x -= lr * mv.x;
    wv.y -= lr * mv.y;
    wv.z -= lr * mv.z;
    wv.w -= lr * mv.w;
    w[i] = wv;
    mom[i] = mv;
  }
  if (step_ptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ptr += 1;
}

__global__ __launch_bounds__(256) void scale_kernel(float4* __restrict__ x, long long n4, float a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = x[i];
    v.x *= a;
    v.y *= a;
    v.z *= a;
    v.w *= a;
    x[i] = v;
  }
}

// bf16 gradient wire (--grad-comm-dtype bf16): fp32 <-> bf16 copies of a
// gradient bucket around its collective (round to nearest even)
__global__ __launch_bounds__(256) void to_bf16_kernel(const float4* __restrict__ x,
                                                     uint2* __restrict__ y, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = x[i];
    __bf16 b[4] = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    y[i] = __builtin_bit_cast(uint2, b);
  }
}

__global__ __launch_bounds__(256) void from_bf16_kernel(const uint2* __restrict__ x,
                                                       float4* __restrict__ y, long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const uint2 u = x[i];
    y[i] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
}

// Replica fingerprint: sum over i (mod 2^64) of splitmix64((i << 32) | word_i)
// of the raw 32-bit words.  Position-keyed and bitwise, so any differing bit,
// sign flip or permutation changes it; integer addition makes the sum
// independent of the reduction order (one number per rank, compared across
// ranks; parallel/sync.py:replica_hash has the identical host version).
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void hash_words_kernel(const uint32_t* __restrict__ x,
                                                        long long n,
                                                        unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[4];
  unsigned long long acc = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    acc += splitmix64(((unsigned long long)i << 32) | x[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}

static inline int grid_for(long long n4) {
  long long b = (n4 + 255) / 256;
  return (int)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
}

void launch_sgd_momentum(float* w, const float* g, float* mom, long long n, long long l2_end,
                         float l2, float momentum, float gscale, const float* lr_ptr,
                         float lr_const, long long* step_ptr, hipStream_t s) {
  const long long n4 = n / 4;
  sgd_momentum_flat_kernel<<<grid_for(n4), 256, 0, s>>>(
      reinterpret_cast<float4*>(w), reinterpret_cast<const float4*>(g),
      reinterpret_cast<float4*>(mom), n4, l2_end / 4, l2, momentum, gscale, lr_ptr, lr_const,
      step_ptr);
}

void launch_to_bf16(const float* x, uint16_t* y, long long n, hipStream_t s) {
  if (n % 4) throw std::runtime_error("to_bf16: n % 4 != 0");
  to_bf16_kernel<<<grid_for(n / 4), 256, 0, s>>>(reinterpret_cast<const float4*>(x),
                                                 reinterpret_cast<uint2*>(y), n / 4);
}

void launch_from_bf16(const uint16_t* x, float* y, long long n, hipStream_t s) {
  if (n % 4) throw std::runtime_error("from_bf16: n % 4 != 0");
  from_bf16_kernel<<<grid_for(n / 4), 256, 0, s>>>(reinterpret_cast<const uint2*>(x),
                                                   reinterpret_cast<float4*>(y), n / 4);
}

void launch_hash_words(const uint32_t* x, long long n, unsigned long long* out, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned long long), s));
  hash_words_kernel<<<grid_for(n / 4 + 1), 256, 0, s>>>(x, n, out);
}

void launch_scale(float* x, long long n, float a, hipStream_t s) {
  const long long n4 = n / 4;
  scale_kernel<<<grid_for(n4), 256, 0, s>>>(reinterpret_cast<float4*>(x), n4, a);
}

}  // namespace optim
