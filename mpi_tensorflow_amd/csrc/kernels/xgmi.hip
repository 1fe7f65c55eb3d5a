// Generic xGMI peer-to-peer kernels (csrc/xgmi_comm.h, kernels/xgmi.h).
#include <stdexcept>
#include <string>

#include "common.h"
#include "xgmi.h"

namespace xgmi {

constexpr int kAllReduceUnroll = 2;  // float4s in flight per thread per rank

template <int NT>
__global__ __launch_bounds__(NT) void allreduce_kernel(const AllReduceArgs a) {
  __shared__ unsigned ep;
  const Sync& s = a.s;
  const int n = s.nranks, me = s.rank, tid = threadIdx.x;
  const bool sgd = a.mom != nullptr;
  const bool reduce_only = a.out != nullptr;
  // every peer-visible byte through system-scope loads / stores (xgmi.h)
  Rsrc br[kMaxRanks], wr[kMaxRanks];
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r)
    if (r < n) {
      br[r] = rsrc(a.buf[r], a.n4 * 16);
      if (sgd) wr[r] = rsrc(a.w[r], a.n4 * 16);
    }
  const unsigned e = next_epoch(s, &ep);
  barrier(s, 0, e, /*release=*/true);  // the buffer comes from earlier kernels
  const float lr = sgd ? *a.lr : 0.f;
  const long long lo = (long long)blockIdx.x * a.per4;
  const long long hi = lo + a.per4 < a.seg4 ? lo + a.per4 : a.seg4;
  long long t0 = now_ticks();
  if (!a.gather_only) {
    const long long base = (long long)me * a.seg4;
    for (long long i0 = lo + tid; i0 < hi; i0 += NT * kAllReduceUnroll) {
      float4 acc[kAllReduceUnroll];
      float4 v[kMaxRanks][kAllReduceUnroll];
      // every rank's loads in flight at once (one round trip per unroll)
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r)
#pragma unroll
        for (int u = 0; u < kAllReduceUnroll; ++u) {
          const long long i = base + i0 + NT * u;
          v[r][u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (contributes(s, r) && i0 + NT * u < hi && i < a.n4)
            v[r][u] = ld4_sys(br[r], (unsigned)(i * 16));
        }
#pragma unroll
      for (int u = 0; u < kAllReduceUnroll; ++u) {
        acc[u] = v[0][u];  // rank order 0..N-1, as a host reduction in rank order
#pragma unroll
        for (int r = 1; r < kMaxRanks; ++r)
          if (r < n) {
            acc[u].x += v[r][u].x;
            acc[u].y += v[r][u].y;
            acc[u].z += v[r][u].z;
            acc[u].w += v[r][u].w;
          }
        const long long i = base + i0 + NT * u;
        if (!(i0 + NT * u < hi && i < a.n4)) continue;
        if (sgd) {  // optim::sgd_momentum_flat_kernel's expression forms
          float4* M4 = reinterpret_cast<float4*>(a.mom);
          float4 wv = reinterpret_cast<const float4*>(a.w[me])[i], gv = acc[u], mv = M4[i];
          const float lc = i < a.l2_end4 ? a.l2 : 0.f;
          gv.x = __builtin_fmaf(lc, wv.x, gv.x * a.gscale);
          gv.y = __builtin_fmaf(lc, wv.y, gv.y * a.gscale);
          gv.z = __builtin_fmaf(lc, wv.z, gv.z * a.gscale);
          gv.w = __builtin_fmaf(lc, wv.w, gv.w * a.gscale);
          mv.x = a.momentum * mv.x + gv.x;
          mv.y = a.momentum * mv.y + gv.y;
          mv.z = a.momentum * mv.z + gv.z;
          mv.w = a.momentum * mv.w + gv.w;
          wv.x -= lr * mv.x;
          wv.y -= lr * mv.y;
          wv.z -= lr * mv.z;
          wv.w -= lr * mv.w;
          st4_sys(wr[me], (unsigned)(i * 16), wv);
          M4[i] = mv;
        } else if (reduce_only) {
          reinterpret_cast<float4*>(a.out)[i - base] = acc[u];  // local: no peer reads it
        } else {
          st4_sys(br[me], (unsigned)(i * 16), acc[u]);
        }
      }
    }
    link_floor(s, t0, a.link_bytes);
  }
  // reduce-scatter: this barrier is the "done reading" one (the peers may
  // rewrite their send buffers after the kernel); gather-only: every segment
  // was final at the arrival barrier, no second one
  if (!a.gather_only) barrier(s, 1, e, false);
  if (reduce_only) return;
  t0 = now_ticks();
  float* const* out = sgd ? a.w : a.buf;  // phase 2 gathers the updated params
  float4* O4 = reinterpret_cast<float4*>(out[me]);
  // every other rank's slice with all loads in flight before the stores (one
  // round trip per unroll, not one per rank)
  for (long long i0 = lo + tid; i0 < hi; i0 += NT * kAllReduceUnroll) {
    float4 v[kMaxRanks][kAllReduceUnroll];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < kAllReduceUnroll; ++u) {
        const long long i = (long long)r * a.seg4 + i0 + NT * u;
        if (r < n && r != me && i0 + NT * u < hi && i < a.n4)
          v[r][u] = ld4_sys(sgd ? wr[r] : br[r], (unsigned)(i * 16));
      }
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
#pragma unroll
      for (int u = 0; u < kAllReduceUnroll; ++u) {
        const long long i = (long long)r * a.seg4 + i0 + NT * u;
        if (r < n && r != me && i0 + NT * u < hi && i < a.n4) O4[i] = v[r][u];
      }
  }
  if (a.step && blockIdx.x == 0 && tid == 0) *a.step += 1;
  link_floor(s, t0, a.link_bytes);
  // closing "done reading" barrier: a plain all-reduce's peers rewrite the
  // buffers this gather reads (their next grads) right after the kernel.  The
  // fused SGD's gather reads the peers' PARAMS, which a peer rewrites only in
  // its next call's phase 1 - after that call's arrival barrier, which this
  // rank reaches only once this kernel (gather included) is done: no barrier
  if (!sgd) barrier(s, 2, e, false);
}

void launch_allreduce(const AllReduceArgs& a, int blocks, int nt, hipStream_t st) {
  if (blocks < 1 || blocks > kMaxBlocks)
    throw std::runtime_error("xgmi all_reduce: grid of " + std::to_string(blocks) + " blocks");
  if (a.s.nranks < 1 || a.s.nranks > kMaxRanks || !a.s.flags || !a.s.epoch || !a.s.error)
    throw std::runtime_error("xgmi all_reduce: communicator not set up");
  for (int r = 0; r < a.s.nranks; ++r)
    if (!a.buf[r] || (!a.s.emulate && !a.s.peer_flags[r]))
      throw std::runtime_error("xgmi all_reduce: rank " + std::to_string(r) + " not mapped");
  if ((long long)blocks * a.per4 < a.seg4 || a.per4 % nt)
    throw std::runtime_error("xgmi all_reduce: grid does not cover the segment");
  if (nt == 64)
    allreduce_kernel<64><<<blocks, 64, 0, st>>>(a);
  else if (nt == 256)
    allreduce_kernel<256><<<blocks, 256, 0, st>>>(a);
  else
    throw std::runtime_error("xgmi all_reduce: 64 or 256 threads a block");
}

// (xgmi.h OneShotArgs) one float4 of every rank a thread, 256 threads a block
__global__ __launch_bounds__(256) void oneshot_sgd_kernel(const OneShotArgs a) {
  __shared__ unsigned ep;
  const Sync& s = a.s;
  const int n = s.nranks, tid = threadIdx.x;
  const long long st = *a.step;  // every block reads it before its completion ticket
  const unsigned slot = (unsigned)((st & 1) * a.n4 * 16);
  Rsrc gr[kMaxRanks];
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r)
    if (r < n) gr[r] = rsrc(a.g[r], 2 * a.n4 * 16);
  const unsigned e = next_epoch(s, &ep);
  barrier(s, 0, e, /*release=*/true);  // the grads come from the update launch
  const long long t0 = now_ticks();
  const long long i = (long long)blockIdx.x * 256 + tid;
  if (i < a.n4) {
    float4 v[kMaxRanks];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      v[r] = r < n ? ld4_peer(s, r, gr[r], slot + (unsigned)(i * 16)) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4* W4 = reinterpret_cast<float4*>(a.w);
    float4* M4 = reinterpret_cast<float4*>(a.mom);
    float4 wv = W4[i], mv = M4[i];
    const float lr = *a.lr;
    float4 gv = v[0];  // rank order 0..N-1
#pragma unroll
    for (int r = 1; r < kMaxRanks; ++r)
      if (r < n) {
        gv.x += v[r].x;
        gv.y += v[r].y;
        gv.z += v[r].z;
        gv.w += v[r].w;
      }
    // optim::sgd_momentum_flat_kernel's expression forms (l2 = 0)
    gv.x = __builtin_fmaf(0.f, wv.x, gv.x * a.gscale);
    gv.y = __builtin_fmaf(0.f, wv.y, gv.y * a.gscale);
    gv.z = __builtin_fmaf(0.f, wv.z, gv.z * a.gscale);
    gv.w = __builtin_fmaf(0.f, wv.w, gv.w * a.gscale);
    mv.x = a.momentum * mv.x + gv.x;
    mv.y = a.momentum * mv.y + gv.y;
    mv.z = a.momentum * mv.z + gv.z;
    mv.w = a.momentum * mv.w + gv.w;
    wv.x -= lr * mv.x;
    wv.y -= lr * mv.y;
    wv.z -= lr * mv.z;
    wv.w -= lr * mv.w;
    W4[i] = wv;
    M4[i] = mv;
  }
  link_floor(s, t0, a.n4 * 16);
  __syncthreads();
  if (tid == 0) {
    const unsigned t =
        __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *a.step = st + 1;
    }
  }
}

void launch_oneshot_sgd(const OneShotArgs& a, hipStream_t st) {
  if (a.s.nranks < 1 || a.s.nranks > kMaxRanks || !a.s.flags || !a.s.epoch || !a.s.error)
    throw std::runtime_error("xgmi one-shot sgd: communicator not set up");
  for (int r = 0; r < a.s.nranks; ++r)
    if (!a.g[r] || (!a.s.emulate && !a.s.peer_flags[r]))
      throw std::runtime_error("xgmi one-shot sgd: rank " + std::to_string(r) + " not mapped");
  if (!a.w || !a.mom || !a.lr || !a.step || !a.done || a.n4 <= 0 || 2 * a.n4 * 16 >= (1LL << 32))
    throw std::runtime_error("xgmi one-shot sgd: arguments");
  const long long blocks = (a.n4 + 255) / 256;
  if (blocks > kMaxBlocks) throw std::runtime_error("xgmi one-shot sgd: buffer too large");
  oneshot_sgd_kernel<<<(int)blocks, 256, 0, st>>>(a);
}

// The dispatch order the barrier argument above relies on (xgmi.h): block b
// goes to XCD b mod 8, and each XCD starts its blocks in increasing id order.
// Each block's first thread records its XCD (hardware register XCC_ID), a
// ticket from its XCD's counter and its start clock, then holds its CU for
// spin_ticks, so a grid several times the resident capacity exercises the
// dispatcher's queue.  out[3 b] = XCD, out[3 b + 1] = ticket, out[3 b + 2] =
// start (100 MHz); ctr: >= 16 x 16 zeroed words.
__global__ __launch_bounds__(64) void dispatch_probe_kernel(unsigned* ctr,
                                                            unsigned long long* out,
                                                            long long spin_ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = now_ticks();
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  x &= 0xfu;
  const unsigned t =
      __hip_atomic_fetch_add(ctr + 16 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  out[3 * blockIdx.x] = x;
  out[3 * blockIdx.x + 1] = t;
  out[3 * blockIdx.x + 2] = (unsigned long long)t0;
  while (now_ticks() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(2);
}

void launch_dispatch_probe(unsigned* ctr, unsigned long long* out, int blocks,
                           long long spin_ticks, hipStream_t st) {
  if (blocks < 1 || blocks > (1 << 20) || spin_ticks < 0 || spin_ticks > 100000)
    throw std::runtime_error("xgmi dispatch probe: 1..2^20 blocks, spin <= 1 ms");
  dispatch_probe_kernel<<<blocks, 64, 0, st>>>(ctr, out, spin_ticks);
}

}  // namespace xgmi
