// Cross-queue edge cost in hipGraph replay vs eager streams (gfx950).
//
// VERDICT r4 asked for the price of one cross-stream event edge, which the
// MNIST sync schedules pay per step (docs/PERF_NOTES.md: "~10 us per
// join").  Each variant runs G "steps" of tiny one-block kernels that spin
// for T us on the 100 MHz real-time clock, so what is left over T x kernels
// is launch / edge overhead:
//   serial   - k1 -> k2 -> k3 on one stream
//   hop      - k1 (s) -> event -> k2 (s2) -> event -> k3 (s): one fork and
//              one join per step, no concurrency (the edges alone)
//   overlap  - k1 (s) -> fork -> [k2 (s2) || k3 (s)] -> join -> k4 (s)
//   serial4  - k1 -> k2 -> k3 -> k4 on one stream (overlap's baseline)
//   flag     - k1 (s) sets a device flag; k2 (s2) polls it (bounded spin,
//              reports a timeout instead of hanging); the two streams fork
//              and join ONCE per graph, not per step
// Every variant is timed eagerly and as one captured graph of G steps.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/edge_lab scripts/microbench/edge_lab.hip
//   /tmp/edge_lab [T_us=2] [G=25] [reps=40]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void spin_kernel(long long ticks) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// producer: spin, then publish flag[i] = epoch (agent-scope release + store)
__global__ void spin_set_kernel(long long ticks, unsigned* flag, const unsigned* epoch) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(flag, *epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// consumer: wait for flag[i] == epoch (bounded: 50 ms, then count a timeout), spin
__global__ void wait_spin_kernel(long long ticks, const unsigned* flag, const unsigned* epoch,
                                 unsigned* timeouts) {
  if (threadIdx.x == 0) {
    const unsigned want = *epoch;
    const long long tw = (long long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - tw > 5000000) {
        atomicAdd(timeouts, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

__global__ void bump_kernel(unsigned* epoch) { *epoch += 1; }

struct Ctx {
  hipStream_t s, s2;
  hipEvent_t e1, e2;
  long long ticks;
  unsigned *flags, *epoch, *timeouts;
};

static void step(const Ctx& c, int variant, int i) {
  const long long t = c.ticks;
  switch (variant) {
    case 0:  // serial
      for (int k = 0; k < 3; ++k) spin_kernel<<<1, 64, 0, c.s>>>(t);
      break;
    case 1:  // hop
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      CK(hipEventRecord(c.e1, c.s));
      CK(hipStreamWaitEvent(c.s2, c.e1, 0));
      spin_kernel<<<1, 64, 0, c.s2>>>(t);
      CK(hipEventRecord(c.e2, c.s2));
      CK(hipStreamWaitEvent(c.s, c.e2, 0));
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      break;
    case 2:  // overlap
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      CK(hipEventRecord(c.e1, c.s));
      CK(hipStreamWaitEvent(c.s2, c.e1, 0));
      spin_kernel<<<1, 64, 0, c.s2>>>(t);
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      CK(hipEventRecord(c.e2, c.s2));
      CK(hipStreamWaitEvent(c.s, c.e2, 0));
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      break;
    case 3:  // serial4
      for (int k = 0; k < 4; ++k) spin_kernel<<<1, 64, 0, c.s>>>(t);
      break;
    case 4:  // flag (streams forked / joined by the caller around all steps)
      spin_set_kernel<<<1, 64, 0, c.s>>>(t, c.flags + i, c.epoch);
      wait_spin_kernel<<<1, 64, 0, c.s2>>>(t, c.flags + i, c.epoch, c.timeouts);
      spin_kernel<<<1, 64, 0, c.s>>>(t);
      break;
  }
}

static void run_steps(const Ctx& c, int variant, int G) {
  if (variant == 4) {
    bump_kernel<<<1, 1, 0, c.s>>>(c.epoch);
    CK(hipEventRecord(c.e1, c.s));
    CK(hipStreamWaitEvent(c.s2, c.e1, 0));
  }
  for (int i = 0; i < G; ++i) step(c, variant, i);
  if (variant == 4) {
    CK(hipEventRecord(c.e2, c.s2));
    CK(hipStreamWaitEvent(c.s, c.e2, 0));
  }
}

int main(int argc, char** argv) {
  const double T = argc > 1 ? atof(argv[1]) : 2.0;
  const int G = argc > 2 ? atoi(argv[2]) : 25;
  const int reps = argc > 3 ? atoi(argv[3]) : 40;
  Ctx c{};
  CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&c.e1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c.e2, hipEventDisableTiming));
  c.ticks = (long long)(T * 100.0);
  CK(hipMalloc(&c.flags, 4096 * sizeof(unsigned)));
  CK(hipMalloc(&c.epoch, sizeof(unsigned)));
  CK(hipMalloc(&c.timeouts, sizeof(unsigned)));
  CK(hipMemset(c.flags, 0, 4096 * sizeof(unsigned)));
  CK(hipMemset(c.epoch, 0, sizeof(unsigned)));
  CK(hipMemset(c.timeouts, 0, sizeof(unsigned)));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const char* names[] = {"serial3", "hop", "overlap", "serial4", "flag"};
  const int kern[] = {3, 3, 4, 4, 3};
  printf("spin per kernel %.1f us, %d steps per graph, %d reps\n", T, G, reps);
  for (int v = 0; v < 5; ++v) {
    // eager
    run_steps(c, v, G);
    CK(hipStreamSynchronize(c.s));
    CK(hipEventRecord(t0, c.s));
    for (int r = 0; r < reps; ++r) run_steps(c, v, G);
    CK(hipEventRecord(t1, c.s));
    CK(hipEventSynchronize(t1));
    float ms_e = 0.f;
    CK(hipEventElapsedTime(&ms_e, t0, t1));
    // graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(c.s, hipStreamCaptureModeGlobal));
    run_steps(c, v, G);
    CK(hipStreamEndCapture(c.s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, c.s));
    CK(hipStreamSynchronize(c.s));
    CK(hipEventRecord(t0, c.s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, c.s));
    CK(hipEventRecord(t1, c.s));
    CK(hipEventSynchronize(t1));
    float ms_g = 0.f;
    CK(hipEventElapsedTime(&ms_g, t0, t1));
    unsigned to = 0;
    CK(hipMemcpy(&to, c.timeouts, 4, hipMemcpyDeviceToHost));
    const double ue = 1000.0 * ms_e / (reps * G), ug = 1000.0 * ms_g / (reps * G);
    const double crit = (v == 2 ? 3 : kern[v]) * T;  // critical-path spin per step
    printf("%-8s eager %7.2f us/step  graph %7.2f us/step  (spin on the critical path %.1f; "
           "graph overhead %.2f us/step)%s\n",
           names[v], ue, ug, crit, ug - crit, to ? "  FLAG TIMEOUTS" : "");
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
