// Grid-barrier cost on MI355X for a persistent decode-layer kernel at B = 1
// ("measure barrier cost at 8 / 16 / 32 / 64 workgroups
// on one XCD first"). Measurement probe, not product code.
//
// Workgroups are placed round-robin over the 8 XCDs by id (id % 8), so a grid
// of 8 n workgroups in which only ids with id % 8 == 0 stay puts n workgroups
// on XCD 0 (the others exit at once). Each iteration is one hand-off of a
// B = 1 decode layer phase: every workgroup stores its slice of the
// activation vector (SLICE floats, write-through `sc1` stores), drains them,
// arrives on a counter (one lane, agent-scope atomic add), polls the counter
// (`sc1` loads, bounded spin), then reads the WHOLE vector (n x SLICE floats,
// `sc1` loads) as the next phase's GEMV input. Reported per iteration from
// HIP events over ITERS iterations; the same with placement over all XCDs.
//
// Usage: xcd_barrier_probe [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define HIPC(x)                                                             \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr int SLICE = 64;  // floats per workgroup per phase (n x 64: d = 512 at n = 8)
constexpr long SPIN_MAX = 1L << 22;

template <bool ONE_XCD>
__global__ __launch_bounds__(256) void barrier_probe(int n, int iters, unsigned* counter,
                                                     float* vec, float* sink, int* err) {
  int a = blockIdx.x;
  if (ONE_XCD) {
    if (blockIdx.x % 8) return;
    a = blockIdx.x / 8;
  }
  const int tid = threadIdx.x;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float* cur = vec + (long)(it & 1) * n * SLICE;
    // this workgroup's slice of the phase output (write-through)
    if (tid < SLICE)
      __hip_atomic_store(cur + a * SLICE + tid, acc + (float)(it + a), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = (unsigned)(it + 1) * (unsigned)n;
      long spins = 0;
      while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_MAX) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    // the whole vector as the next phase's input
    for (int i = tid; i < n * SLICE; i += 256)
      acc += __hip_atomic_load(cur + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) sink[a] = acc;
}

// the launch-boundary alternative: one tiny kernel per phase (graph-captured)
__global__ __launch_bounds__(256) void phase_kernel(const float* in, float* out, int n) {
  const int tid = threadIdx.x;
  float acc = 0.0f;
  for (int i = tid; i < n * SLICE; i += 256) acc += in[i];
  if (tid < SLICE) out[blockIdx.x * SLICE + tid] = acc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  unsigned* counter;
  float *vec, *sink;
  int* err;
  HIPC(hipMalloc(&counter, 4));
  HIPC(hipMalloc(&vec, 2L * 256 * SLICE * 4));
  HIPC(hipMalloc(&sink, 256 * 4));
  HIPC(hipMalloc(&err, 4));
  hipStream_t st;
  HIPC(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  HIPC(hipEventCreate(&e0));
  HIPC(hipEventCreate(&e1));
  printf("| placement | workgroups | us per hand-off (store slice, barrier, read vector) |\n|---|---|---|\n");
  auto run = [&](bool one, int n) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      HIPC(hipMemsetAsync(counter, 0, 4, st));
      HIPC(hipMemsetAsync(err, 0, 4, st));
      HIPC(hipEventRecord(e0, st));
      if (one)
        barrier_probe<true><<<8 * n, 256, 0, st>>>(n, iters, counter, vec, sink, err);
      else
        barrier_probe<false><<<n, 256, 0, st>>>(n, iters, counter, vec, sink, err);
      HIPC(hipEventRecord(e1, st));
      HIPC(hipStreamSynchronize(st));
      int he = 0;
      HIPC(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
      if (he) {
        printf("| %s | %d | spin limit hit |\n", one ? "one XCD" : "all XCDs", n);
        return;
      }
      float ms = 0;
      HIPC(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("| %s | %d | %.2f |\n", one ? "one XCD" : "all XCDs", n, best * 1e3f / iters);
    fflush(stdout);
  };
  for (int n : {8, 16, 32, 64}) run(true, n);
  for (int n : {8, 16, 32, 64, 128, 256}) run(false, n);
  // launch-boundary reference: a graph of `G` dependent tiny kernels
  for (int n : {8, 32}) {
    const int G = 200;
    hipGraph_t g;
    hipGraphExec_t ge;
    HIPC(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < G; ++i)
      phase_kernel<<<n, 256, 0, st>>>(vec + (long)(i & 1) * n * SLICE, vec + (long)((i + 1) & 1) * n * SLICE, n);
    HIPC(hipStreamEndCapture(st, &g));
    HIPC(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      HIPC(hipEventRecord(e0, st));
      HIPC(hipGraphLaunch(ge, st));
      HIPC(hipEventRecord(e1, st));
      HIPC(hipStreamSynchronize(st));
      float ms = 0;
      HIPC(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("| launch boundary (graph of %d dependent kernels) | %d | %.2f |\n", G, n, best * 1e3f / G);
    HIPC(hipGraphExecDestroy(ge));
    HIPC(hipGraphDestroy(g));
  }
  return 0;
}
