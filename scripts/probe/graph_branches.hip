// Probe: do independent branches of a captured hipGraph run concurrently?
// Two spin kernels (~50 us each, 8 WGs) on forked streams inside one capture;
// replayed graph time ~50 us => concurrent, ~100 us => serialized.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(long long cycles, int* sink) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) atomicAdd(sink, 1);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  int* sink;
  CK(hipMalloc(&sink, 4));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, j1, j2, a, b;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const long long cyc = 100000;  // ~50 us at ~2 GHz shader clock (clock64 rate differs; relative only)
  // single kernel time
  spin<<<8, 64, 0, s0>>>(cyc, sink);
  CK(hipStreamSynchronize(s0));
  CK(hipEventRecord(a, s0));
  for (int i = 0; i < 10; ++i) spin<<<8, 64, 0, s0>>>(cyc, sink);
  CK(hipEventRecord(b, s0));
  CK(hipEventSynchronize(b));
  float one;
  CK(hipEventElapsedTime(&one, a, b));
  // graph with two parallel branches, each: 4 spins in sequence
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(fork, s0));
  CK(hipStreamWaitEvent(s1, fork, 0));
  CK(hipStreamWaitEvent(s2, fork, 0));
  for (int i = 0; i < 4; ++i) spin<<<8, 64, 0, s1>>>(cyc, sink);
  for (int i = 0; i < 4; ++i) spin<<<8, 64, 0, s2>>>(cyc, sink);
  CK(hipEventRecord(j1, s1));
  CK(hipEventRecord(j2, s2));
  CK(hipStreamWaitEvent(s0, j1, 0));
  CK(hipStreamWaitEvent(s0, j2, 0));
  CK(hipStreamEndCapture(s0, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s0));
  CK(hipStreamSynchronize(s0));
  CK(hipEventRecord(a, s0));
  for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s0));
  CK(hipEventRecord(b, s0));
  CK(hipEventSynchronize(b));
  float gt;
  CK(hipEventElapsedTime(&gt, a, b));
  printf("single spin kernel: %.1f us; graph (2 branches x 4 spins): %.1f us per replay "
         "(serial would be ~%.1f, concurrent ~%.1f)\n",
         one * 100.0f, gt * 100.0f, 8 * one * 100.0f, 4 * one * 100.0f);
  return 0;
}
