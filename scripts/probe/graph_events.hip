// Probe: can HIP events recorded inside a captured graph be timed?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(float* x, int n) { int i = blockIdx.x * 256 + threadIdx.x; if (i < n) for (int k = 0; k < 200; ++k) x[i] = x[i] * 0.999f + 1.0f; }
int main() {
  float* x; hipMalloc(&x, 1 << 24);
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int mode = 0; mode < 3; ++mode) {
    for (int flags = 0; flags < 2; ++flags) {
      hipEvent_t a, b;
      if (flags) { hipEventCreateWithFlags(&a, hipEventDefault); hipEventCreateWithFlags(&b, hipEventDefault); }
      else { hipEventCreate(&a); hipEventCreate(&b); }
      hipGraph_t g; hipGraphExec_t e;
      hipStreamCaptureMode m = mode == 0 ? hipStreamCaptureModeGlobal : mode == 1 ? hipStreamCaptureModeThreadLocal : hipStreamCaptureModeRelaxed;
      hipError_t r0 = hipStreamBeginCapture(s, m);
      spin<<<1024, 256, 0, s>>>(x, 1 << 18);
      hipError_t r1 = hipEventRecord(a, s);
      spin<<<1024, 256, 0, s>>>(x, 1 << 18);
      hipError_t r2 = hipEventRecord(b, s);
      hipError_t r3 = hipStreamEndCapture(s, &g);
      hipError_t r4 = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
      for (int it = 0; it < 3; ++it) {
        hipError_t r5 = hipGraphLaunch(e, s);
        hipStreamSynchronize(s);
        float ms = -1; hipError_t r6 = hipEventElapsedTime(&ms, a, b);
        printf("mode %d flags %d it %d: begin %d rec %d %d end %d inst %d launch %d elapsed %d (%s) ms=%f\n", mode, flags, it, r0, r1, r2, r3, r4, r5, r6, hipGetErrorString(r6), ms);
      }
      // alternative: explicit event record nodes added to the graph
      hipGraphExecDestroy(e); hipGraphDestroy(g);
      hipGraph_t g2; hipGraphCreate(&g2, 0);
      hipGraphNode_t n1, n2, n3;
      hipKernelNodeParams kp = {}; void* args[] = {&x, nullptr}; int n = 1 << 18; args[1] = &n;
      kp.func = (void*)spin; kp.gridDim = dim3(1024); kp.blockDim = dim3(256); kp.kernelParams = args;
      hipGraphAddEventRecordNode(&n1, g2, nullptr, 0, a);
      hipGraphAddKernelNode(&n2, g2, &n1, 1, &kp);
      hipGraphAddEventRecordNode(&n3, g2, &n2, 1, b);
      hipGraphExec_t e2; hipError_t q = hipGraphInstantiate(&e2, g2, nullptr, nullptr, 0);
      hipGraphLaunch(e2, s); hipStreamSynchronize(s);
      float ms = -1; hipError_t r6 = hipEventElapsedTime(&ms, a, b);
      printf("  explicit nodes: inst %d elapsed %d (%s) ms=%f\n", q, r6, hipGetErrorString(r6), ms);
      hipGraphExecDestroy(e2); hipGraphDestroy(g2);
      // eager record after graph launch (bracketing the whole graph)
      hipEventRecord(a, s); spin<<<1024, 256, 0, s>>>(x, 1 << 18); hipEventRecord(b, s); hipStreamSynchronize(s);
      r6 = hipEventElapsedTime(&ms, a, b);
      printf("  eager: elapsed %d ms=%f\n", r6, ms);
      hipEventDestroy(a); hipEventDestroy(b);
    }
  }
  return 0;
}
