// Probe: read rate of the cross-attention's byte pattern (R rows x H heads,
// each (row, head) streams its K rows then its V rows: 1500 x 128 B each) under
// load-issue variants: loads in flight per lane, non-temporal loads, workgroup
// size, and the share of the chip the grid covers. Time per launch from a
// hipGraph of 32 launches over two alternating buffer copies (no MALL reuse).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = (uint32_t)i * 2654435761u ^ seed;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// one workgroup per (row, head) unit; NT threads; U 16-B loads in flight per lane
template <int NT, int U, bool NTL>
__global__ __launch_bounds__(NT) void stream_kernel(const uint4* __restrict__ K,
                                                    const uint4* __restrict__ V, int n16,
                                                    int units, float* out) {
  uint32_t acc = 0;
  for (int unit = blockIdx.x; unit < units; unit += gridDim.x) {
    const long base = (long)unit * n16;
    for (int pass = 0; pass < 2; ++pass) {
      const uint4* p = (pass ? V : K) + base;
      for (int i = threadIdx.x; i < n16; i += NT * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const u32x4* a = reinterpret_cast<const u32x4*>(p + min(i + u * NT, n16 - 1));
          v[u] = NTL ? __builtin_nontemporal_load(a) : *a;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u][0] ^ v[u][3];
      }
    }
  }
  if (acc == 0x12345u) out[threadIdx.x] = (float)acc;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 32;
  const int H = 20, Lc = 1500, L = 32, reps = 10;
  const size_t unit_elems = (size_t)Lc * 64;  // f16 per (row, head)
  const size_t elems = (size_t)R * H * unit_elems;
  uint16_t *ck, *cv;
  CK(hipMalloc(&ck, 2 * elems * 2));
  CK(hipMalloc(&cv, 2 * elems * 2));
  fill_kernel<<<4096, 256>>>((uint32_t*)ck, elems, 7);
  fill_kernel<<<4096, 256>>>((uint32_t*)cv, elems, 8);
  float* out;
  CK(hipMalloc(&out, 4096));
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n16 = (int)(unit_elems * 2 / 16), units = R * H;
  const double bytes = 2.0 * elems * 2;
  struct Op {
    std::string name;
    std::function<void(int)> f;
  };
  auto K = [&](int l) { return (const uint4*)(ck + (l & 1) * elems); };
  auto Vp = [&](int l) { return (const uint4*)(cv + (l & 1) * elems); };
#define OP(NT, U, NTL, G) \
  {#NT " thr, " #U " in flight, nt=" #NTL ", grid " #G, [&](int l) { stream_kernel<NT, U, NTL><<<(G) ? (G) : units, NT, 0, s>>>(K(l), Vp(l), n16, units, out); }}
  std::vector<Op> ops = {
      OP(256, 8, false, 0),  OP(256, 8, true, 0),   OP(256, 16, false, 0), OP(256, 16, true, 0),
      OP(256, 4, false, 0),  OP(512, 8, false, 0),  OP(512, 8, true, 0),   OP(128, 16, false, 0),
      OP(256, 8, false, 512), OP(256, 8, false, 256), OP(256, 16, true, 512), OP(512, 8, true, 256),
  };
  printf("R=%d: %zu MB per launch\n", R, (size_t)(bytes / 1e6));
  for (auto& op : ops) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 0; l < L; ++l) op.f(l);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps / L;
    printf("%-44s %8.2f us  %6.2f TB/s\n", op.name.c_str(), us, bytes / us / 1e6);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
