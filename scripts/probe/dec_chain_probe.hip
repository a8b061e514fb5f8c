// Probe: unprofiled per-launch time of the decode-step GEMM / LayerNorm
// kernels of libmwx.so at large-v3 shapes (R rows, d 1280), each chain
// captured in a hipGraph (32 layers of distinct weights, so the weights stream
// from HBM as in a real decode step) and replayed; time = graph wall / launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include
//        -I../../sentiric-stt-whisper-service_amd/csrc dec_chain_probe.hip
//        -L../../sentiric-stt-whisper-service_amd -lmwx -o dec_chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "kernels.h"

using T = __bf16;
using namespace mwx;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void empty_kernel(float* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1.0f;
}

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * 256ull + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    // bf16 in [-0.03, 0.03): exponent 0x3c (2^-7..), random mantissa / sign
    p[i] = (uint16_t)(((h & 1) << 15) | (0x3c << 7) | ((h >> 1) & 0x7f));
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int d = 1280, L = 32;
  const size_t wq = 3ul * d * d, wd = 1ul * d * d, wf = 4ul * d * d;
  const size_t per_layer = wq + 3 * wd + 2 * wf;  // qkv, o, cq, co, fc1, fc2
  uint16_t* W;
  CK(hipMalloc(&W, per_layer * L * 2));
  fill_kernel<<<4096, 256>>>(W, per_layer * L, 1234);
  auto wl = [&](int l, int which) -> const T* {
    size_t off = per_layer * l;
    const size_t sz[6] = {wq, wd, wd, wd, wf, wf};
    for (int i = 0; i < which; ++i) off += sz[i];
    return reinterpret_cast<const T*>(W + off);
  };
  float *x, *bias, *lnw, *lnb, *slab;
  CK(hipMalloc(&x, (size_t)R * d * 4));
  CK(hipMalloc(&bias, 4 * d * 4));
  CK(hipMalloc(&lnw, d * 4));
  CK(hipMalloc(&lnb, d * 4));
  CK(hipMalloc(&slab, (size_t)8 * R * 3 * d * 4));
  std::vector<float> h(4 * d, 0.01f), ones(d, 1.0f);
  CK(hipMemcpy(bias, h.data(), 4 * d * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(lnw, ones.data(), d * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(lnb, h.data(), d * 4, hipMemcpyHostToDevice));
  std::vector<float> hx((size_t)R * d);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.0f - 1.0f;
  CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  const size_t R64 = (R + 63) / 64 * 64;
  T *od, *ffd, *hd;
  CK(hipMalloc(&od, R64 * d * 2));
  CK(hipMalloc(&ffd, R64 * 4 * d * 2));
  CK(hipMalloc(&hd, R64 * d * 2));
  CK(hipMemset(od, 0, R64 * d * 2));
  CK(hipMemset(ffd, 0, R64 * 4 * d * 2));
  CK(hipMemset(hd, 0, R64 * d * 2));
  int* act;
  CK(hipMalloc(&act, R * 4));
  std::vector<int> ha(R, 1);
  CK(hipMemcpy(act, ha.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  auto ep_slab = [&](int ldc) {
    EpiParams e;
    e.c32 = slab;
    e.ldc = ldc;
    return e;
  };
  auto ep_res = [&]() {
    EpiParams e;
    e.c32 = x;
    e.r32 = x;
    e.ldc = d;
    e.bias = bias;
    e.active = act;
    return e;
  };
  auto ep_gelu = [&]() {
    EpiParams e;
    e.c16 = ffd;
    e.ldc = 4 * d;
    e.bias = bias;
    e.pack_out = true;
    return e;
  };
  struct Op {
    std::string name;
    int launches_per_layer;
    std::function<void(int)> f;
  };
  std::vector<Op> ops = {
      {"empty 512 WG", 1, [&](int) { empty_kernel<<<512, 256, 0, s>>>(nullptr); }},
      {"ln_qkv (gemm_ln QKV)", 1,
       [&](int l) { gemm_ln_launch<T>(EPI_F32, x, lnw, lnb, wl(l, 0), R, 3 * d, d, ep_slab(3 * d), s); }},
      {"ln_cq (gemm_ln d x d)", 1,
       [&](int l) { gemm_ln_launch<T>(EPI_F32, x, lnw, lnb, wl(l, 2), R, d, d, ep_slab(d), s); }},
      {"ln_fc1 (gemm_ln FFN1+GELU)", 1,
       [&](int l) { gemm_ln_launch<T>(EPI_GELU, x, lnw, lnb, wl(l, 4), R, 4 * d, d, ep_gelu(), s); }},
      {"res_o (skinny RES K=d)", 1, [&](int l) { gemm_decode<T>(EPI_RES, od, wl(l, 1), R, d, d, ep_res(), s); }},
      {"res_fc2 (skinny RES K=4d)", 1,
       [&](int l) { gemm_decode<T>(EPI_RES, ffd, wl(l, 5), R, d, 4 * d, ep_res(), s); }},
      {"skinny_fc1 (GELU pack)", 1,
       [&](int l) { gemm_decode<T>(EPI_GELU, hd, wl(l, 4), R, 4 * d, d, ep_gelu(), s); }},
      {"splitk_qkv", 1, [&](int l) { gemm_splitk_partials<T>(hd, wl(l, 0), R, 3 * d, d, slab, s); }},
      {"splitk_o", 1, [&](int l) { gemm_splitk_partials<T>(od, wl(l, 1), R, d, d, slab, s); }},
      {"splitk_fc2", 1, [&](int l) { gemm_splitk_partials<T>(ffd, wl(l, 5), R, d, 4 * d, slab, s); }},
      {"ln_dec (KS 5 slabs)", 1,
       [&](int) { layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias); }},
      {"FUSED layer GEMMs (6 launches)", 6,
       [&](int l) {
         gemm_ln_launch<T>(EPI_F32, x, lnw, lnb, wl(l, 0), R, 3 * d, d, ep_slab(3 * d), s);
         gemm_decode<T>(EPI_RES, od, wl(l, 1), R, d, d, ep_res(), s);
         gemm_ln_launch<T>(EPI_F32, x, lnw, lnb, wl(l, 2), R, d, d, ep_slab(d), s);
         gemm_decode<T>(EPI_RES, od, wl(l, 3), R, d, d, ep_res(), s);
         gemm_ln_launch<T>(EPI_GELU, x, lnw, lnb, wl(l, 4), R, 4 * d, d, ep_gelu(), s);
         gemm_decode<T>(EPI_RES, ffd, wl(l, 5), R, d, 4 * d, ep_res(), s);
       }},
      {"LEGACY layer GEMMs+LN (9 launches)", 9,
       [&](int l) {
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 8, bias);
         gemm_splitk_partials<T>(hd, wl(l, 0), R, 3 * d, d, slab, s);
         gemm_splitk_partials<T>(od, wl(l, 1), R, d, d, slab, s);
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
         gemm_splitk_partials<T>(hd, wl(l, 2), R, d, d, slab, s);
         gemm_splitk_partials<T>(od, wl(l, 3), R, d, d, slab, s);
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
         gemm_decode<T>(EPI_GELU, hd, wl(l, 4), R, 4 * d, d, ep_gelu(), s);
         gemm_splitk_partials<T>(ffd, wl(l, 5), R, d, 4 * d, slab, s);
       }},
  };
  const char* only = getenv("PROBE_ONLY");
  printf("R=%d rows, d=%d, %d layers of distinct weights per graph, %d replays\n", R, d, L, reps);
  printf("%-38s %10s %12s\n", "chain", "us/launch", "us/layer");
  for (auto& op : ops) {
    if (only && op.name.find(only) == std::string::npos) continue;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 0; l < L; ++l) op.f(l);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));  // warm-up
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
    const double per_layer = ms * 1e3 / reps / L;
    printf("%-38s %10.2f %12.2f\n", op.name.c_str(), per_layer / op.launches_per_layer, per_layer);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
