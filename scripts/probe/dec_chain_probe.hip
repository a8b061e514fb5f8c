// Probe: unprofiled per-launch time of the decode-step GEMM / LayerNorm
// kernels of libmwx.so at large-v3 shapes (R rows, d 1280), each chain
// captured in a hipGraph (32 layers of distinct weights, so the weights stream
// from HBM as in a real decode step) and replayed; time = graph wall / launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include
//        -I../../sentiric-stt-whisper-service_amd/csrc dec_chain_probe.hip
//        -L../../sentiric-stt-whisper-service_amd -lmwx -o dec_chain_probe
// (k_chain.hip, the fused GEMM -> LayerNorm -> GEMM seam, is compiled in:
// `verify seam` checks it bit for bit against the three launches)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "kernels.h"
#include "k_chain.hip"  // (the fused-seam probe kernel)

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

// launch-cost probes: an empty kernel's cost in a graph
// chain against its grid size, its LDS allocation and its kernarg size, and the
// cost of the dirty L2 lines a kernel leaves behind (end-of-kernel release)
__global__ void empty_lds_kernel(float* p) {
  extern __shared__ float lds[];
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = lds[0];
}
struct BigArg {
  float v[256];  // 1 KB of kernel arguments
};
__global__ void empty_bigarg_kernel(BigArg a, float* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = a.v[threadIdx.x & 255];
}
// each workgroup stores 4 KB (256 lanes x 16 B): plain stores (dirty L2 lines)
// or non-temporal stores
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void store_kernel(f4v* p) {
  const f4v v = {1.0f, 2.0f, 3.0f, (float)blockIdx.x};
  f4v* q = p + (size_t)blockIdx.x * 256 + threadIdx.x;
  if (NT)
    __builtin_nontemporal_store(v, q);
  else
    *q = v;
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

// pure streaming read of the cross-attention's bytes: one workgroup per
// (row, head) reads its K rows then its V rows (1500 x 128 B each), 16 B per
// lane, 8 loads in flight per lane, one value kept so nothing is elided
__global__ __launch_bounds__(256) void stream_kv_kernel(const uint4* __restrict__ K,
                                                        const uint4* __restrict__ V, int n16,
                                                        float* out) {
  const long base = (long)blockIdx.x * n16;
  uint32_t acc = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const uint4* p = (pass ? V : K) + base;
    for (int i = threadIdx.x; i < n16; i += 256 * 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[min(i + u * 256, n16 - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u].x ^ v[u].w;
    }
  }
  if (acc == 0x12345u) out[threadIdx.x] = (float)acc;
}

// reads [p, p + n16 * 16) once (brings it into the Infinity Cache / L2)
__global__ __launch_bounds__(256) void touch_kernel(const uint4* __restrict__ p, long n16, float* out) {
  uint32_t acc = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256 * 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[min(i + u * (long)gridDim.x * 256, n16 - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u].x ^ v[u].w;
  }
  if (acc == 0x12345u) out[threadIdx.x] = (float)acc;
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
  // attention / logits operands (large-v3: 20 heads x 64, 1500 audio ctx, 448 text ctx)
  const int H = 20, Lc = 1500, Tctx = 448, V = 51866;
  const size_t cross_elems = (size_t)R * H * Lc * 64;
  uint16_t *ck, *cv, *kself, *vself;
  CK(hipMalloc(&ck, 2 * cross_elems * 2));  // two layer copies (alternating: no MALL reuse)
  CK(hipMalloc(&cv, 2 * cross_elems * 2));
  fill_kernel<<<4096, 256>>>(ck, 2 * cross_elems, 7);
  fill_kernel<<<4096, 256>>>(cv, 2 * cross_elems, 8);
  const size_t self_elems = (size_t)R * H * Tctx * 64;
  CK(hipMalloc(&kself, 2 * self_elems * 2));
  CK(hipMalloc(&vself, 2 * self_elems * 2));
  fill_kernel<<<4096, 256>>>(kself, 2 * self_elems, 9);
  fill_kernel<<<4096, 256>>>(vself, 2 * self_elems, 10);
  int *pos, *xidx, *kvmap, *kvown;
  CK(hipMalloc(&pos, R * 4));
  CK(hipMalloc(&xidx, R * 4));
  CK(hipMalloc(&kvmap, (size_t)R * Tctx * 4));
  CK(hipMalloc(&kvown, R * 4));
  std::vector<int> hp(R, 112), hxi(R);
  for (int r = 0; r < R; ++r) hxi[r] = r;
  CK(hipMemcpy(pos, hp.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(xidx, hxi.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemset(kvmap, 0, (size_t)R * Tctx * 4));
  CK(hipMemset(kvown, 0, R * 4));
  uint16_t* temb;
  const size_t Vp = (V + 15) / 16 * 16;
  CK(hipMalloc(&temb, Vp * d * 2));
  fill_kernel<<<4096, 256>>>(temb, Vp * d, 11);
  float *logits, *smask, *flt;
  CK(hipMalloc(&logits, (size_t)R * V * 4));
  CK(hipMalloc(&smask, (size_t)V * 4));
  CK(hipMalloc(&flt, (size_t)R * V * 4));
  CK(hipMemset(smask, 0, (size_t)V * 4));
  RowCtl* ctl;
  TokOut* tout;
  LPPart* parts;
  LPRes* lres;
  CK(hipMalloc(&ctl, R * sizeof(RowCtl)));
  CK(hipMalloc(&tout, R * sizeof(TokOut)));
  CK(hipMalloc(&parts, R * LP_G * sizeof(LPPart)));
  CK(hipMalloc(&lres, R * LP_G * sizeof(LPRes)));
  std::vector<RowCtl> hc(R);
  for (auto& c : hc) {
    c = RowCtl{};
    c.active = 1;
    c.sample = 1;
    c.penult_ts = 1;
    c.seek_delta = 3000;
  }
  CK(hipMemcpy(ctl, hc.data(), R * sizeof(RowCtl), hipMemcpyHostToDevice));
  LogitsConst LCo{V, 50257, 50365, 220, 1, -1, 50363};
  const float kqs = 0.35355339f;
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
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fk, jn;
  CK(hipEventCreateWithFlags(&fk, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&jn, hipEventDisableTiming));
  // one whole decoder layer (11 launches); pf: a side-stream kernel reads
  // layer l+1's weights while layer l runs (0 none, 1 at layer start, 2 after
  // the cross-attention's launch)
  auto full_layer = [&](int l, int pf) {
    auto prefetch = [&]() {
      CK(hipEventRecord(fk, s));
      CK(hipStreamWaitEvent(s2, fk, 0));
      const int ln = (l + 1) % L;
      touch_kernel<<<512, 256, 0, s2>>>((const uint4*)wl(ln, 0), (long)(per_layer * 2 / 16), x + 4 * d);
    };
    if (pf == 1) prefetch();
    layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 8, bias);
    gemm_splitk_partials<T>(hd, wl(l, 0), R, 3 * d, d, slab, s);
    dec_attention<T>(slab, 5, 3 * d, bias, kqs, kqs, (_Float16*)kself + (l & 1) * self_elems,
                     (_Float16*)vself + (l & 1) * self_elems, nullptr, pos, act, 0, Tctx, od, R, H,
                     1.0f, s, kvmap, kvown, 0, 1);
    gemm_splitk_partials<T>(od, wl(l, 1), R, d, d, slab, s);
    layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
    gemm_splitk_partials<T>(hd, wl(l, 2), R, d, d, slab, s);
    dec_attention<T>(slab, 5, d, bias, 1.0f, 1.0f, (_Float16*)ck + (l & 1) * cross_elems,
                     (_Float16*)cv + (l & 1) * cross_elems, xidx, pos, act, Lc, Lc, od, R, H, kqs, s);
    if (pf == 2) prefetch();
    gemm_splitk_partials<T>(od, wl(l, 3), R, d, d, slab, s);
    layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
    gemm_decode<T>(EPI_GELU, hd, wl(l, 4), R, 4 * d, d, ep_gelu(), s);
    gemm_splitk_partials<T>(ffd, wl(l, 5), R, d, 4 * d, slab, s);
    if (pf && l == L - 1) {  // join the side stream
      CK(hipEventRecord(jn, s2));
      CK(hipStreamWaitEvent(s, jn, 0));
    }
  };
  // fused seams (k_chain.hip): counters [L][3][8], zeroed at the head of each
  // replay by a memset node (the engine zeroes them in the step's embedding)
  unsigned *ctrs, *cerr;
  CK(hipMalloc(&ctrs, (size_t)L * 3 * chain_slot_words() * 4));
  CK(hipMalloc(&cerr, 4));
  CK(hipMemset(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4));
  CK(hipMemset(cerr, 0, 4));
  float* slab2;
  CK(hipMalloc(&slab2, (size_t)8 * R * 3 * d * 4));
  auto chain = [&](int l, int site, const T* pA, const T* pW, int pK, const T* cW, int cN,
                   bool skinny, float* cP) {
    ChainArgs a;
    a.M = R;
    a.d = d;
    a.p_A = pA;
    a.p_W = pW;
    a.p_K = pK;
    a.ln.x = x;
    a.ln.w = lnw;
    a.ln.b = lnb;
    a.ln.P = slab;
    a.ln.pbias = bias;
    a.ln.y = hd;
    a.ln.active = act;
    a.c_W = cW;
    a.c_N = cN;
    a.c_skinny = skinny;
    a.c_P = cP;
    a.c_epi = ep_gelu();
    a.ctr = ctrs + ((size_t)l * 3 + site) * chain_slot_words();
    a.err = cerr;
    if (!chain_launch<T>(a, s)) {
      fprintf(stderr, "chain_launch unsupported\n");
      exit(1);
    }
  };
  auto chain_layer = [&](int l) {
    if (l == 0) CK(hipMemsetAsync(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4, s));
    dec_attention<T>(slab2, 5, 3 * d, bias, kqs, kqs, (_Float16*)kself + (l & 1) * self_elems,
                     (_Float16*)vself + (l & 1) * self_elems, nullptr, pos, act, 0, Tctx, od, R, H,
                     1.0f, s, kvmap, kvown, 0, 1);
    chain(l, 0, od, wl(l, 1), d, wl(l, 2), d, false, slab2);  // out -> LN2 -> cross-Q
    dec_attention<T>(slab2, 5, d, bias, 1.0f, 1.0f, (_Float16*)ck + (l & 1) * cross_elems,
                     (_Float16*)cv + (l & 1) * cross_elems, xidx, pos, act, Lc, Lc, od, R, H, kqs, s);
    chain(l, 1, od, wl(l, 3), d, wl(l, 4), 4 * d, true, nullptr);  // cross-out -> LN3 -> FFN1
    chain(l, 2, ffd, wl(l, 5), 4 * d, wl((l + 1) % L, 0), 3 * d, false, slab2);  // FFN2 -> LN1 -> QKV
  };
  // ---- bit-exactness: each fused seam == its three launches (same inputs) ----
  if (R <= 64) {  // (the fused seams support <= 64 rows)
    fill_kernel<<<1024, 256>>>((uint16_t*)od, R64 * d, 21);
    fill_kernel<<<1024, 256>>>((uint16_t*)ffd, R64 * 4 * d, 22);
    // slab rows of the producer must be finite garbage-free: the producers write them
    CK(hipDeviceSynchronize());
    std::vector<float> x0((size_t)R * d);
    CK(hipMemcpy(x0.data(), x, x0.size() * 4, hipMemcpyDeviceToHost));
    const size_t hdn = R64 * d, ffn = R64 * 4 * d, sln = (size_t)8 * R * 3 * d;
    auto snap = [&](std::vector<float>& hx, std::vector<uint16_t>& hh, std::vector<uint16_t>& hf,
                    std::vector<float>& hs) {
      CK(hipDeviceSynchronize());
      hx.resize((size_t)R * d);
      hh.resize(hdn);
      hf.resize(ffn);
      hs.resize(sln);
      CK(hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hh.data(), hd, hdn * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hf.data(), ffd, ffn * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hs.data(), slab2, sln * 4, hipMemcpyDeviceToHost));
    };
    auto reset = [&]() {
      CK(hipMemcpy(x, x0.data(), x0.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemset(hd, 0, hdn * 2));
      CK(hipMemset(slab2, 0, sln * 4));
      CK(hipMemset(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4));
      fill_kernel<<<1024, 256>>>((uint16_t*)ffd, ffn, 22);
      CK(hipDeviceSynchronize());
    };
    const char* names[3] = {"o+ln+cq", "co+ln+fc1", "fc2+ln+qkv"};
    for (int site = 0; site < 3; ++site) {
      std::vector<float> ax, as, bx, bs;
      std::vector<uint16_t> ah, af, bh, bf;
      reset();
      if (site == 0) {
        gemm_splitk_partials<T>(od, wl(0, 1), R, d, d, slab, s);
        layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
        gemm_splitk_partials<T>(hd, wl(0, 2), R, d, d, slab2, s);
      } else if (site == 1) {
        gemm_splitk_partials<T>(od, wl(0, 3), R, d, d, slab, s);
        layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
        EpiParams e = ep_gelu();
        e.nw = 4;
        gemm_decode<T>(EPI_GELU, hd, wl(0, 4), R, 4 * d, d, e, s);
      } else {
        gemm_splitk_partials<T>(ffd, wl(0, 5), R, d, 4 * d, slab, s);
        layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 8, bias);
        gemm_splitk_partials<T>(hd, wl(1, 0), R, 3 * d, d, slab2, s);
      }
      snap(ax, ah, af, as);
      reset();
      if (site == 0) chain(0, 0, od, wl(0, 1), d, wl(0, 2), d, false, slab2);
      if (site == 1) chain(0, 1, od, wl(0, 3), d, wl(0, 4), 4 * d, true, nullptr);
      if (site == 2) chain(0, 2, ffd, wl(0, 5), 4 * d, wl(1, 0), 3 * d, false, slab2);
      snap(bx, bh, bf, bs);
      unsigned herr = 0;
      CK(hipMemcpy(&herr, cerr, 4, hipMemcpyDeviceToHost));
      const bool ok = ax == bx && ah == bh && af == bf && memcmp(as.data(), bs.data(), as.size() * 4) == 0;
      size_t dx = 0, dh = 0, df = 0, ds = 0;
      for (size_t i = 0; i < ax.size(); ++i) dx += memcmp(&ax[i], &bx[i], 4) != 0;
      for (size_t i = 0; i < ah.size(); ++i) dh += ah[i] != bh[i];
      for (size_t i = 0; i < af.size(); ++i) df += af[i] != bf[i];
      for (size_t i = 0; i < as.size(); ++i) ds += memcmp(&as[i], &bs[i], 4) != 0;
      printf("verify seam %-12s %s (diff x %zu, hd %zu, ffd %zu, slabs %zu; err %u)\n", names[site],
             ok ? "BIT-EXACT" : "MISMATCH", dx, dh, df, ds, herr);
    }
  }
  struct Op {
    std::string name;
    int launches_per_layer;
    std::function<void(int)> f;
  };
  std::vector<Op> ops = {
      {"empty 512 WG", 1, [&](int) { empty_kernel<<<512, 256, 0, s>>>(nullptr); }},
      {"launch: empty 1 WG", 1, [&](int) { empty_kernel<<<1, 256, 0, s>>>(nullptr); }},
      {"launch: empty 64 WG", 1, [&](int) { empty_kernel<<<64, 256, 0, s>>>(nullptr); }},
      {"launch: empty 128 WG", 1, [&](int) { empty_kernel<<<128, 256, 0, s>>>(nullptr); }},
      {"launch: empty 256 WG", 1, [&](int) { empty_kernel<<<256, 256, 0, s>>>(nullptr); }},
      {"launch: empty 1024 WG", 1, [&](int) { empty_kernel<<<1024, 256, 0, s>>>(nullptr); }},
      {"launch: empty 2048 WG", 1, [&](int) { empty_kernel<<<2048, 256, 0, s>>>(nullptr); }},
      {"launch: empty 512 WG x 64 thr", 1, [&](int) { empty_kernel<<<512, 64, 0, s>>>(nullptr); }},
      {"launch: empty 512 WG x 1024 thr", 1, [&](int) { empty_kernel<<<512, 1024, 0, s>>>(nullptr); }},
      {"launch: empty 512 WG, 64 KB LDS", 1,
       [&](int) { empty_lds_kernel<<<512, 256, 65536, s>>>(nullptr); }},
      {"launch: empty 512 WG, 1 KB kernarg", 1,
       [&](int) { empty_bigarg_kernel<<<512, 256, 0, s>>>(BigArg{}, nullptr); }},
      {"launch: 40 WG store 160 KB", 1, [&](int) { store_kernel<false><<<40, 256, 0, s>>>((f4v*)slab2); }},
      {"launch: 40 WG store 160 KB nt", 1, [&](int) { store_kernel<true><<<40, 256, 0, s>>>((f4v*)slab2); }},
      {"launch: 640 WG store 2.6 MB", 1, [&](int) { store_kernel<false><<<640, 256, 0, s>>>((f4v*)slab2); }},
      {"launch: 640 WG store 2.6 MB nt", 1, [&](int) { store_kernel<true><<<640, 256, 0, s>>>((f4v*)slab2); }},
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
      // the same weights every launch: they stay in L2 / the Infinity Cache
      // (what a perfect prefetch of the next GEMM's weights could give)
      {"WARM splitk_qkv", 1, [&](int) { gemm_splitk_partials<T>(hd, wl(0, 0), R, 3 * d, d, slab, s); }},
      {"WARM splitk_o", 1, [&](int) { gemm_splitk_partials<T>(od, wl(0, 1), R, d, d, slab, s); }},
      {"WARM splitk_fc2", 1, [&](int) { gemm_splitk_partials<T>(ffd, wl(0, 5), R, d, 4 * d, slab, s); }},
      {"WARM skinny_fc1", 1,
       [&](int) { gemm_decode<T>(EPI_GELU, hd, wl(0, 4), R, 4 * d, d, ep_gelu(), s); }},
      {"stream_kv (cross bytes, pure read)", 1,
       [&](int l) {
         stream_kv_kernel<<<R * H, 256, 0, s>>>((const uint4*)(ck + (l & 1) * cross_elems),
                                                (const uint4*)(cv + (l & 1) * cross_elems), Lc * 64 * 2 / 16,
                                                x);
       }},
      {"cross_attn (KS 5 query slabs)", 1,
       [&](int l) {
         dec_attention<T>(slab, 5, d, bias, 1.0f, 1.0f, (_Float16*)ck + (l & 1) * cross_elems,
                          (_Float16*)cv + (l & 1) * cross_elems, xidx, pos, act, Lc, Lc, od, R, H, kqs, s);
       }},
      {"self_attn (pos 112, KS 5)", 1,
       [&](int l) {
         dec_attention<T>(slab, 5, 3 * d, bias, kqs, kqs, (_Float16*)kself + (l & 1) * self_elems,
                          (_Float16*)vself + (l & 1) * self_elems, nullptr, pos, act, 0, Tctx, od, R, H,
                          1.0f, s, kvmap, kvown, 0, 1);
       }},
      {"logits GEMM (per step)", 1,
       [&](int l) {
         EpiParams e;
         e.c32 = logits;
         e.ldc = V;
         gemm_decode<T>(EPI_F32, hd, (const T*)temb, R, V, d, e, s);
       }},
      {"logits_process (per step)", 1,
       [&](int) {
         logits_process(logits, smask, ctl, tout, nullptr, nullptr, LCo, R, LPScratch{flt, parts, lres}, s);
       }},
      {"FULL layer (11 launches)", 11, [&](int l) { full_layer(l, 0); }},
      {"CHAIN layer (5 launches)", 5, [&](int l) { chain_layer(l); }},
      {"seam o+ln+cq (3 launches)", 3,
       [&](int l) {
         gemm_splitk_partials<T>(od, wl(l, 1), R, d, d, slab, s);
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
         gemm_splitk_partials<T>(hd, wl(l, 2), R, d, d, slab2, s);
       }},
      {"CHAIN seam o+ln+cq (1 launch)", 1,
       [&](int l) {
         if (l == 0) CK(hipMemsetAsync(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4, s));
         chain(l, 0, od, wl(l, 1), d, wl(l, 2), d, false, slab2);
       }},
      {"seam fc2+ln+qkv (3 launches)", 3,
       [&](int l) {
         gemm_splitk_partials<T>(ffd, wl(l, 5), R, d, 4 * d, slab, s);
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 8, bias);
         gemm_splitk_partials<T>(hd, wl((l + 1) % L, 0), R, 3 * d, d, slab2, s);
       }},
      {"CHAIN seam fc2+ln+qkv (1 launch)", 1,
       [&](int l) {
         if (l == 0) CK(hipMemsetAsync(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4, s));
         chain(l, 2, ffd, wl(l, 5), 4 * d, wl((l + 1) % L, 0), 3 * d, false, slab2);
       }},
      {"seam co+ln+fc1 (3 launches)", 3,
       [&](int l) {
         gemm_splitk_partials<T>(od, wl(l, 3), R, d, d, slab, s);
         layer_norm_dec<T>(x, lnw, lnb, hd, R, d, act, s, slab, 5, bias);
         EpiParams e = ep_gelu();
         e.nw = 4;
         gemm_decode<T>(EPI_GELU, hd, wl(l, 4), R, 4 * d, d, e, s);
       }},
      {"CHAIN seam co+ln+fc1 (1 launch)", 1,
       [&](int l) {
         if (l == 0) CK(hipMemsetAsync(ctrs, 0, (size_t)L * 3 * chain_slot_words() * 4, s));
         chain(l, 1, od, wl(l, 3), d, wl(l, 4), 4 * d, true, nullptr);
       }},
      {"FULL layer + prefetch next at start", 11, [&](int l) { full_layer(l, 1); }},
      {"FULL layer + prefetch next after xattn", 11, [&](int l) { full_layer(l, 2); }},
      {"touch one layer's weights", 1,
       [&](int l) { touch_kernel<<<512, 256, 0, s>>>((const uint4*)wl(l, 0), (long)(per_layer * 2 / 16), x + 4 * d); }},
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
    if (R > 64 && op.name.find("CHAIN") != std::string::npos) continue;
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
    unsigned herr = 0;
    CK(hipMemcpy(&herr, cerr, 4, hipMemcpyDeviceToHost));
    if (herr) {
      printf("  !! chain hand-off wait timed out\n");
      CK(hipMemset(cerr, 0, 4));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // ---- concurrency: a GEMM chain of row group A beside the cross-attention of
  // row group B (R/2 rows each): one stream (sequential), two streams with two
  // graphs, one graph with two branches
  if (!only || std::string(only) == "conc") {
    const int Rh = R / 2;
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto chainA = [&](hipStream_t st) {
      for (int l = 0; l < L; ++l) {
        layer_norm_dec<T>(x, lnw, lnb, hd, Rh, d, act, st, slab, 8, bias);
        gemm_splitk_partials<T>(hd, wl(l, 0), Rh, 3 * d, d, slab, st);
        gemm_splitk_partials<T>(od, wl(l, 1), Rh, d, d, slab, st);
        layer_norm_dec<T>(x, lnw, lnb, hd, Rh, d, act, st, slab, 5, bias);
        gemm_splitk_partials<T>(hd, wl(l, 2), Rh, d, d, slab, st);
        gemm_splitk_partials<T>(od, wl(l, 3), Rh, d, d, slab, st);
        layer_norm_dec<T>(x, lnw, lnb, hd, Rh, d, act, st, slab, 5, bias);
        gemm_decode<T>(EPI_GELU, hd, wl(l, 4), Rh, 4 * d, d, ep_gelu(), st);
        gemm_splitk_partials<T>(ffd, wl(l, 5), Rh, d, 4 * d, slab, st);
      }
    };
    T* od2;
    float* slab2;
    CK(hipMalloc(&od2, R64 * d * 2));
    CK(hipMalloc(&slab2, (size_t)8 * R * 3 * d * 4));
    auto chainB = [&](hipStream_t st) {
      for (int l = 0; l < L; ++l)
        dec_attention<T>(slab2, 5, d, bias, 1.0f, 1.0f, (_Float16*)ck + (l & 1) * cross_elems,
                         (_Float16*)cv + (l & 1) * cross_elems, xidx + Rh, pos, act, Lc, Lc, od2, Rh, H,
                         kqs, st);
    };
    auto time_graph = [&](hipGraphExec_t ge, hipStream_t st) {
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(b, st));
      CK(hipStreamSynchronize(st));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      return ms * 1e3 / reps / L;
    };
    auto capture = [&](hipStream_t st, const std::function<void()>& f) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      f();
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      return ge;
    };
    hipGraphExec_t gA = capture(s, [&] { chainA(s); });
    hipGraphExec_t gB = capture(s, [&] { chainB(s); });
    hipGraphExec_t gAB = capture(s, [&] { chainA(s); chainB(s); });
    printf("concurrency (%d + %d rows), us per layer:\n", Rh, Rh);
    printf("  A alone (GEMM+LN chain)            %8.2f\n", time_graph(gA, s));
    printf("  B alone (cross-attention)          %8.2f\n", time_graph(gB, s));
    printf("  A then B, one stream               %8.2f\n", time_graph(gAB, s));
    // two graphs on two streams
    hipGraphExec_t gB2 = capture(s2, [&] { chainB(s2); });
    CK(hipGraphLaunch(gA, s));
    CK(hipGraphLaunch(gB2, s2));
    CK(hipDeviceSynchronize());
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    CK(hipEventRecord(a, s));
    CK(hipStreamWaitEvent(s2, a, 0));
    for (int r = 0; r < reps; ++r) {
      CK(hipGraphLaunch(gA, s));
      CK(hipGraphLaunch(gB2, s2));
    }
    CK(hipEventRecord(c, s2));
    CK(hipStreamWaitEvent(s, c, 0));
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("  A || B, two streams / two graphs   %8.2f\n", ms * 1e3 / reps / L);
    // one graph, two branches (fork / join through events during capture)
    hipEvent_t fk, jn;
    CK(hipEventCreateWithFlags(&fk, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&jn, hipEventDisableTiming));
    hipGraphExec_t gF = capture(s, [&] {
      CK(hipEventRecord(fk, s));
      CK(hipStreamWaitEvent(s2, fk, 0));
      chainB(s2);
      CK(hipEventRecord(jn, s2));
      chainA(s);
      CK(hipStreamWaitEvent(s, jn, 0));
    });
    printf("  A || B, one graph, two branches    %8.2f\n", time_graph(gF, s));
  }
  return 0;
}
