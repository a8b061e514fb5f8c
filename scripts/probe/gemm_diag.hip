// Probe: encoder-GEMM structure variants on gfx950 (bf16 in, f32 out, C = A W^T,
// A [M][K], W [N][K] row-major). Times each variant on the large-v3 QKV /
// FC1 / FC2 shapes of a 32-clip batch and checks sampled outputs against a
// double-precision host dot product.
//
// Variant template: BM x BN tile, WM x WN waves (each wave (BM/WM) x (BN/WN)
// outputs as 16x16 fragments), NST-stage LDS ring filled by global_load_lds
// (16 B/lane, XOR-swizzled via the source address), NST-1 tiles in flight,
// counted vmcnt + raw s_barrier. REG = register-staged 2-buffer reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int BK = 64;
__device__ int g_store = 1;  // 0: timing runs skip the C stores (main loop only)

template <int N_>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N_ == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N_ == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N_ == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N_ == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N_ == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N_ == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N_ == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BM, int BN, int WM, int WN, int NST, int MINB, int DIAG = 0>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_v(const __bf16* __restrict__ A,
                                                            const __bf16* __restrict__ W,
                                                            float* __restrict__ C, int M, int N,
                                                            int K, int remap) {
  constexpr int NW = WM * WN, FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int GA = BM / 8 / NW, GB = BN / 8 / NW;  // DMA instrs per wave per tile
  constexpr int GT = GA + GB;
  __shared__ __attribute__((aligned(16))) __bf16 lds[NST][(BM + BN) * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int bid = blockIdx.x;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM, nb = nbn * nbm;
  if (remap) {  // bijective XCD remap: blocks sharing an XCD get consecutive ids
    const int q = nb / 8, r = nb % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  // M-tile groups of 8 along N for L2 reuse of the A rows
  const int bm = bid / nbn, bn = bid % nbn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int lr = lane >> 3, ls = lane & 7;
  const __bf16* asrc[GA];
  const __bf16* wsrc[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = (wid * GA + i) * 8 + lr;
    asrc[i] = A + (long)min(m0 + r, M - 1) * K + (ls ^ (r & 7)) * 8;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = (wid * GB + i) * 8 + lr;
    wsrc[i] = W + (long)min(n0 + r, N - 1) * K + (ls ^ (r & 7)) * 8;
  }
  auto issue = [&](int kt, int st) {
    const int ko = kt * BK;
#pragma unroll
    for (int i = 0; i < GA; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(asrc[i] + ko),
          (void __attribute__((address_space(3)))*)(&lds[st][((wid * GA + i) * 8) * BK]), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < GB; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(wsrc[i] + ko),
          (void __attribute__((address_space(3)))*)(&lds[st][(BM + (wid * GB + i) * 8) * BK]), 16,
          0, 0);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const int nk = K / BK;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) issue(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NST;
    const int left = nk - 1 - kt;
    if (DIAG == 0) {
      if (NST >= 3 && left >= NST - 2)
        vm_wait<GT * (NST - 2)>();
      else if (NST >= 4 && left >= 1)
        vm_wait<GT>();
      else
        vm_wait<0>();
    } else {
      vm_wait<24>();  // diagnostic: DMA latency not waited for (results wrong)
    }
    __builtin_amdgcn_sched_barrier(0);
    if (DIAG != 2) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NST - 1 < nk) issue(kt + NST - 1, (kt + NST - 1) % NST);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
      const int kc = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(&lds[cur][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = BM + wn * (BN / WN) + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(&lds[cur][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N && g_store) C[(long)m * N + n] = acc[i][j][r];
      }
    }
}


// 256x256 tile, 32-deep K steps through a 4-stage LDS-DMA ring (3 steps in
// flight), fragments of step k+1 read from LDS while the MFMAs of step k run
// (two register sets, loop unrolled by 2), one barrier per step.
template <int DIAG>
__global__ __launch_bounds__(512, 1) void gemm_pf4(const __bf16* __restrict__ A,
                                                  const __bf16* __restrict__ W,
                                                  float* __restrict__ C, int M, int N, int K,
                                                  int remap) {
  constexpr int BM = 256, BN = 256, BKE = 32, NST = 4, CPR = 4, RPI = 16;
  constexpr int GDA = BM / RPI / 8, GDB = BN / RPI / 8;  // 2 + 2 DMA instrs per wave per step
  constexpr int FM = 8, FN = 4;
  __shared__ __attribute__((aligned(16))) __bf16 lds[NST][(BM + BN) * BKE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / 4, wn = wid % 4;
  int bid = blockIdx.x;
  const int nbn = (N + BN - 1) / BN, nbm = (M + BM - 1) / BM, nb = nbn * nbm;
  if (remap) {
    const int q = nb / 8, r = nb % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int m0 = (bid / nbn) * BM, n0 = (bid % nbn) * BN;
  auto swz = [](int row) { return (row >> 2) & 3; };
  const int lr = lane / CPR, ls = lane % CPR;
  const __bf16* asrc[GDA];
  const __bf16* wsrc[GDB];
#pragma unroll
  for (int i = 0; i < GDA; ++i) {
    const int r = (wid * GDA + i) * RPI + lr;
    asrc[i] = A + (long)min(m0 + r, M - 1) * K + (ls ^ swz(r)) * 8;
  }
#pragma unroll
  for (int i = 0; i < GDB; ++i) {
    const int r = (wid * GDB + i) * RPI + lr;
    wsrc[i] = W + (long)min(n0 + r, N - 1) * K + (ls ^ swz(r)) * 8;
  }
  auto issue = [&](int kt, int st) {
    const int ko = kt * BKE;
#pragma unroll
    for (int i = 0; i < GDA; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(asrc[i] + ko),
          (void __attribute__((address_space(3)))*)(&lds[st][((wid * GDA + i) * RPI) * BKE]), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < GDB; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(wsrc[i] + ko),
          (void __attribute__((address_space(3)))*)(&lds[st][(BM + (wid * GDB + i) * RPI) * BKE]), 16,
          0, 0);
  };
  // per-lane fragment offsets within a stage (elements)
  int aoff[FM], boff[FN];
  const int kc = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wm * 128 + i * 16 + (lane & 15);
    aoff[i] = row * BKE + ((kc ^ swz(row)) << 3);
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int row = BM + wn * 64 + j * 16 + (lane & 15);
    boff[j] = row * BKE + ((kc ^ swz(row)) << 3);
  }
  bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
  auto read = [&](int st, bf16x8* fa, bf16x8* fb) {
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(&lds[st][boff[j]]);
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(&lds[st][aoff[i]]);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  auto mfma = [&](const bf16x8* fa, const bf16x8* fb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const int nk = K / BKE;  // (even, >= 4 on every shape here)
  issue(0, 0);
  issue(1, 1);
  issue(2, 2);
  __builtin_amdgcn_s_waitcnt(0x0F78);  // step 0 landed (this wave)
  __builtin_amdgcn_s_barrier();
  read(0, fa0, fb0);
  // one step: wait for step kt+1's DMA, barrier, refill the freed stage with
  // step kt+3, read step kt+1's fragments, MFMAs of step kt (compile-time
  // variants for the last steps, so the steady-state loop has no branches and
  // the counted lgkmcnt survives)
#define PF4_STEP(KT, ISSUE, WAITN, READ, FA, FB, NA, NB)                      \
  do {                                                                        \
    if (DIAG == 0) {                                                          \
      if (WAITN == 4) __builtin_amdgcn_s_waitcnt(0x0F74);        \
      else if (WAITN == 0) __builtin_amdgcn_s_waitcnt(0x0F70);   \
    }                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                        \
    __builtin_amdgcn_s_barrier();                                             \
    __builtin_amdgcn_sched_barrier(0);                                        \
    if (ISSUE) issue((KT) + 3, ((KT) + 3) & 3);                               \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* step KT's reads */ \
    if (READ) read(((KT) + 1) & 3, NA, NB);                                   \
    mfma(FA, FB);                                                             \
  } while (0)
  int kt = 0;
  for (; kt + 4 < nk; kt += 2) {
    PF4_STEP(kt, 1, 4, 1, fa0, fb0, fa1, fb1);
    PF4_STEP(kt + 1, 1, 4, 1, fa1, fb1, fa0, fb0);
  }
  PF4_STEP(kt, 1, 4, 1, fa0, fb0, fa1, fb1);      // nk-4: issues nk-1
  PF4_STEP(kt + 1, 0, 4, 1, fa1, fb1, fa0, fb0);  // nk-3
  PF4_STEP(kt + 2, 0, 0, 1, fa0, fb0, fa1, fb1);  // nk-2
  PF4_STEP(kt + 3, 0, -1, 0, fa1, fb1, fa0, fb0); // nk-1
#undef PF4_STEP
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N && g_store) C[(long)m * N + n] = acc[i][j][r];
      }
    }
}

// register-staged reference (the engine's gemm_big main loop)
__global__ __launch_bounds__(256, 2) void gemm_reg(const __bf16* __restrict__ A,
                                                   const __bf16* __restrict__ W,
                                                   float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 128;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][BM * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BM;
  const int srow = tid >> 3, kc0 = tid & 7;
  const __bf16* a[4];
  const __bf16* w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = A + (long)min(m0 + srow + 32 * i, M - 1) * K + kc0 * 8;
    w[i] = W + (long)min(n0 + srow + 32 * i, N - 1) * K + kc0 * 8;
  }
  const int soff0 = srow * BK + ((kc0 ^ (srow & 7)) << 3);
  uint4 ra[4], rw[4];
  f32x4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ra[i] = *reinterpret_cast<const uint4*>(a[i]);
    rw[i] = *reinterpret_cast<const uint4*>(w[i]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    *reinterpret_cast<uint4*>(&lds[0][0][soff0 + i * 32 * BK]) = ra[i];
    *reinterpret_cast<uint4*>(&lds[0][1][soff0 + i * 32 * BK]) = rw[i];
  }
  __syncthreads();
  const int nk = K / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ra[i] = *reinterpret_cast<const uint4*>(a[i] + (kt + 1) * BK);
        rw[i] = *reinterpret_cast<const uint4*>(w[i] + (kt + 1) * BK);
      }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
      const int kc = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(&lds[cur][0][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(&lds[cur][1][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<uint4*>(&lds[cur ^ 1][0][soff0 + i * 32 * BK]) = ra[i];
        *reinterpret_cast<uint4*>(&lds[cur ^ 1][1][soff0 + i * 32 * BK]) = rw[i];
      }
    __syncthreads();
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N && g_store) C[(long)m * N + n] = acc[i][j][r];
      }
    }
}

static float bf2f(__bf16 h) { return (float)h; }

struct Shape {
  const char* name;
  int M, N, K;
};

int main() {
  const Shape shapes[] = {{"qkv", 48000, 3840, 1280}, {"fc1", 48000, 5120, 1280},
                          {"fc2", 48000, 1280, 5120}};
  const long maxA = 48000L * 5120, maxW = 5120L * 5120, maxC = 48000L * 5120;
  std::vector<__bf16> hA(maxA), hW(maxW);
  unsigned s = 12345;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f;
  };
  for (auto& x : hA) x = (__bf16)rnd();
  for (auto& x : hW) x = (__bf16)(rnd() * 0.05f);
  __bf16 *dA, *dW;
  float* dC;
  CK(hipMalloc(&dA, maxA * 2));
  CK(hipMalloc(&dW, maxW * 2));
  CK(hipMalloc(&dC, maxC * 4));
  CK(hipMemcpy(dA, hA.data(), maxA * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, hW.data(), maxW * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> hC(64);
  for (const Shape& sh : shapes) {
    const double flop = 2.0 * sh.M * sh.N * sh.K;
    auto run = [&](const char* name, auto launch) {
      int one = 1, zero = 0;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_store), &zero, 4));
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      const int reps = 5;
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_store), &one, 4));
      CK(hipMemset(dC, 0, 4096));
      launch();
      CK(hipDeviceSynchronize());
      // sampled check
      double maxerr = 0;
      for (int t = 0; t < 16; ++t) {
        const int m = (t * 7919 + 13) % sh.M, n = (t * 104729 + 7) % sh.N;
        float got;
        CK(hipMemcpy(&got, dC + (long)m * sh.N + n, 4, hipMemcpyDeviceToHost));
        double ref = 0;
        for (int k = 0; k < sh.K; ++k)
          ref += (double)bf2f(hA[(long)m * sh.K + k]) * bf2f(hW[(long)n * sh.K + k]);
        maxerr = fmax(maxerr, fabs(ref - got));
      }
      printf("%-4s %-34s %8.1f us %7.1f TF/s  maxerr %.2e\n", sh.name, name, ms * 1e3,
             flop / (ms * 1e-3) / 1e12, maxerr);
      fflush(stdout);
    };
    const int M = sh.M, N = sh.N, K = sh.K;

#define V(BM_, BN_, WM_, WN_, NST_, MINB_, REMAP)                                              \
    run("glds " #BM_ "x" #BN_ " w" #WM_ "x" #WN_ " st" #NST_ " mb" #MINB_ " rm" #REMAP, [&] { \
      const int nb = ((M + BM_ - 1) / BM_) * ((N + BN_ - 1) / BN_);                           \
      gemm_v<BM_, BN_, WM_, WN_, NST_, MINB_><<<nb, 64 * WM_ * WN_>>>(dA, dW, dC, M, N, K,  \
                                                                     REMAP);               \
    })
    V(256, 256, 2, 4, 2, 1, 1);
    run("pf4 256x256 bk32 st4 frag-prefetch", [&] {
      const int nb = ((M + 255) / 256) * ((N + 255) / 256);
      gemm_pf4<0><<<nb, 512>>>(dA, dW, dC, M, N, K, 1);
    });
    run("pf4 DIAG1 no DMA wait", [&] {
      const int nb = ((M + 255) / 256) * ((N + 255) / 256);
      gemm_pf4<1><<<nb, 512>>>(dA, dW, dC, M, N, K, 1);
    });
    run("glds 256x256 DIAG1 no DMA wait", [&] {
      const int nb = ((M + 255) / 256) * ((N + 255) / 256);
      gemm_v<256, 256, 2, 4, 2, 1, 1><<<nb, 512>>>(dA, dW, dC, M, N, K, 1);
    });
    run("glds 256x256 DIAG2 no wait/barrier", [&] {
      const int nb = ((M + 255) / 256) * ((N + 255) / 256);
      gemm_v<256, 256, 2, 4, 2, 1, 2><<<nb, 512>>>(dA, dW, dC, M, N, K, 1);
    });
  }
  return 0;
}
