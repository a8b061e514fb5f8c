// PROBE (measured, not kept in libmwx.so; compiled into dec_chain_probe.hip):
// decoder-layer seams in one launch (gfx950): [producer split-K GEMM] ->
// LayerNorm of the step's rows -> consumer GEMM. Bit-identical to the three
// separate launches, but not faster: at large-v3 / 32 rows the fused seam took
// 10.4 / 17.2 / 13.3 us against 8.8 / 13.9 / 13.8 us for the three launches
// (out-proj / FFN2 / cross-out seams; a whole layer 89.1 vs 85.0 us,
// profiles/r04_chain_seams.txt): every in-launch hand-off pays a write-through
// drain, an atomic and a poll (about three memory round trips) where a launch
// boundary costs ~1.8 us (MI355X_MICROARCH.md price list, "splitk-seam").
//
// A decode step of a large-v3 layer at 32 rows is a chain of latency-bound
// launches (~1.8 us per launch boundary, scripts/probe/dec_chain_probe.hip);
// three of them are LayerNorms that sit between two GEMMs (out-proj -> LN2 ->
// cross-Q, cross-out -> LN3 -> FFN1, FFN2 -> LN1 -> QKV). This kernel runs
// such a triple as one grid of three block roles, ordered by block id:
//
//   [0, n1)          producer split-K GEMM blocks (exactly gemm_splitk's
//                    per-block arithmetic); each stores its f32 slab tile
//                    write-through (sc1) and adds 1 to its row block's counter;
//   [n1, n1 + M)     one LayerNorm block per row (exactly ln_dec_kernel's
//                    arithmetic): loads what does not depend on the producer
//                    (x, bias, LN weights), waits until the producer blocks of
//                    its row block have all arrived, reads their slabs (sc1),
//                    writes x and the packed normalised row (sc1) and arrives;
//   [n1 + M, ...)    consumer GEMM blocks (gemm_splitk's or, for FFN1, the
//                    4-wave gemm_skinny's arithmetic): issue their weight loads
//                    first, wait until the LayerNorm rows of their row block
//                    have arrived, then read the A fragments (sc1).
//
// So the consumer's weight stream overlaps the producer and the LayerNorm,
// and two launch boundaries go away. Hand-off form (MI355X_MICROARCH.md,
// "Valid forms", table row 1): the payload is stored sc1 (write-through) and
// loaded sc1 (L2-served, L1 bypassed); every storing wave waits vmcnt(0)
// before the one lane per block that adds to an agent-scope counter (behind
// a workgroup barrier when several waves stored); the block whose add came
// last (told by the value the add returned) signals onward; a waiter polls
// with sc1 loads and loads the payload only afterwards. To keep hundreds of
// arrivals and pollers off one cache line (the first version, one counter per
// row block, took 40 us per seam against 8.9 us for the three launches): the
// producer arrivals go to 8 shard counters (block id % 8), each shard's last
// arriver adds to a top counter the LayerNorm blocks poll, and the LayerNorm
// blocks' last arriver sets 32 ready-flag replicas the consumer blocks poll
// (block id % 32); every word on its own 128-B line. Blocks only ever wait
// for blocks of lower id (dispatched before them), and every wait is bounded
// (CHAIN_SPIN_TICKS of the 100-MHz device clock): a wait that runs out sets
// *err instead of hanging the GPU, and the host turns that into an error. A
// seam's counter slot is zeroed by the LayerNorm blocks of the seam launched
// after it (a.zero: the previous launch's slot, idle by stream order) and by
// the host before each decode loop.
#include <type_traits>

#include "kcommon.h"
#include "kernels.h"

namespace mwx {

// Decoder-layer seam in one launch (k_chain.hip): [producer split-K GEMM
// p_A x p_W -> slabs ln.P] -> LayerNorm of the M rows (x completed in place
// from the slabs + ln.pbias when there is a producer) into ln.y (packed A
// tiles) -> consumer GEMM ln.y x c_W: split-K slabs c_P [c_ks][M][c_N], or
// (c_skinny) the full-K 4-wave GEMM with c_epi's EPI_GELU packed epilogue.
// Same per-element arithmetic as gemm_splitk_partials + layer_norm_dec +
// gemm_splitk_partials / gemm_decode(EPI_GELU, nw = 4). M <= 64, d % 128 == 0,
// 16-bit weights. err: set if a hand-off wait timed out. Returns false if the
// shape is unsupported.
struct ChainLn {
  float* x = nullptr;
  const float* w = nullptr;
  const float* b = nullptr;
  const float* P = nullptr;  // the producer's slab buffer [KS][M][d] (KS set by chain_launch)
  int KS = 0;
  const float* pbias = nullptr;
  void* y = nullptr;
  const int* active = nullptr;
};
struct ChainArgs {
  int M = 0, d = 0;
  const void* p_A = nullptr;
  const void* p_W = nullptr;  // nullptr: no producer (x complete)
  int p_K = 0, p_ks = 0, p_kch = 0;
  ChainLn ln;
  const void* c_W = nullptr;
  int c_N = 0;
  bool c_skinny = false;
  int c_ks = 0, c_kch = 0;
  float* c_P = nullptr;
  EpiParams c_epi;
  unsigned* ctr = nullptr;   // this seam's counter slot (chain_slot_words(), zero at launch)
  unsigned* zero = nullptr;  // a slot to zero (the previous seam launch's), or nullptr
  int nzero = 0;
  unsigned* err = nullptr;
};
int chain_slot_words();
template <typename T>
bool chain_launch(const ChainArgs& a, hipStream_t st);

constexpr uint64_t CHAIN_SPIN_TICKS = 10000000;  // 100 ms at 100 MHz

__device__ __forceinline__ void st_sc1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1_16(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// (the caller waits vmcnt(0) before using the value: the compiler does not
// track loads issued by inline asm)
__device__ __forceinline__ u32x4 ld_sc1_16(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// counter slot of one seam: per row block (<= 4) CH_RB_WORDS words, one
// counter per 128-B line (32 words): lines 0-7 producer shard counters, 8 the
// producer top counter, 9 the LayerNorm arrivals, 10-41 the ready replicas
constexpr int CH_LINE = 32, CH_SHARDS = 8, CH_REPL = 32;
constexpr int CH_RB_WORDS = (CH_SHARDS + 2 + CH_REPL) * CH_LINE;
__device__ __forceinline__ unsigned* ch_shard(unsigned* slot, int rb, int sh) {
  return slot + rb * CH_RB_WORDS + sh * CH_LINE;
}
__device__ __forceinline__ unsigned* ch_top(unsigned* slot, int rb) {
  return slot + rb * CH_RB_WORDS + CH_SHARDS * CH_LINE;
}
__device__ __forceinline__ unsigned* ch_lncnt(unsigned* slot, int rb) {
  return slot + rb * CH_RB_WORDS + (CH_SHARDS + 1) * CH_LINE;
}
__device__ __forceinline__ unsigned* ch_ready(unsigned* slot, int rb, int r) {
  return slot + rb * CH_RB_WORDS + (CH_SHARDS + 2 + r) * CH_LINE;
}
// ids in [lo, hi) congruent to sh mod 8
__device__ __forceinline__ int ch_count_mod8(int lo, int hi, int sh) {
  auto f = [sh](int x) { return x > sh ? (x - sh + 7) / 8 : 0; };
  return f(hi) - f(lo);
}

// thread 0 polls *ctr (sc1 loads, s_sleep `nap` between polls) until it
// reaches `target`, then the whole block proceeds; bounded: on time-out *err
// is set and the block goes on
__device__ __forceinline__ void chain_wait(const unsigned* ctr, unsigned target, unsigned* err,
                                           int nap) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (nap >= 4)
        __builtin_amdgcn_s_sleep(4);
      else
        __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > CHAIN_SPIN_TICKS) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}
// after every storing wave's vmcnt(0) wait and a workgroup barrier, one lane
// adds 1 to *ctr; returns (to every thread) whether this block's add was the
// `n`-th, i.e. the last
__device__ __forceinline__ bool chain_arrive(unsigned* ctr, unsigned n, unsigned* flag) {
  vm_drain();
  __syncthreads();
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == n;
  __syncthreads();
  return *flag != 0;
}

template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 as_v8(u32x4 u) {
  return __builtin_bit_cast(typename Elt<T>::v8, u);
}

constexpr int CH_KMAX = 5;   // split-K k-steps per wave (splitk_factor: 1..5)
constexpr int CH_SKMAX = 10; // skinny (4 waves) k-steps per wave

// ---- split-K block (gemm_splitk<T, 1, kch> arithmetic, MT = 1) ----
// A_SC1: the A fragments were handed off in this launch (sc1 loads after the
// wait); P_SC1: the slab tile is handed off in this launch (sc1 stores).
template <typename T, bool A_SC1, bool P_SC1>
__device__ __forceinline__ void ch_splitk_block(const T* __restrict__ Ap, const T* __restrict__ W,
                                                int KT, int M, int N, int kslice, int kch,
                                                float* __restrict__ P, int bx, int ks, int bz,
                                                const unsigned* wait_ctr, unsigned wait_target,
                                                unsigned* err, f32x4 (*red)[64]) {
  using V8 = typename Elt<T>::v8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = bx * 16;
  const int m_base = bz * 16;
  const int Mb = min(16, M - m_base);
  const int kt0 = (ks * kslice >> 5) + wid * kch;
  const long f0 = (long)bx * KT + kt0;
  const T* at = Ap + ((long)bz * KT + kt0) * 512 + lane * 8;
  V8 bfr[CH_KMAX], afr[CH_KMAX];
  const T* wt = W + f0 * 512 + lane * 8;
#pragma unroll
  for (int c = 0; c < CH_KMAX; ++c)
    if (c < kch) bfr[c] = *reinterpret_cast<const V8*>(wt + c * 512);
  if constexpr (A_SC1) {
    chain_wait(wait_ctr, wait_target, err, 4);
    u32x4 raw[CH_KMAX];
#pragma unroll
    for (int c = 0; c < CH_KMAX; ++c)
      if (c < kch) raw[c] = ld_sc1_16(at + c * 512);
    vm_drain();
#pragma unroll
    for (int c = 0; c < CH_KMAX; ++c)
      if (c < kch) afr[c] = as_v8<T>(raw[c]);
  } else {
#pragma unroll
    for (int c = 0; c < CH_KMAX; ++c)
      if (c < kch) afr[c] = *reinterpret_cast<const V8*>(at + c * 512);
  }
  f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < CH_KMAX; ++c)
    if (c < kch) acc = Elt<T>::mfma(afr[c], bfr[c], acc);
  red[wid][lane] = acc;
  __syncthreads();
  if (wid != 0) return;
  const int n = n0 + (lane & 15);
  if (n >= N) return;
  float* Pk = P + (long)ks * M * N;
  const f32x4 v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = (lane >> 4) * 4 + r;
    if (m < Mb) {
      if constexpr (P_SC1)
        st_sc1(Pk + (long)(m_base + m) * N + n, v[r]);
      else
        Pk[(long)(m_base + m) * N + n] = v[r];
    }
  }
}

// ---- skinny block, 4 waves x kch k-steps (gemm_skinny<T, 1, kch> with NW = 4) ----
// epilogue EPI_GELU with packed output (FFN1)
template <typename T>
__device__ __forceinline__ void ch_skinny_block(const T* __restrict__ Ap, const T* __restrict__ W,
                                                int KT, int M, int N, int kch, const EpiParams& E,
                                                int bx, int by, const unsigned* wait_ctr,
                                                unsigned wait_target, unsigned* err,
                                                f32x4 (*red)[64]) {
  using V8 = typename Elt<T>::v8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = bx * 16;
  const int m_base = by * 16;
  const int Mb = min(16, M - m_base);
  const int kt0 = wid * kch;
  const long f0 = (long)bx * KT + kt0;
  const T* at = Ap + ((long)by * KT + kt0) * 512 + lane * 8;
  V8 bfr[CH_SKMAX], afr[CH_SKMAX];
  const T* wt = W + f0 * 512 + lane * 8;
#pragma unroll
  for (int c = 0; c < CH_SKMAX; ++c)
    if (c < kch) bfr[c] = *reinterpret_cast<const V8*>(wt + c * 512);
  chain_wait(wait_ctr, wait_target, err, 4);
  {
    u32x4 raw[CH_SKMAX];
#pragma unroll
    for (int c = 0; c < CH_SKMAX; ++c)
      if (c < kch) raw[c] = ld_sc1_16(at + c * 512);
    vm_drain();
#pragma unroll
    for (int c = 0; c < CH_SKMAX; ++c)
      if (c < kch) afr[c] = as_v8<T>(raw[c]);
  }
  f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < CH_SKMAX; ++c)
    if (c < kch) acc = Elt<T>::mfma(afr[c], bfr[c], acc);
  red[wid][lane] = acc;
  __syncthreads();
  if (wid != 0) return;
  for (int w = 1; w < 4; ++w) acc += red[w][lane];
  const int n = n0 + (lane & 15);
  if (n >= N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ml = (lane >> 4) * 4 + r;
    if (ml >= Mb) continue;
    const int m = m_base + ml;
    const float g = gelu_ggml(acc[r] + E.bias[n]);
    ((T*)E.c16)[pack_index(m, n, E.ldc)] = to_t<T>(g);
  }
}

// ---- LayerNorm block of one row (ln_dec_kernel arithmetic) ----
template <typename T>
__device__ __forceinline__ void ch_ln_block(const ChainLn& L, int row, int N, int M,
                                            const unsigned* wait_ctr, unsigned wait_target,
                                            unsigned* slot, unsigned* err, double (*red)[4],
                                            unsigned* flag) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool own = tid * 8 < N;
  const int i0 = own ? tid * 8 : 0;
  float* xr = L.x + (long)row * N + i0;
  const f32x4 xa = *reinterpret_cast<const f32x4*>(xr);
  const f32x4 xc = *reinterpret_cast<const f32x4*>(xr + 4);
  f32x4 pb0 = {0, 0, 0, 0}, pb1 = {0, 0, 0, 0};
  if (L.P) {
    pb0 = *reinterpret_cast<const f32x4*>(L.pbias + i0);
    pb1 = *reinterpret_cast<const f32x4*>(L.pbias + i0 + 4);
  }
  const f32x4 w0 = *reinterpret_cast<const f32x4*>(L.w + i0);
  const f32x4 w1 = *reinterpret_cast<const f32x4*>(L.w + i0 + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(L.b + i0);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(L.b + i0 + 4);
  const int act_r = L.active ? L.active[row] : 1;
  f32x4 pk[8][2];
  if (L.P) {
    chain_wait(wait_ctr, wait_target, err, 2);
    const long pstride = (long)M * N;
    const float* pp = L.P + (long)row * N + i0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < L.KS) {
        pk[k][0] = __builtin_bit_cast(f32x4, ld_sc1_16(pp + k * pstride));
        pk[k][1] = __builtin_bit_cast(f32x4, ld_sc1_16(pp + k * pstride + 4));
      }
    vm_drain();
  }
  const int rb = row / 16;
  const unsigned rows_rb = (unsigned)min(16, M - 16 * rb);
  // the row block's last LayerNorm block sets the consumers' ready replicas
  auto arrive = [&]() {
    if (chain_arrive(ch_lncnt(slot, rb), rows_rb, flag) && threadIdx.x < CH_REPL) {
      vm_drain();
      asm volatile("global_store_dword %0, %1, off sc1" ::"v"(ch_ready(slot, rb, threadIdx.x)),
                   "v"(1u) : "memory");
    }
  };
  if (!act_r) {
    arrive();
    return;
  }
  float v[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = xa[e];
    v[4 + e] = xc[e];
  }
  if (L.P) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float acc = pk[0][e >> 2][e & 3];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (k < L.KS) acc += pk[k][e >> 2][e & 3];
      v[e] = (acc + (e < 4 ? pb0[e] : pb1[e - 4])) + v[e];
    }
    if (own) {
      *reinterpret_cast<f32x4*>(xr) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(xr + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
  double s = 0.0;
  if (own) {
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (double)v[e];
  }
  s = wave_sum_d_dpp(s);
  if (lane == 0) red[0][wid] = s;
  __syncthreads();
  s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const float mean = (float)(s / N);
  double s2 = 0.0;
  if (own) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - mean;
      s2 += (double)(d * d);
    }
  }
  s2 = wave_sum_d_dpp(s2);
  if (lane == 0) red[1][wid] = s2;
  __syncthreads();
  s2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const float variance = (float)(s2 / N);
  const float scale = 1.0f / sqrtf(variance + 1e-5f);
  if (own) {
    typename Elt<T>::v8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      o[e] = to_t<T>(((v[e] - mean) * scale) * (e < 4 ? w0[e] : w1[e - 4]) +
                     (e < 4 ? b0[e] : b1[e - 4]));
    st_sc1_16((T*)L.y + pack_index(row, i0, N), __builtin_bit_cast(u32x4, o));
  }
  arrive();
}

template <typename T, bool PROD, bool SKINNY>
__global__ __launch_bounds__(256) void chain_kernel(ChainArgs a) {
  __shared__ f32x4 red[4][64];
  __shared__ double lred[2][4];
  __shared__ unsigned flag;
  const int N = a.d;  // LayerNorm width = producer N = consumer K
  int b = blockIdx.x;
  unsigned* slot = a.ctr;
  const int nx = (N + 15) / 16;
  const int per_rb = PROD ? nx * a.p_ks : 0;  // producer blocks per row block
  const int nrb = (a.M + 15) / 16;
  const int n1 = per_rb * nrb;
  if (PROD && b < n1) {
    const int bx = b % nx, ks = (b / nx) % a.p_ks, bz = b / per_rb;
    ch_splitk_block<T, false, true>((const T*)a.p_A, (const T*)a.p_W, a.p_K / 32, a.M, N,
                                    a.p_K / a.p_ks, a.p_kch, (float*)a.ln.P, bx, ks, bz, nullptr,
                                    0, a.err, red);
    // (only wave 0 stored the slab tile: its own drain suffices, the other
    // waves returned from the block body; the barrier in chain_arrive needs
    // every wave, so the drain and the adds are done by wave 0 alone here)
    if ((threadIdx.x >> 6) == 0) {
      vm_drain();
      if (threadIdx.x == 0) {
        const int sh = b % CH_SHARDS;
        const unsigned n_sh = (unsigned)ch_count_mod8(bz * per_rb, (bz + 1) * per_rb, sh);
        if (__hip_atomic_fetch_add(ch_shard(slot, bz, sh), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) + 1 == n_sh)
          __hip_atomic_fetch_add(ch_top(slot, bz), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  b -= n1;
  if (b < a.M) {
    // (zero the previous seam launch's counter slot: idle by stream order)
    if (a.zero)
      for (int i = b * 256 + threadIdx.x; i < a.nzero; i += a.M * 256) a.zero[i] = 0u;
    const int rb = b / 16;
    unsigned shards = 0;
    for (int sh = 0; sh < CH_SHARDS; ++sh)
      shards += ch_count_mod8(rb * per_rb, (rb + 1) * per_rb, sh) > 0 ? 1u : 0u;
    ch_ln_block<T>(a.ln, b, N, a.M, ch_top(slot, rb), shards, slot, a.err, lred, &flag);
    return;
  }
  b -= a.M;
  {
    const int nxc = (a.c_N + 15) / 16;
    const int KT = N / 32;
    const int rep = blockIdx.x % CH_REPL;
    if (SKINNY) {
      const int bx = b % nxc, by = b / nxc;
      ch_skinny_block<T>((const T*)a.ln.y, (const T*)a.c_W, KT, a.M, a.c_N, a.c_kch, a.c_epi, bx,
                         by, ch_ready(slot, by, rep), 1u, a.err, red);
    } else {
      const int bx = b % nxc, ks = (b / nxc) % a.c_ks, bz = b / (nxc * a.c_ks);
      ch_splitk_block<T, true, false>((const T*)a.ln.y, (const T*)a.c_W, KT, a.M, a.c_N,
                                      N / a.c_ks, a.c_kch, a.c_P, bx, ks, bz,
                                      ch_ready(slot, bz, rep), 1u, a.err, red);
    }
  }
}

int chain_slot_words() { return 4 * CH_RB_WORDS; }

template <typename T>
bool chain_launch(const ChainArgs& a0, hipStream_t st) {
  ChainArgs a = a0;
  const int N = a.d;
  if (a.M < 1 || a.M > 64 || N % 128 || N > 2048) return false;
  const int nrb = (a.M + 15) / 16;
  const bool prod = a.p_W != nullptr;
  if (prod) {
    a.p_ks = splitk_factor(a.p_K);
    if (a.p_ks == 0) return false;
    a.p_kch = a.p_K / a.p_ks / 128;
    if (a.p_kch < 1 || a.p_kch > CH_KMAX) return false;
    a.ln.KS = a.p_ks;
  } else {
    a.ln.P = nullptr;
    a.ln.KS = 0;
  }
  const bool skinny = a.c_skinny;
  int nc = 0;
  if (skinny) {
    if ((N / 32) % 4) return false;
    a.c_kch = N / 32 / 4;
    if (a.c_kch > CH_SKMAX) return false;
    nc = (a.c_N + 15) / 16 * nrb;
  } else {
    a.c_ks = splitk_factor(N);
    if (a.c_ks == 0) return false;
    a.c_kch = N / a.c_ks / 128;
    if (a.c_kch < 1 || a.c_kch > CH_KMAX) return false;
    nc = (a.c_N + 15) / 16 * a.c_ks * nrb;
  }
  const int n1 = prod ? (N + 15) / 16 * a.p_ks * nrb : 0;
  const dim3 g(n1 + a.M + nc), blk(256);
  if (prod) {
    if (skinny)
      chain_kernel<T, true, true><<<g, blk, 0, st>>>(a);
    else
      chain_kernel<T, true, false><<<g, blk, 0, st>>>(a);
  } else {
    if (skinny)
      chain_kernel<T, false, true><<<g, blk, 0, st>>>(a);
    else
      chain_kernel<T, false, false><<<g, blk, 0, st>>>(a);
  }
  return true;
}

template bool chain_launch<_Float16>(const ChainArgs&, hipStream_t);
template bool chain_launch<__bf16>(const ChainArgs&, hipStream_t);

}  // namespace mwx
