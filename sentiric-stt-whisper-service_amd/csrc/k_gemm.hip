// MFMA GEMMs for gfx950 with ggml-faithful fused epilogues.
//
// C[m][n] = sum_k A[m][k] * W[n][k]: both operands K-contiguous (W is the ggml
// [out][in] weight layout), f16 or bf16 inputs, f32 accumulation on
// v_mfma_f32_16x16x32_{f16,bf16}. Replaces ggml_mul_mat (+ the ggml_add /
// ggml_scale / ggml_gelu / ggml_cpy nodes that follow it in whisper.cpp's
// encoder, cross and decoder graphs — SURVEY.md §2.2 rows 2-11).
//
// Two kernels:
//  * gemm_big:    128x128x64 tiles, 4 waves (2x2, 64x64 per wave), operands
//                 staged through double-buffered LDS with an XOR swizzle (16-B
//                 chunk ^= row & 7) so the ds_read_b128 fragment reads are
//                 bank-conflict free; register-staged prefetch of tile k+1
//                 during the MFMAs of tile k, one barrier per K tile.
//                 Encoder / conv / cross-KV GEMMs (M = clips x 1500).
//  * gemm_skinny: decode GEMMs (M <= 64 rows): weight-streaming, fragments
//                 loaded straight to VGPRs (no LDS round trip), 4 waves split
//                 K (or N for wide outputs), LDS reduction, one 16-column
//                 strip per wave.
#include <algorithm>

#include "kcommon.h"
#include "kernels.h"

namespace mwx {

template <int EPI, typename T, bool OUT16>
__device__ __forceinline__ void epi_store(const EpiParams& P, int bz, int m, int n, float acc) {
  if constexpr (EPI == EPI_ENC_QKV) {
    const int d = P.d;
    const int part = n / d;
    const int nn = n - part * d;
    const int h = nn >> 6, e = nn & 63;
    const int b = m / P.L, t = m - b * P.L;
    const _Float16 hv = (_Float16)(acc + P.bias[n]);
    if (part == 0)
      P.q[(((long)b * P.H + h) * P.L + t) * 64 + e] = hv;
    else if (part == 1)
      P.k[(((long)b * P.H + h) * P.L + t) * 64 + e] = hv;
    else
      P.v[(((long)b * P.H + h) * 64 + e) * P.ldv + t] = hv;
  } else if constexpr (EPI == EPI_GELU) {
    const float g = gelu_ggml(acc + P.bias[n]);
    const long idx = P.pack_out ? pack_index(m, n, P.ldc)
                                : (long)bz * P.c_bstride + (long)m * P.ldc + n;
    if constexpr (OUT16)
      ((_Float16*)P.c16)[idx] = (_Float16)g;
    else
      ((T*)P.c16)[idx] = to_t<T>(g);
  } else if constexpr (EPI == EPI_RES) {
    const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + n;
    const float b = P.bias ? P.bias[n] : 0.0f;
    P.c32[idx] = (acc + b) + P.r32[idx];
  } else if constexpr (EPI == EPI_CONV2) {
    const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + n;
    P.c32[idx] = P.pe[(long)m * P.ldc + n] + gelu_ggml(acc + P.bias[n]);
  } else if constexpr (EPI == EPI_F32) {
    P.c32[(long)bz * P.c_bstride + (long)m * P.ldc + n] = acc;
  } else if constexpr (EPI == EPI_CROSS_KV) {
    const int d = P.d;
    const int layer = n / (2 * d);
    const int r = n - layer * 2 * d;
    const int kv = r >= d;
    const int nn = r - kv * d;
    const int h = nn >> 6, e = nn & 63;
    const int bl = m / P.L, t = m - bl * P.L;
    const long idx = ((((long)layer * P.ncap + P.slot[bl]) * P.H + h) * P.L + t) * 64 + e;
    if (!kv)
      P.k[idx] = (_Float16)(acc * P.kscale);
    else
      P.v[idx] = (_Float16)(acc + P.bias[n]);
  } else if constexpr (EPI == EPI_DEC_QKV) {
    if (!P.active[m]) return;
    const int d = P.d;
    const int part = n / d;
    const int nn = n - part * d;
    const int h = nn >> 6, e = nn & 63;
    if (part == 0) {
      P.q[(long)m * d + nn] = (_Float16)((acc + P.bias[n]) * P.qscale);
    } else {
      const long idx = (((long)m * P.H + h) * P.L + P.pos[m]) * 64 + e;
      if (part == 1)
        P.k[idx] = (_Float16)(acc * P.kscale);
      else
        P.v[idx] = (_Float16)(acc + P.bias[n]);
    }
  } else if constexpr (EPI == EPI_STORE16) {
    ((_Float16*)P.c16)[(long)m * P.ldc + n] = (_Float16)(acc + P.bias[n]);
  }
}

template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 ld8(const T* p) {
  return *reinterpret_cast<const typename Elt<T>::v8*>(p);
}

// ---------------------------------------------------------------------------
// big tile GEMM
// ---------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;

template <typename T, int EPI, bool OUT16>
__global__ __launch_bounds__(256, 2) void gemm_big(const T* __restrict__ A, long lda,
                                                   long a_bstride, const T* __restrict__ W,
                                                   long ldw, int M, int N, int K, EpiParams P) {
  using V8 = typename Elt<T>::v8;
  __shared__ __attribute__((aligned(16))) T lds[2][2][BM * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int bz = blockIdx.z;
  A += (long)bz * a_bstride;

  // staging: thread t moves 16-B chunk (row = t/8 + 32 i, kc = t%8) of both
  // 128x64 tiles; rows past M / N are clamped (their outputs are discarded)
  const int srow = tid >> 3, kc0 = tid & 7;
  const T* a0 = A + (long)min(m0 + srow, M - 1) * lda + kc0 * 8;
  const T* a1 = A + (long)min(m0 + srow + 32, M - 1) * lda + kc0 * 8;
  const T* a2 = A + (long)min(m0 + srow + 64, M - 1) * lda + kc0 * 8;
  const T* a3 = A + (long)min(m0 + srow + 96, M - 1) * lda + kc0 * 8;
  const T* w0 = W + (long)min(n0 + srow, N - 1) * ldw + kc0 * 8;
  const T* w1 = W + (long)min(n0 + srow + 32, N - 1) * ldw + kc0 * 8;
  const T* w2 = W + (long)min(n0 + srow + 64, N - 1) * ldw + kc0 * 8;
  const T* w3 = W + (long)min(n0 + srow + 96, N - 1) * ldw + kc0 * 8;
  // swizzled LDS offsets: (row & 7) is the same for rows srow + 32 i
  const int soff0 = srow * BK + ((kc0 ^ (srow & 7)) << 3);
  constexpr int SROW32 = 32 * BK;
  uint4 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define GLOAD(kt)                                                   \
  do {                                                              \
    const int ko = (kt) * BK;                                       \
    ra0 = *reinterpret_cast<const uint4*>(a0 + ko);                 \
    ra1 = *reinterpret_cast<const uint4*>(a1 + ko);                 \
    ra2 = *reinterpret_cast<const uint4*>(a2 + ko);                 \
    ra3 = *reinterpret_cast<const uint4*>(a3 + ko);                 \
    rw0 = *reinterpret_cast<const uint4*>(w0 + ko);                 \
    rw1 = *reinterpret_cast<const uint4*>(w1 + ko);                 \
    rw2 = *reinterpret_cast<const uint4*>(w2 + ko);                 \
    rw3 = *reinterpret_cast<const uint4*>(w3 + ko);                 \
  } while (0)
#define SSTORE(buf)                                                                 \
  do {                                                                              \
    *reinterpret_cast<uint4*>(&lds[buf][0][soff0]) = ra0;                           \
    *reinterpret_cast<uint4*>(&lds[buf][0][soff0 + SROW32]) = ra1;                  \
    *reinterpret_cast<uint4*>(&lds[buf][0][soff0 + 2 * SROW32]) = ra2;              \
    *reinterpret_cast<uint4*>(&lds[buf][0][soff0 + 3 * SROW32]) = ra3;              \
    *reinterpret_cast<uint4*>(&lds[buf][1][soff0]) = rw0;                           \
    *reinterpret_cast<uint4*>(&lds[buf][1][soff0 + SROW32]) = rw1;                  \
    *reinterpret_cast<uint4*>(&lds[buf][1][soff0 + 2 * SROW32]) = rw2;              \
    *reinterpret_cast<uint4*>(&lds[buf][1][soff0 + 3 * SROW32]) = rw3;              \
  } while (0)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  GLOAD(0);
  SSTORE(0);
  __syncthreads();
  const int nk = K / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) GLOAD(kt + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      V8 af[4], bf[4];
      const int kc = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const V8*>(&lds[cur][0][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + (lane & 15);
        bf[j] = *reinterpret_cast<const V8*>(&lds[cur][1][row * BK + ((kc ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Elt<T>::mfma(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < nk) SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef GLOAD
#undef SSTORE
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N) epi_store<EPI, T, OUT16>(P, bz, m, n, acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------
// skinny (decode) GEMM: M <= 16*MT rows. One workgroup = one 16-column strip;
// its NW waves split K, each wave owns KCH consecutive 32-deep k-steps and
// issues all of its W and A fragment loads before the first MFMA (one memory
// round trip per launch), then the NW partial tiles are summed through LDS.
// ---------------------------------------------------------------------------
template <int EPI, typename T, bool OUT16>
__device__ __forceinline__ void skinny_store(const EpiParams& P, int m, int n, float v) {
  epi_store<EPI, T, OUT16>(P, 0, m, n, v);
}

template <typename T, int MT, int KCH>
__global__ __launch_bounds__(1024) void gemm_skinny(int epi, const T* __restrict__ Ap,
                                                    const T* __restrict__ Wp, int KT, int M,
                                                    int N, EpiParams P) {
  using V8 = typename Elt<T>::v8;
  __shared__ f32x4 red[16][MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int n0 = blockIdx.x * 16;
  // row block of 64 (grid.y): per-row arithmetic does not depend on M
  const int m_base = blockIdx.y * 64;
  const int Mb = min(64, M - m_base);
  const int kt0 = wid * KCH;
  const T* wt = Wp + ((long)blockIdx.x * KT + kt0) * 512 + lane * 8;
  const T* at = Ap + ((long)(blockIdx.y * 4) * KT + kt0) * 512 + lane * 8;
  V8 bfr[KCH];
  V8 afr[MT][KCH];
#pragma unroll
  for (int c = 0; c < KCH; ++c) bfr[c] = ld8(wt + c * 512);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < KCH; ++c) afr[mt][c] = ld8(at + ((long)mt * KT + c) * 512);
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < KCH; ++c) acc[mt] = Elt<T>::mfma(afr[mt][c], bfr[c], acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    for (int w = 1; w < NW; ++w) acc[mt] += red[w][mt][lane];
  const int n = n0 + (lane & 15);
  if (n >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ml = mt * 16 + (lane >> 4) * 4 + r;
      if (ml >= Mb) continue;
      const int m = m_base + ml;
      const float v = acc[mt][r];
      switch (epi) {
        case EPI_GELU: skinny_store<EPI_GELU, T, false>(P, m, n, v); break;
        case EPI_RES: skinny_store<EPI_RES, T, false>(P, m, n, v); break;
        case EPI_F32: skinny_store<EPI_F32, T, false>(P, m, n, v); break;
        case EPI_DEC_QKV: skinny_store<EPI_DEC_QKV, T, false>(P, m, n, v); break;
        case EPI_STORE16: skinny_store<EPI_STORE16, T, false>(P, m, n, v); break;
        default: break;
      }
    }
}

// (waves, k-steps per wave) for a K: all 32-deep k-steps split evenly over at
// most 16 waves with at most 10 k-steps each.
static bool skinny_split(int K, int& nw, int& kch) {
  if (K % 32) return false;
  const int S = K / 32;
  for (int w = 16; w >= 1; --w) {
    if (S % w) continue;
    const int c = S / w;
    if (c == 1 || c == 2 || c == 3 || c == 4 || c == 6 || c == 8 || c == 10) {
      nw = w;
      kch = c;
      return true;
    }
  }
  return false;
}

template <typename T, int MT>
static bool skinny_launch(int epi, const T* Ap, const T* Wp, int M, int N, int K,
                          const EpiParams& P, hipStream_t st) {
  int nw = 0, kch = 0;
  if (!skinny_split(K, nw, kch)) return false;
  const dim3 g((N + 15) / 16, (M + 63) / 64), b(64 * nw);
  switch (kch) {
#define SK(C) \
  case C: gemm_skinny<T, MT, C><<<g, b, 0, st>>>(epi, Ap, Wp, K / 32, M, N, P); return true;
    SK(1) SK(2) SK(3) SK(4) SK(6) SK(8) SK(10)
#undef SK
    default: return false;
  }
}

// ---------------------------------------------------------------------------
// split-K decode GEMM: P[ks][m][n] = sum_{k in slice ks} A[m][k] * W[n][k]
// (raw f32 partials, no epilogue). Grid (N/16, KS): far more workgroups than
// 16-column strips alone, each reading only its K slice of A and W, so every
// CU streams a small share of the weights. The KS partials are summed (in ks
// order) by the consumer kernel together with the epilogue ggml applies
// (bias, residual, scale, f16 rounding), so the reduction costs no launch.
// ---------------------------------------------------------------------------
template <typename T, int MT, int KCH>
__global__ __launch_bounds__(256) void gemm_splitk(const T* __restrict__ Ap,
                                                   const T* __restrict__ Wp, int KT, int M,
                                                   int N, int kslice, float* __restrict__ P) {
  using V8 = typename Elt<T>::v8;
  __shared__ f32x4 red[4][MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16, ks = blockIdx.y;
  const int m_base = blockIdx.z * 64;  // row block (64 rows per grid.z slice)
  const int Mb = min(64, M - m_base);
  const int kt0 = (ks * kslice >> 5) + wid * KCH;
  const T* wt = Wp + ((long)blockIdx.x * KT + kt0) * 512 + lane * 8;
  const T* at = Ap + ((long)(blockIdx.z * 4) * KT + kt0) * 512 + lane * 8;
  V8 bfr[KCH];
  V8 afr[MT][KCH];
#pragma unroll
  for (int c = 0; c < KCH; ++c) bfr[c] = ld8(wt + c * 512);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < KCH; ++c) afr[mt][c] = ld8(at + ((long)mt * KT + c) * 512);
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < KCH; ++c) acc[mt] = Elt<T>::mfma(afr[mt][c], bfr[c], acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
  const int n = n0 + (lane & 15);
  if (n >= N) return;
  float* Pk = P + (long)ks * M * N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 v = (red[0][mt][lane] + red[1][mt][lane]) + (red[2][mt][lane] + red[3][mt][lane]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 16 + (lane >> 4) * 4 + r;
      if (m < Mb) Pk[(long)(m_base + m) * N + n] = v[r];
    }
  }
}

int splitk_factor(int K) {
  if (K % 128) return 0;
  const int S = K / 32;  // 32-deep k-steps
  for (int ks = 8; ks >= 1; --ks)
    if (S % ks == 0 && (S / ks) % 4 == 0 && (S / ks) / 4 <= 5) return ks;
  return 0;
}

template <typename T>
int gemm_splitk_partials(const T* Ap, const T* Wp, int M, int N, int K, float* P,
                         hipStream_t st) {
  const int ks = splitk_factor(K);
  if (ks == 0) return 0;
  const int kslice = K / ks;
  const int kch = kslice / 128;
  const int MT = (std::min(M, 64) + 15) / 16;
  const dim3 g((N + 15) / 16, ks, (M + 63) / 64);
#define SKL(MTV, C)                                                                       \
  if (MT == MTV && kch == C) {                                                            \
    gemm_splitk<T, MTV, C><<<g, 256, 0, st>>>(Ap, Wp, K / 32, M, N, kslice, P);        \
    return ks;                                                                            \
  }
#define SKM(MTV) SKL(MTV, 1) SKL(MTV, 2) SKL(MTV, 3) SKL(MTV, 4) SKL(MTV, 5)
  SKM(1) SKM(2) SKM(3) SKM(4)
#undef SKM
#undef SKL
  return 0;
}

template int gemm_splitk_partials<_Float16>(const _Float16*, const _Float16*, int, int, int, float*,
                                            hipStream_t);
template int gemm_splitk_partials<__bf16>(const __bf16*, const __bf16*, int, int, int, float*,
                                          hipStream_t);

template <typename T>
bool gemm_decode(int epi, const T* Ap, const T* Wp, int M, int N, int K, const EpiParams& P,
                 hipStream_t st) {
  const int MT = (std::min(M, 64) + 15) / 16;
  if (MT == 1) return skinny_launch<T, 1>(epi, Ap, Wp, M, N, K, P, st);
  if (MT == 2) return skinny_launch<T, 2>(epi, Ap, Wp, M, N, K, P, st);
  if (MT == 3) return skinny_launch<T, 3>(epi, Ap, Wp, M, N, K, P, st);
  return skinny_launch<T, 4>(epi, Ap, Wp, M, N, K, P, st);
}
template bool gemm_decode<_Float16>(int, const _Float16*, const _Float16*, int, int, int,
                                    const EpiParams&, hipStream_t);
template bool gemm_decode<__bf16>(int, const __bf16*, const __bf16*, int, int, int,
                                  const EpiParams&, hipStream_t);

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
template <typename T, int EPI, bool OUT16>
static void gemm_dispatch(const T* A, long lda, long a_bstride, const T* W, long ldw, int M,
                          int N, int K, int batch, const EpiParams& P, hipStream_t st) {
  dim3 g((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  gemm_big<T, EPI, OUT16><<<g, 256, 0, st>>>(A, lda, a_bstride, W, ldw, M, N, K, P);
}

template <typename T>
void gemm(int epi, bool out_f16, const T* A, long lda, long a_bstride, const T* W, long ldw,
          int M, int N, int K, int batch, const EpiParams& P, hipStream_t st) {
  switch (epi) {
    case EPI_ENC_QKV: gemm_dispatch<T, EPI_ENC_QKV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_GELU:
      if (out_f16)
        gemm_dispatch<T, EPI_GELU, true>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st);
      else
        gemm_dispatch<T, EPI_GELU, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st);
      break;
    case EPI_RES: gemm_dispatch<T, EPI_RES, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_CONV2: gemm_dispatch<T, EPI_CONV2, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_F32: gemm_dispatch<T, EPI_F32, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_CROSS_KV: gemm_dispatch<T, EPI_CROSS_KV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_DEC_QKV: gemm_dispatch<T, EPI_DEC_QKV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_STORE16: gemm_dispatch<T, EPI_STORE16, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    default: break;
  }
}

template void gemm<_Float16>(int, bool, const _Float16*, long, long, const _Float16*, long, int,
                             int, int, int, const EpiParams&, hipStream_t);
template void gemm<__bf16>(int, bool, const __bf16*, long, long, const __bf16*, long, int, int,
                           int, int, const EpiParams&, hipStream_t);

}  // namespace mwx
