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
    const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + n;
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

  uint4 ra[4], rw[4];
  const T* ap[4];
  const T* wp[4];
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 3, kc = c & 7;
    const int gm = min(m0 + row, M - 1);
    const int gn = min(n0 + row, N - 1);
    ap[i] = A + (long)gm * lda + kc * 8;
    wp[i] = W + (long)gn * ldw + kc * 8;
    soff[i] = row * BK + ((kc ^ (row & 7)) << 3);
  }
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const uint4*>(ap[i] + kt * BK);
      rw[i] = *reinterpret_cast<const uint4*>(wp[i] + kt * BK);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(&lds[buf][0][soff[i]]) = ra[i];
      *reinterpret_cast<uint4*>(&lds[buf][1][soff[i]]) = rw[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  gload(0);
  sstore(0);
  __syncthreads();
  const int nk = K / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
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
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
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
// skinny (decode) GEMM: M <= 16*MT rows
// ---------------------------------------------------------------------------
template <typename T, int EPI, bool OUT16, int MT, int WN>
__global__ __launch_bounds__(256) void gemm_skinny(const T* __restrict__ A, long lda,
                                                   const T* __restrict__ W, long ldw, int M,
                                                   int N, int K, EpiParams P) {
  using V8 = typename Elt<T>::v8;
  constexpr int WK = 4 / WN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wn = wid % WN, wk = wid / WN;
  const int n0 = (blockIdx.x * WN + wn) * 16;
  const int ncol = min(n0 + (lane & 15), N - 1);
  const T* wrow = W + (long)ncol * ldw + (lane >> 4) * 8;
  const T* arow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = min(mt * 16 + (lane & 15), M - 1);
    arow[mt] = A + (long)row * lda + (lane >> 4) * 8;
  }
  const int kper = K / WK;
  const int kb = wk * kper;
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0, 0, 0, 0};
  for (int k = kb; k < kb + kper; k += 32) {
    const V8 b = ld8(wrow + k);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = Elt<T>::mfma(ld8(arow[mt] + k), b, acc[mt]);
  }
  if constexpr (WK > 1) {
    __shared__ f32x4 red[4][MT][64];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
    __syncthreads();
    if (wk != 0) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int w = 1; w < WK; ++w) acc[mt] += red[w * WN + wn][mt][lane];
  }
  const int n = n0 + (lane & 15);
  if (n >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 16 + (lane >> 4) * 4 + r;
      if (m < M) epi_store<EPI, T, OUT16>(P, 0, m, n, acc[mt][r]);
    }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
template <typename T, int EPI, bool OUT16>
static void gemm_dispatch(const T* A, long lda, long a_bstride, const T* W, long ldw, int M,
                          int N, int K, int batch, const EpiParams& P, hipStream_t st) {
  if (batch == 1 && M <= 64 && (K % 128) == 0) {
    const int MT = (M + 15) / 16;
    const bool wide = N >= 4096;
#define SKINNY(MTV)                                                                         \
  if (MT == MTV) {                                                                          \
    if (wide)                                                                               \
      gemm_skinny<T, EPI, OUT16, MTV, 4><<<(N + 63) / 64, 256, 0, st>>>(A, lda, W, ldw, M, \
                                                                         N, K, P);          \
    else                                                                                    \
      gemm_skinny<T, EPI, OUT16, MTV, 1><<<(N + 15) / 16, 256, 0, st>>>(A, lda, W, ldw, M, \
                                                                         N, K, P);          \
    return;                                                                                 \
  }
    SKINNY(1)
    SKINNY(2)
    SKINNY(3)
    SKINNY(4)
#undef SKINNY
  }
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
