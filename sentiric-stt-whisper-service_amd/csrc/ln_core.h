// The decode LayerNorm's per-row arithmetic (whisper.cpp ggml_norm(eps 1e-5)
// + ggml_mul + ggml_add after the residual add of the producing projection),
// shared by ln_dec_kernel (k_misc.hip) and the LayerNorm folded into the next
// split-K GEMM at one row (gemm_splitk LNF, k_gemm.hip): one 256-thread
// workgroup per row, thread t owns elements 8t .. 8t+7 (t < N / 8). Both
// callers inline the same statements, so their results are bit-identical
// (the library is built with -ffp-contract=off).
#pragma once

#include "kcommon.h"
#include "kernels.h"

namespace mwx {

// v += (sum of the KS split-K partials, in ks order) + pbias (ggml: the
// matmul + bias, then the residual add)
__device__ __forceinline__ void ln_fold8(float (&v)[8], const f32x4 (&pk)[8][2], int KS,
                                         const f32x4& pb0, const f32x4& pb1) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float acc = pk[0][e >> 2][e & 3];
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (k < KS) acc += pk[k][e >> 2][e & 3];
    v[e] = (acc + (e < 4 ? pb0[e] : pb1[e - 4])) + v[e];
  }
}

// mean and 1/sqrt(var + eps) of the row: double sums of the thread's 8
// elements, DPP wave sums, the four waves' sums combined in a fixed order.
// Every thread of the workgroup calls it (two __syncthreads inside); in a
// workgroup of more than 4 waves (gemm_skinny LNF) waves 4.. own no elements.
__device__ __forceinline__ void ln_stats(const float (&v)[8], bool own, int N,
                                         double (&red)[2][4], int lane, int wid, float& mean,
                                         float& scale) {
  double s = 0.0;
  if (own) {
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (double)v[e];
  }
  s = wave_sum_d_dpp(s);
  if (lane == 0 && wid < 4) red[0][wid] = s;
  __syncthreads();
  s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  mean = (float)(s / N);
  double s2 = 0.0;
  if (own) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - mean;
      s2 += (double)(d * d);
    }
  }
  s2 = wave_sum_d_dpp(s2);
  if (lane == 0 && wid < 4) red[1][wid] = s2;
  __syncthreads();
  s2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const float variance = (float)(s2 / N);
  scale = 1.0f / sqrtf(variance + 1e-5f);
}

template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 ln_out8(const float (&v)[8], float mean, float scale,
                                                       const f32x4& w0, const f32x4& w1,
                                                       const f32x4& b0, const f32x4& b1) {
  typename Elt<T>::v8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    o[e] = to_t<T>(((v[e] - mean) * scale) * (e < 4 ? w0[e] : w1[e - 4]) + (e < 4 ? b0[e] : b1[e - 4]));
  return o;
}

// The folded LayerNorm's prologue in a decode GEMM at one row (LnFuse,
// kernels.h): the row's residual and LayerNorm into srow (natural order, K
// elements); workgroup `writer` stores the residual to x_out. Every thread of
// the workgroup calls it (barriers inside, srow complete on return).
template <typename T>
__device__ __forceinline__ void ln_fold_prologue(const LnFuse& ln, int K, bool writer, T* srow,
                                                 double (&red)[2][4]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool own = tid * 8 < K;
  const int i0 = own ? tid * 8 : 0;
  const f32x4 xa = *reinterpret_cast<const f32x4*>(ln.x_in + i0);
  const f32x4 xc = *reinterpret_cast<const f32x4*>(ln.x_in + i0 + 4);
  f32x4 pk[8][2];
  f32x4 pb0, pb1;
  if (ln.P) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < ln.KS) {
        pk[k][0] = *reinterpret_cast<const f32x4*>(ln.P + k * ln.pstride + i0);
        pk[k][1] = *reinterpret_cast<const f32x4*>(ln.P + k * ln.pstride + i0 + 4);
      }
    pb0 = *reinterpret_cast<const f32x4*>(ln.pbias + i0);
    pb1 = *reinterpret_cast<const f32x4*>(ln.pbias + i0 + 4);
  }
  const f32x4 w0 = *reinterpret_cast<const f32x4*>(ln.w + i0);
  const f32x4 w1 = *reinterpret_cast<const f32x4*>(ln.w + i0 + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(ln.b + i0);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(ln.b + i0 + 4);
  const int act = ln.active ? ln.active[0] : 1;
  float v[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = xa[e];
    v[4 + e] = xc[e];
  }
  if (ln.P) ln_fold8(v, pk, ln.KS, pb0, pb1);
  if (writer && own) {
    // (an inactive row keeps its residual, as ln_dec_kernel leaves it)
    *reinterpret_cast<f32x4*>(ln.x_out + i0) = act ? f32x4{v[0], v[1], v[2], v[3]} : xa;
    *reinterpret_cast<f32x4*>(ln.x_out + i0 + 4) = act ? f32x4{v[4], v[5], v[6], v[7]} : xc;
  }
  float mean, scale;
  ln_stats(v, own, K, red, lane, wid, mean, scale);
  if (own)
    *reinterpret_cast<typename Elt<T>::v8*>(srow + i0) = ln_out8<T>(v, mean, scale, w0, w1, b0, b1);
  __syncthreads();
}

// lane l's A fragment of k-step kt at one row: row l & 15 (row 0 only is
// real, the others zero), k = 32 kt + 8 (l >> 4)
template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 ln_fold_frag(const T* srow, int kt, int lane) {
  typename Elt<T>::v8 z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (T)0.0f;
  return (lane & 15) == 0 ? *reinterpret_cast<const typename Elt<T>::v8*>(srow + kt * 32 + (lane >> 4) * 8)
                          : z;
}

}  // namespace mwx
