// MX-fp8 activation quantization for the encoder GEMMs (OCP MX block format:
// 32 consecutive k share one E8M0 power-of-two scale, elements are e4m3fn).
// Scale choice (no clipping): X = 2^e with e the smallest integer such that
// amax <= 448 * 2^e; element codes are e4m3 round-to-nearest-even of x / X.
// The host weight quantizer (quant.cpp mx_quantize_row) and the oracle
// restate the same rule.
#include "kcommon.h"
#include "kernels.h"

namespace mwx {

template <typename T>
__global__ __launch_bounds__(256) void mx_quantize_kernel(const T* __restrict__ x, long ld, int M,
                                                          int nb, uint8_t* __restrict__ q,
                                                          uint8_t* __restrict__ s, int K) {
  const long blk = (long)blockIdx.x * 256 + threadIdx.x;
  if (blk >= (long)M * nb) return;
  const long row = blk / nb;
  const int b = (int)(blk - row * nb);
  const T* src = x + row * ld + b * 32;
  float v[32];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const typename Elt<T>::v8 w = *reinterpret_cast<const typename Elt<T>::v8*>(src + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[c * 8 + e] = (float)w[e];
  }
  float amax = 0.0f;
#pragma unroll
  for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
  const int ex = mx_exp(amax);
  const float inv = ldexpf(1.0f, -ex);  // exact: x / 2^ex
  uint32_t pk[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) word |= (uint32_t)e4m3_rne(v[w * 4 + e] * inv) << (8 * e);
    pk[w] = word;
  }
  uint4* dst = reinterpret_cast<uint4*>(q + row * (long)K + b * 32);
  dst[0] = uint4{pk[0], pk[1], pk[2], pk[3]};
  dst[1] = uint4{pk[4], pk[5], pk[6], pk[7]};
  s[row * nb + b] = (uint8_t)(127 + ex);
}

template <typename T>
void mx_quantize(const T* x, long ld, int M, int K, uint8_t* q, uint8_t* s, hipStream_t st) {
  const int nb = K / 32;
  const long n = (long)M * nb;
  mx_quantize_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(x, ld, M, nb, q, s, K);
}

template void mx_quantize<_Float16>(const _Float16*, long, int, int, uint8_t*, uint8_t*,
                                    hipStream_t);
template void mx_quantize<__bf16>(const __bf16*, long, int, int, uint8_t*, uint8_t*, hipStream_t);

}  // namespace mwx
