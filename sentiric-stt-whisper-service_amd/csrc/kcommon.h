// Device-side helpers shared by the gfx950 kernels of the mwx engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace mwx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-/8-byte loads of bytes one CU reads once per launch (the decode cross K/V
// streams): NT = non-temporal (`nt` cache policy), which keeps them from
// displacing reusable lines; measured 43.3 -> 38.5 us for the large-v3 cross
// K/V byte pattern at 32 rows (scripts/probe/stream_probe.hip)
template <bool NT, typename V>
__device__ __forceinline__ V ld_stream(const V* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// Element type traits: T is _Float16 (ggml f16 files) or __bf16.
template <typename T>
struct Elt;
template <>
struct Elt<_Float16> {
  using v8 = f16x8;
  __device__ static inline f32x4 mfma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Elt<__bf16> {
  using v8 = bf16x8;
  __device__ static inline f32x4 mfma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

// f32 -> f16 of a value computed in f32. ggml stores the f32 result and then
// converts it (two roundings: the f32 op, then f16). The empty asm keeps the
// value materialised as f32, so the compiler cannot fuse the producing
// multiply / add into v_fma_mix{lo,hi}_f16, which rounds a*b(+c) to f16 once
// (it does so even with -ffp-contract=off; seen on the decode K scaling and
// the softmax's P).
__device__ __forceinline__ _Float16 f16r(float x) {
  asm volatile("" : "+v"(x));
  return (_Float16)x;
}
template <typename T>
__device__ __forceinline__ T to_t(float x) {
  asm volatile("" : "+v"(x));  // (as f16r)
  return (T)x;  // v_cvt_f16_f32 / v_cvt_pk_bf16_f32: round to nearest even
}
template <typename T>
__device__ __forceinline__ float to_f(T x) {
  return (float)x;
}

// ggml GELU (tanh approximation) as evaluated by the ggml CPU backend with
// GGML_GELU_FP16: the input is rounded to f16, the f32 formula is applied and
// the result is rounded to f16 again (table lookup); saturates outside ±10.
__device__ __forceinline__ float gelu_f32(float x) {
  const float GELU_COEF_A = 0.044715f;
  const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
  return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
}
__device__ __forceinline__ float gelu_ggml(float x) {
  if (x <= -10.0f) return 0.0f;
  if (x >= 10.0f) return x;
  const float xh = (float)f16r(x);
  return (float)f16r(gelu_f32(xh));
}

// gelu_ggml(x) by table lookup (gelu_table_build fills the table with the
// f16(gelu_f32(h)) gelu_ggml computes for every f16 h with |h| <= 10): the
// same value for every x (NaN passes through as in gelu_f32)
template <typename TP>
__device__ __forceinline__ float gelu_ggml_tab(float x, TP tab) {
  if (x <= -10.0f) return 0.0f;
  if (x >= 10.0f) return x;
  if (x != x) return x;
  const uint16_t hb = __builtin_bit_cast(uint16_t, f16r(x));
  const int idx = (hb & 0x7fff) + (hb >> 15) * GELU_TAB_HALF;
  return (float)__builtin_bit_cast(_Float16, tab[idx]);
}

// OCP MX-fp8 block rule (k_mx.hip, the cross K/V cache epilogue; host:
// quant.cpp mx_quantize_row, oracle mx_round_rows): the E8M0 exponent of a
// 32-element block is the smallest e with amax <= 448 * 2^e (no clipping);
// codes are e4m3fn round-to-nearest-even of x / 2^e.
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.0f)) return 0;
  int e0;
  const float m = frexpf(amax, &e0);  // amax = m * 2^e0, m in [0.5, 1)
  int e = (e0 - 1) - 8 + (2.0f * m > 1.75f ? 1 : 0);
  return max(-127, min(127, e));
}

__device__ __forceinline__ uint8_t e4m3_rne(float v) {
  const uint8_t sgn = v < 0.0f ? 0x80 : 0;
  const float a = fabsf(v);
  if (a < 0.015625f) return sgn | (uint8_t)rintf(a * 512.0f);  // subnormals (8 -> 2^-6)
  int E;
  const float m = frexpf(a, &E);  // a = m * 2^E
  int q = (int)rintf(m * 16.0f);   // a / 2^(E-1-3), in [8, 16]
  int ex = E - 1;
  if (q == 16) {
    q = 8;
    ++ex;
  }
  return sgn | (uint8_t)(((ex + 7) << 3) | (q - 8));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave reductions without LDS round trips: DPP steps inside each 16-lane row
// (xor 1, xor 2 by quad_perm, then row_half_mirror and row_mirror pair lanes
// i and 7-i / 15-i), then the four row results read with v_readlane and
// combined as (r0 + r1) + (r2 + r3); every lane gets the result. A
// ds_bpermute shuffle costs an LDS round trip per step (six per reduction,
// twelve for a double); these cost a few cycles each.
// (update_dpp with bound_ctrl: every lane of these row-local patterns has a
// valid source, so the result is mov_dpp's, and the compiler can fold the
// move into the consuming add / max as one v_*_dpp instruction)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint64_t lo = dpp_u32<CTRL>((uint32_t)u), hi = dpp_u32<CTRL>((uint32_t)(u >> 32));
  return __longlong_as_double((long long)((hi << 32) | lo));
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __double_as_longlong(v);
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
  return __longlong_as_double((long long)((hi << 32) | lo));
}
// x (op) x-of-lane^m for m = 8, 16, 32 without an LDS round trip (the same
// values as __shfl_xor, which compiles to ds_bpermute): m = 8 by DPP
// row_ror:8 inside a 16-lane row; m = 16 / 32 by gfx950's row swaps
// v_permlane16_swap / v_permlane32_swap, whose two results hold the lane's
// own value and its partner's (in an order that depends on the row: the ops
// used here are commutative, so the result is the same bits either way)
__device__ __forceinline__ float add_xor8(float a) {
  return a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_xor16(float a) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(a), __float_as_int(a), false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float a) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(a), false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}
__device__ __forceinline__ float max_xor16(float a) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(a), __float_as_int(a), false, false);
  return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float a) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(a), false, false);
  return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ int max_xor16_i(int a) {
  const auto r = __builtin_amdgcn_permlane16_swap(a, a, false, false);
  return max((int)r[0], (int)r[1]);
}
__device__ __forceinline__ int max_xor32_i(int a) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, a, false, false);
  return max((int)r[0], (int)r[1]);
}

__device__ __forceinline__ double wave_sum_d_dpp(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, __uint_as_float(dpp_u32<0xB1>(__float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<0x4E>(__float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<0x141>(__float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(dpp_u32<0x140>(__float_as_uint(v))));
  return fmaxf(fmaxf(__uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 0)),
                     __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 16))),
               fmaxf(__uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 32)),
                     __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 48))));
}

// Launch span stamps (perf classes "<class>.span", engine.cpp span_slot): the
// earliest workgroup start and the latest workgroup end of a launch on the
// constant-rate device clock (s_memrealtime), i.e. the launch's duration as a
// kernel trace measures it, without the queueing in front of it that a HIP
// event bracket also counts when another stream's kernels hold the CUs. A
// slot holds SPAN_SHARDS pairs, 128 B apart (workgroup id % SPAN_SHARDS picks
// one), so the per-workgroup atomics do not queue on one address: pair[0] =
// max of ~start (= ~earliest start), pair[1] = max of the ends; all zeroed
// before the launch; the host reduces over the shards. Thread 0 of the
// workgroup (of its wave 0 for the end stamp) stamps.
__device__ __forceinline__ unsigned long long* span_pair(unsigned long long* span) {
  const unsigned wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  return span + (wg % SPAN_SHARDS) * 16;
}
__device__ __forceinline__ void span_start(unsigned long long* span) {
  if (span && threadIdx.x == 0)
    atomicMax(span_pair(span), ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void span_end(unsigned long long* span) {
  if (span && threadIdx.x == 0)
    atomicMax(span_pair(span) + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

}  // namespace mwx
