// ggml block-quantized tensor types of whisper .bin files (host side).
//
// whisper.cpp's `quantize` tool (examples/common-ggml.cpp ggml_common_quantize_0
// at v1.8.2) rewrites every 2-D tensor except the conv biases and positional
// embeddings as one of the legacy 32-element block formats below; the
// distributed ggml-*-q5_0 / -q5_1 / -q8_0 models are of this kind. The engine
// dequantizes them once at load (ggml dequantize_row_q* semantics, f32) and
// rounds to f16, the compute type of whisper.cpp's GPU backends for these
// types (dequantize + f16 GEMM). The writer below restates ggml's
// quantize_row_q*_ref so test models can be produced without whisper.cpp.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"

namespace mwx {

namespace {
constexpr int QK = 32;

// bytes per 32-element block (ggml-common.h block_q4_0 ... block_q8_0)
int block_bytes(int type) {
  switch (type) {
    case GGML_Q4_0: return 2 + QK / 2;          // d, qs[16]
    case GGML_Q4_1: return 2 + 2 + QK / 2;      // d, m, qs[16]
    case GGML_Q5_0: return 2 + 4 + QK / 2;      // d, qh[4], qs[16]
    case GGML_Q5_1: return 2 + 2 + 4 + QK / 2;  // d, m, qh[4], qs[16]
    case GGML_Q8_0: return 2 + QK;              // d, qs[32]
    default: return 0;
  }
}

inline float rd16(const uint8_t* p) {
  uint16_t h;
  memcpy(&h, p, 2);
  return f16_to_f32(h);
}
inline void wr16(uint8_t* p, float f) {
  const uint16_t h = f32_to_f16(f);
  memcpy(p, &h, 2);
}
}  // namespace

bool ggml_type_is_quant(int type) { return block_bytes(type) > 0; }

int ggml_ftype_of(int type) {
  switch (type) {  // GGML_FTYPE_MOSTLY_*; quantized files add GGML_QNT_VERSION (2) * 1000
    case GGML_F16: return 1;
    case GGML_BF16: return 24;
    case GGML_Q4_0: return 2000 + 2;
    case GGML_Q4_1: return 2000 + 3;
    case GGML_Q8_0: return 2000 + 7;
    case GGML_Q5_0: return 2000 + 8;
    case GGML_Q5_1: return 2000 + 9;
    default: return -1;
  }
}

size_t ggml_tensor_bytes(int type, int64_t ne0, int64_t n) {
  switch (type) {
    case GGML_F32: return (size_t)n * 4;
    case GGML_F16:
    case GGML_BF16: return (size_t)n * 2;
    default: break;
  }
  const int bb = block_bytes(type);
  if (bb == 0 || ne0 % QK != 0) return 0;
  return (size_t)(n / QK) * bb;
}

// ggml dequantize_row_q4_0 / _q4_1 / _q5_0 / _q5_1 / _q8_0
void ggml_dequantize(int type, const uint8_t* src, float* dst, int64_t n) {
  const int bb = block_bytes(type);
  for (int64_t b = 0; b < n / QK; ++b) {
    const uint8_t* x = src + b * bb;
    float* y = dst + b * QK;
    const float d = rd16(x);
    switch (type) {
      case GGML_Q4_0: {
        const uint8_t* qs = x + 2;
        for (int j = 0; j < QK / 2; ++j) {
          y[j] = (float)((qs[j] & 0x0F) - 8) * d;
          y[j + QK / 2] = (float)((qs[j] >> 4) - 8) * d;
        }
        break;
      }
      case GGML_Q4_1: {
        const float m = rd16(x + 2);
        const uint8_t* qs = x + 4;
        for (int j = 0; j < QK / 2; ++j) {
          y[j] = (float)(qs[j] & 0x0F) * d + m;
          y[j + QK / 2] = (float)(qs[j] >> 4) * d + m;
        }
        break;
      }
      case GGML_Q5_0:
      case GGML_Q5_1: {
        const bool q51 = type == GGML_Q5_1;
        const float m = q51 ? rd16(x + 2) : 0.0f;
        uint32_t qh;
        memcpy(&qh, x + (q51 ? 4 : 2), 4);
        const uint8_t* qs = x + (q51 ? 8 : 6);
        for (int j = 0; j < QK / 2; ++j) {
          const uint8_t xh0 = ((qh >> j) << 4) & 0x10;
          const uint8_t xh1 = (qh >> (j + 12)) & 0x10;
          const int x0 = (qs[j] & 0x0F) | xh0;
          const int x1 = (qs[j] >> 4) | xh1;
          if (q51) {
            y[j] = (float)x0 * d + m;
            y[j + QK / 2] = (float)x1 * d + m;
          } else {
            y[j] = (float)(x0 - 16) * d;
            y[j + QK / 2] = (float)(x1 - 16) * d;
          }
        }
        break;
      }
      case GGML_Q8_0: {
        const int8_t* qs = reinterpret_cast<const int8_t*>(x + 2);
        for (int j = 0; j < QK; ++j) y[j] = (float)qs[j] * d;
        break;
      }
      default: break;
    }
  }
}

// ggml quantize_row_q4_0_ref / _q4_1_ref / _q5_0_ref / _q5_1_ref / _q8_0_ref
void ggml_quantize(int type, const float* src, uint8_t* dst, int64_t n) {
  const int bb = block_bytes(type);
  for (int64_t b = 0; b < n / QK; ++b) {
    const float* x = src + b * QK;
    uint8_t* y = dst + b * bb;
    memset(y, 0, bb);
    switch (type) {
      case GGML_Q4_0:
      case GGML_Q5_0: {
        float amax = 0.0f, mx = 0.0f;  // the value of largest magnitude
        for (int j = 0; j < QK; ++j)
          if (amax < fabsf(x[j])) {
            amax = fabsf(x[j]);
            mx = x[j];
          }
        const bool q5 = type == GGML_Q5_0;
        const float d = mx / (q5 ? -16.0f : -8.0f);
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        wr16(y, d);
        uint8_t* qs = y + (q5 ? 6 : 2);
        uint32_t qh = 0;
        for (int j = 0; j < QK / 2; ++j) {
          const float x0 = x[j] * id, x1 = x[QK / 2 + j] * id;
          if (q5) {
            const uint8_t xi0 = (uint8_t)std::min(31, (int)(int8_t)(x0 + 16.5f));
            const uint8_t xi1 = (uint8_t)std::min(31, (int)(int8_t)(x1 + 16.5f));
            qs[j] = (xi0 & 0x0F) | ((xi1 & 0x0F) << 4);
            qh |= ((xi0 & 0x10u) >> 4) << j;
            qh |= ((xi1 & 0x10u) >> 4) << (j + QK / 2);
          } else {
            const uint8_t xi0 = (uint8_t)std::min(15, (int)(int8_t)(x0 + 8.5f));
            const uint8_t xi1 = (uint8_t)std::min(15, (int)(int8_t)(x1 + 8.5f));
            qs[j] = xi0 | (xi1 << 4);
          }
        }
        if (q5) memcpy(y + 2, &qh, 4);
        break;
      }
      case GGML_Q4_1:
      case GGML_Q5_1: {
        float mn = FLT_MAX, mx = -FLT_MAX;
        for (int j = 0; j < QK; ++j) {
          mn = std::min(mn, x[j]);
          mx = std::max(mx, x[j]);
        }
        const bool q5 = type == GGML_Q5_1;
        const float d = (mx - mn) / (q5 ? 31.0f : 15.0f);
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        wr16(y, d);
        wr16(y + 2, mn);
        uint8_t* qs = y + (q5 ? 8 : 4);
        uint32_t qh = 0;
        for (int j = 0; j < QK / 2; ++j) {
          const float x0 = (x[j] - mn) * id, x1 = (x[QK / 2 + j] - mn) * id;
          if (q5) {
            const uint8_t xi0 = (uint8_t)(x0 + 0.5f), xi1 = (uint8_t)(x1 + 0.5f);
            qs[j] = (xi0 & 0x0F) | ((xi1 & 0x0F) << 4);
            qh |= ((xi0 & 0x10u) >> 4) << j;
            qh |= ((xi1 & 0x10u) >> 4) << (j + QK / 2);
          } else {
            const uint8_t xi0 = (uint8_t)std::min(15, (int)(int8_t)(x0 + 0.5f));
            const uint8_t xi1 = (uint8_t)std::min(15, (int)(int8_t)(x1 + 0.5f));
            qs[j] = xi0 | (xi1 << 4);
          }
        }
        if (q5) memcpy(y + 4, &qh, 4);
        break;
      }
      case GGML_Q8_0: {
        float amax = 0.0f;
        for (int j = 0; j < QK; ++j) amax = std::max(amax, fabsf(x[j]));
        const float d = amax / 127.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        wr16(y, d);
        int8_t* qs = reinterpret_cast<int8_t*>(y + 2);
        for (int j = 0; j < QK; ++j) qs[j] = (int8_t)roundf(x[j] * id);
        break;
      }
      default: break;
    }
  }
}


// ---------------------------------------------------------------------------
// MX-fp8 (OCP MX: 32 consecutive k share an E8M0 scale, elements e4m3fn) for
// the fp8 compute mode's encoder / cross-K/V weights. Scale rule (no
// clipping): X = 2^e, e the smallest integer with amax <= 448 * 2^e; codes are
// e4m3 round-to-nearest-even of x / X (same rule as k_mx.hip).
// ---------------------------------------------------------------------------
static int mx_exp_host(float amax) {
  if (!(amax > 0.0f)) return 0;
  int e0;
  const float m = frexpf(amax, &e0);
  const int e = (e0 - 1) - 8 + (2.0f * m > 1.75f ? 1 : 0);
  return std::max(-127, std::min(127, e));
}

static uint8_t e4m3_rne_host(float v) {
  const uint8_t sgn = v < 0.0f ? 0x80 : 0;
  const float a = fabsf(v);
  if (a < 0.015625f) return sgn | (uint8_t)rintf(a * 512.0f);
  int E;
  const float m = frexpf(a, &E);
  int q = (int)rintf(m * 16.0f);
  int ex = E - 1;
  if (q == 16) {
    q = 8;
    ++ex;
  }
  return sgn | (uint8_t)(((ex + 7) << 3) | (q - 8));
}

// value of an e4m3fn code times the E8M0 scale 2^(s - 127)
float mx_dequant(uint8_t code, uint8_t s) {
  const int e = (code >> 3) & 15, m = code & 7;
  const float a = e == 0 ? ldexpf((float)m, -9) : ldexpf((float)(8 + m), e - 10);
  return ldexpf(code & 0x80 ? -a : a, (int)s - 127);
}

void mx_quantize_row(const float* x, int K, uint8_t* q, uint8_t* s) {
  for (int b = 0; b < K / 32; ++b) {
    float amax = 0.0f;
    for (int j = 0; j < 32; ++j) amax = std::max(amax, fabsf(x[b * 32 + j]));
    const int e = mx_exp_host(amax);
    const float inv = ldexpf(1.0f, -e);
    for (int j = 0; j < 32; ++j) q[b * 32 + j] = e4m3_rne_host(x[b * 32 + j] * inv);
    s[b] = (uint8_t)(127 + e);
  }
}

}  // namespace mwx
