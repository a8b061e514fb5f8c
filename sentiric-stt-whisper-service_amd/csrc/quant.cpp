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
//
// The K types (q2_K .. q6_K: 256-element super-blocks with 16- or 32-element
// sub-block scales, ggml-common.h block_q2_K .. block_q6_K) are read the same
// way (ggml-quants.c dequantize_row_q2_K .. q6_K). Their writer is NOT ggml's
// quantize_row_q*_K_ref (whose scale search, make_qkx2_quants / make_q3_quants
// / make_qx_quants, is not restated): it produces valid blocks from a plain
// min/max (or signed absmax) rule so that test files exist. Loading is the
// parity surface: a file from whisper.cpp's tool is read by the same
// dequantizer. ggml requires ne0 % 256 == 0 for these types (tiny's 384-wide
// rows cannot be K-quantized by whisper.cpp either).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"

namespace mwx {

namespace {
constexpr int QK = 32;
constexpr int QK_K = 256;

// bytes per 32-element block (ggml-common.h block_q4_0 ... block_q8_0)
int block_bytes(int type) {
  switch (type) {
    case GGML_Q4_0: return 2 + QK / 2;          // d, qs[16]
    case GGML_Q4_1: return 2 + 2 + QK / 2;      // d, m, qs[16]
    case GGML_Q5_0: return 2 + 4 + QK / 2;      // d, qh[4], qs[16]
    case GGML_Q5_1: return 2 + 2 + 4 + QK / 2;  // d, m, qh[4], qs[16]
    case GGML_Q8_0: return 2 + QK;              // d, qs[32]
    // K super-blocks of 256 (ggml-common.h)
    case GGML_Q2_K: return 16 + 64 + 2 + 2;        // scales[16], qs[64], d, dmin
    case GGML_Q3_K: return 32 + 64 + 12 + 2;       // hmask[32], qs[64], scales[12], d
    case GGML_Q4_K: return 2 + 2 + 12 + 128;       // d, dmin, scales[12], qs[128]
    case GGML_Q5_K: return 2 + 2 + 12 + 32 + 128;  // d, dmin, scales[12], qh[32], qs[128]
    case GGML_Q6_K: return 128 + 64 + 16 + 2;      // ql[128], qh[64], scales[16], d
    default: return 0;
  }
}

bool is_k(int type) { return type >= GGML_Q2_K && type <= GGML_Q6_K; }

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

int ggml_block_elems(int type) {
  if (type == GGML_F32 || type == GGML_F16 || type == GGML_BF16) return 1;
  if (block_bytes(type) == 0) return 0;
  return is_k(type) ? QK_K : QK;
}

int ggml_ftype_of(int type) {
  switch (type) {  // GGML_FTYPE_MOSTLY_*; quantized files add GGML_QNT_VERSION (2) * 1000
    case GGML_F16: return 1;
    case GGML_BF16: return 24;
    case GGML_Q4_0: return 2000 + 2;
    case GGML_Q4_1: return 2000 + 3;
    case GGML_Q8_0: return 2000 + 7;
    case GGML_Q5_0: return 2000 + 8;
    case GGML_Q5_1: return 2000 + 9;
    case GGML_Q2_K: return 2000 + 10;  // GGML_FTYPE_MOSTLY_Q2_K .. Q6_K = 10 .. 14
    case GGML_Q3_K: return 2000 + 11;
    case GGML_Q4_K: return 2000 + 12;
    case GGML_Q5_K: return 2000 + 13;
    case GGML_Q6_K: return 2000 + 14;
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
  const int bb = block_bytes(type), be = ggml_block_elems(type);
  if (bb == 0 || ne0 % be != 0) return 0;
  return (size_t)(n / be) * bb;
}

namespace {
// ggml-quants.c get_scale_min_k4: sub-block j's 6-bit scale and min of the
// 12-byte packed table of q4_K / q5_K
void scale_min_k4(int j, const uint8_t* q, uint8_t& d, uint8_t& m) {
  if (j < 4) {
    d = q[j] & 63;
    m = q[j + 4] & 63;
  } else {
    d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

// ggml-quants.c dequantize_row_q2_K .. q6_K, one super-block (256 values)
void dequant_k(int type, const uint8_t* x, float* y) {
  switch (type) {
    case GGML_Q2_K: {
      const uint8_t* sc = x;
      const uint8_t* q = x + 16;
      const float d = rd16(x + 80), dmin = rd16(x + 82);
      int is = 0;
      for (int n = 0; n < QK_K; n += 128, q += 32)
        for (int sh = 0; sh < 8; sh += 2)
          for (int half = 0; half < 2; ++half, ++is) {
            const float dl = d * (float)(sc[is] & 0xF), ml = dmin * (float)(sc[is] >> 4);
            for (int l = 0; l < 16; ++l) *y++ = dl * (float)((q[l + 16 * half] >> sh) & 3) - ml;
          }
      break;
    }
    case GGML_Q3_K: {
      const uint8_t* hm = x;
      const uint8_t* q = x + 32;
      const uint8_t* raw = x + 96;
      const float d_all = rd16(x + 108);
      // the 16 6-bit scales: low nibbles in bytes 0..7, top two bits in 8..11
      int8_t scales[16];
      for (int s = 0; s < 16; ++s) {
        const int lo = s < 8 ? raw[s] & 0xF : raw[s - 8] >> 4;
        const int hi = (raw[8 + (s & 3)] >> (2 * (s >> 2))) & 3;
        scales[s] = (int8_t)(lo | (hi << 4));
      }
      int is = 0;
      uint8_t m = 1;
      for (int n = 0; n < QK_K; n += 128, q += 32)
        for (int sh = 0; sh < 8; sh += 2, m <<= 1)
          for (int half = 0; half < 2; ++half, ++is) {
            const float dl = d_all * (float)(scales[is] - 32);
            for (int l = 0; l < 16; ++l) {
              const int k = l + 16 * half;
              *y++ = dl * (float)(((q[k] >> sh) & 3) - ((hm[k] & m) ? 0 : 4));
            }
          }
      break;
    }
    case GGML_Q4_K:
    case GGML_Q5_K: {
      const bool q5 = type == GGML_Q5_K;
      const float d = rd16(x), dmin = rd16(x + 2);
      const uint8_t* scales = x + 4;
      const uint8_t* qh = x + 16;
      const uint8_t* ql = x + (q5 ? 48 : 16);
      uint8_t u1 = 1, u2 = 2;
      for (int j = 0, is = 0; j < QK_K; j += 64, ql += 32, is += 2, u1 <<= 2, u2 <<= 2) {
        uint8_t sc, mn;
        scale_min_k4(is, scales, sc, mn);
        const float d1 = d * (float)sc, m1 = dmin * (float)mn;
        scale_min_k4(is + 1, scales, sc, mn);
        const float d2 = d * (float)sc, m2 = dmin * (float)mn;
        for (int l = 0; l < 32; ++l)
          *y++ = d1 * (float)((ql[l] & 0xF) + (q5 && (qh[l] & u1) ? 16 : 0)) - m1;
        for (int l = 0; l < 32; ++l)
          *y++ = d2 * (float)((ql[l] >> 4) + (q5 && (qh[l] & u2) ? 16 : 0)) - m2;
      }
      break;
    }
    case GGML_Q6_K: {
      const uint8_t* ql = x;
      const uint8_t* qh = x + 128;
      const int8_t* sc = reinterpret_cast<const int8_t*>(x + 192);
      const float d = rd16(x + 208);
      for (int n = 0; n < QK_K; n += 128, y += 128, ql += 64, qh += 32, sc += 8)
        for (int l = 0; l < 32; ++l) {
          const int is = l / 16;
          const int q1 = ((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
          const int q2 = ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
          const int q3 = ((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
          const int q4 = ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
          y[l] = d * (float)sc[is] * (float)q1;
          y[l + 32] = d * (float)sc[is + 2] * (float)q2;
          y[l + 64] = d * (float)sc[is + 4] * (float)q3;
          y[l + 96] = d * (float)sc[is + 6] * (float)q4;
        }
      break;
    }
    default: break;
  }
}

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
inline int nearest(float v) { return (int)lrintf(v); }

// A plain valid K encoder (see the file comment): per sub-block of `sub`
// values an unsigned scale and min (q2_K / q4_K / q5_K: x ~ d*sc*q - dmin*m,
// q in [0, qmax]) or a signed scale (q3_K / q6_K: x ~ d*sc*q, q in
// [-half, half-1]); the super-block scales are f16 and the codes are taken
// against the f16-rounded values, so the blocks decode to the nearest
// representable value under their own scales.
void quant_k(int type, const float* x, uint8_t* y) {
  const int sub = (type == GGML_Q4_K || type == GGML_Q5_K) ? 32 : 16;
  const int nsub = QK_K / sub;
  const bool has_min = type == GGML_Q2_K || type == GGML_Q4_K || type == GGML_Q5_K;
  const int qmax = type == GGML_Q2_K ? 3 : type == GGML_Q4_K ? 15 : type == GGML_Q5_K ? 31
                 : type == GGML_Q3_K ? 4 : 32;  // signed: magnitude of the lowest code
  const int smax = type == GGML_Q2_K ? 15 : type == GGML_Q6_K ? 127 : type == GGML_Q3_K ? 31 : 63;
  float fs[16], fm[16];  // per sub-block real scale and min (>= 0)
  for (int s = 0; s < nsub; ++s) {
    const float* v = x + s * sub;
    if (has_min) {
      float mn = 0.0f, mx = 0.0f;
      for (int i = 0; i < sub; ++i) {
        mn = std::min(mn, v[i]);
        mx = std::max(mx, v[i]);
      }
      fs[s] = (mx - mn) / (float)qmax;
      fm[s] = -mn;
    } else {
      float amax = 0.0f, big = 0.0f;
      for (int i = 0; i < sub; ++i)
        if (fabsf(v[i]) > amax) {
          amax = fabsf(v[i]);
          big = v[i];
        }
      fs[s] = big / -(float)qmax;  // the largest magnitude maps to the lowest code
      fm[s] = 0.0f;
    }
  }
  float smaxv = 0.0f, mmaxv = 0.0f;
  for (int s = 0; s < nsub; ++s) {
    smaxv = std::max(smaxv, fabsf(fs[s]));
    mmaxv = std::max(mmaxv, fm[s]);
  }
  const float d = f16_to_f32(f32_to_f16(smaxv / (float)smax));
  const float dmin = f16_to_f32(f32_to_f16(mmaxv / (float)smax));
  int isc[16], imn[16];
  for (int s = 0; s < nsub; ++s) {
    isc[s] = d > 0.0f ? clampi(nearest(fs[s] / d), has_min ? 0 : -smax - 1, smax) : 0;
    if (type == GGML_Q3_K) isc[s] = clampi(isc[s], -32, 31);
    imn[s] = dmin > 0.0f ? clampi(nearest(fm[s] / dmin), 0, smax) : 0;
  }
  // integer code of element e (0..255) under its sub-block's scales
  auto code = [&](int e) {
    const int s = e / sub;
    const float step = d * (float)isc[s];
    if (step == 0.0f) return 0;
    if (has_min) return clampi(nearest((x[e] + dmin * (float)imn[s]) / step), 0, qmax);
    return clampi(nearest(x[e] / step), -qmax, qmax - 1);
  };
  memset(y, 0, block_bytes(type));
  switch (type) {
    case GGML_Q2_K:
      for (int s = 0; s < 16; ++s) y[s] = (uint8_t)(isc[s] | (imn[s] << 4));
      for (int e = 0; e < QK_K; ++e) {  // byte (e/128)*32 + (e%32), bits 2*((e%128)/32)
        const int r = e % 128;
        y[16 + (e / 128) * 32 + (r % 32)] |= (uint8_t)(code(e) << (2 * (r / 32)));
      }
      wr16(y + 80, d);
      wr16(y + 82, dmin);
      break;
    case GGML_Q3_K: {
      for (int s = 0; s < 16; ++s) {
        const int v = isc[s] + 32;  // 6 bits
        y[96 + (s & 7)] |= (uint8_t)((v & 0xF) << (s < 8 ? 0 : 4));
        y[96 + 8 + (s & 3)] |= (uint8_t)((v >> 4) << (2 * (s >> 2)));
      }
      for (int e = 0; e < QK_K; ++e) {
        const int r = e % 128, c = code(e) + 4;  // 0..7: low 2 bits + high-mask bit
        y[32 + (e / 128) * 32 + (r % 32)] |= (uint8_t)((c & 3) << (2 * (r / 32)));
        if (c & 4) y[r % 32] |= (uint8_t)(1u << ((e / 128) * 4 + r / 32));
      }
      wr16(y + 108, d);
      break;
    }
    case GGML_Q4_K:
    case GGML_Q5_K: {
      const bool q5 = type == GGML_Q5_K;
      wr16(y, d);
      wr16(y + 2, dmin);
      uint8_t* sc = y + 4;
      for (int j = 0; j < 4; ++j) {
        sc[j] = (uint8_t)((isc[j] & 63) | ((isc[j + 4] >> 4) << 6));
        sc[j + 4] = (uint8_t)((imn[j] & 63) | ((imn[j + 4] >> 4) << 6));
        sc[j + 8] = (uint8_t)((isc[j + 4] & 0xF) | ((imn[j + 4] & 0xF) << 4));
      }
      uint8_t* ql = y + (q5 ? 48 : 16);
      for (int e = 0; e < QK_K; ++e) {  // sub-block s = e/32: byte (s/2)*32 + e%32, nibble s&1
        const int s = e / 32, c = code(e);
        ql[(s / 2) * 32 + (e % 32)] |= (uint8_t)((c & 0xF) << (4 * (s & 1)));
        if (q5 && (c & 16)) y[16 + (e % 32)] |= (uint8_t)(1u << s);
      }
      break;
    }
    case GGML_Q6_K:
      for (int s = 0; s < 16; ++s) y[192 + s] = (uint8_t)(int8_t)isc[s];
      for (int e = 0; e < QK_K; ++e) {
        const int n = e / 128, r = e % 128, k = r / 32, l = r % 32, c = code(e) + 32;
        y[n * 64 + (k & 1) * 32 + l] |= (uint8_t)((c & 0xF) << (4 * (k >> 1)));
        y[128 + n * 32 + l] |= (uint8_t)((c >> 4) << (2 * k));
      }
      wr16(y + 208, d);
      break;
    default: break;
  }
}
}  // namespace

// ggml dequantize_row_q4_0 / _q4_1 / _q5_0 / _q5_1 / _q8_0 / _q2_K .. _q6_K
void ggml_dequantize(int type, const uint8_t* src, float* dst, int64_t n) {
  const int bb = block_bytes(type);
  if (is_k(type)) {
    for (int64_t b = 0; b < n / QK_K; ++b) dequant_k(type, src + b * bb, dst + b * QK_K);
    return;
  }
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

// ggml quantize_row_q4_0_ref / _q4_1_ref / _q5_0_ref / _q5_1_ref / _q8_0_ref;
// K types: the plain encoder above
void ggml_quantize(int type, const float* src, uint8_t* dst, int64_t n) {
  const int bb = block_bytes(type);
  if (is_k(type)) {
    for (int64_t b = 0; b < n / QK_K; ++b) quant_k(type, src + b * QK_K, dst + b * bb);
    return;
  }
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
