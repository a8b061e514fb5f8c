// ============================================================================
// mwx ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference hot path: whisper.cpp v1.8.2 (the
// third-party dependency of sentiric-stt-whisper-service, pinned by
// `ARG WHISPER_CPP_VERSION=v1.8.2` at Dockerfile:24 / Dockerfile.gpu:24 and
// called from src/stt_engine.cpp:245-246). whisper.cpp is not vendored in the
// reference and is absent from this container, so every function below
// restates its published algorithm at the level of *where values are rounded*
// (f16/bf16 conversion points of the ggml CPU backend), not instruction order.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker. The product (libmwx.so) never
// links or calls it.
//
// PARITY STATUS: the reference ships no tests, fixtures or golden vectors for
// this path, and whisper.cpp cannot be built offline.
// Parity with whisper.cpp itself is therefore UNPINNED; the restatement is
// cross-checked against an independent implementation (HF transformers
// Whisper, in-container) through the fixtures in tests/golden/.
//
// Numeric mode ("ggml-cpu"): weights are the exact 16-bit values of the file;
// matmul inputs are rounded to the weight type (ggml vec_dot_type); attention
// Q/K/V/P are rounded to f16 (ggml itype); GELU is the ggml f16-table GELU;
// LayerNorm accumulates in double (ggml_float); softmax follows
// ggml_compute_forward_soft_max_f32. An "exact" mode (flag ORC_EXACT) skips
// all 16-bit rounding of activations and uses f32 tanh-GELU, for comparisons
// against fp32 implementations.
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <sys/stat.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <random>
#include <regex>
#include <string>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// ---------------------------------------------------------------------------
// 16-bit conversions (round to nearest even)
// ---------------------------------------------------------------------------
static inline float f16_round(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = x & 0x80000000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return f;  // inf / nan
  // values >= 65520 round to inf
  if (ax >= 0x477ff000u) {
    uint32_t r = sign | 0x7f800000u;
    float o;
    memcpy(&o, &r, 4);
    return o;
  }
  float a;
  memcpy(&a, &ax, 4);
  float out;
  if (a < 6.103515625e-05f) {
    // subnormal f16 range: quantum 2^-24
    const float q = 5.9604644775390625e-08f;
    out = std::nearbyint(a / q) * q;  // a/q exact (power of two), RNE
  } else {
    uint32_t m = ax;
    const uint32_t rem = m & 0x1fffu;
    m &= ~0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (m & 0x2000u))) m += 0x2000u;
    memcpy(&out, &m, 4);
  }
  uint32_t o;
  memcpy(&o, &out, 4);
  o |= sign;
  memcpy(&out, &o, 4);
  return out;
}

static inline float bf16_round(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  if ((x & 0x7fffffffu) > 0x7f800000u) return f;
  x += 0x7fffu + ((x >> 16) & 1u);
  x &= 0xffff0000u;
  float o;
  memcpy(&o, &x, 4);
  return o;
}

static inline float h2f(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t mant = h & 0x3ffu;
  uint32_t x;
  if (exp == 0) {
    if (mant == 0) {
      x = sign;
    } else {
      float v = (float)mant * 5.9604644775390625e-08f;
      memcpy(&x, &v, 4);
      x |= sign;
    }
  } else if (exp == 31) {
    x = sign | 0x7f800000u | (mant << 13);
  } else {
    x = sign | ((exp + 112u) << 23) | (mant << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}
static inline float b2f(uint16_t h) {
  uint32_t x = (uint32_t)h << 16;
  float f;
  memcpy(&f, &x, 4);
  return f;
}

enum { T_F32 = 0, T_F16 = 1, T_BF16 = 30 };
enum { ORC_EXACT = 1, ORC_MXFP8 = 2 };

// ---------------------------------------------------------------------------
// model
// ---------------------------------------------------------------------------
struct Tensor {
  std::vector<int64_t> ne;
  std::vector<float> v;  // exact values of the stored type
};

struct Model {
  int32_t hp[11];
  int n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
  int n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels;
  int wtype = T_F16;
  int n_fft = 201;
  std::vector<float> filters;
  // vocab
  std::vector<std::string> id_to_token;
  std::map<std::string, int> token_to_id;
  int eot = 50256, sot = 50257, translate = 50357, transcribe = 50358,
      solm = 50359, prev = 50360, nosp = 50361, not_ = 50362, beg = 50363;
  bool multilingual = false;
  int num_languages = 0;
  std::map<std::string, Tensor> t;
  int flags = 0;
  std::string key;  // file identity + flags: the encoder / cross-K/V caches' key

  const float* w(const std::string& n) const {
    auto it = t.find(n);
    if (it == t.end()) {
      fprintf(stderr, "oracle: missing tensor %s\n", n.c_str());
      abort();
    }
    return it->second.v.data();
  }
  float rw(float x) const {  // round a matmul input to the weight type
    if (flags & ORC_EXACT) return x;
    return wtype == T_BF16 ? bf16_round(x) : f16_round(x);
  }
  float r16(float x) const {  // round to ggml itype (f16)
    if (flags & ORC_EXACT) return x;
    return f16_round(x);
  }
};

static const char* kLang[] = {
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca",
    "nl", "ar", "sv", "it", "id", "hi", "fi", "vi", "he", "uk", "el", "ms",
    "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg", "lt", "la",
    "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn",
    "et", "mk", "br", "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw",
    "gl", "mr", "pa", "si", "km", "sn", "yo", "so", "af", "oc", "ka", "be",
    "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn",
    "mt", "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha",
    "ba", "jw", "su", "yue"};
static const int kNLang = 100;
static int lang_id(const std::string& s) {
  for (int i = 0; i < kNLang; ++i)
    if (s == kLang[i]) return i;
  return -1;
}

static inline float h2f_at(const uint8_t* p) {
  uint16_t h;
  memcpy(&h, p, 2);
  return h2f(h);
}

// ggml legacy block quantizations (ggml-common.h block_q4_0 .. block_q8_0;
// type ids Q4_0 = 2, Q4_1 = 3, Q5_0 = 6, Q5_1 = 7, Q8_0 = 8): 32 elements per
// block, f16 scale d (and min m for the _1 variants), ggml dequantize_row_q*.
// K super-blocks (ggml-common.h block_q2_K .. block_q6_K, type ids 10 .. 14):
// 256 elements, ggml-quants.c dequantize_row_q*_K, restated per element below.
static int quant_block_bytes(int tt) {
  switch (tt) {
    case 2: return 18;
    case 3: return 20;
    case 6: return 22;
    case 7: return 24;
    case 8: return 34;
    case 10: return 84;
    case 11: return 110;
    case 12: return 144;
    case 13: return 176;
    case 14: return 210;
    default: return 0;
  }
}
static int quant_block_elems(int tt) { return tt >= 10 && tt <= 14 ? 256 : 32; }

// Element e (0..255) of one K super-block. Within a 128-element half h = e/128
// the 2-bit planes of q2_K / q3_K interleave four 32-element groups g in one
// 32-byte run (bits 2g..2g+1 of byte e%32); q3_K's sign-offset bit sits in
// hmask[e%32] at bit 4h+g; q4_K / q5_K pair 32-element sub-blocks in nibbles
// of a 32-byte run (sub-block e/32: byte (e/64)*32 + e%32, high nibble when
// odd; q5_K's fifth bit at qh[e%32] bit e/32); q6_K keeps the low nibbles of
// groups 0/1 and 2/3 in two 32-byte runs per half and the top two bits of
// all four groups in one (byte h*32 + e%32, bits 2g..2g+1). Scales belong to
// 16-element sub-blocks (e/16) except q4_K / q5_K's 32-element ones.
static float dequant_k_elem(int tt, const uint8_t* b, int e) {
  const int h = e / 128, g = (e % 128) / 32, l = e % 32;
  switch (tt) {
    case 10: {  // scales[16] (scale | min << 4), qs[64], d, dmin
      const int s = b[e / 16];
      const int q = (b[16 + h * 32 + l] >> (2 * g)) & 3;
      return h2f_at(b + 80) * (float)(s & 15) * (float)q - h2f_at(b + 82) * (float)(s >> 4);
    }
    case 11: {  // hmask[32], qs[64], scales[12] (6-bit, offset 32), d
      const int s = e / 16;
      const int lo = (s < 8 ? b[96 + s] : b[96 + s - 8] >> 4) & 15;
      const int hi = (b[104 + s % 4] >> (2 * (s / 4))) & 3;
      const int q = ((b[32 + h * 32 + l] >> (2 * g)) & 3) - ((b[l] >> (4 * h + g)) & 1 ? 0 : 4);
      return h2f_at(b + 108) * (float)((lo | (hi << 4)) - 32) * (float)q;
    }
    case 12:
    case 13: {  // d, dmin, scales[12] (6-bit scale / min pairs), [qh[32]], qs[128]
      const int s = e / 32;
      const uint8_t* t = b + 4;
      const int sc = s < 4 ? t[s] & 63 : (t[s + 4] & 15) | ((t[s - 4] >> 6) << 4);
      const int mn = s < 4 ? t[s + 4] & 63 : (t[s + 4] >> 4) | ((t[s] >> 6) << 4);
      const uint8_t* qs = b + (tt == 13 ? 48 : 16);
      int q = (qs[(s / 2) * 32 + l] >> (4 * (s & 1))) & 15;
      if (tt == 13) q += ((b[16 + l] >> s) & 1) << 4;
      return h2f_at(b) * (float)sc * (float)q - h2f_at(b + 2) * (float)mn;
    }
    case 14: {  // ql[128], qh[64], scales[16] (int8), d
      const int lo = (b[h * 64 + (g & 1) * 32 + l] >> (4 * (g >> 1))) & 15;
      const int hi = (b[128 + h * 32 + l] >> (2 * g)) & 3;
      return h2f_at(b + 208) * (float)(int8_t)b[192 + e / 16] * (float)((lo | (hi << 4)) - 32);
    }
    default: return 0.0f;
  }
}

static void dequant_blocks(int tt, const uint8_t* q, float* y, int64_t n) {
  const int bb = quant_block_bytes(tt);
  if (quant_block_elems(tt) == 256) {
    for (int64_t b = 0; b < n / 256; ++b, q += bb, y += 256)
      for (int e = 0; e < 256; ++e) y[e] = dequant_k_elem(tt, q, e);
    return;
  }
  for (int64_t b = 0; b < n / 32; ++b, q += bb, y += 32) {
    uint16_t hd, hm = 0;
    memcpy(&hd, q, 2);
    const float d = h2f(hd);
    const bool has_min = tt == 3 || tt == 7;
    if (has_min) memcpy(&hm, q + 2, 2);
    const float m = has_min ? h2f(hm) : 0.0f;
    for (int j = 0; j < 32; ++j) {
      int v;  // the quantized integer of element j
      if (tt == 8) {
        v = (int8_t)q[2 + j];
      } else {
        const int hi = j >= 16;
        const uint8_t* qs = q + (tt == 2 ? 2 : tt == 3 ? 4 : tt == 6 ? 6 : 8);
        v = hi ? (qs[j - 16] >> 4) : (qs[j] & 0x0F);
        if (tt == 6 || tt == 7) {  // fifth bit from qh, element j at bit j
          uint32_t qh;
          memcpy(&qh, q + (tt == 6 ? 2 : 4), 4);
          v |= (int)((qh >> j) & 1u) << 4;
        }
      }
      if (has_min) y[j] = (float)v * d + m;
      else y[j] = (float)(v - (tt == 2 ? 8 : tt == 6 ? 16 : 0)) * d;
    }
  }
}

static bool load(const char* path, Model& m) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  uint32_t magic;
  f.read((char*)&magic, 4);
  if (magic != 0x67676d6cu) return false;
  f.read((char*)m.hp, 44);
  m.n_vocab = m.hp[0];
  m.n_audio_ctx = m.hp[1];
  m.n_audio_state = m.hp[2];
  m.n_audio_head = m.hp[3];
  m.n_audio_layer = m.hp[4];
  m.n_text_ctx = m.hp[5];
  m.n_text_state = m.hp[6];
  m.n_text_head = m.hp[7];
  m.n_text_layer = m.hp[8];
  m.n_mels = m.hp[9];
  int32_t fn_mel, fn_fft;
  f.read((char*)&fn_mel, 4);
  f.read((char*)&fn_fft, 4);
  m.n_fft = fn_fft;
  m.filters.resize((size_t)fn_mel * fn_fft);
  f.read((char*)m.filters.data(), m.filters.size() * 4);
  int32_t nv;
  f.read((char*)&nv, 4);
  m.id_to_token.assign(m.n_vocab, "");
  for (int i = 0; i < nv; ++i) {
    uint32_t len;
    f.read((char*)&len, 4);
    std::string s(len, '\0');
    if (len) f.read(&s[0], len);
    m.token_to_id[s] = i;
    m.id_to_token[i] = s;
  }
  m.multilingual = m.n_vocab >= 51865;
  m.num_languages = m.n_vocab - 51765 - (m.multilingual ? 1 : 0);
  if (m.multilingual) {
    m.eot++;
    m.sot++;
    const int dt = m.num_languages - 98;
    m.translate += dt;
    m.transcribe += dt;
    m.solm += dt;
    m.prev += dt;
    m.nosp += dt;
    m.not_ += dt;
    m.beg += dt;
  }
  for (int i = nv; i < m.n_vocab; ++i) {
    std::string w;
    if (i > m.beg) w = "[_TT_" + std::to_string(i - m.beg) + "]";
    else if (i == m.eot) w = "[_EOT_]";
    else if (i == m.sot) w = "[_SOT_]";
    else if (i == m.translate) w = "[_TRANSLATE_]";
    else if (i == m.transcribe) w = "[_TRANSCRIBE_]";
    else if (i == m.solm) w = "[_SOLM_]";
    else if (i == m.prev) w = "[_PREV_]";
    else if (i == m.nosp) w = "[_NOSP_]";
    else if (i == m.not_) w = "[_NOT_]";
    else if (i == m.beg) w = "[_BEG_]";
    else if (i > m.sot && i <= m.sot + m.num_languages) {
      const int li = i - m.sot - 1;
      w = std::string("[_LANG_") + (li < kNLang ? kLang[li] : "") + "]";
    } else w = "[_extra_token_" + std::to_string(i) + "]";
    m.token_to_id[w] = i;
    m.id_to_token[i] = w;
  }
  while (true) {
    int32_t nd, nl, tt;
    f.read((char*)&nd, 4);
    if (f.eof()) break;
    f.read((char*)&nl, 4);
    f.read((char*)&tt, 4);
    Tensor T;
    int64_t n = 1;
    for (int i = 0; i < nd; ++i) {
      int32_t e;
      f.read((char*)&e, 4);
      T.ne.push_back(e);
      n *= e;
    }
    std::string name(nl, '\0');
    f.read(&name[0], nl);
    T.v.resize(n);
    if (tt == T_F32) {
      f.read((char*)T.v.data(), n * 4);
    } else if (quant_block_bytes(tt) > 0) {
      // whisper.cpp quantize-tool output: dequantized (ggml dequantize_row_q*)
      // and rounded once to f16, the engine's compute type for these files
      if (T.ne[0] % quant_block_elems(tt)) return false;
      std::vector<uint8_t> q((size_t)(n / quant_block_elems(tt)) * quant_block_bytes(tt));
      f.read((char*)q.data(), q.size());
      dequant_blocks(tt, q.data(), T.v.data(), n);
      for (int64_t i = 0; i < n; ++i) T.v[i] = f16_round(T.v[i]);
      if (name == "decoder.token_embedding.weight") m.wtype = T_F16;
    } else {
      std::vector<uint16_t> h(n);
      f.read((char*)h.data(), n * 2);
      for (int64_t i = 0; i < n; ++i) T.v[i] = tt == T_F16 ? h2f(h[i]) : b2f(h[i]);
      if (name == "decoder.token_embedding.weight") m.wtype = tt;
    }
    if (!f) return false;
    m.t[name] = std::move(T);
  }
  return true;
}

// ---------------------------------------------------------------------------
// primitive ops
// ---------------------------------------------------------------------------
static inline float dotf(const float* a, const float* b, int n) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int i = 0;
  for (; i + 8 <= n; i += 8)
    for (int j = 0; j < 8; ++j) acc[j] += a[i + j] * b[i + j];
  float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  for (; i < n; ++i) s += a[i] * b[i];
  return s;
}

// dotf of 2 input rows against 4 weight rows at once (8 independent
// accumulator vectors instead of one dependent chain): every output is summed
// exactly as dotf sums it (lane j of the 8-wide accumulator = acc[j], the
// same pairwise tree, then the tail), so results are bit-identical to dotf
typedef float v8f __attribute__((vector_size(32)));
static inline v8f ld8f(const float* p) {
  v8f v;
  memcpy(&v, p, 32);
  return v;
}
static inline float hsum8(v8f a) {
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}
static void dot_2x4(const float* x0, const float* x1, const float* w0, int K, int ldw, float* y0,
                    float* y1) {
  v8f acc[2][4];
  for (int r = 0; r < 2; ++r)
    for (int j = 0; j < 4; ++j) acc[r][j] = v8f{0, 0, 0, 0, 0, 0, 0, 0};
  int i = 0;
  for (; i + 8 <= K; i += 8) {
    const v8f a0 = ld8f(x0 + i), a1 = ld8f(x1 + i);
    for (int j = 0; j < 4; ++j) {
      const v8f b = ld8f(w0 + (size_t)j * ldw + i);
      acc[0][j] += a0 * b;
      acc[1][j] += a1 * b;
    }
  }
  for (int j = 0; j < 4; ++j) {
    const float* wj = w0 + (size_t)j * ldw;
    float s0 = hsum8(acc[0][j]), s1 = hsum8(acc[1][j]);
    for (int t = i; t < K; ++t) {
      s0 += x0[t] * wj[t];
      s1 += x1[t] * wj[t];
    }
    y0[j] = s0;
    y1[j] = s1;
  }
}

// ---------------------------------------------------------------------------
// MX-fp8 (engine compute mode MWX_COMPUTE_MXFP8; not a whisper.cpp mode):
// every 32 consecutive k of a row share a power-of-two scale 2^E, E the
// smallest integer with max|x| <= 448 * 2^E (no clipping); elements are
// rounded to e4m3fn (round to nearest even, subnormal step 2^-9).
// ---------------------------------------------------------------------------
static float e4m3_round(float v) {
  const float a = fabsf(v);
  if (a == 0.0f) return v;
  const int e = ilogbf(a);
  const float step = e < -6 ? ldexpf(1.0f, -9) : ldexpf(1.0f, e - 3);
  const float q = rintf(a / step) * step;
  return v < 0.0f ? -q : q;
}
static void mx_round_rows(float* x, size_t rows, int K) {
  for (size_t r = 0; r < rows; ++r)
    for (int b = 0; b < K / 32; ++b) {
      float* p = x + r * K + b * 32;
      float amax = 0.0f;
      for (int j = 0; j < 32; ++j) amax = std::max(amax, fabsf(p[j]));
      int E = 0;
      if (amax > 0.0f) {
        E = ilogbf(amax) - 8;
        while (amax > 448.0f * ldexpf(1.0f, E)) ++E;
        while (amax <= 448.0f * ldexpf(1.0f, E - 1)) --E;
        E = std::max(-127, std::min(127, E));
      }
      const float X = ldexpf(1.0f, E);
      for (int j = 0; j < 32; ++j) p[j] = e4m3_round(p[j] / X) * X;
    }
}

// y[M][N] = round_w(x)[M][K] . W[N][K]^T  (ggml_mul_mat, src0 = W); mx: the
// rounded input is further MX-fp8 quantized (W was quantized at load)
// y[r][n] = dotf(x[r], W[n]) for x [M][K], W [N][K]: blocks of NB weight rows
// (L2-resident) against every input row, so the inputs stream once per block
// instead of once per weight row, 2 x 4 outputs per register block; each
// output is still exactly one dotf (same summation order)
static void dot_rows(const float* x, int M, int K, const float* W, int N, float* y) {
  constexpr int NB = 16;
#pragma omp parallel for schedule(dynamic, 1)
  for (int n0 = 0; n0 < N; n0 += NB) {
    const int n1 = std::min(N, n0 + NB);
    int r = 0;
    for (; r + 2 <= M; r += 2) {
      const float* x0 = x + (size_t)r * K;
      int n = n0;
      for (; n + 4 <= n1; n += 4) {
        float o0[4], o1[4];
        dot_2x4(x0, x0 + K, W + (size_t)n * K, K, K, o0, o1);
        for (int j = 0; j < 4; ++j) {
          y[(size_t)r * N + n + j] = o0[j];
          y[(size_t)(r + 1) * N + n + j] = o1[j];
        }
      }
      for (; n < n1; ++n) {
        y[(size_t)r * N + n] = dotf(x0, W + (size_t)n * K, K);
        y[(size_t)(r + 1) * N + n] = dotf(x0 + K, W + (size_t)n * K, K);
      }
    }
    for (; r < M; ++r) {
      const float* x_r = x + (size_t)r * K;
      for (int n = n0; n < n1; ++n) y[(size_t)r * N + n] = dotf(x_r, W + (size_t)n * K, K);
    }
  }
}

static void matmul(const Model& m, const float* W, const float* x, int M, int N,
                   int K, float* y, bool mx = false) {
  std::vector<float> xr((size_t)M * K);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)xr.size(); ++i) xr[i] = m.rw(x[i]);
  if (mx) mx_round_rows(xr.data(), M, K);
  dot_rows(xr.data(), M, K, W, N, y);
}

static void add_bias(float* y, const float* b, int M, int N) {
#pragma omp parallel for schedule(static)
  for (int r = 0; r < M; ++r)
    for (int n = 0; n < N; ++n) y[(size_t)r * N + n] += b[n];
}

// ggml_norm (eps) followed by *w + b
static void layer_norm(const float* x, const float* w, const float* b, int M,
                       int N, float* y) {
  const float eps = 1e-5f;
#pragma omp parallel for schedule(static)
  for (int r = 0; r < M; ++r) {
    const float* xr = x + (size_t)r * N;
    float* yr = y + (size_t)r * N;
    double sum = 0.0;
    for (int i = 0; i < N; ++i) sum += (double)xr[i];
    const float mean = (float)(sum / N);
    double sum2 = 0.0;
    for (int i = 0; i < N; ++i) {
      const float v = xr[i] - mean;
      yr[i] = v;
      sum2 += (double)(v * v);
    }
    const float variance = (float)(sum2 / N);
    const float scale = 1.0f / sqrtf(variance + eps);
    for (int i = 0; i < N; ++i) yr[i] = (yr[i] * scale) * w[i] + b[i];
  }
}

static inline float gelu_f32(float x) {
  const float GELU_COEF_A = 0.044715f;
  const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
  return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
}
// ggml_vec_gelu_f32 with GGML_GELU_FP16 (f16 lookup table)
static inline float gelu(const Model& m, float x) {
  if (m.flags & ORC_EXACT) return gelu_f32(x);
  if (x <= -10.0f) return 0.0f;
  if (x >= 10.0f) return x;
  return f16_round(gelu_f32(f16_round(x)));
}

// softmax of n values with scale (ggml_compute_forward_soft_max_f32); masked
// entries (mask == true) get -inf.
static void softmax(float* w, int n, float scale) {
  for (int i = 0; i < n; ++i) w[i] *= scale;
  float mx = -INFINITY;
  for (int i = 0; i < n; ++i) mx = std::max(mx, w[i]);
  double sum = 0.0;
  for (int i = 0; i < n; ++i) {
    const float v = expf(w[i] - mx);
    sum += (double)v;
    w[i] = v;
  }
  const float inv = (float)(1.0 / sum);
  for (int i = 0; i < n; ++i) w[i] *= inv;
}

// ---------------------------------------------------------------------------
// mel spectrogram (log_mel_spectrogram + worker + fft/dft of whisper.cpp)
// ---------------------------------------------------------------------------
struct Cache {
  float sin_vals[400], cos_vals[400], hann[400];
  Cache() {
    for (int i = 0; i < 400; ++i) {
      const double theta = (2 * M_PI * i) / 400;
      sin_vals[i] = sinf((float)theta);
      cos_vals[i] = cosf((float)theta);
      hann[i] = (float)(0.5 * (1.0 - cosf((float)((2.0 * M_PI * i) / 400))));
    }
  }
};
static const Cache& gcache() {
  static Cache c;
  return c;
}

static void dft(const float* in, int N, float* out) {
  const int step = 400 / N;
  for (int k = 0; k < N; ++k) {
    float re = 0, im = 0;
    for (int n = 0; n < N; ++n) {
      const int idx = (k * n * step) % 400;
      re += in[n] * gcache().cos_vals[idx];
      im -= in[n] * gcache().sin_vals[idx];
    }
    out[k * 2 + 0] = re;
    out[k * 2 + 1] = im;
  }
}

static void fft(float* in, int N, float* out) {
  if (N == 1) {
    out[0] = in[0];
    out[1] = 0;
    return;
  }
  const int half_N = N / 2;
  if (N - half_N * 2 == 1) {
    dft(in, N, out);
    return;
  }
  float* even = in + N;
  for (int i = 0; i < half_N; ++i) even[i] = in[2 * i];
  float* even_fft = out + 2 * N;
  fft(even, half_N, even_fft);
  float* odd = even;
  for (int i = 0; i < half_N; ++i) odd[i] = in[2 * i + 1];
  float* odd_fft = even_fft + N;
  fft(odd, half_N, odd_fft);
  const int step = 400 / N;
  for (int k = 0; k < half_N; k++) {
    const int idx = k * step;
    const float re = gcache().cos_vals[idx];
    const float im = -gcache().sin_vals[idx];
    const float re_odd = odd_fft[2 * k + 0];
    const float im_odd = odd_fft[2 * k + 1];
    out[2 * k + 0] = even_fft[2 * k + 0] + re * re_odd - im * im_odd;
    out[2 * k + 1] = even_fft[2 * k + 1] + re * im_odd + im * re_odd;
    out[2 * (k + half_N) + 0] = even_fft[2 * k + 0] - re * re_odd + im * im_odd;
    out[2 * (k + half_N) + 1] = even_fft[2 * k + 1] - re * im_odd - im * re_odd;
  }
}

struct Mel {
  int n_mel = 0, n_len = 0, n_len_org = 0;
  std::vector<float> data;  // [n_mel][n_len]
};

static void log_mel(const Model& m, const float* samples, int n_samples, Mel& mel) {
  const int frame_size = 400, frame_step = 160;
  const int64_t stage_1_pad = 16000 * 30, stage_2_pad = frame_size / 2;
  std::vector<float> padded(n_samples + stage_1_pad + stage_2_pad * 2, 0.0f);
  std::copy(samples, samples + n_samples, padded.begin() + stage_2_pad);
  for (int i = 0; i < stage_2_pad; ++i) padded[i] = samples[stage_2_pad - i];  // reverse_copy(s+1, s+201)
  mel.n_mel = m.n_mels;
  mel.n_len = (int)((padded.size() - frame_size) / frame_step);
  mel.n_len_org = 1 + (int)((n_samples + stage_2_pad - frame_size) / frame_step);
  mel.data.assign((size_t)mel.n_mel * mel.n_len, 0.0f);
  const int n_samp = n_samples + (int)stage_2_pad;
  const int n_fft = m.n_fft;
  const int n_fft_frames = std::min(n_samp / frame_step + 1, mel.n_len);
#pragma omp parallel
  {
    std::vector<float> fft_in(frame_size * 2, 0.0f), fft_out(frame_size * 2 * 2 * 2);
#pragma omp for schedule(static)
    for (int i = 0; i < n_fft_frames; ++i) {
      const int offset = i * frame_step;
      std::fill(fft_in.begin(), fft_in.end(), 0.0f);
      for (int j = 0; j < std::min(frame_size, n_samp - offset); j++)
        fft_in[j] = gcache().hann[j] * padded[offset + j];
      fft(fft_in.data(), frame_size, fft_out.data());
      for (int j = 0; j < n_fft; j++)
        fft_out[j] = fft_out[2 * j + 0] * fft_out[2 * j + 0] + fft_out[2 * j + 1] * fft_out[2 * j + 1];
      for (int j = 0; j < mel.n_mel; j++) {
        double sum = 0.0;
        int k = 0;
        const float* fl = m.filters.data() + (size_t)j * n_fft;
        for (k = 0; k < n_fft - 3; k += 4)
          sum += fft_out[k + 0] * fl[k + 0] + fft_out[k + 1] * fl[k + 1] +
                 fft_out[k + 2] * fl[k + 2] + fft_out[k + 3] * fl[k + 3];
        for (; k < n_fft; k++) sum += fft_out[k] * fl[k];
        sum = log10(std::max(sum, 1e-10));
        mel.data[(size_t)j * mel.n_len + i] = (float)sum;
      }
    }
  }
  const float floor_v = (float)log10(1e-10);
  for (int i = n_fft_frames; i < mel.n_len; ++i)
    for (int j = 0; j < mel.n_mel; ++j) mel.data[(size_t)j * mel.n_len + i] = floor_v;
  double mmax = -1e20;
  for (float v : mel.data)
    if (v > mmax) mmax = v;
  mmax -= 8.0;
  for (float& v : mel.data) {
    if (v < mmax) v = (float)mmax;
    v = (float)((v + 4.0) / 4.0);
  }
}

// ---------------------------------------------------------------------------
// encoder (whisper_build_graph_conv + _encoder + _cross, non-flash path)
// ---------------------------------------------------------------------------
// conv1d with kernel 3, padding 1, stride s; input x[C][T] (channel-major),
// output y[T_out][D] (time-major); inputs rounded to the weight type (im2col).
static void conv1d(const Model& m, const float* W /*[D][C][3]*/, const float* b,
                   const float* x, int C, int T, int D, int stride, float* y) {
  const int T_out = T / stride;
  std::vector<float> col((size_t)T_out * C * 3);
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T_out; ++t)
    for (int c = 0; c < C; ++c)
      for (int k = 0; k < 3; ++k) {
        const int ti = t * stride + k - 1;
        const float v = (ti >= 0 && ti < T) ? x[(size_t)c * T + ti] : 0.0f;
        col[((size_t)t * C + c) * 3 + k] = m.rw(v);
      }
  dot_rows(col.data(), T_out, C * 3, W, D, y);
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T_out; ++t)
    for (int d = 0; d < D; ++d) y[(size_t)t * D + d] += b[d];
}

// multi-head attention, one query block; Q[Lq][D], K[Lk][D], V[Lk][D] (f32);
// scores scaled by `scale` inside softmax; causal: mask keys > q_pos0 + i.
// khp / vtp (optional): K and V of every head already laid out as the loop
// below builds them ([H][Lk][dh] and [H][dh][Lk], r16-rounded): the cross
// K/V of a window, prepared once (cross_heads) instead of on every decode
static void attention(const Model& m, const float* Q, const float* K, const float* V,
                      int Lq, int Lk, int D, int H, float scale, int causal_pos0,
                      float* O, const float* khp = nullptr, const float* vtp = nullptr) {
  const int dh = D / H;
#pragma omp parallel
  {
    // vt: V of the head transposed [e][j] (the P.V sums read it contiguously,
    // in the same order as before)
    std::vector<float> q(dh), w(Lk), khb(khp ? 0 : (size_t)Lk * dh), vtb(vtp ? 0 : (size_t)dh * Lk);
#pragma omp for schedule(static)
    for (int h = 0; h < H; ++h) {
      const float* kh = khp ? khp + (size_t)h * Lk * dh : khb.data();
      const float* vt = vtp ? vtp + (size_t)h * dh * Lk : vtb.data();
      if (!khp)
        for (int j = 0; j < Lk; ++j)
          for (int e = 0; e < dh; ++e) khb[(size_t)j * dh + e] = m.r16(K[(size_t)j * D + h * dh + e]);
      if (!vtp)
        for (int j = 0; j < Lk; ++j)
          for (int e = 0; e < dh; ++e) vtb[(size_t)e * Lk + j] = m.r16(V[(size_t)j * D + h * dh + e]);
      for (int i = 0; i < Lq; ++i) {
        for (int e = 0; e < dh; ++e) q[e] = m.r16(Q[(size_t)i * D + h * dh + e]);
        const int nk = causal_pos0 >= 0 ? std::min(Lk, causal_pos0 + i + 1) : Lk;
        for (int j = 0; j < nk; ++j) w[j] = dotf(kh + (size_t)j * dh, q.data(), dh);
        softmax(w.data(), nk, scale);
        for (int j = 0; j < nk; ++j) w[j] = m.r16(w[j]);
        for (int e = 0; e < dh; ++e) {
          const float* ve = vt + (size_t)e * Lk;
          float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          int j = 0;
          for (; j + 8 <= nk; j += 8)
            for (int u = 0; u < 8; ++u) acc[u] += ve[j + u] * w[j + u];
          float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
          for (; j < nk; ++j) s += ve[j] * w[j];
          O[(size_t)i * D + h * dh + e] = s;
        }
      }
    }
  }
}

// Encoder layer cap used only by the bounded CPU-baseline sample (bench.py):
// < 0 runs all layers.
static int g_enc_layer_limit = -1;

// Results cache of the oracle's most expensive pure functions (the encoder
// and the cross K/V of a window): at large-v3 depth one encode costs a minute
// of CPU and the GPU test suite asks for the same window (same model file,
// same mel frames) in several tests. Keyed by the model's identity and an
// FNV-1a hash of the exact input bytes; a few entries, oldest dropped first.
static uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}
template <class V>
struct ResultCache {
  size_t cap;
  std::vector<std::pair<std::string, V>> e;
  const V* get(const std::string& k) const {
    for (const auto& x : e)
      if (x.first == k) return &x.second;
    return nullptr;
  }
  void put(const std::string& k, const V& v) {
    if (e.size() >= cap) e.erase(e.begin());
    e.emplace_back(k, v);
  }
};
static ResultCache<std::vector<float>> g_enc_cache{8, {}};

// the conv stem: mel window x [n_mels][2 n_ctx] -> residual stream inp [n_ctx][D]
static void encode_stem(const Model& m, const std::vector<float>& x, std::vector<float>& inp) {
  const int n_ctx = m.n_audio_ctx, D = m.n_audio_state;
  const int T = 2 * n_ctx;
  std::vector<float> h1((size_t)T * D), h2((size_t)n_ctx * D);
  conv1d(m, m.w("encoder.conv1.weight"), m.w("encoder.conv1.bias"), x.data(), m.n_mels, T, D, 1, h1.data());
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)h1.size(); ++i) h1[i] = gelu(m, h1[i]);
  // conv2 consumes channel-major input
  std::vector<float> h1c((size_t)D * T);
  for (int t = 0; t < T; ++t)
    for (int d = 0; d < D; ++d) h1c[(size_t)d * T + t] = h1[(size_t)t * D + d];
  conv1d(m, m.w("encoder.conv2.weight"), m.w("encoder.conv2.bias"), h1c.data(), D, T, D, 2, h2.data());
  const float* pe = m.w("encoder.positional_embedding");
  inp.resize((size_t)n_ctx * D);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)inp.size(); ++i) inp[i] = pe[i] + gelu(m, h2[i]);
}

// Test hook of one encoder layer (orc_encode_layer): ext[g] non-null takes
// GEMM g's A operand (0: attn LN output, 1: attention output, 2: mlp LN
// output, 3: GELU output) from the caller instead of computing it; out[g]
// non-null receives the A operand used.
struct EncLayerIO {
  const float* ext[4];
  float* out[4];
};

// one encoder layer on the residual stream inp [n_ctx][D], in place
static void encode_layer(const Model& m, int il, std::vector<float>& inp, const EncLayerIO* io) {
  const int M = m.n_audio_ctx, D = m.n_audio_state, H = m.n_audio_head;
  std::vector<float> cur((size_t)M * D), q((size_t)M * D), k((size_t)M * D),
      v((size_t)M * D), o((size_t)M * D), ff((size_t)M * 4 * D);
  const float KQscale = 1.0f / sqrtf((float)(D / H));
  const bool mx = (m.flags & ORC_MXFP8) != 0;
  auto operand = [&](int g, std::vector<float>& a) {
    if (io && io->ext[g]) std::copy(io->ext[g], io->ext[g] + a.size(), a.begin());
    if (io && io->out[g]) std::copy(a.begin(), a.end(), io->out[g]);
  };
  const std::string p = "encoder.blocks." + std::to_string(il);
  layer_norm(inp.data(), m.w(p + ".attn_ln.weight"), m.w(p + ".attn_ln.bias"), M, D, cur.data());
  operand(0, cur);
  matmul(m, m.w(p + ".attn.query.weight"), cur.data(), M, D, D, q.data(), mx);
  add_bias(q.data(), m.w(p + ".attn.query.bias"), M, D);
  matmul(m, m.w(p + ".attn.key.weight"), cur.data(), M, D, D, k.data(), mx);
  matmul(m, m.w(p + ".attn.value.weight"), cur.data(), M, D, D, v.data(), mx);
  add_bias(v.data(), m.w(p + ".attn.value.bias"), M, D);
  attention(m, q.data(), k.data(), v.data(), M, M, D, H, KQscale, -1, o.data());
  operand(1, o);
  matmul(m, m.w(p + ".attn.out.weight"), o.data(), M, D, D, cur.data(), mx);
  add_bias(cur.data(), m.w(p + ".attn.out.bias"), M, D);
  for (size_t i = 0; i < inp.size(); ++i) inp[i] = cur[i] + inp[i];
  layer_norm(inp.data(), m.w(p + ".mlp_ln.weight"), m.w(p + ".mlp_ln.bias"), M, D, cur.data());
  operand(2, cur);
  matmul(m, m.w(p + ".mlp.0.weight"), cur.data(), M, 4 * D, D, ff.data(), mx);
  add_bias(ff.data(), m.w(p + ".mlp.0.bias"), M, 4 * D);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)ff.size(); ++i) ff[i] = gelu(m, ff[i]);
  operand(3, ff);
  matmul(m, m.w(p + ".mlp.2.weight"), ff.data(), M, D, 4 * D, cur.data(), mx);
  add_bias(cur.data(), m.w(p + ".mlp.2.bias"), M, D);
  for (size_t i = 0; i < inp.size(); ++i) inp[i] = cur[i] + inp[i];
}

// Encodes the 2*n_ctx mel frames starting at `seek`; out = embd_enc [n_ctx][D].
static void encode(const Model& m, const Mel& mel, int seek, std::vector<float>& out) {
  const int n_ctx = m.n_audio_ctx, D = m.n_audio_state;
  const int T = 2 * n_ctx;
  std::vector<float> x((size_t)m.n_mels * T, 0.0f);
  const int i0 = std::min(seek, mel.n_len), i1 = std::min(seek + T, mel.n_len);
  for (int j = 0; j < m.n_mels; ++j)
    for (int i = i0; i < i1; ++i) x[(size_t)j * T + (i - i0)] = mel.data[(size_t)j * mel.n_len + i];
  const std::string ckey = m.key + "|enc|" + std::to_string(g_enc_layer_limit) + "|" +
                           std::to_string(fnv1a(x.data(), x.size() * sizeof(float)));
  if (const auto* hit = m.key.empty() ? nullptr : g_enc_cache.get(ckey)) {
    out = *hit;
    return;
  }
  std::vector<float> inp;
  encode_stem(m, x, inp);
  const int M = n_ctx;
  const int n_layers = g_enc_layer_limit >= 0 ? std::min(g_enc_layer_limit, m.n_audio_layer)
                                             : m.n_audio_layer;
  for (int il = 0; il < n_layers; ++il) encode_layer(m, il, inp, nullptr);
  out.resize((size_t)M * D);
  layer_norm(inp.data(), m.w("encoder.ln_post.weight"), m.w("encoder.ln_post.bias"), M, D, out.data());
  if (!m.key.empty()) g_enc_cache.put(ckey, out);
}

// kv_cross: per decoder layer K = f16(Kscale * Wk enc), V = f16(Wv enc + b)
struct Cross {
  std::vector<float> k, v;  // [n_layer][n_ctx][D]
  // per head, as attention() lays them out: kh [n_layer][H][n_ctx][dh],
  // vt [n_layer][H][dh][n_ctx] (cross_heads)
  std::vector<float> kh, vt;
};
static void cross_heads(const Model& m, Cross& c) {
  const int M = m.n_audio_ctx, D = m.n_text_state, L = m.n_text_layer, H = m.n_text_head;
  const int dh = D / H;
  c.kh.resize(c.k.size());
  c.vt.resize(c.v.size());
#pragma omp parallel for schedule(static)
  for (int lh = 0; lh < L * H; ++lh) {
    const int il = lh / H, h = lh % H;
    const float* K = c.k.data() + (size_t)il * M * D;
    const float* V = c.v.data() + (size_t)il * M * D;
    float* kh = c.kh.data() + (size_t)lh * M * dh;
    float* vt = c.vt.data() + (size_t)lh * dh * M;
    for (int j = 0; j < M; ++j)
      for (int e = 0; e < dh; ++e) {
        kh[(size_t)j * dh + e] = m.r16(K[(size_t)j * D + h * dh + e]);
        vt[(size_t)e * M + j] = m.r16(V[(size_t)j * D + h * dh + e]);
      }
  }
}
static ResultCache<Cross> g_cross_cache{2, {}};
static void cross(const Model& m, const std::vector<float>& enc, Cross& c) {
  const std::string ckey = m.key + "|cross|" + std::to_string(fnv1a(enc.data(), enc.size() * sizeof(float)));
  if (const auto* hit = m.key.empty() ? nullptr : g_cross_cache.get(ckey)) {
    c = *hit;
    return;
  }
  struct Put {
    const std::string& k;
    Cross& c;
    const bool on;
    ~Put() {
      if (on) g_cross_cache.put(k, c);
    }
  } put{ckey, c, !m.key.empty()};
  const int M = m.n_audio_ctx, D = m.n_text_state, L = m.n_text_layer;
  const float Kscale = powf((float)(D / m.n_text_head), -0.25f);
  c.k.resize((size_t)L * M * D);
  c.v.resize((size_t)L * M * D);
  std::vector<float> tmp((size_t)M * D);
  for (int il = 0; il < L; ++il) {
    const std::string p = "decoder.blocks." + std::to_string(il);
    matmul(m, m.w(p + ".cross_attn.key.weight"), enc.data(), M, D, m.n_audio_state, tmp.data(),
           m.flags & ORC_MXFP8);
    for (size_t i = 0; i < tmp.size(); ++i) c.k[(size_t)il * M * D + i] = m.r16(tmp[i] * Kscale);
    matmul(m, m.w(p + ".cross_attn.value.weight"), enc.data(), M, D, m.n_audio_state, tmp.data(),
           m.flags & ORC_MXFP8);
    add_bias(tmp.data(), m.w(p + ".cross_attn.value.bias"), M, D);
    for (size_t i = 0; i < tmp.size(); ++i) c.v[(size_t)il * M * D + i] = m.r16(tmp[i]);
    if (m.flags & ORC_MXFP8) {
      // fp8 cross K/V cache: the f16 values of each 32-block of a (time,
      // head) row MX-rounded (the engine stores codes + E8M0 scales)
      mx_round_rows(c.k.data() + (size_t)il * M * D, M, D);
      mx_round_rows(c.v.data() + (size_t)il * M * D, M, D);
    }
  }
  cross_heads(m, c);
}

// ---------------------------------------------------------------------------
// decoder with KV cache (whisper_build_graph_decoder, non-flash path)
// ---------------------------------------------------------------------------
struct KV {
  // per layer [n][D] (f16-rounded values), grown as tokens are decoded (a
  // beam hand-over copies what is stored, not n_text_ctx rows)
  std::vector<std::vector<float>> k, v;
  int n = 0;  // tokens stored
};

// Decodes `n_tok` tokens at positions n_past.. and returns logits of every
// token [n_tok][n_vocab].
static void decode(const Model& m, const Cross& cr, KV& kv, const int* tokens, int n_tok,
                   int n_past, std::vector<float>& logits) {
  const int D = m.n_text_state, H = m.n_text_head, L = m.n_text_layer, V = m.n_vocab;
  const int n_ctx = m.n_text_ctx, n_actx = m.n_audio_ctx;
  const int dh = D / H;
  const float KQscale = powf((float)dh, -0.25f);
  if (kv.k.empty()) {
    kv.k.resize(L);
    kv.v.resize(L);
  }
  (void)n_ctx;
  const int M = n_tok;
  const float* te = m.w("decoder.token_embedding.weight");
  const float* pe = m.w("decoder.positional_embedding");
  std::vector<float> inp((size_t)M * D), cur((size_t)M * D), q((size_t)M * D),
      k((size_t)M * D), v((size_t)M * D), o((size_t)M * D), ff((size_t)M * 4 * D);
  for (int i = 0; i < M; ++i)
    for (int d = 0; d < D; ++d)
      inp[(size_t)i * D + d] = te[(size_t)tokens[i] * D + d] + pe[(size_t)(n_past + i) * D + d];
  for (int il = 0; il < L; ++il) {
    const std::string p = "decoder.blocks." + std::to_string(il);
    layer_norm(inp.data(), m.w(p + ".attn_ln.weight"), m.w(p + ".attn_ln.bias"), M, D, cur.data());
    matmul(m, m.w(p + ".attn.query.weight"), cur.data(), M, D, D, q.data());
    add_bias(q.data(), m.w(p + ".attn.query.bias"), M, D);
    for (auto& e : q) e *= KQscale;
    matmul(m, m.w(p + ".attn.key.weight"), cur.data(), M, D, D, k.data());
    for (auto& e : k) e *= KQscale;
    matmul(m, m.w(p + ".attn.value.weight"), cur.data(), M, D, D, v.data());
    add_bias(v.data(), m.w(p + ".attn.value.bias"), M, D);
    kv.k[il].resize((size_t)(n_past + M) * D);
    kv.v[il].resize((size_t)(n_past + M) * D);
    float* kc = kv.k[il].data();
    float* vc = kv.v[il].data();
    for (int i = 0; i < M; ++i)
      for (int d = 0; d < D; ++d) {
        kc[(size_t)(n_past + i) * D + d] = m.r16(k[(size_t)i * D + d]);
        vc[(size_t)(n_past + i) * D + d] = m.r16(v[(size_t)i * D + d]);
      }
    attention(m, q.data(), kc, vc, M, n_past + M, D, H, 1.0f, n_past, o.data());
    matmul(m, m.w(p + ".attn.out.weight"), o.data(), M, D, D, cur.data());
    add_bias(cur.data(), m.w(p + ".attn.out.bias"), M, D);
    for (size_t i = 0; i < inp.size(); ++i) inp[i] = cur[i] + inp[i];
    // cross-attention
    layer_norm(inp.data(), m.w(p + ".cross_attn_ln.weight"), m.w(p + ".cross_attn_ln.bias"), M, D, cur.data());
    matmul(m, m.w(p + ".cross_attn.query.weight"), cur.data(), M, D, D, q.data());
    add_bias(q.data(), m.w(p + ".cross_attn.query.bias"), M, D);
    attention(m, q.data(), cr.k.data() + (size_t)il * n_actx * D, cr.v.data() + (size_t)il * n_actx * D,
              M, n_actx, D, H, KQscale, -1, o.data(),
              cr.kh.empty() ? nullptr : cr.kh.data() + (size_t)il * n_actx * D,
              cr.vt.empty() ? nullptr : cr.vt.data() + (size_t)il * n_actx * D);
    matmul(m, m.w(p + ".cross_attn.out.weight"), o.data(), M, D, D, cur.data());
    add_bias(cur.data(), m.w(p + ".cross_attn.out.bias"), M, D);
    for (size_t i = 0; i < inp.size(); ++i) inp[i] = cur[i] + inp[i];
    // mlp
    layer_norm(inp.data(), m.w(p + ".mlp_ln.weight"), m.w(p + ".mlp_ln.bias"), M, D, cur.data());
    matmul(m, m.w(p + ".mlp.0.weight"), cur.data(), M, 4 * D, D, ff.data());
    add_bias(ff.data(), m.w(p + ".mlp.0.bias"), M, 4 * D);
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)ff.size(); ++i) ff[i] = gelu(m, ff[i]);
    matmul(m, m.w(p + ".mlp.2.weight"), ff.data(), M, D, 4 * D, cur.data());
    add_bias(cur.data(), m.w(p + ".mlp.2.bias"), M, D);
    for (size_t i = 0; i < inp.size(); ++i) inp[i] = cur[i] + inp[i];
  }
  layer_norm(inp.data(), m.w("decoder.ln.weight"), m.w("decoder.ln.bias"), M, D, cur.data());
  logits.resize((size_t)M * V);
  matmul(m, te, cur.data(), M, V, D, logits.data());
  kv.n = n_past + M;
}

// ---------------------------------------------------------------------------
// whisper_full restatement
// ---------------------------------------------------------------------------
struct TokenData {
  int id = 0, tid = 0;
  float p = 0, plog = 0, pt = 0, ptsum = 0;
  int64_t t0 = -1, t1 = -1, t_dtw = -1;
  float vlen = 0;
};
struct Segment {
  int64_t t0, t1;
  std::string text;
  float no_speech_prob;
  std::vector<TokenData> tokens;
  bool speaker_turn_next;
};
struct Sequence {
  std::vector<TokenData> tokens;
  int result_len = 0;
  double sum_logprobs_all = 0, sum_logprobs = -INFINITY, avg_logprobs = -INFINITY,
         entropy = 0, score = -INFINITY;
};
struct Decoder {
  Sequence seq;
  bool failed = false, completed = false, has_ts = false;
  int seek_delta = 3000;
  KV kv;
  std::vector<float> probs, logits, logprobs;
  std::mt19937 rng;
};

struct Params {
  int strategy = 0;
  int n_max_text_ctx = 16384;
  int offset_ms = 0, duration_ms = 0;
  bool translate = false, no_context = true, no_timestamps = false,
       single_segment = false, print_special = false, token_timestamps = false;
  float thold_pt = 0.01f, thold_ptsum = 0.01f;
  int max_tokens = 0;
  bool tdrz_enable = false;
  std::string language = "en";
  std::vector<int> prompt_tokens;
  std::string initial_prompt;
  bool suppress_blank = true, suppress_nst = false;
  float temperature = 0.0f, max_initial_ts = 1.0f, length_penalty = -1.0f,
        temperature_inc = 0.2f, entropy_thold = 2.4f, logprob_thold = -1.0f,
        no_speech_thold = 0.6f;
  int best_of = 5, beam_size = 5;
  int bench_fixed_steps = 0;
};

struct Result {
  std::vector<Segment> segs;
  int lang_id = 0;
  std::vector<std::vector<int>> window_tokens;  // raw tokens of every window (debug)
};

// Decision trace (test hook, orc_trace_*): every float-sensitive decision
// full() takes, in order, with the oracle-side margin by which it was taken.
// Two runs on different logits (the oracle's own arithmetic and the device's
// logits, replayed) agree up to their first differing event; that event's
// margin against the measured logits error says whether the divergence is a
// near-tie or a differing rule (tests/test_gpu_beam_oracle.py).
enum TraceKind {
  TR_DRAW = 1,      // discrete_distribution draw: a = draw index, b = id; margin = distance
                    // of the uniform to the nearest cumulative boundary of id's interval
  TR_ARGMAX = 2,    // greedy pick: b = id; margin = top-1 - top-2 logprob
  TR_ASSIGN = 3,    // beam hand-over: a = source decoder, b = last token id; margin = the
                    // smallest sum_logprobs_all gap to a neighbouring distinct candidate
  TR_TSMASS = 4,    // timestamp-mass rule: a = forced; margin = |log sum p(ts) - max text logprob|
  TR_BEST = 5,      // best decoder: a = id; margin = best score - runner-up score
  TR_FALLBACK = 6,  // a = success; margin = distance of the deciding quantity to its threshold
  TR_NOSPEECH = 7,  // window is_no_speech: a = value; margin as above
  TR_EXACT_TIE = 8, // two DISTINCT beam candidates tied exactly on (sum_logprobs_all, decoder)
                    // (upstream std::sort leaves their order unspecified: DESIGN §2 D5)
  TR_STATUS = 9,    // decoder state after a step: a = completed + 2 failed, b = result_len
};
// a, b: the outcome taken. Follow mode (below) may override the oracle's own
// outcome: then forced = 1, (own_a, own_b) is what the oracle's arithmetic
// decided and fmargin how far that arithmetic is from the taken outcome (in
// the kind's own units: cumulative probability for draws, log-prob for argmax
// / ts_mass, summed log-prob for assign, score for best, the threshold
// quantity for fallback / no_speech). Draws also record [lo, hi), the taken
// id's interval of the normalised cumulative probabilities.
struct TraceEv {
  int kind, seek, it, step, dec, a, b;
  double margin, v;
  int forced = 0, own_a = 0, own_b = 0;
  double fmargin = 0.0, lo = 0.0, hi = 0.0;
};
static bool g_trace_on = false;
static std::vector<TraceEv> g_trace;
static struct { int seek = 0, it = 0, step = -1, dec = 0; } g_tctx;
static TraceEv& trace(int kind, int a, int b, double margin, double v = 0.0) {
  static TraceEv sink;
  if (!g_trace_on) return sink = TraceEv{};
  g_trace.push_back({kind, g_tctx.seek, g_tctx.it, g_tctx.step, g_tctx.dec, a, b, margin, v});
  return g_trace.back();
}

// Follow mode (test hook, orc_trace_follow): full() runs on its own logits but
// takes, at every traced decision, the outcome a guide trace recorded — the
// oracle's loop replayed on the device's logits. Where the two outcomes differ
// the event is marked forced, so the run continues on the device's path and
// every later decision is still compared against the oracle's own arithmetic
// on that path (tests/test_gpu_beam_oracle.py). A guide event of another kind
// or place, or a structural event (status, exact tie) that differs, ends
// following: g_follow_break = that event's index.
static bool g_follow_on = false;
static std::vector<TraceEv> g_follow;
static long g_follow_break = -1;
static const TraceEv* follow(int kind) {
  if (!g_follow_on || !g_trace_on) return nullptr;
  const size_t i = g_trace.size();  // the index the event about to be traced gets
  const TraceEv* g = i < g_follow.size() ? &g_follow[i] : nullptr;
  if (!g || g->kind != kind || g->seek != g_tctx.seek || g->it != g_tctx.it ||
      g->step != g_tctx.step || g->dec != g_tctx.dec) {
    g_follow_on = false;
    g_follow_break = (long)i;
    return nullptr;
  }
  return g;
}
static void follow_structural(int a, int b) {  // after tracing a status / tie event
  if (!g_follow_on) return;
  const TraceEv& e = g_trace.back();
  const TraceEv& g = g_follow[g_trace.size() - 1];
  if (g.a != a || g.b != b) {
    g_follow_on = false;
    g_follow_break = (long)g_trace.size() - 1;
    (void)e;
  }
}
static void mark_forced(TraceEv& e, int own_a, int own_b, double fmargin) {
  e.forced = 1;
  e.own_a = own_a;
  e.own_b = own_b;
  e.fmargin = fmargin;
}

// The decision of a libstdc++ discrete_distribution draw. rng is the
// generator state BEFORE the draw (its uniform is generate_canonical<double,
// 53>, the search lower_bound over the normalised partial sums), id the
// oracle's own outcome. Traces the draw (margin = distance of u to the nearest
// boundary of id's interval) and returns the id to take: in follow mode the
// guide's, with fmargin = the distance of u to that id's interval.
static int trace_draw(const std::vector<float>& probs, std::mt19937 rng, int k, int id) {
  if (!g_trace_on) return id;
  const TraceEv* g = follow(TR_DRAW);
  const int take = g ? g->b : id;
  const double u = std::generate_canonical<double, std::numeric_limits<double>::digits>(rng);
  double sum = 0.0;
  for (float p : probs) sum += p;
  auto interval = [&](int j, double& lo, double& hi) {
    lo = 0.0;
    for (int i = 0; i < j; ++i) lo += probs[i] / sum;
    hi = lo + probs[j] / sum;
  };
  double lo, hi;
  interval(id, lo, hi);
  const double margin = std::min(u - lo, hi - u);
  if (take == id) {
    TraceEv& e = trace(TR_DRAW, k, id, margin, u);
    e.lo = lo;
    e.hi = hi;
    return id;
  }
  double flo, fhi;
  interval(take, flo, fhi);
  TraceEv& e = trace(TR_DRAW, k, take, margin, u);
  e.lo = flo;
  e.hi = fhi;
  mark_forced(e, k, id, u < flo ? flo - u : u - fhi);
  return take;
}

static const std::vector<std::string> kNonSpeech = {
    "\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^",
    "_", "`", "{", "|", "}", "~", "「", "」", "『", "』", "<<", ">>", "<<<", ">>>", "--",
    "---", "-(", "-[", "('", "(\"", "((", "))", "(((", ")))", "[[", "]]", "{{", "}}", "♪♪",
    "♪♪♪", "♩", "♪", "♫", "♬", "♭", "♮", "♯"};

static void compute_logprobs(const std::vector<float>& logits, int n, std::vector<float>& lp) {
  const float mx = *std::max_element(logits.begin(), logits.end());
  float lse = 0.0f;
  for (int i = 0; i < n; ++i)
    if (logits[i] > -INFINITY) lse += expf(logits[i] - mx);
  lse = logf(lse) + mx;
  for (int i = 0; i < n; ++i) lp[i] = logits[i] > -INFINITY ? logits[i] - lse : -INFINITY;
}
static void compute_probs(const std::vector<float>& logits, int n, const std::vector<float>& lp,
                          std::vector<float>& pr) {
  for (int i = 0; i < n; ++i) pr[i] = logits[i] == -INFINITY ? 0.0f : expf(lp[i]);
}

// ts_mass_rule = false leaves out the last step (the timestamp-mass rule), a
// test hook of orc_process_logits
static void process_logits(const Model& m, const Params& P, Decoder& dec, const float* raw,
                           float temperature, bool ts_mass_rule = true) {
  const int n = m.n_vocab;
  const auto& toks = dec.seq.tokens;
  const bool is_initial = toks.empty();
  auto& logits = dec.logits;
  logits.assign(raw, raw + n);
  dec.probs.resize(n);
  dec.logprobs.resize(n);
  if (temperature > 0.0f)
    for (int i = 0; i < n; ++i) logits[i] /= temperature;
  if (P.suppress_blank && is_initial) {
    logits[m.eot] = -INFINITY;
    logits[m.token_to_id.at(" ")] = -INFINITY;
  }
  logits[m.not_] = -INFINITY;
  if (P.no_timestamps)
    for (int i = m.beg; i < n; ++i) logits[i] = -INFINITY;
  logits[m.sot] = -INFINITY;
  logits[m.nosp] = -INFINITY;
  if (!P.tdrz_enable) logits[m.solm] = -INFINITY;
  logits[m.translate] = -INFINITY;
  logits[m.transcribe] = -INFINITY;
  logits[m.prev] = -INFINITY;
  for (int i = 0; i < kNLang; ++i) logits[m.sot + 1 + i] = -INFINITY;
  logits[m.prev] = -INFINITY;
  if (P.suppress_nst) {
    for (const auto& t : kNonSpeech) {
      for (const std::string& s : {t, " " + t}) {
        auto it = m.token_to_id.find(s);
        if (it != m.token_to_id.end()) logits[it->second] = -INFINITY;
      }
    }
    auto it = m.token_to_id.find(" -");
    if (it != m.token_to_id.end()) logits[it->second] = -INFINITY;
    it = m.token_to_id.find(" '");
    if (it != m.token_to_id.end()) logits[it->second] = -INFINITY;
  }
  if (P.bench_fixed_steps > 0) {  // benchmark workload: no EOT, no timestamps
    logits[m.eot] = -INFINITY;
    for (int i = m.beg; i < n; ++i) logits[i] = -INFINITY;
  }
  {
    const bool last_ts = !toks.empty() && toks.back().id >= m.beg;
    const bool penult_ts = toks.size() < 2 || toks[toks.size() - 2].id >= m.beg;
    if (last_ts) {
      if (penult_ts) {
        for (int i = m.beg; i < n; ++i) logits[i] = -INFINITY;
      } else {
        for (int i = 0; i < m.eot; ++i) logits[i] = -INFINITY;
      }
    }
  }
  if (is_initial && P.max_initial_ts > 0.0f) {
    const float precision = float(30) / m.n_audio_ctx;
    const int tid0 = (int)std::round(P.max_initial_ts / precision);
    for (int i = m.beg + tid0 + 1; i < n; ++i) logits[i] = -INFINITY;
  }
  if (dec.has_ts) {
    const int tid0 = dec.seek_delta / 2;
    for (int i = m.beg; i < m.beg + tid0; ++i) logits[i] = -INFINITY;
  }
  compute_logprobs(logits, n, dec.logprobs);
  if (ts_mass_rule) {
    float ts_logprob = -INFINITY;
    {
      float lse = 0.0f;
      const float lmax = *std::max_element(dec.logprobs.begin() + m.beg, dec.logprobs.end());
      for (int i = m.beg; i < n; ++i)
        if (dec.logprobs[i] > -INFINITY) lse += expf(dec.logprobs[i] - lmax);
      if (lse > 0.0f) ts_logprob = logf(lse) + lmax;
    }
    const float max_text = *std::max_element(dec.logprobs.begin(), dec.logprobs.begin() + m.beg);
    bool forced_ts = ts_logprob > max_text;
    {
      const TraceEv* g = follow(TR_TSMASS);
      const double mg = fabs((double)ts_logprob - (double)max_text);
      if (g && g->a != (int)forced_ts) {
        mark_forced(trace(TR_TSMASS, g->a, 0, mg), forced_ts, 0, mg);
        forced_ts = g->a != 0;
      } else {
        trace(TR_TSMASS, forced_ts, 0, mg);
      }
    }
    if (forced_ts) {
      for (int i = 0; i < m.beg; ++i) {
        logits[i] = -INFINITY;
        dec.logprobs[i] = -INFINITY;
      }
    }
  }
  compute_probs(logits, n, dec.logprobs, dec.probs);
}

static TokenData sample_token(const Model& m, Decoder& dec, bool best) {
  TokenData r;
  r.t0 = r.t1 = r.t_dtw = -1;
  const int n = m.n_vocab;
  const auto& probs = dec.probs;
  const auto& lp = dec.logprobs;
  {
    double sum_ts = 0.0, max_ts = 0.0;
    for (int i = m.beg; i < n; i++) {
      if (probs[i] == -INFINITY) continue;
      sum_ts += probs[i];
      if (max_ts < probs[i]) {
        max_ts = probs[i];
        r.tid = i;
      }
    }
    r.pt = (float)(max_ts / (sum_ts + 1e-10));
    r.ptsum = (float)sum_ts;
  }
  if (best) {
    for (int i = 0; i < n; ++i) {
      if (r.p < probs[i]) {
        r.id = i;
        r.p = probs[i];
        r.plog = lp[i];
      }
    }
    if (g_trace_on) {
      float second = -INFINITY;
      for (int i = 0; i < n; ++i)
        if (i != r.id && lp[i] > second) second = lp[i];
      const TraceEv* g = follow(TR_ARGMAX);
      if (g && g->b != r.id) {
        mark_forced(trace(TR_ARGMAX, 0, g->b, (double)r.plog - (double)second), 0, r.id,
                    (double)r.plog - (double)lp[g->b]);
        r.id = g->b;
        r.p = probs[r.id];
        r.plog = lp[r.id];
      } else {
        trace(TR_ARGMAX, 0, r.id, (double)r.plog - (double)second);
      }
    }
  } else {
    std::discrete_distribution<> dist(probs.begin(), probs.end());
    const std::mt19937 before = dec.rng;
    r.id = dist(dec.rng);
    r.id = trace_draw(probs, before, 0, r.id);
    r.p = probs[r.id];
    r.plog = lp[r.id];
  }
  if (r.id >= m.beg) {
    r.tid = r.id;
    r.pt = r.p;
  }
  return r;
}

// whisper_sample_token_topk (whisper.cpp v1.8.2): the timestamp statistics of
// whisper_sample_token, then k draws with replacement from
// std::discrete_distribution over the decoder's probs with the decoder's RNG
// (upstream also partial-sorts the logits here, but the candidates come from
// the draws).
static std::vector<TokenData> sample_topk(const Model& m, Decoder& dec, int k) {
  const int n = m.n_vocab;
  const auto& probs = dec.probs;
  const auto& lp = dec.logprobs;
  int tid = m.beg;
  float pt = 0.0f, ptsum = 0.0f;
  {
    double sum_ts = 0.0, max_ts = 0.0;
    for (int i = m.beg; i < n; i++) {
      if (probs[i] == -INFINITY) continue;
      sum_ts += probs[i];
      if (max_ts < probs[i]) {
        max_ts = probs[i];
        tid = i;
      }
    }
    pt = (float)(max_ts / (sum_ts + 1e-10));
    ptsum = (float)sum_ts;
  }
  std::discrete_distribution<> dist(probs.begin(), probs.end());
  std::vector<TokenData> out;
  for (int i = 0; i < k; ++i) {
    TokenData r;
    const std::mt19937 before = dec.rng;
    r.id = dist(dec.rng);
    r.id = trace_draw(probs, before, i, r.id);
    r.tid = tid;
    r.p = probs[r.id];
    r.plog = lp[r.id];
    r.pt = pt;
    r.ptsum = ptsum;
    if (r.id >= m.beg) {
      r.tid = r.id;
      r.pt = r.p;
    }
    out.push_back(r);
  }
  return out;
}

// whisper_sequence_tokens_equal
static bool tokens_equal(const Sequence& a, const Sequence& b) {
  if (a.tokens.size() != b.tokens.size()) return false;
  for (int i = (int)a.tokens.size() - 1; i >= 0; i--)
    if (a.tokens[i].id != b.tokens[i].id) return false;
  return true;
}

struct BeamCand {
  int decoder_idx;
  int seek_delta;
  bool has_ts;
  Sequence seq;
};


static void sequence_score(const Params& P, Sequence& s) {
  if (s.result_len == 0) return;
  double result = 0.0;
  for (int i = 0; i < s.result_len; ++i) result += s.tokens[i].plog;
  s.sum_logprobs = result;
  s.avg_logprobs = result / s.result_len;
  double penalty = s.result_len;
  if (P.length_penalty > 0.0f) penalty = pow((5.0 + penalty) / 6.0, P.length_penalty);
  s.score = result / penalty;
  const int n = 32;
  int cnt = 0;
  double entropy = 0.0;
  std::map<int, int> counts;
  for (int i = std::max(0, s.result_len - n); i < s.result_len; ++i) {
    counts[s.tokens[i].id]++;
    cnt++;
  }
  for (const auto& kv : counts) {
    const double p = kv.second / (double)cnt;
    entropy -= p * log(p);
  }
  s.entropy = entropy;
}

static std::vector<float> signal_energy(const float* sig, int n, int hw) {
  std::vector<float> r(n);
  for (int i = 0; i < n; i++) {
    float sum = 0;
    for (int j = -hw; j <= hw; j++)
      if (i + j >= 0 && i + j < n) sum += fabsf(sig[i + j]);
    r[i] = sum / (2 * hw + 1);
  }
  return r;
}

static float voice_length(const std::string& text) {
  float res = 0.0f;
  for (char c : text) {
    if (c == ' ') res += 0.01f;
    else if (c == ',') res += 2.00f;
    else if (c == '.' || c == '!' || c == '?') res += 3.00f;
    else if (c >= '0' && c <= '9') res += 3.00f;
    else res += 1.00f;
  }
  return res;
}
static int ts_to_sample(int64_t t, int n) {
  return std::max(0, std::min(n - 1, (int)((t * 16000) / 100)));
}
static int64_t sample_to_ts(int i) { return (100ll * i) / 16000; }

struct TsState {
  int64_t t_beg = 0, t_last = 0;
  int tid_last = 0;
  std::vector<float> energy;
};

static void token_level_timestamps(const Model& m, TsState& st, Segment& seg, float thold_pt,
                                   float thold_ptsum) {
  auto& tokens = seg.tokens;
  const int n_samples = (int)st.energy.size();
  if (n_samples == 0) return;
  const int64_t t0 = seg.t0, t1 = seg.t1;
  const int n = (int)tokens.size();
  if (n == 0) return;
  if (n == 1) {
    tokens[0].t0 = t0;
    tokens[0].t1 = t1;
    return;
  }
  for (int j = 0; j < n; ++j) {
    auto& token = tokens[j];
    if (j == 0) {
      if (token.id == m.beg) {
        tokens[j].t0 = t0;
        tokens[j].t1 = t0;
        tokens[j + 1].t0 = t0;
        st.t_beg = t0;
        st.t_last = t0;
        st.tid_last = m.beg;
      } else {
        tokens[j].t0 = st.t_last;
      }
    }
    const int64_t tt = st.t_beg + 2 * (token.tid - m.beg);
    tokens[j].vlen = voice_length(m.id_to_token[token.id]);
    if (token.pt > thold_pt && token.ptsum > thold_ptsum && token.tid > st.tid_last && tt <= t1) {
      if (j > 0) tokens[j - 1].t1 = tt;
      tokens[j].t0 = tt;
      st.tid_last = token.tid;
    }
  }
  tokens[n - 2].t1 = t1;
  tokens[n - 1].t0 = t1;
  tokens[n - 1].t1 = t1;
  st.t_last = t1;
  {
    int p0 = 0, p1 = 0;
    while (true) {
      while (p1 < n && tokens[p1].t1 < 0) p1++;
      if (p1 >= n) p1--;
      if (p1 > p0) {
        double psum = 0.0;
        for (int j = p0; j <= p1; j++) psum += tokens[j].vlen;
        const double dt = tokens[p1].t1 - tokens[p0].t0;
        for (int j = p0 + 1; j <= p1; j++) {
          const double ct = tokens[j - 1].t0 + dt * tokens[j - 1].vlen / psum;
          tokens[j - 1].t1 = (int64_t)ct;
          tokens[j].t0 = (int64_t)ct;
        }
      }
      p1++;
      p0 = p1;
      if (p1 >= n) break;
    }
  }
  for (int j = 0; j < n - 1; j++) {
    if (tokens[j].t1 < 0) tokens[j + 1].t0 = tokens[j].t1;
    if (j > 0) {
      if (tokens[j - 1].t1 > tokens[j].t0) {
        tokens[j].t0 = tokens[j - 1].t1;
        tokens[j].t1 = std::max(tokens[j].t0, tokens[j].t1);
      }
    }
  }
  {
    const int hw = 16000 / 8;
    for (int j = 0; j < n; j++) {
      if (tokens[j].id >= m.eot) continue;
      int s0 = ts_to_sample(tokens[j].t0, n_samples);
      int s1 = ts_to_sample(tokens[j].t1, n_samples);
      const int ss0 = std::max(s0 - hw, 0);
      const int ss1 = std::min(s1 + hw, n_samples);
      const int ns = ss1 - ss0;
      float sum = 0.0f;
      for (int k = ss0; k < ss1; k++) sum += st.energy[k];
      const float thold = 0.5 * sum / ns;
      {
        int k = s0;
        if (st.energy[k] > thold && j > 0) {
          while (k > 0 && st.energy[k] > thold) k--;
          tokens[j].t0 = sample_to_ts(k);
          if (tokens[j].t0 < tokens[j - 1].t1) {
            tokens[j].t0 = tokens[j - 1].t1;
          } else {
            s0 = k;
          }
        } else {
          while (st.energy[k] < thold && k < s1) k++;
          s0 = k;
          tokens[j].t0 = sample_to_ts(k);
        }
      }
      {
        int k = s1;
        if (st.energy[k] > thold) {
          while (k < n_samples - 1 && st.energy[k] > thold) k++;
          tokens[j].t1 = sample_to_ts(k);
          // upstream tests `j < ns - 1` (ns = samples, not tokens) and so reads
          // tokens[j + 1] past the end for a trailing text token (UB); guarded
          if (j < ns - 1 && j + 1 < n && tokens[j].t1 > tokens[j + 1].t0) {
            tokens[j].t1 = tokens[j + 1].t0;
          } else {
            s1 = k;
          }
        } else {
          while (st.energy[k] < thold && k > s0) k--;
          s1 = k;
          tokens[j].t1 = sample_to_ts(k);
        }
      }
    }
  }
}

static std::vector<int> tokenize(const Model& m, const std::string& text) {
  std::vector<std::string> words;
  std::string str = text;
  static const std::regex re(
      R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
  std::smatch mt;
  while (std::regex_search(str, mt, re)) {
    for (auto x : mt) words.push_back(x);
    str = mt.suffix();
  }
  std::vector<int> out;
  for (const auto& w : words) {
    int i = 0, n = (int)w.size();
    while (i < n) {
      int j = n;
      bool found = false;
      while (j > i) {
        auto it = m.token_to_id.find(w.substr(i, j - i));
        if (it != m.token_to_id.end()) {
          out.push_back(it->second);
          i = j;
          found = true;
          break;
        }
        --j;
      }
      if (!found) ++i;
    }
  }
  return out;
}

static int lang_auto_detect(const Model& m, const Cross& cr) {
  KV kv;
  std::vector<float> logits;
  const int tok = m.sot;
  decode(m, cr, kv, &tok, 1, 0, logits);
  // g_lang is a std::map keyed by code: iterate codes in sorted order
  std::vector<std::pair<std::string, int>> langs;
  for (int i = 0; i < kNLang; ++i) langs.emplace_back(kLang[i], i);
  std::sort(langs.begin(), langs.end());
  std::vector<std::pair<float, int>> lid;
  for (const auto& kv2 : langs) lid.emplace_back(logits[m.sot + 1 + kv2.second], kv2.second);
  std::sort(lid.begin(), lid.end(), [](const std::pair<float, int>& a, const std::pair<float, int>& b) {
    return a.first > b.first;
  });
  return lid[0].second;
}

// External decoder (test replay): when set, full() takes the logits of every
// decode from these callbacks instead of its own encoder/decoder — used to run
// the token-loop logic (logits rules, sampling, beam search) on logits
// produced by the device, so that logic is compared exactly.
typedef void (*ExtEncodeFn)(void* user, int seek);
typedef void (*ExtLogitsFn)(void* user, const int* tokens, int n, float* logits_last);
static ExtEncodeFn g_ext_encode = nullptr;
static ExtLogitsFn g_ext_logits = nullptr;
static void* g_ext_user = nullptr;
// Logits tap (test hook): full() on its own logits hands every decoded row
// (the context it was decoded for, its last-position logits) to this callback,
// so a test measures the oracle-vs-device logits error on exactly the prefixes
// both runs decoded.
typedef void (*TapFn)(void* user, const int* tokens, int n, const float* logits_last);
static TapFn g_tap = nullptr;
static void* g_tap_user = nullptr;

static int full(const Model& m, Params P, const float* samples, int n_samples, Result& R) {
  R.segs.clear();
  const bool ext = g_ext_logits != nullptr;
  Mel mel;
  if (n_samples > 0 && !ext) log_mel(m, samples, n_samples, mel);
  if (ext && n_samples > 0) {  // only n_len_org is needed from the mel
    mel.n_len_org = 1 + (n_samples + 200 - 400) / 160;
  }
  std::vector<float> enc;
  Cross cr;
  int cached_seek = -1;
  auto encode_at = [&](int seek) {
    if (cached_seek == seek) return;
    if (ext) {
      g_ext_encode(g_ext_user, seek);
    } else {
      encode(m, mel, seek, enc);
      cross(m, enc, cr);
    }
    cached_seek = seek;
  };
  std::string language = P.language;
  if (language.empty() || language == "auto") {
    encode_at(0);
    R.lang_id = lang_auto_detect(m, cr);
    language = kLang[R.lang_id];
  }
  TsState ts;
  if (P.token_timestamps && n_samples > 0) ts.energy = signal_energy(samples, n_samples, 32);
  const int seek_start = P.offset_ms / 10;
  const int seek_end = P.duration_ms == 0 ? mel.n_len_org : seek_start + P.duration_ms / 10;
  const int delta_min = 10;
  if (seek_end < seek_start + delta_min) return 0;
  std::vector<float> temps;
  if (P.temperature_inc > 0.0f && P.bench_fixed_steps <= 0) {
    for (float t = P.temperature; t < 1.0f + 1e-6f; t += P.temperature_inc) temps.push_back(t);
  } else {
    temps.push_back(P.temperature);
  }
  int n_decoders = P.strategy == 0 ? P.best_of : std::max(P.best_of, P.beam_size);
  n_decoders = std::max(1, n_decoders);
  std::vector<Decoder> decs(n_decoders);
  for (int j = 1; j < n_decoders; ++j) decs[j].rng = std::mt19937(j);
  decs[0].rng = std::mt19937(0);
  std::vector<int> prompt_past;
  {
    std::vector<int> pt = P.prompt_tokens;
    if (pt.empty() && !P.initial_prompt.empty()) pt = tokenize(m, P.initial_prompt);
    if (!pt.empty()) {
      for (int t : pt) prompt_past.push_back(t);
      std::rotate(prompt_past.begin(), prompt_past.end() - pt.size(), prompt_past.end());
    }
  }
  std::vector<int> prompt_init = {m.sot};
  if (m.multilingual) {
    const int li = lang_id(language);
    R.lang_id = li;
    prompt_init.push_back(m.sot + 1 + li);
    prompt_init.push_back(P.translate ? m.translate : m.transcribe);
  }
  {
    const bool is_distil = m.n_text_layer == 2 && m.n_vocab != 51866;
    if (is_distil && !P.no_timestamps) P.no_timestamps = true;
  }
  if (P.no_timestamps) prompt_init.push_back(m.not_);
  int seek = seek_start;
  std::vector<int> prompt;
  std::vector<float> logits;
  while (true) {
    if (seek + delta_min >= seek_end) break;
    encode_at(seek);
    g_tctx.seek = seek;
    if (seek > seek_start && seek + 500 >= seek_end) prompt_past.clear();
    int best_id = 0;
    float no_speech_prob = 0.0f;
    for (int it = 0; it < (int)temps.size(); ++it) {
      const float t_cur = temps[it];
      g_tctx.it = it;
      g_tctx.step = -1;
      g_tctx.dec = 0;
      int n_cur = 1;
      if (P.strategy == 0) {
        if (t_cur > 0.0f) n_cur = P.best_of;
      } else {
        n_cur = t_cur > 0.0f ? P.best_of : P.beam_size;
      }
      n_cur = std::max(1, n_cur);
      for (int j = 0; j < n_cur; ++j) {
        auto& d = decs[j];
        d.seq = Sequence();
        d.seek_delta = 100 * 30;
        d.failed = d.completed = d.has_ts = false;
      }
      prompt.clear();
      if (!prompt_past.empty() && t_cur < 0.5f && P.n_max_text_ctx > 0) {
        const int n_take = std::min(std::min(P.n_max_text_ctx, m.n_text_ctx / 2), (int)prompt_past.size());
        prompt = {m.prev};
        prompt.insert(prompt.begin() + 1, prompt_past.end() - n_take, prompt_past.end());
      }
      prompt.insert(prompt.end(), prompt_init.begin(), prompt_init.end());
      decs[0].kv = KV();
      const float* last;
      if (ext) {
        logits.resize(m.n_vocab);
        g_ext_logits(g_ext_user, prompt.data(), (int)prompt.size(), logits.data());
        last = logits.data();
      } else {
        decode(m, cr, decs[0].kv, prompt.data(), (int)prompt.size(), 0, logits);
        last = logits.data() + (size_t)(prompt.size() - 1) * m.n_vocab;
        if (g_tap) g_tap(g_tap_user, prompt.data(), (int)prompt.size(), last);
      }
      {
        std::vector<float> l(last, last + m.n_vocab), lp(m.n_vocab), pr(m.n_vocab);
        compute_logprobs(l, m.n_vocab, lp);
        compute_probs(l, m.n_vocab, lp, pr);
        no_speech_prob = pr[m.nosp];
      }
      process_logits(m, P, decs[0], last, t_cur);
      for (int j = 1; j < n_cur; ++j) {
        decs[j].kv = decs[0].kv;
        decs[j].probs = decs[0].probs;
        decs[j].logits = decs[0].logits;
        decs[j].logprobs = decs[0].logprobs;
      }
      const int n_max = P.bench_fixed_steps > 0 ? P.bench_fixed_steps : m.n_text_ctx / 2 - 4;
      for (int i = 0; i < n_max; ++i) {
        g_tctx.step = i;
        if (P.strategy == 1) {
          // beam search: beam_size candidates per live decoder, sorted by
          // sum_logprobs_all (desc, then decoder index), assigned in order,
          // skipping candidates equal to the one just taken (from i > 0);
          // each decoder takes over its candidate's KV cache
          std::vector<BeamCand> cands;
          for (int j = 0; j < n_cur; ++j) {
            auto& d = decs[j];
            if (d.completed || d.failed) continue;
            g_tctx.dec = j;
            for (const auto& tok : sample_topk(m, d, P.beam_size)) {
              cands.push_back({j, d.seek_delta, d.has_ts, d.seq});
              cands.back().seq.tokens.push_back(tok);
              cands.back().seq.sum_logprobs_all += tok.plog;
            }
          }
          // upstream std::sort: candidates tied on both keys come out in an
          // unspecified order; the engine keeps their draw
          // order. Such a tie between DISTINCT sequences is traced
          // (TR_EXACT_TIE): where none occurs, the two orders agree.
          std::sort(cands.begin(), cands.end(), [](const BeamCand& a, const BeamCand& b) {
            if (a.seq.sum_logprobs_all != b.seq.sum_logprobs_all)
              return a.seq.sum_logprobs_all > b.seq.sum_logprobs_all;
            return a.decoder_idx < b.decoder_idx;
          });
          if (g_trace_on) {
            for (size_t c = 1; c < cands.size(); ++c)
              if (cands[c].seq.sum_logprobs_all == cands[c - 1].seq.sum_logprobs_all &&
                  cands[c].decoder_idx == cands[c - 1].decoder_idx &&
                  !tokens_equal(cands[c].seq, cands[c - 1].seq)) {
                if (follow(TR_EXACT_TIE)) {
                  trace(TR_EXACT_TIE, cands[c].decoder_idx, cands[c].seq.tokens.back().id, 0.0);
                  follow_structural(cands[c].decoder_idx, cands[c].seq.tokens.back().id);
                } else {
                  trace(TR_EXACT_TIE, cands[c].decoder_idx, cands[c].seq.tokens.back().id, 0.0);
                }
              }
          }
          // distance in sum_logprobs_all from candidate c to the nearest
          // candidate before / after it that is a different sequence
          auto assign_margin = [&](size_t c) {
            double g = INFINITY;
            for (size_t e = c; e-- > 0;)
              if (!tokens_equal(cands[e].seq, cands[c].seq)) {
                g = std::min(g, cands[e].seq.sum_logprobs_all - cands[c].seq.sum_logprobs_all);
                break;
              }
            for (size_t e = c + 1; e < cands.size(); ++e)
              if (!tokens_equal(cands[e].seq, cands[c].seq)) {
                g = std::min(g, cands[c].seq.sum_logprobs_all - cands[e].seq.sum_logprobs_all);
                break;
              }
            return g;
          };
          size_t cur_c = 0;
          std::vector<int> src(n_cur, -1);
          for (int j = 0; j < n_cur; ++j) {
            auto& d = decs[j];
            if (d.completed || d.failed) continue;
            if (cur_c >= cands.size()) cur_c = 0;
            const size_t cur_pos = cur_c;
            g_tctx.dec = j;
            const double own_margin = assign_margin(cur_pos);
            const TraceEv* g = follow(TR_ASSIGN);
            if (g && (g->a != cands[cur_pos].decoder_idx || g->b != cands[cur_pos].seq.tokens.back().id)) {
              // the guide took another candidate here: the first one after this
              // position with its (source decoder, last token) moves up to it
              // (the device ranked it higher: a reorder within the logits noise)
              size_t f = cur_pos + 1;
              while (f < cands.size() &&
                     !(cands[f].decoder_idx == g->a && cands[f].seq.tokens.back().id == g->b))
                ++f;
              if (f < cands.size()) {
                const int oa = cands[cur_pos].decoder_idx, ob = cands[cur_pos].seq.tokens.back().id;
                const double gap = cands[cur_pos].seq.sum_logprobs_all - cands[f].seq.sum_logprobs_all;
                std::rotate(cands.begin() + cur_pos, cands.begin() + f, cands.begin() + f + 1);
                mark_forced(trace(TR_ASSIGN, g->a, g->b, own_margin, cands[cur_pos].seq.sum_logprobs_all),
                            oa, ob, gap);
              } else {  // not among this step's candidates: a structural difference
                trace(TR_ASSIGN, cands[cur_pos].decoder_idx, cands[cur_pos].seq.tokens.back().id,
                      own_margin, cands[cur_pos].seq.sum_logprobs_all);
                g_follow_on = false;
                g_follow_break = (long)g_trace.size() - 1;
              }
            } else {
              trace(TR_ASSIGN, cands[cur_pos].decoder_idx, cands[cur_pos].seq.tokens.back().id,
                    own_margin, cands[cur_pos].seq.sum_logprobs_all);
            }
            const BeamCand& cur = cands[cur_c++];
            while (cands.size() > cur_c && tokens_equal(cands[cur_c].seq, cur.seq) && i > 0) ++cur_c;
            d.seek_delta = cur.seek_delta;
            d.has_ts = cur.has_ts;
            d.seq = cur.seq;
            src[j] = cur.decoder_idx;
          }
          std::vector<KV> kv_new(n_cur);
          for (int j = 0; j < n_cur; ++j)
            if (src[j] >= 0 && src[j] != j) kv_new[j] = decs[src[j]].kv;
          for (int j = 0; j < n_cur; ++j)
            if (src[j] >= 0 && src[j] != j) decs[j].kv = std::move(kv_new[j]);
        } else {
          for (int j = 0; j < n_cur; ++j) {
            auto& d = decs[j];
            if (d.completed || d.failed) continue;
            g_tctx.dec = j;
            d.seq.tokens.push_back(sample_token(m, d, t_cur < 1e-6f));
            d.seq.sum_logprobs_all += d.seq.tokens.back().plog;
          }
        }
        for (int j = 0; j < n_cur; ++j) {
          auto& d = decs[j];
          if (d.completed || d.failed) continue;
          const auto& tok = d.seq.tokens.back();
          if (tok.id > m.beg) {
            const int sd_new = 2 * (tok.id - m.beg);
            if (d.has_ts && d.seek_delta > sd_new && d.seq.result_len < i) {
              d.failed = true;
              continue;
            }
            d.seek_delta = sd_new;
            d.seq.result_len = i + 1;
            d.has_ts = true;
          }
          if (tok.id == m.eot || (P.max_tokens > 0 && i >= P.max_tokens) ||
              (d.has_ts && seek + d.seek_delta + delta_min >= seek_end)) {
            if (d.seq.result_len == 0 && !P.no_timestamps) {
              if (seek + d.seek_delta + delta_min >= seek_end) {
                d.seq.result_len = i + 1;
              } else {
                d.failed = true;
                continue;
              }
            }
            if (P.single_segment || P.no_timestamps) {
              d.seq.result_len = i + 1;
              d.seek_delta = 100 * 30;
            }
            d.completed = true;
            continue;
          }
          if (i == n_max - 1 && (d.seq.result_len == 0 || d.seek_delta < 100 * 30 / 2)) {
            d.failed = true;
            continue;
          }
        }
        bool all = true;
        for (int j = 0; j < n_cur; ++j) {
          if (!(decs[j].completed || decs[j].failed)) all = false;
          g_tctx.dec = j;
          const int st = decs[j].completed + 2 * decs[j].failed;
          const bool fl = follow(TR_STATUS) != nullptr;
          trace(TR_STATUS, st, decs[j].seq.result_len, INFINITY);
          if (fl) follow_structural(st, decs[j].seq.result_len);
        }
        if (all) break;
        const int n_past = (int)prompt.size() + i;
        for (int j = 0; j < n_cur; ++j) {
          auto& d = decs[j];
          if (d.failed || d.completed) continue;
          g_tctx.dec = j;
          const int tok = d.seq.tokens.back().id;
          if (ext) {
            std::vector<int> ctxt(prompt);
            for (const auto& t : d.seq.tokens) ctxt.push_back(t.id);
            logits.resize(m.n_vocab);
            g_ext_logits(g_ext_user, ctxt.data(), (int)ctxt.size(), logits.data());
          } else {
            decode(m, cr, d.kv, &tok, 1, n_past, logits);
            if (g_tap) {
              std::vector<int> ctxt(prompt);
              for (const auto& t : d.seq.tokens) ctxt.push_back(t.id);
              g_tap(g_tap_user, ctxt.data(), (int)ctxt.size(), logits.data());
            }
          }
          process_logits(m, P, d, logits.data(), t_cur);
        }
      }
      double best_score = -INFINITY;
      for (int j = 0; j < n_cur; ++j) {
        auto& d = decs[j];
        if (d.failed) continue;
        d.seq.tokens.resize(d.seq.result_len);
        sequence_score(P, d.seq);
        if (d.seq.result_len > 32 && d.seq.entropy < P.entropy_thold) {
          d.failed = true;
          continue;
        }
        if (best_score < d.seq.score) {
          best_score = d.seq.score;
          best_id = j;
        }
      }
      g_tctx.step = n_max;
      g_tctx.dec = best_id;
      if (g_trace_on) {
        double runner = -INFINITY;
        for (int j = 0; j < n_cur; ++j)
          if (!decs[j].failed && j != best_id && !tokens_equal(decs[j].seq, decs[best_id].seq))
            runner = std::max(runner, decs[j].seq.score);
        const TraceEv* g = follow(TR_BEST);
        if (g && g->a != best_id && g->a >= 0 && g->a < n_cur && !decs[g->a].failed) {
          const int own = best_id;
          best_id = g->a;
          mark_forced(trace(TR_BEST, best_id, decs[best_id].seq.result_len, best_score - runner,
                            decs[best_id].seq.score),
                      own, decs[own].seq.result_len, best_score - decs[best_id].seq.score);
        } else {
          trace(TR_BEST, best_id, decs[best_id].seq.result_len, best_score - runner, best_score);
          if (g && g->a != best_id) {  // the guide's best decoder failed here
            g_follow_on = false;
            g_follow_break = (long)g_trace.size() - 1;
          }
        }
      }
      bool success = true;
      if (it != (int)temps.size() - 1) {
        const auto& d = decs[best_id];
        if (d.failed || (d.seq.avg_logprobs < P.logprob_thold && no_speech_prob < P.no_speech_thold))
          success = false;
        if (g_trace_on) {
          const double ga = (double)P.logprob_thold - d.seq.avg_logprobs;  // > 0: below
          const double gn = (double)P.no_speech_thold - no_speech_prob;
          const double mg = d.failed ? INFINITY
                                     : (success ? std::max(ga > 0 ? 0.0 : -ga, gn > 0 ? 0.0 : -gn)
                                                : std::min(ga, gn));
          const TraceEv* g = follow(TR_FALLBACK);
          if (g && g->a != (int)success && !d.failed) {
            mark_forced(trace(TR_FALLBACK, g->a, d.failed, mg), success, d.failed, mg);
            success = g->a != 0;
          } else {
            trace(TR_FALLBACK, success, d.failed, mg);
            if (g && g->a != (int)success) {
              g_follow_on = false;
              g_follow_break = (long)g_trace.size() - 1;
            }
          }
        }
      }
      if (success) break;
    }
    {
      const auto& best = decs[best_id];
      auto seek_delta = best.seek_delta;
      const auto result_len = best.seq.result_len;
      const auto& toks = best.seq.tokens;
      {
        std::vector<int> ids;
        for (const auto& t : toks) ids.push_back(t.id);
        R.window_tokens.push_back(ids);
      }
      bool is_no_speech = no_speech_prob > P.no_speech_thold && best.seq.avg_logprobs < P.logprob_thold;
      if (g_trace_on) {
        const double gn = (double)no_speech_prob - P.no_speech_thold;  // > 0: above
        const double ga = (double)P.logprob_thold - best.seq.avg_logprobs;
        const double mg =
            is_no_speech ? std::min(gn, ga) : std::max(gn > 0 ? 0.0 : -gn, ga > 0 ? 0.0 : -ga);
        const TraceEv* g = follow(TR_NOSPEECH);
        if (g && g->a != (int)is_no_speech) {
          mark_forced(trace(TR_NOSPEECH, g->a, 0, mg), is_no_speech, 0, mg);
          is_no_speech = g->a != 0;
        } else {
          trace(TR_NOSPEECH, is_no_speech, 0, mg);
        }
      }
      prompt_past.clear();
      if (prompt.front() == m.prev)
        prompt_past.insert(prompt_past.end(), prompt.begin() + 1, prompt.end() - prompt_init.size());
      for (int i = 0; i < result_len && !is_no_speech; ++i) prompt_past.push_back(toks[i].id);
      if (!toks.empty() && !is_no_speech) {
        int i0 = 0;
        auto t0 = seek + 2 * (toks.front().tid - m.beg);
        std::string text;
        bool stn = false;
        for (int i = 0; i < (int)toks.size(); i++) {
          if (P.print_special || toks[i].id < m.eot) text += m.id_to_token[toks[i].id];
          if (P.tdrz_enable && toks[i].id == m.solm) stn = true;
          if (toks[i].id > m.beg && !P.single_segment) {
            const auto t1 = seek + 2 * (toks[i].tid - m.beg);
            if (!text.empty()) {
              Segment s{t0, t1, text, no_speech_prob, {}, stn};
              for (int j = i0; j <= i; j++) s.tokens.push_back(toks[j]);
              R.segs.push_back(s);
              if (P.token_timestamps)
                token_level_timestamps(m, ts, R.segs.back(), P.thold_pt, P.thold_ptsum);
            }
            text = "";
            while (i < (int)toks.size() && toks[i].id > m.beg) i++;
            i--;
            t0 = t1;
            i0 = i + 1;
            stn = false;
          }
        }
        if (!text.empty()) {
          const auto t1 = seek + seek_delta;
          Segment s{t0, t1, text, no_speech_prob, {}, stn};
          for (int j = i0; j < (int)toks.size(); j++) s.tokens.push_back(toks[j]);
          R.segs.push_back(s);
          if (P.token_timestamps) token_level_timestamps(m, ts, R.segs.back(), P.thold_pt, P.thold_ptsum);
        }
      }
      // benchmark workload (bench_fixed_steps): every window decodes the fixed
      // step count and the clip advances by a whole window (long-form clips
      // run window after window)
      seek += P.bench_fixed_steps > 0 ? 100 * 30 : seek_delta;
    }
  }
  return 0;
}

}  // namespace orc

// ============================================================================
// C ABI (ctypes) — test infrastructure only
// ============================================================================
using namespace orc;

struct OrcFull {
  Result r;
};

extern "C" {

void* orc_load(const char* path, int flags) {
  auto* m = new Model();
  m->flags = flags;
  {
    struct stat st;
    if (stat(path, &st) == 0)
      m->key = std::string(path) + "|" + std::to_string((long long)st.st_size) + "|" +
               std::to_string((long long)st.st_mtim.tv_sec) + "." +
               std::to_string((long long)st.st_mtim.tv_nsec) + "|" + std::to_string(flags);
  }
  if (!load(path, *m)) {
    delete m;
    return nullptr;
  }
  if (flags & ORC_MXFP8) {
    // the engine quantizes these (16-bit) weights to MX-fp8 at load: the
    // encoder projections, the cross K/V projections, and (bf16 models) every
    // decoder projection plus the tied token embedding (decoder GEMMs on fp8
    // weights dequantized in registers; the embedding rows are gathered from
    // the same rounded values)
    const bool dec_w = m->wtype == 30;  // GGML_BF16
    for (auto& kv : m->t) {
      const std::string& n = kv.first;
      const bool wt = n.size() > 7 && n.compare(n.size() - 7, 7, ".weight") == 0;
      const bool enc = n.rfind("encoder.blocks.", 0) == 0 &&
                       (n.find(".attn.") != std::string::npos || n.find(".mlp.") != std::string::npos) &&
                       wt;
      const bool cross = n.find(".cross_attn.key.weight") != std::string::npos ||
                         n.find(".cross_attn.value.weight") != std::string::npos;
      const bool dec = dec_w && wt && n.rfind("decoder.blocks.", 0) == 0 &&
                       (n.find(".attn.") != std::string::npos ||
                        n.find(".cross_attn.query.") != std::string::npos ||
                        n.find(".cross_attn.out.") != std::string::npos ||
                        n.find(".mlp.") != std::string::npos);
      const bool emb = dec_w && n == "decoder.token_embedding.weight";
      if (!enc && !cross && !dec && !emb) continue;
      Tensor& t = kv.second;
      const int K = (int)t.ne[0];
      if (K % 32) {
        delete m;
        return nullptr;
      }
      mx_round_rows(t.v.data(), t.v.size() / K, K);
    }
  }
  return m;
}
void orc_free(void* h) { delete (Model*)h; }
void orc_set_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n);
#else
  (void)n;
#endif
}
void orc_set_enc_layer_limit(int n) { g_enc_layer_limit = n; }
// decision trace (TraceKind above): on = 1 clears and starts recording
void orc_trace_enable(int on) {
  g_trace_on = on != 0;
  if (on) g_trace.clear();
}
int orc_trace_count() { return (int)g_trace.size(); }
// where full() stands (for an external-logits callback): {seek, it, step, dec}
void orc_trace_ctx(int* out) {
  out[0] = g_tctx.seek;
  out[1] = g_tctx.it;
  out[2] = g_tctx.step;
  out[3] = g_tctx.dec;
}
// ints[10] = {kind, seek, it, step, dec, a, b, forced, own_a, own_b};
// dbls[5] = {margin, v, fmargin, lo, hi}
void orc_trace_get(int i, int* ints, double* dbls) {
  const TraceEv& e = g_trace.at(i);
  int v[10] = {e.kind, e.seek, e.it, e.step, e.dec, e.a, e.b, e.forced, e.own_a, e.own_b};
  for (int k = 0; k < 10; ++k) ints[k] = v[k];
  double d[5] = {e.margin, e.v, e.fmargin, e.lo, e.hi};
  for (int k = 0; k < 5; ++k) dbls[k] = d[k];
}
// follow mode: the guide trace, 7 ints per event {kind, seek, it, step, dec,
// a, b}; n = 0 turns following off. Takes effect for the next traced run.
void orc_trace_follow(const int* ints, int n) {
  g_follow.clear();
  for (int i = 0; i < n; ++i) {
    const int* e = ints + 7 * i;
    TraceEv ev{e[0], e[1], e[2], e[3], e[4], e[5], e[6], 0.0, 0.0};
    g_follow.push_back(ev);
  }
  g_follow_on = n > 0;
  g_follow_break = -1;
}
// index of the event where following ended (-1: followed to the end)
long orc_trace_follow_break() { return g_follow_break; }
void orc_set_logits_tap(TapFn fn, void* user) {
  g_tap = fn;
  g_tap_user = user;
}
void orc_set_external(ExtEncodeFn enc, ExtLogitsFn lg, void* user) {
  g_ext_encode = enc;
  g_ext_logits = lg;
  g_ext_user = user;
}
void orc_hparams(void* h, int* out) {
  auto* m = (Model*)h;
  for (int i = 0; i < 11; ++i) out[i] = m->hp[i];
}
int orc_wtype(void* h) { return ((Model*)h)->wtype; }
// copies the (loaded, dequantized) values of tensor `name`; returns its size
long orc_tensor(void* h, const char* name, float* out, long cap) {
  const Model* m = (const Model*)h;
  auto it = m->t.find(name);
  if (it == m->t.end()) return -1;
  const long n = (long)it->second.v.size();
  if (out) memcpy(out, it->second.v.data(), sizeof(float) * std::min(n, cap));
  return n;
}
void orc_special(void* h, int* out) {
  auto* m = (Model*)h;
  int v[9] = {m->eot, m->sot, m->translate, m->transcribe, m->solm, m->prev, m->nosp, m->not_, m->beg};
  for (int i = 0; i < 9; ++i) out[i] = v[i];
}
const char* orc_token_str(void* h, int id) { return ((Model*)h)->id_to_token.at(id).c_str(); }
const float* orc_filters(void* h) { return ((Model*)h)->filters.data(); }

// mel: returns n_len; out (may be null) receives [n_mels][n_len]
int orc_mel(void* h, const float* pcm, int n, float* out, int out_cap, int* n_len_org) {
  Mel mel;
  log_mel(*(Model*)h, pcm, n, mel);
  if (n_len_org) *n_len_org = mel.n_len_org;
  if (out && (int64_t)out_cap >= (int64_t)mel.data.size())
    memcpy(out, mel.data.data(), mel.data.size() * 4);
  return mel.n_len;
}

// encoder on a mel [n_mels][n_len]; out = [n_audio_ctx][n_audio_state]
// test hooks of the encoder's parts (tests/test_gpu_c5.py per-layer check):
// the conv stem's residual stream for the window at `seek`, and one layer on
// a given residual stream x_in [n_ctx][D] -> x_out, with optional external /
// returned GEMM A operands (EncLayerIO: attn LN out, attention out, mlp LN
// out [n_ctx][D]; GELU out [n_ctx][4D])
void orc_encode_stem(void* h, const float* mel_data, int n_len, int seek, float* x_out) {
  const Model& m = *(const Model*)h;
  const int T = 2 * m.n_audio_ctx;
  std::vector<float> x((size_t)m.n_mels * T, 0.0f);
  const int i0 = std::min(seek, n_len), i1 = std::min(seek + T, n_len);
  for (int j = 0; j < m.n_mels; ++j)
    for (int i = i0; i < i1; ++i) x[(size_t)j * T + (i - i0)] = mel_data[(size_t)j * n_len + i];
  std::vector<float> inp;
  encode_stem(m, x, inp);
  std::copy(inp.begin(), inp.end(), x_out);
}
void orc_encode_post(void* h, const float* x, float* out) {
  const Model& m = *(const Model*)h;
  layer_norm(x, m.w("encoder.ln_post.weight"), m.w("encoder.ln_post.bias"), m.n_audio_ctx,
             m.n_audio_state, out);
}
void orc_encode_layer(void* h, int il, const float* x_in, const float* const* ext, float* const* outs,
                      float* x_out) {
  const Model& m = *(const Model*)h;
  std::vector<float> inp(x_in, x_in + (size_t)m.n_audio_ctx * m.n_audio_state);
  EncLayerIO io{};
  for (int g = 0; g < 4; ++g) {
    io.ext[g] = ext ? ext[g] : nullptr;
    io.out[g] = outs ? outs[g] : nullptr;
  }
  encode_layer(m, il, inp, &io);
  std::copy(inp.begin(), inp.end(), x_out);
}
void orc_encode(void* h, const float* mel_data, int n_len, int seek, float* out) {
  auto* m = (Model*)h;
  Mel mel;
  mel.n_mel = m->n_mels;
  mel.n_len = n_len;
  mel.data.assign(mel_data, mel_data + (size_t)m->n_mels * n_len);
  std::vector<float> enc;
  encode(*m, mel, seek, enc);
  memcpy(out, enc.data(), enc.size() * 4);
}

// cross K/V for all decoder layers: k_out/v_out = [n_text_layer][n_audio_ctx][D]
void orc_cross(void* h, const float* enc, float* k_out, float* v_out) {
  auto* m = (Model*)h;
  std::vector<float> e(enc, enc + (size_t)m->n_audio_ctx * m->n_audio_state);
  Cross c;
  cross(*m, e, c);
  memcpy(k_out, c.k.data(), c.k.size() * 4);
  memcpy(v_out, c.v.data(), c.v.size() * 4);
}

// teacher-forced decode of tokens (one at a time, positions 0..n-1) given
// cross K/V; logits_out = [n][n_vocab]
void orc_decode_seq(void* h, const float* k_cross, const float* v_cross, const int* tokens,
                    int n, float* logits_out) {
  auto* m = (Model*)h;
  Cross c;
  const size_t sz = (size_t)m->n_text_layer * m->n_audio_ctx * m->n_text_state;
  c.k.assign(k_cross, k_cross + sz);
  c.v.assign(v_cross, v_cross + sz);
  cross_heads(*m, c);
  KV kv;
  std::vector<float> lg;
  for (int i = 0; i < n; ++i) {
    decode(*m, c, kv, tokens + i, 1, i, lg);
    memcpy(logits_out + (size_t)i * m->n_vocab, lg.data(), (size_t)m->n_vocab * 4);
  }
}

// full pipeline. iparams: [strategy, best_of, beam_size, translate, no_timestamps,
//   token_timestamps, suppress_nst, suppress_blank, tdrz, bench_fixed_steps, no_context]
// fparams: [temperature, temperature_inc, entropy_thold, logprob_thold,
//   no_speech_thold, max_initial_ts, length_penalty, thold_pt, thold_ptsum]
void* orc_full(void* h, const int* ip, const float* fp, const char* language,
               const char* initial_prompt, const float* pcm, int n, int* rc) {
  auto* m = (Model*)h;
  Params P;
  P.strategy = ip[0];
  P.best_of = ip[1];
  P.beam_size = ip[2];
  P.translate = ip[3];
  P.no_timestamps = ip[4];
  P.token_timestamps = ip[5];
  P.suppress_nst = ip[6];
  P.suppress_blank = ip[7];
  P.tdrz_enable = ip[8];
  P.bench_fixed_steps = ip[9];
  P.no_context = ip[10];
  P.temperature = fp[0];
  P.temperature_inc = fp[1];
  P.entropy_thold = fp[2];
  P.logprob_thold = fp[3];
  P.no_speech_thold = fp[4];
  P.max_initial_ts = fp[5];
  P.length_penalty = fp[6];
  P.thold_pt = fp[7];
  P.thold_ptsum = fp[8];
  P.language = language ? language : "en";
  if (initial_prompt) P.initial_prompt = initial_prompt;
  auto* r = new OrcFull();
  *rc = full(*m, P, pcm, n, r->r);
  return r;
}
void orc_full_free(void* r) { delete (OrcFull*)r; }
int orc_full_n_segments(void* r) { return (int)((OrcFull*)r)->r.segs.size(); }
const char* orc_full_segment_text(void* r, int i) { return ((OrcFull*)r)->r.segs[i].text.c_str(); }
void orc_full_segment_times(void* r, int i, int64_t* t) {
  t[0] = ((OrcFull*)r)->r.segs[i].t0;
  t[1] = ((OrcFull*)r)->r.segs[i].t1;
}
int orc_full_n_tokens(void* r, int i) { return (int)((OrcFull*)r)->r.segs[i].tokens.size(); }
// token: ids[2] = {id, tid}; f[4] = {p, plog, pt, ptsum}; t[2] = {t0, t1}
void orc_full_token(void* r, int i, int j, int* ids, float* f, int64_t* t) {
  const auto& tk = ((OrcFull*)r)->r.segs[i].tokens[j];
  ids[0] = tk.id;
  ids[1] = tk.tid;
  f[0] = tk.p;
  f[1] = tk.plog;
  f[2] = tk.pt;
  f[3] = tk.ptsum;
  t[0] = tk.t0;
  t[1] = tk.t1;
}
// whisper_process_logits + whisper_sample_token(best = true) on ONE raw logits
// row for a decoder whose sampled tokens so far are hist[0..n_hist) (the
// token-loop rules pinned against HF's Whisper logits processors,
// tests/test_oracle_golden.py). has_ts / seek_delta are the decoder state the
// loop derives from hist (full() above). ip: [suppress_blank, suppress_nst,
// no_timestamps, tdrz, bench_fixed_steps, skip_ts_mass]; skip_ts_mass = 1
// returns the logits before the "sum p(timestamps) > max p(text)" rule (a
// test hook: that rule is the last step of process_logits). fp: [temperature,
// max_initial_ts]. out_logits / out_logprobs / out_probs: [n_vocab];
// tok_i = {id, tid}, tok_f = {p, plog, pt, ptsum}.
void orc_process_logits(void* h, const float* raw, const int* hist, int n_hist, int has_ts,
                        int seek_delta, const int* ip, const float* fp, float* out_logits,
                        float* out_logprobs, float* out_probs, int* tok_i, float* tok_f) {
  const Model& m = *(const Model*)h;
  Params P;
  P.suppress_blank = ip[0];
  P.suppress_nst = ip[1];
  P.no_timestamps = ip[2];
  P.tdrz_enable = ip[3];
  P.bench_fixed_steps = ip[4];
  P.max_initial_ts = fp[1];
  Decoder d;
  for (int i = 0; i < n_hist; ++i) {
    TokenData t;
    t.id = hist[i];
    d.seq.tokens.push_back(t);
  }
  d.has_ts = has_ts != 0;
  d.seek_delta = seek_delta;
  const int n = m.n_vocab;
  process_logits(m, P, d, raw, fp[0], ip[5] == 0);
  memcpy(out_logits, d.logits.data(), (size_t)n * 4);
  memcpy(out_logprobs, d.logprobs.data(), (size_t)n * 4);
  memcpy(out_probs, d.probs.data(), (size_t)n * 4);
  const TokenData t = sample_token(m, d, true);
  tok_i[0] = t.id;
  tok_i[1] = t.tid;
  tok_f[0] = t.p;
  tok_f[1] = t.plog;
  tok_f[2] = t.pt;
  tok_f[3] = t.ptsum;
}
int orc_full_lang_id(void* r) { return ((OrcFull*)r)->r.lang_id; }
int orc_full_n_windows(void* r) { return (int)((OrcFull*)r)->r.window_tokens.size(); }
int orc_full_window_tokens(void* r, int w, int* out, int cap) {
  const auto& v = ((OrcFull*)r)->r.window_tokens[w];
  for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
  return (int)v.size();
}

}  // extern "C"
