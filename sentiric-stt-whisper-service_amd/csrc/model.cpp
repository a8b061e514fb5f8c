// ggml .bin model file reader, synthetic model writer, vocabulary, language
// table, tokenizer and logging for the mwx engine.
//
// The file layout is the one whisper.cpp's whisper_model_load reads and the
// upstream converter (models/convert-pt-to-ggml.py) writes; the service
// provisions such files through ModelManager (src/model_manager.cpp:15-31,
// default ggml-medium.bin per src/config.h:18,112-114).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <fstream>
#include <functional>
#include <regex>

#include "common.h"
#include "mwx_test.h"

namespace mwx {

// ---------------------------------------------------------------------------
// logging
// ---------------------------------------------------------------------------
static mwx_log_callback g_log_cb = nullptr;
static void* g_log_user = nullptr;

void log_msg(mwx_log_level level, const char* fmt, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (g_log_cb) {
    g_log_cb(level, buf, g_log_user);
  } else if (level >= MWX_LOG_LEVEL_WARN) {
    fputs(buf, stderr);
  }
}

// ---------------------------------------------------------------------------
// 16-bit float conversions (round to nearest even, as F16C / v_cvt_f16_f32)
// ---------------------------------------------------------------------------
uint16_t f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t exp = (x >> 23) & 0xffu;
  uint32_t mant = x & 0x7fffffu;
  if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
  const int32_t e = (int32_t)exp - 127 + 15;
  if (e >= 31) return (uint16_t)(sign | 0x7c00u);
  if (e <= 0) {
    if (e < -10) return (uint16_t)sign;
    mant |= 0x800000u;
    const uint32_t shift = (uint32_t)(14 - e);
    uint32_t hm = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1u);
    const uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
    return (uint16_t)(sign | hm);
  }
  uint32_t h = sign | ((uint32_t)e << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)h;
}

float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t mant = h & 0x3ffu;
  uint32_t x;
  if (exp == 0) {
    if (mant == 0) {
      x = sign;
    } else {
      int e = -1;
      do {
        e++;
        mant <<= 1;
      } while (!(mant & 0x400u));
      x = sign | ((uint32_t)(127 - 15 - e) << 23) | ((mant & 0x3ffu) << 13);
    }
  } else if (exp == 31) {
    x = sign | 0x7f800000u | (mant << 13);
  } else {
    x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}

uint16_t f32_to_bf16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40u);
  x += 0x7fffu + ((x >> 16) & 1u);
  return (uint16_t)(x >> 16);
}

float bf16_to_f32(uint16_t h) {
  uint32_t x = (uint32_t)h << 16;
  float f;
  memcpy(&f, &x, 4);
  return f;
}

// ---------------------------------------------------------------------------
// language table (code, id) — the g_lang map of whisper.cpp
// ---------------------------------------------------------------------------
static const char* kLangCodes[] = {
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca",
    "nl", "ar", "sv", "it", "id", "hi", "fi", "vi", "he", "uk", "el", "ms",
    "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg", "lt", "la",
    "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn",
    "et", "mk", "br", "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw",
    "gl", "mr", "pa", "si", "km", "sn", "yo", "so", "af", "oc", "ka", "be",
    "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn",
    "mt", "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha",
    "ba", "jw", "su", "yue"};
static const int kNumLang = (int)(sizeof(kLangCodes) / sizeof(kLangCodes[0]));

int lang_id(const std::string& code) {
  for (int i = 0; i < kNumLang; ++i)
    if (code == kLangCodes[i]) return i;
  return -1;
}
const char* lang_str(int id) {
  if (id < 0 || id >= kNumLang) return nullptr;
  return kLangCodes[id];
}
int lang_max_id() { return kNumLang - 1; }

const std::vector<std::pair<std::string, int>>& lang_table_sorted() {
  static std::vector<std::pair<std::string, int>> t = [] {
    std::vector<std::pair<std::string, int>> v;
    for (int i = 0; i < kNumLang; ++i) v.emplace_back(kLangCodes[i], i);
    std::sort(v.begin(), v.end());
    return v;
  }();
  return t;
}

// ---------------------------------------------------------------------------
// tokenizer (whisper_tokenize: regex split + greedy longest match)
// ---------------------------------------------------------------------------
std::vector<int32_t> tokenize(const Vocab& vocab, const std::string& text) {
  std::vector<std::string> words;
  {
    std::string str = text;
    static const std::regex re(
        R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
    std::smatch m;
    while (std::regex_search(str, m, re)) {
      for (auto x : m) words.push_back(x);
      str = m.suffix();
    }
  }
  std::vector<int32_t> tokens;
  for (const auto& word : words) {
    if (word.empty()) continue;
    int i = 0;
    const int n = (int)word.size();
    while (i < n) {
      int j = n;
      bool found = false;
      while (j > i) {
        auto it = vocab.token_to_id.find(word.substr(i, j - i));
        if (it != vocab.token_to_id.end()) {
          tokens.push_back(it->second);
          i = j;
          found = true;
          break;
        }
        --j;
      }
      if (!found) {
        MWX_LOG_ERROR("mwx_tokenize: unknown token\n");
        ++i;
      }
    }
  }
  return tokens;
}

// ---------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------
template <typename T>
static bool rd(std::ifstream& f, T& v) {
  f.read(reinterpret_cast<char*>(&v), sizeof(T));
  return (bool)f;
}

static void finalize_vocab(Vocab& vocab, int32_t n_vocab_file) {
  if (vocab.is_multilingual()) {
    vocab.token_eot++;
    vocab.token_sot++;
    const int dt = vocab.num_languages() - 98;
    vocab.token_translate += dt;
    vocab.token_transcribe += dt;
    vocab.token_solm += dt;
    vocab.token_prev += dt;
    vocab.token_nosp += dt;
    vocab.token_not += dt;
    vocab.token_beg += dt;
  }
  for (int i = n_vocab_file; i < vocab.n_vocab; i++) {
    std::string word;
    if (i > vocab.token_beg) {
      word = "[_TT_" + std::to_string(i - vocab.token_beg) + "]";
    } else if (i == vocab.token_eot) {
      word = "[_EOT_]";
    } else if (i == vocab.token_sot) {
      word = "[_SOT_]";
    } else if (i == vocab.token_translate) {
      word = "[_TRANSLATE_]";
    } else if (i == vocab.token_transcribe) {
      word = "[_TRANSCRIBE_]";
    } else if (i == vocab.token_solm) {
      word = "[_SOLM_]";
    } else if (i == vocab.token_prev) {
      word = "[_PREV_]";
    } else if (i == vocab.token_nosp) {
      word = "[_NOSP_]";
    } else if (i == vocab.token_not) {
      word = "[_NOT_]";
    } else if (i == vocab.token_beg) {
      word = "[_BEG_]";
    } else if (i > vocab.token_sot &&
               i <= vocab.token_sot + vocab.num_languages()) {
      const char* ls = lang_str(i - vocab.token_sot - 1);
      word = std::string("[_LANG_") + (ls ? ls : "") + "]";
    } else {
      word = "[_extra_token_" + std::to_string(i) + "]";
    }
    vocab.token_to_id[word] = i;
    vocab.id_to_token[i] = word;
  }
}

bool read_model_file(const char* path, ModelFile& mf) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    MWX_LOG_ERROR("mwx: failed to open '%s'\n", path);
    return false;
  }
  uint32_t magic = 0;
  if (!rd(f, magic) || magic != 0x67676d6cu) {
    MWX_LOG_ERROR("mwx: invalid model file '%s' (bad magic)\n", path);
    return false;
  }
  Hparams& hp = mf.hp;
  int32_t* hpf[] = {&hp.n_vocab,      &hp.n_audio_ctx,  &hp.n_audio_state,
                    &hp.n_audio_head, &hp.n_audio_layer, &hp.n_text_ctx,
                    &hp.n_text_state, &hp.n_text_head,  &hp.n_text_layer,
                    &hp.n_mels,       &hp.ftype};
  for (auto* p : hpf)
    if (!rd(f, *p)) return false;
  hp.ftype %= 1000;  // GGML_QNT_VERSION_FACTOR

  if (!rd(f, mf.filt_n_mel) || !rd(f, mf.filt_n_fft)) return false;
  if (mf.filt_n_mel <= 0 || mf.filt_n_fft != 1 + MWX_N_FFT / 2 ||
      mf.filt_n_mel != hp.n_mels) {
    MWX_LOG_ERROR("mwx: unexpected mel filter shape %d x %d\n", mf.filt_n_mel,
                  mf.filt_n_fft);
    return false;
  }
  mf.filters.resize((size_t)mf.filt_n_mel * mf.filt_n_fft);
  f.read(reinterpret_cast<char*>(mf.filters.data()),
         mf.filters.size() * sizeof(float));

  int32_t n_vocab_file = 0;
  if (!rd(f, n_vocab_file) || n_vocab_file < 0 || n_vocab_file > hp.n_vocab)
    return false;
  Vocab& vocab = mf.vocab;
  vocab.n_vocab = hp.n_vocab;
  vocab.id_to_token.assign(hp.n_vocab, std::string());
  std::vector<char> tmp;
  for (int i = 0; i < n_vocab_file; ++i) {
    uint32_t len = 0;
    if (!rd(f, len)) return false;
    std::string word;
    if (len > 0) {
      tmp.resize(len);
      f.read(tmp.data(), len);
      word.assign(tmp.data(), len);
    }
    vocab.token_to_id[word] = i;
    vocab.id_to_token[i] = word;
  }
  finalize_vocab(vocab, n_vocab_file);

  while (true) {
    int32_t n_dims = 0, name_len = 0, ttype = 0;
    f.read(reinterpret_cast<char*>(&n_dims), 4);
    if (f.eof()) break;
    if (!rd(f, name_len) || !rd(f, ttype)) return false;
    if (n_dims < 1 || n_dims > 4 || name_len <= 0 || name_len > 256) {
      MWX_LOG_ERROR("mwx: corrupt tensor header\n");
      return false;
    }
    FileTensor t;
    t.type = ttype;
    for (int i = 0; i < n_dims; ++i) {
      int32_t ne = 0;
      if (!rd(f, ne)) return false;
      t.ne.push_back(ne);
    }
    t.name.resize(name_len);
    f.read(&t.name[0], name_len);
    const size_t bytes = ggml_tensor_bytes(ttype, t.ne[0], t.nelements());
    if (bytes == 0) {
      MWX_LOG_ERROR("mwx: tensor '%s' has unsupported type %d (or inner dim %lld)\n",
                    t.name.c_str(), ttype, (long long)t.ne[0]);
      return false;
    }
    t.data.resize(bytes);
    f.read(reinterpret_cast<char*>(t.data.data()), t.data.size());
    if (!f) {
      MWX_LOG_ERROR("mwx: truncated tensor '%s'\n", t.name.c_str());
      return false;
    }
    mf.tensors[t.name] = std::move(t);
  }
  return true;
}

// ---------------------------------------------------------------------------
// synthetic model writer
// ---------------------------------------------------------------------------
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x100000001b3ull;
  }
  return h;
}

// librosa.filters.mel(sr=16000, n_fft=400, n_mels, htk=False, norm="slaney")
static double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3.0;
  double mels = f / f_sp;
  const double min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  if (f >= min_log_hz) mels = min_log_mel + std::log(f / min_log_hz) / logstep;
  return mels;
}
static double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3.0;
  double freqs = f_sp * m;
  const double min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  if (m >= min_log_mel) freqs = min_log_hz * std::exp(logstep * (m - min_log_mel));
  return freqs;
}
static std::vector<float> mel_filterbank(int n_mels) {
  const int n_fft_bins = 1 + MWX_N_FFT / 2;
  std::vector<double> fftfreqs(n_fft_bins);
  for (int i = 0; i < n_fft_bins; ++i)
    fftfreqs[i] = (double)i * (MWX_SAMPLE_RATE / 2.0) / (n_fft_bins - 1);
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
  std::vector<double> mel_f(n_mels + 2);
  for (int i = 0; i < n_mels + 2; ++i)
    mel_f[i] = mel_to_hz(mmin + (mmax - mmin) * i / (double)(n_mels + 1));
  std::vector<float> w((size_t)n_mels * n_fft_bins);
  for (int i = 0; i < n_mels; ++i) {
    const double fd0 = mel_f[i + 1] - mel_f[i];
    const double fd1 = mel_f[i + 2] - mel_f[i + 1];
    const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
    for (int k = 0; k < n_fft_bins; ++k) {
      const double lower = -(mel_f[i] - fftfreqs[k]) / fd0;
      const double upper = (mel_f[i + 2] - fftfreqs[k]) / fd1;
      const double v = std::max(0.0, std::min(lower, upper));
      w[(size_t)i * n_fft_bins + k] = (float)(v * enorm);
    }
  }
  return w;
}

// GPT-2 byte-level order for ids 0..255 (bytes_to_unicode), then unique
// pseudo-syllable words; the multilingual vocab ends with an empty token.
static std::vector<std::string> synthetic_vocab(int n) {
  std::vector<std::string> v;
  std::vector<int> bs;
  for (int b = 33; b <= 126; ++b) bs.push_back(b);
  for (int b = 161; b <= 172; ++b) bs.push_back(b);
  for (int b = 174; b <= 255; ++b) bs.push_back(b);
  for (int b = 0; b < 256; ++b)
    if (std::find(bs.begin(), bs.end(), b) == bs.end()) bs.push_back(b);
  for (int b : bs) v.push_back(std::string(1, (char)b));
  static const char* cons = "bdfgklmnprstvz";
  static const char* vows = "aeiou";
  for (int id = 256; (int)v.size() < n; ++id) {
    long long q = (id - 256) / 2;
    std::string w;
    while (true) {
      const int d = (int)(q % 70);
      w.push_back(cons[d / 5]);
      w.push_back(vows[d % 5]);
      q = q / 70 - 1;
      if (q < 0) break;
    }
    if (id % 2 == 0) w = " " + w;
    v.push_back(w);
  }
  return v;
}

struct ArchSpec {
  const char* name;
  Hparams hp;
};

static bool arch_hparams(const std::string& arch, Hparams& hp) {
  // n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer,
  // n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels
  struct A {
    const char* n;
    int v, ac, as, ah, al, tc, ts, th, tl, nm;
  };
  static const A t[] = {
      {"micro", 51864, 1500, 128, 2, 2, 448, 128, 2, 3, 80},
      {"micro-ml", 51865, 1500, 128, 2, 2, 448, 128, 2, 3, 80},
      {"micro-v3", 51866, 1500, 128, 2, 2, 448, 128, 2, 3, 128},
      // test geometry for the 256-element K quantizations (rows of 256)
      {"micro256", 51864, 1500, 256, 4, 2, 448, 256, 4, 3, 80},
      {"tiny.en", 51864, 1500, 384, 6, 4, 448, 384, 6, 4, 80},
      {"tiny", 51865, 1500, 384, 6, 4, 448, 384, 6, 4, 80},
      {"base.en", 51864, 1500, 512, 8, 6, 448, 512, 8, 6, 80},
      {"base", 51865, 1500, 512, 8, 6, 448, 512, 8, 6, 80},
      {"small", 51865, 1500, 768, 12, 12, 448, 768, 12, 12, 80},
      {"medium", 51865, 1500, 1024, 16, 24, 448, 1024, 16, 24, 80},
      {"large-v3", 51866, 1500, 1280, 20, 32, 448, 1280, 20, 32, 128},
      // large-v3 geometry (d 1280, 20 heads, 128 mels, vocab 51866) with 2 + 2
      // layers: every large-v3 kernel instantiation at an oracle-checkable cost
      {"large-v3-l2", 51866, 1500, 1280, 20, 2, 448, 1280, 20, 2, 128},
  };
  for (const auto& a : t) {
    if (arch == a.n) {
      hp.n_vocab = a.v;
      hp.n_audio_ctx = a.ac;
      hp.n_audio_state = a.as;
      hp.n_audio_head = a.ah;
      hp.n_audio_layer = a.al;
      hp.n_text_ctx = a.tc;
      hp.n_text_state = a.ts;
      hp.n_text_head = a.th;
      hp.n_text_layer = a.tl;
      hp.n_mels = a.nm;
      return true;
    }
  }
  return false;
}

namespace {
struct Writer {
  std::ofstream f;
  uint64_t seed;
  int wtype;
  std::vector<uint8_t> buf;

  template <typename T>
  void put(const T& v) {
    f.write(reinterpret_cast<const char*>(&v), sizeof(T));
  }

  // ne in numpy order (outermost first); written reversed (ggml order).
  // the seeded value of element i of tensor `name` (uniform center +- scale)
  float gen(const std::string& name, int64_t i, float center, float scale) const {
    const uint64_t key = fnv1a64(name) ^ seed;
    const uint64_t r = splitmix64(key + (uint64_t)i * 0xD1B54A32D192ED03ull);
    const float u = (float)((double)(r >> 40) * (1.0 / 8388608.0) - 1.0);
    return center + scale * u;
  }

  void tensor(const std::string& name, std::vector<int64_t> shape, int ttype,
              float center, float scale, const float* explicit_vals = nullptr,
              const std::function<float(int64_t, float)>& adjust = nullptr) {
    const int32_t nd = (int32_t)shape.size();
    put(nd);
    put((int32_t)name.size());
    put((int32_t)ttype);
    for (int i = nd - 1; i >= 0; --i) put((int32_t)shape[i]);
    f.write(name.data(), name.size());
    int64_t n = 1;
    for (auto s : shape) n *= s;
    const uint64_t key = fnv1a64(name) ^ seed;
    const bool quant = ggml_type_is_quant(ttype);
    const size_t esz = ttype == GGML_F32 ? 4 : 2;
    const int64_t chunk = 1 << 20;  // a multiple of the 32-element quant block
    buf.resize((size_t)std::min<int64_t>(n, chunk) * (quant ? 4 : esz));
    for (int64_t i0 = 0; i0 < n; i0 += chunk) {
      const int64_t i1 = std::min(n, i0 + chunk);
      for (int64_t i = i0; i < i1; ++i) {
        float v;
        if (explicit_vals) {
          v = explicit_vals[i];
        } else {
          const uint64_t r = splitmix64(key + (uint64_t)i * 0xD1B54A32D192ED03ull);
          const float u = (float)((double)(r >> 40) * (1.0 / 8388608.0) - 1.0);
          v = center + scale * u;
        }
        if (adjust) v = adjust(i, v);
        if (quant) {
          reinterpret_cast<float*>(buf.data())[i - i0] = v;
          continue;
        }
        uint8_t* p = buf.data() + (size_t)(i - i0) * esz;
        if (ttype == GGML_F32) {
          memcpy(p, &v, 4);
        } else {
          const uint16_t h = ttype == GGML_F16 ? f32_to_f16(v) : f32_to_bf16(v);
          memcpy(p, &h, 2);
        }
      }
      if (quant) {
        std::vector<uint8_t> q(ggml_tensor_bytes(ttype, shape.back(), i1 - i0));
        ggml_quantize(ttype, reinterpret_cast<const float*>(buf.data()), q.data(), i1 - i0);
        f.write(reinterpret_cast<const char*>(q.data()), q.size());
        continue;
      }
      f.write(reinterpret_cast<const char*>(buf.data()), (size_t)(i1 - i0) * esz);
    }
  }
};
}  // namespace

}  // namespace mwx

extern "C" int mwx_write_synthetic_model(const char* path, const char* arch,
                                         int wtype, uint64_t seed) {
  using namespace mwx;
  Hparams hp;
  std::string an = arch ? arch : "";
  const bool rich = an.size() > 5 && an.compare(an.size() - 5, 5, "-rich") == 0;
  if (rich) an.resize(an.size() - 5);
  if (!arch_hparams(an, hp)) {
    MWX_LOG_ERROR("mwx_write_synthetic_model: unknown arch '%s'\n",
                  arch ? arch : "(null)");
    return -1;
  }
  hp.ftype = ggml_ftype_of(wtype);
  if (hp.ftype < 0) return -2;
  // K super-blocks need rows of a multiple of 256 (ggml_row_size)
  const int be = ggml_block_elems(wtype);
  if (hp.n_audio_state % be || hp.n_text_state % be) {
    MWX_LOG_ERROR("mwx_write_synthetic_model: %s rows (%d) are not a multiple of the %d-element "
                  "blocks of type %d\n", an.c_str(), hp.n_text_state, be, wtype);
    return -2;
  }
  // quantized files keep the 3-D conv kernels in f16 (the quantize tool only
  // rewrites 2-D tensors)
  const int conv_type = ggml_type_is_quant(wtype) ? GGML_F16 : wtype;
  Writer w;
  w.f.open(path, std::ios::binary | std::ios::trunc);
  if (!w.f) return -3;
  w.seed = seed;
  w.wtype = wtype;
  w.put((uint32_t)0x67676d6cu);
  const int32_t hpv[] = {hp.n_vocab,      hp.n_audio_ctx,  hp.n_audio_state,
                         hp.n_audio_head, hp.n_audio_layer, hp.n_text_ctx,
                         hp.n_text_state, hp.n_text_head,  hp.n_text_layer,
                         hp.n_mels,       hp.ftype};
  for (int32_t v : hpv) w.put(v);
  const auto filt = mel_filterbank(hp.n_mels);
  w.put((int32_t)hp.n_mels);
  w.put((int32_t)(1 + MWX_N_FFT / 2));
  w.f.write(reinterpret_cast<const char*>(filt.data()), filt.size() * 4);
  const int n_base = hp.n_vocab >= 51865 ? 50257 : 50256;
  const auto words = synthetic_vocab(n_base);
  w.put((int32_t)n_base);
  for (int i = 0; i < n_base; ++i) {
    const std::string& s = (hp.n_vocab >= 51865 && i == 50256) ? std::string() : words[i];
    w.put((uint32_t)s.size());
    w.f.write(s.data(), s.size());
  }

  const int64_t da = hp.n_audio_state, dt = hp.n_text_state;
  // residual-branch outputs (attn.out, mlp.2) get gain 3 so the decoder state
  // is not dominated by the input token's own (tied) embedding
  auto lin = [&](const std::string& pfx, int64_t out, int64_t in, bool bias, float gain = 1.0f) {
    w.tensor(pfx + ".weight", {out, in}, wtype, 0.0f, gain * std::sqrt(3.0f / (float)in));
    if (bias) w.tensor(pfx + ".bias", {out}, GGML_F32, 0.0f, 0.05f);
  };
  auto ln = [&](const std::string& pfx, int64_t d) {
    w.tensor(pfx + ".weight", {d}, GGML_F32, 1.0f, 0.1f);
    w.tensor(pfx + ".bias", {d}, GGML_F32, 0.0f, 0.05f);
  };
  // encoder positional embedding: whisper sinusoids(n_ctx, n_state)
  {
    std::vector<float> pe((size_t)hp.n_audio_ctx * da);
    const int64_t half = da / 2;
    const double inc = std::log(10000.0) / (double)(half - 1);
    for (int64_t t = 0; t < hp.n_audio_ctx; ++t)
      for (int64_t j = 0; j < half; ++j) {
        const double st = (double)t * std::exp(-inc * (double)j);
        pe[(size_t)t * da + j] = (float)std::sin(st);
        pe[(size_t)t * da + half + j] = (float)std::cos(st);
      }
    w.tensor("encoder.positional_embedding", {hp.n_audio_ctx, da}, GGML_F32,
             0, 0, pe.data());
  }
  w.tensor("encoder.conv1.weight", {da, hp.n_mels, 3}, conv_type, 0.0f,
           std::sqrt(3.0f / (float)(hp.n_mels * 3)));
  w.tensor("encoder.conv1.bias", {da, 1}, GGML_F32, 0.0f, 0.05f);
  w.tensor("encoder.conv2.weight", {da, da, 3}, conv_type, 0.0f,
           std::sqrt(3.0f / (float)(da * 3)));
  w.tensor("encoder.conv2.bias", {da, 1}, GGML_F32, 0.0f, 0.05f);
  for (int l = 0; l < hp.n_audio_layer; ++l) {
    const std::string p = "encoder.blocks." + std::to_string(l);
    lin(p + ".attn.query", da, da, true);
    lin(p + ".attn.key", da, da, false);
    lin(p + ".attn.value", da, da, true);
    lin(p + ".attn.out", da, da, true, 3.0f);
    ln(p + ".attn_ln", da);
    lin(p + ".mlp.0", 4 * da, da, true);
    lin(p + ".mlp.2", da, 4 * da, true, 3.0f);
    ln(p + ".mlp_ln", da);
  }
  ln("encoder.ln_post", da);
  // tied token embedding: logit std ~8 for unit-variance final activations.
  // "-rich" test variants: the final LayerNorm bias b is large and the
  // timestamp / EOT embeddings get +beta / +gamma * b/|b|^2, so timestamp and
  // EOT logits are lifted by about beta / gamma: the token loop then emits
  // timestamps, segment splits, EOT and seeks (with peaked, well-separated
  // logits, so device and oracle agree token for token).
  const float ln_b_scale = rich ? 1.0f : 0.05f;
  const float beta = 12.0f, gamma = 30.0f;
  std::vector<float> bdir(dt, 0.0f);
  if (rich) {
    double nb = 0.0;
    for (int64_t j = 0; j < dt; ++j) {
      bdir[j] = w.gen("decoder.ln.bias", j, 0.0f, ln_b_scale);
      nb += (double)bdir[j] * bdir[j];
    }
    for (auto& x : bdir) x = (float)(x / nb);
  }
  const int64_t beg_id = hp.n_vocab >= 51866 ? 50365 : hp.n_vocab == 51865 ? 50364 : 50363;
  const int64_t eot_id = hp.n_vocab >= 51865 ? 50257 : 50256;
  std::function<float(int64_t, float)> boost = nullptr;
  if (rich)
    boost = [&](int64_t i, float v) {
      const int64_t row = i / dt, col = i % dt;
      if (row >= beg_id) return v + beta * bdir[col];
      if (row == eot_id) return v + gamma * bdir[col];
      return v;
    };
  w.tensor("decoder.token_embedding.weight", {hp.n_vocab, dt}, wtype, 0.0f,
           8.0f * std::sqrt(3.0f / (float)dt), nullptr, boost);
  const float pos_std = rich ? 1.5f : 0.2f;
  w.tensor("decoder.positional_embedding", {hp.n_text_ctx, dt}, GGML_F32, 0.0f, pos_std);
  for (int l = 0; l < hp.n_text_layer; ++l) {
    const std::string p = "decoder.blocks." + std::to_string(l);
    lin(p + ".attn.query", dt, dt, true);
    lin(p + ".attn.key", dt, dt, false);
    lin(p + ".attn.value", dt, dt, true);
    lin(p + ".attn.out", dt, dt, true, 3.0f);
    ln(p + ".attn_ln", dt);
    lin(p + ".cross_attn.query", dt, dt, true);
    lin(p + ".cross_attn.key", dt, da, false);
    lin(p + ".cross_attn.value", dt, da, true);
    lin(p + ".cross_attn.out", dt, dt, true, 3.0f);
    ln(p + ".cross_attn_ln", dt);
    lin(p + ".mlp.0", 4 * dt, dt, true);
    lin(p + ".mlp.2", dt, 4 * dt, true, 3.0f);
    ln(p + ".mlp_ln", dt);
  }
  w.tensor("decoder.ln.weight", {dt}, GGML_F32, 1.0f, 0.1f);
  w.tensor("decoder.ln.bias", {dt}, GGML_F32, 0.0f, ln_b_scale);
  w.f.close();
  return w.f ? 0 : -4;
}

// ---------------------------------------------------------------------------
// model quantizer: whisper.cpp's `quantize` tool (examples/quantize +
// examples/common-ggml.cpp ggml_common_quantize_0 at v1.8.2; K types: valid
// blocks from quant.cpp's plain encoder, not ggml's scale search) — every 2-D
// tensor except the positional embeddings (and conv biases, which are not
// 2-D in ggml's sense for the rule below) is rewritten as `type` blocks from
// its f32 (or f16 / bf16 widened) values; everything else is copied
// unchanged; hparams.ftype becomes GGML_QNT_VERSION * 1000 + ftype. Streams
// one tensor at a time.
// ---------------------------------------------------------------------------
extern "C" int mwx_model_quantize(const char* in_path, const char* out_path, int type) {
  using namespace mwx;
  if (!in_path || !out_path || !ggml_type_is_quant(type)) return -1;
  std::ifstream fi(in_path, std::ios::binary);
  if (!fi) return -2;
  std::ofstream fo(out_path, std::ios::binary | std::ios::trunc);
  if (!fo) return -3;
  auto copy = [&](size_t n) {
    std::vector<char> b(n);
    fi.read(b.data(), (std::streamsize)n);
    fo.write(b.data(), (std::streamsize)n);
    return (bool)fi;
  };
  uint32_t magic = 0;
  int32_t hp[11];
  if (!rd(fi, magic) || magic != 0x67676d6cu) return -4;
  for (int32_t& v : hp)
    if (!rd(fi, v)) return -4;
  if (hp[10] % 1000 != 1 && hp[10] % 1000 != 0 && hp[10] % 1000 != 24) {
    MWX_LOG_ERROR("mwx_model_quantize: input must be f32 / f16 / bf16 (ftype %d)\n", hp[10]);
    return -5;
  }
  hp[10] = ggml_ftype_of(type);
  fo.write(reinterpret_cast<const char*>(&magic), 4);
  fo.write(reinterpret_cast<const char*>(hp), sizeof hp);
  int32_t n_mel = 0, n_fft = 0;
  if (!rd(fi, n_mel) || !rd(fi, n_fft) || n_mel <= 0 || n_fft <= 0) return -4;
  fo.write(reinterpret_cast<const char*>(&n_mel), 4);
  fo.write(reinterpret_cast<const char*>(&n_fft), 4);
  if (!copy((size_t)n_mel * n_fft * 4)) return -4;
  int32_t n_vocab = 0;
  if (!rd(fi, n_vocab) || n_vocab < 0) return -4;
  fo.write(reinterpret_cast<const char*>(&n_vocab), 4);
  for (int i = 0; i < n_vocab; ++i) {
    uint32_t len = 0;
    if (!rd(fi, len)) return -4;
    fo.write(reinterpret_cast<const char*>(&len), 4);
    if (len && !copy(len)) return -4;
  }
  std::vector<uint8_t> data, qout;
  std::vector<float> f32;
  while (true) {
    int32_t nd = 0, nl = 0, tt = 0;
    fi.read(reinterpret_cast<char*>(&nd), 4);
    if (fi.eof()) break;
    if (!rd(fi, nl) || !rd(fi, tt) || nd < 1 || nd > 4 || nl <= 0 || nl > 256) return -4;
    int32_t ne[4] = {1, 1, 1, 1};
    for (int i = 0; i < nd; ++i)
      if (!rd(fi, ne[i])) return -4;
    std::string name(nl, '\0');
    fi.read(&name[0], nl);
    int64_t n = 1;
    for (int i = 0; i < nd; ++i) n *= ne[i];
    const size_t bytes = ggml_tensor_bytes(tt, ne[0], n);
    if (bytes == 0) return -6;
    data.resize(bytes);
    fi.read(reinterpret_cast<char*>(data.data()), (std::streamsize)bytes);
    if (!fi) return -4;
    const bool skip = name == "encoder.positional_embedding" ||
                      name == "decoder.positional_embedding" ||
                      name == "encoder.conv1.bias" || name == "encoder.conv2.bias";
    const bool quant = nd == 2 && !skip &&
                       (tt == GGML_F32 || tt == GGML_F16 || tt == GGML_BF16);
    if (quant && ne[0] % ggml_block_elems(type) != 0) {
      // ggml_quantize_chunk asserts on such rows: whisper.cpp's tool fails too
      MWX_LOG_ERROR("mwx_model_quantize: '%s' rows of %d are not a multiple of the %d-element "
                    "blocks of type %d\n", name.c_str(), ne[0], ggml_block_elems(type), type);
      return -8;
    }
    const int32_t ot = quant ? type : tt;
    fo.write(reinterpret_cast<const char*>(&nd), 4);
    fo.write(reinterpret_cast<const char*>(&nl), 4);
    fo.write(reinterpret_cast<const char*>(&ot), 4);
    fo.write(reinterpret_cast<const char*>(ne), 4 * nd);
    fo.write(name.data(), nl);
    if (!quant) {
      fo.write(reinterpret_cast<const char*>(data.data()), (std::streamsize)bytes);
      continue;
    }
    f32.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      if (tt == GGML_F32) {
        memcpy(&f32[i], &data[4 * i], 4);
      } else {
        uint16_t h;
        memcpy(&h, &data[2 * i], 2);
        f32[i] = tt == GGML_F16 ? f16_to_f32(h) : bf16_to_f32(h);
      }
    }
    qout.resize(ggml_tensor_bytes(type, ne[0], n));
    ggml_quantize(type, f32.data(), qout.data(), n);
    fo.write(reinterpret_cast<const char*>(qout.data()), (std::streamsize)qout.size());
  }
  fo.close();
  return fo ? 0 : -7;
}

extern "C" int mwx_test_dequantize(int type, const void* src, long n, float* dst) {
  using namespace mwx;
  const int be = ggml_block_elems(type);
  if (!ggml_type_is_quant(type) || n < 0 || n % be || !src || !dst) return -1;
  ggml_dequantize(type, static_cast<const uint8_t*>(src), dst, n);
  return 0;
}

extern "C" void mwx_log_set(mwx_log_callback cb, void* user_data) {
  mwx::g_log_cb = cb;
  mwx::g_log_user = user_data;
}

extern "C" int mwx_lang_id(const char* lang) {
  return lang ? mwx::lang_id(lang) : -1;
}
extern "C" const char* mwx_lang_str(int id) { return mwx::lang_str(id); }
extern "C" int mwx_lang_max_id(void) { return mwx::lang_max_id(); }
