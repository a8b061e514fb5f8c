// Shared host-side definitions of the mwx engine (model hyper-parameters,
// vocabulary, logging). Device code lives in the *.hip files.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "mwx.h"

namespace mwx {

// ggml tensor types used by whisper .bin files (ggml.h enum ggml_type values):
// f32 / f16 / bf16, the legacy 32-element block quantizations and the
// 256-element "K" super-block quantizations written by whisper.cpp's quantize
// tool.
enum GgmlType : int32_t {
  GGML_F32 = 0,
  GGML_F16 = 1,
  GGML_Q4_0 = 2,
  GGML_Q4_1 = 3,
  GGML_Q5_0 = 6,
  GGML_Q5_1 = 7,
  GGML_Q8_0 = 8,
  GGML_Q2_K = 10,
  GGML_Q3_K = 11,
  GGML_Q4_K = 12,
  GGML_Q5_K = 13,
  GGML_Q6_K = 14,
  GGML_BF16 = 30
};

// quant.cpp: block formats (ggml-common.h) and ggml's reference (de)quantizers
bool ggml_type_is_quant(int type);
// elements per block: 32 (legacy), 256 (K super-blocks), 1 (f32/f16/bf16), 0 unknown
int ggml_block_elems(int type);
// bytes of an n-element tensor with inner dim ne0 (0: unsupported type/shape)
size_t ggml_tensor_bytes(int type, int64_t ne0, int64_t n);
void ggml_dequantize(int type, const uint8_t* src, float* dst, int64_t n);
void ggml_quantize(int type, const float* src, uint8_t* dst, int64_t n);
// whisper hparams.ftype (ggml_ftype) of a file whose 2-D weights are `type`
int ggml_ftype_of(int type);
// one row of K (multiple of 32) values -> MX-fp8 codes q[K] + E8M0 scales s[K/32]
void mx_quantize_row(const float* x, int K, uint8_t* q, uint8_t* s);
float mx_dequant(uint8_t code, uint8_t s);  // e4m3fn code x 2^(s - 127)

// The 11 int32 header fields of a whisper ggml .bin file, in file order
// (whisper.cpp whisper_model_load; upstream converter convert-pt-to-ggml.py).
struct Hparams {
  int32_t n_vocab = 51864;
  int32_t n_audio_ctx = 1500;
  int32_t n_audio_state = 384;
  int32_t n_audio_head = 6;
  int32_t n_audio_layer = 4;
  int32_t n_text_ctx = 448;
  int32_t n_text_state = 384;
  int32_t n_text_head = 6;
  int32_t n_text_layer = 4;
  int32_t n_mels = 80;
  int32_t ftype = 1;
};

// Special-token layout of whisper_vocab (whisper.cpp), including the shift the
// loader applies to multilingual vocabularies.
struct Vocab {
  int n_vocab = 51864;
  int32_t token_eot = 50256;
  int32_t token_sot = 50257;
  int32_t token_translate = 50357;
  int32_t token_transcribe = 50358;
  int32_t token_solm = 50359;
  int32_t token_prev = 50360;
  int32_t token_nosp = 50361;
  int32_t token_not = 50362;
  int32_t token_beg = 50363;
  std::vector<std::string> id_to_token;
  std::map<std::string, int32_t> token_to_id;

  bool is_multilingual() const { return n_vocab >= 51865; }
  int num_languages() const {
    return n_vocab - 51765 - (is_multilingual() ? 1 : 0);
  }
};

// Host copy of one tensor as read from the .bin file.
struct FileTensor {
  std::string name;
  int32_t type = GGML_F32;
  std::vector<int64_t> ne;  // ggml order: ne[0] is contiguous
  std::vector<uint8_t> data;
  int64_t nelements() const {
    int64_t n = 1;
    for (auto v : ne) n *= v;
    return n;
  }
};

struct ModelFile {
  Hparams hp;
  int32_t filt_n_mel = 0, filt_n_fft = 0;
  std::vector<float> filters;  // [n_mel][n_fft]
  Vocab vocab;
  std::map<std::string, FileTensor> tensors;
};

// Parses a whisper ggml .bin file. Returns false (and logs) on any error.
bool read_model_file(const char* path, ModelFile& mf);

// Language table (g_lang of whisper.cpp: std::map keyed by language code,
// iterated in code order by whisper_lang_auto_detect_with_state).
int lang_id(const std::string& code);
const char* lang_str(int id);
int lang_max_id();
// (code, id) pairs in std::map iteration order.
const std::vector<std::pair<std::string, int>>& lang_table_sorted();

// whisper_tokenize semantics: regex pre-split, greedy longest-match.
std::vector<int32_t> tokenize(const Vocab& vocab, const std::string& text);

// Logging (whisper_log_set compatible).
void log_msg(mwx_log_level level, const char* fmt, ...);

// f32 <-> 16-bit float helpers (round to nearest even).
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);
uint16_t f32_to_bf16(float f);
float bf16_to_f32(uint16_t h);

}  // namespace mwx

#define MWX_LOG_INFO(...) ::mwx::log_msg(MWX_LOG_LEVEL_INFO, __VA_ARGS__)
#define MWX_LOG_WARN(...) ::mwx::log_msg(MWX_LOG_LEVEL_WARN, __VA_ARGS__)
#define MWX_LOG_ERROR(...) ::mwx::log_msg(MWX_LOG_LEVEL_ERROR, __VA_ARGS__)
#define MWX_LOG_DEBUG(...) ::mwx::log_msg(MWX_LOG_LEVEL_DEBUG, __VA_ARGS__)
