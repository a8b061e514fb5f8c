// TEST INFRASTRUCTURE ONLY — a CPU stand-in for libmwx.so, linked into the
// sanitizer build of the host SttEngine (tests/san/Makefile) and nowhere else.
//
// It decodes nothing. It exists so that the host side of the drop-in — the
// SttEngine state pool and EngineBusy timeout, the dynamic request batcher,
// the streaming re-transcription loop, the text post-filters, the speaker
// clusterer and the C shim — can run under AddressSanitizer + UBSan and
// ThreadSanitizer in a container without a GPU. Every result is a
// deterministic function of the audio: one segment per 1.5 s, three text
// tokens and one timestamp token per segment, texts cycling through normal
// phrases and the reference's hallucination list, token probabilities that
// sometimes fall below the 0.40 average cut.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mwx.h"

namespace {

const int kEot = 50256;
const char* const kWords[] = {" hello", " world", " this", " is", " a", " test", " of", " the",
                              " stream", " engine", " Thank", " you", ".", "[", "Music", "]"};
const char* const kTexts[] = {" hello world this", " is a test", " Thank you.", " of the stream",
                              "[Music]",          " engine test", " .",          " a world"};

struct Token {
  int id;
  float p;
  int64_t t0, t1;
};
struct Segment {
  std::string text;
  int64_t t0, t1;
  bool turn;
  std::vector<Token> tokens;
};

}  // namespace

struct mwx_context {
  std::string path;
};
struct mwx_state {
  std::vector<Segment> segs;
};

namespace {

int run(mwx_state* st, const mwx_full_params& p, const float* x, int n) {
  st->segs.clear();
  if (!x || n < 0) return -1;
  const int per = 24000;
  const int nseg = n / per + (n % per >= 8000 ? 1 : 0);
  double e = 0.0;
  for (int i = 0; i < n; i += 97) e += std::fabs(x[i]);
  const int salt = (int)(e * 7.0) & 7;
  for (int i = 0; i < nseg; ++i) {
    if (p.abort_callback && p.abort_callback(p.abort_callback_user_data)) return -6;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    Segment s;
    s.text = kTexts[(i + salt) & 7];
    s.t0 = 150 * (int64_t)i;
    s.t1 = std::min<int64_t>(150 * (int64_t)(i + 1), (int64_t)n * 100 / 16000);
    s.turn = p.tdrz_enable && (i % 3 == 2);
    for (int k = 0; k < 3; ++k) {
      const float pr = ((i + k + salt) % 5 == 0) ? 0.2f : 0.9f - 0.05f * k;
      s.tokens.push_back({(i * 3 + k + salt) % 16, pr, s.t0 + 50 * k, s.t0 + 50 * (k + 1)});
    }
    s.tokens.push_back({kEot + 1 + i, 0.99f, s.t1, s.t1});
    st->segs.push_back(std::move(s));
  }
  return 0;
}

}  // namespace

extern "C" {

mwx_context_params mwx_context_default_params(void) {
  mwx_context_params p;
  std::memset(&p, 0, sizeof p);
  p.use_gpu = true;
  p.flash_attn = true;
  return p;
}

mwx_context* mwx_init_from_file_with_params(const char* path, mwx_context_params params) {
  if (!params.use_gpu || !path) return nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) return nullptr;
  std::fclose(f);
  return new mwx_context{path};
}

mwx_state* mwx_init_state(mwx_context* ctx) { return ctx ? new mwx_state() : nullptr; }
void mwx_free_state(mwx_state* st) { delete st; }
void mwx_free(mwx_context* ctx) { delete ctx; }

mwx_full_params mwx_full_default_params(int strategy) {
  mwx_full_params p;
  std::memset(&p, 0, sizeof p);
  p.strategy = strategy;
  p.greedy.best_of = 5;
  p.beam_search.beam_size = 5;
  return p;
}

int mwx_full_with_state(mwx_context* ctx, mwx_state* st, mwx_full_params p, const float* x, int n) {
  if (!ctx || !st) return -1;
  return run(st, p, x, n);
}

int mwx_full_batch(mwx_context* ctx, mwx_state* const* states, mwx_full_params p,
                   const float* const* x, const int* n, int n_clips) {
  if (!ctx || n_clips <= 0) return -1;
  for (int b = 0; b < n_clips; ++b) {
    const int r = run(states[b], p, x[b], n[b]);
    if (r) return r;
  }
  return 0;
}

int mwx_full_n_segments_from_state(mwx_state* st) { return (int)st->segs.size(); }
const char* mwx_full_get_segment_text_from_state(mwx_state* st, int i) {
  return st->segs.at(i).text.c_str();
}
int64_t mwx_full_get_segment_t0_from_state(mwx_state* st, int i) { return st->segs.at(i).t0; }
int64_t mwx_full_get_segment_t1_from_state(mwx_state* st, int i) { return st->segs.at(i).t1; }
bool mwx_full_get_segment_speaker_turn_next_from_state(mwx_state* st, int i) {
  return st->segs.at(i).turn;
}
int mwx_full_n_tokens_from_state(mwx_state* st, int i) { return (int)st->segs.at(i).tokens.size(); }
mwx_token_data mwx_full_get_token_data_from_state(mwx_state* st, int i, int j) {
  const Token& t = st->segs.at(i).tokens.at(j);
  mwx_token_data d;
  std::memset(&d, 0, sizeof d);
  d.id = t.id;
  d.p = t.p;
  d.plog = std::log(t.p);
  d.t0 = t.t0;
  d.t1 = t.t1;
  d.t_dtw = -1;
  return d;
}

const char* mwx_token_to_str(mwx_context*, mwx_token id) {
  return id >= 0 && id < 16 ? kWords[id] : nullptr;
}
mwx_token mwx_token_eot(mwx_context*) { return kEot; }

mwx_prosody_params mwx_prosody_default_params(void) { return {0.07f, 170.0f, 60.0f, 500.0f}; }

int mwx_prosody_batch(mwx_context* ctx, mwx_state* st, const float* pcm, int64_t n_pcm,
                      const int64_t* start, const int64_t* len, int n_seg, int sample_rate,
                      const mwx_prosody_params* params, mwx_prosody* out) {
  if (!ctx || !st || !pcm || !params || sample_rate < 100) return -1;
  for (int i = 0; i < n_seg; ++i) {
    if (start[i] < 0 || len[i] < 0 || start[i] + len[i] > n_pcm) return -1;
    mwx_prosody r;
    std::memset(&r, 0, sizeof r);
    double e = 0.0, z = 0.0;
    for (int64_t k = 0; k < len[i]; ++k) {
      const float v = pcm[start[i] + k];
      e += (double)v * v;
      if (k && (v >= 0) != (pcm[start[i] + k - 1] >= 0)) z += 1.0;
    }
    r.energy_mean = len[i] ? (float)std::sqrt(e / (double)len[i]) : 0.0f;
    r.zero_crossing_rate = len[i] ? (float)(z / (double)len[i]) : 0.0f;
    r.pitch_mean = 100.0f + 40.0f * (float)(i % 4);
    for (int k = 0; k < 8; ++k) r.speaker_vec[k] = 1.0f + (float)((i / 2 + k) % 3);
    r.gender = r.pitch_mean > params->gender_threshold ? MWX_GENDER_F : MWX_GENDER_M;
    r.emotion = i % 4;
    out[i] = r;
  }
  return 0;
}

long mwx_resample_max_frames(int n_in, int src, int dst) {
  if (n_in < 0 || src <= 0 || dst <= 0) return -1;
  return (long)((double)n_in * dst / src) + 100;
}

int mwx_resample(mwx_context* ctx, mwx_state* st, const float* in, int n_in, int src, int dst,
                 float* out, int out_cap) {
  if (!ctx || !st || !in || src <= 0 || dst <= 0) return -1;
  if (src == dst || n_in == 0) return 0;
  int n = 0;
  for (; n < out_cap; ++n) {  // linear interpolation, holding back one sample
    const double pos = (double)n * src / dst;
    const int i = (int)pos;
    if (i + 1 >= n_in) break;
    out[n] = (float)(in[i] + (pos - i) * (in[i + 1] - in[i]));
  }
  return n;
}

}  // extern "C"
