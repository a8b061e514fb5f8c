// Plain-C entry points over mwx_host::SttEngine for the Python tests (ctypes).
// Results are returned as JSON with every string hex-encoded (token text may
// be a partial UTF-8 sequence).
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "stt_engine.h"
#include "stt_stream.h"
#include "text_filters.h"

using namespace mwx_host;

namespace {

std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  o.reserve(s.size() * 2);
  for (unsigned char c : s) {
    o.push_back(d[c >> 4]);
    o.push_back(d[c & 15]);
  }
  return o;
}

std::string to_json(const std::vector<TranscriptionResult>& rs) {
  std::string o = "[";
  char buf[1024];
  for (size_t i = 0; i < rs.size(); ++i) {
    const TranscriptionResult& r = rs[i];
    std::snprintf(buf, sizeof buf, "%s{\"prob\":%.9g,\"t0\":%lld,\"t1\":%lld,\"turn\":%d,\"n\":%d,",
                  i ? "," : "", r.prob, (long long)r.t0, (long long)r.t1, (int)r.speaker_turn_next,
                  r.token_count);
    o += buf;
    o += "\"text\":\"" + hex(r.text) + "\",\"language\":\"" + hex(r.language) + "\",";
    const AffectiveTags& a = r.affective;
    std::snprintf(buf, sizeof buf,
                  "\"gender\":\"%s\",\"emotion\":\"%s\",\"speaker\":\"%s\",\"arousal\":%.9g,"
                  "\"valence\":%.9g,\"pitch_mean\":%.9g,\"pitch_std\":%.9g,\"energy_mean\":%.9g,"
                  "\"energy_std\":%.9g,\"spectral_centroid\":%.9g,\"zero_crossing_rate\":%.9g,",
                  r.gender_proxy.c_str(), r.emotion_proxy.c_str(), r.speaker_id.c_str(), r.arousal,
                  r.valence, a.pitch_mean, a.pitch_std, a.energy_mean, a.energy_std,
                  a.spectral_centroid, a.zero_crossing_rate);
    o += buf;
    o += "\"speaker_vec\":[";
    for (size_t j = 0; j < a.speaker_vec.size(); ++j) {
      std::snprintf(buf, sizeof buf, "%s%.9g", j ? "," : "", a.speaker_vec[j]);
      o += buf;
    }
    o += "],\"tokens\":[";
    for (size_t j = 0; j < r.tokens.size(); ++j) {
      const TokenData& t = r.tokens[j];
      std::snprintf(buf, sizeof buf, "%s{\"p\":%.9g,\"t0\":%lld,\"t1\":%lld,\"text\":\"", j ? "," : "",
                    t.p, (long long)t.t0, (long long)t.t1);
      o += buf;
      o += hex(t.text) + "\"}";
    }
    o += "]}";
  }
  return o + "]";
}

int emit(const std::string& s, char* out, int cap) {
  if ((int)s.size() + 1 > cap) return -(int)(s.size() + 1);
  std::memcpy(out, s.c_str(), s.size() + 1);
  return (int)s.size();
}

}  // namespace

extern "C" {

int mwx_stt_is_hallucination(const char* text) { return is_hallucination(text ? text : "") ? 1 : 0; }

void* mwx_stt_new(const char* model_dir, const char* model_filename, int parallel_requests,
                  int queue_timeout_ms, int beam_size, const char* language, int vad_ms_min,
                  int gpu_device) {
  Settings s;
  s.model_dir = model_dir;
  s.model_filename = model_filename;
  s.parallel_requests = parallel_requests;
  s.request_queue_timeout_ms = queue_timeout_ms;
  s.beam_size = beam_size;
  s.language = language;
  s.vad_ms_min_duration = vad_ms_min;
  s.gpu_device = gpu_device;
  try {
    return new SttEngine(s);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "SttEngine: %s\n", e.what());
    return nullptr;
  }
}

// As mwx_stt_new, with dynamic request batching (Settings::max_batch /
// batch_window_us).
void* mwx_stt_new_batched(const char* model_dir, const char* model_filename,
                          int parallel_requests, int queue_timeout_ms, int beam_size,
                          const char* language, int vad_ms_min, int gpu_device, int max_batch,
                          int batch_window_us) {
  Settings s;
  s.model_dir = model_dir;
  s.model_filename = model_filename;
  s.parallel_requests = parallel_requests;
  s.request_queue_timeout_ms = queue_timeout_ms;
  s.beam_size = beam_size;
  s.language = language;
  s.vad_ms_min_duration = vad_ms_min;
  s.gpu_device = gpu_device;
  s.max_batch = max_batch;
  s.batch_window_us = batch_window_us;
  try {
    return new SttEngine(s);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "SttEngine: %s\n", e.what());
    return nullptr;
  }
}

// SpeakerClusterer over n 8-D vectors in order: writes the ids, one per line.
int mwx_stt_cluster_ids(const float* vecs, int n, float threshold, char* out, int cap) {
  SpeakerClusterer c(threshold);
  std::string o;
  for (int i = 0; i < n; ++i)
    o += c.assign_or_add(std::vector<float>(vecs + 8 * i, vecs + 8 * i + 8)) + "\n";
  return emit(o, out, cap);
}

// As mwx_stt_new_batched, with Settings::stream_buffer_samples.
void* mwx_stt_new_ex(const char* model_dir, const char* model_filename, int parallel_requests,
                     int queue_timeout_ms, int beam_size, const char* language, int vad_ms_min,
                     int gpu_device, int max_batch, int batch_window_us,
                     int stream_buffer_samples) {
  Settings s;
  s.model_dir = model_dir;
  s.model_filename = model_filename;
  s.parallel_requests = parallel_requests;
  s.request_queue_timeout_ms = queue_timeout_ms;
  s.beam_size = beam_size;
  s.language = language;
  s.vad_ms_min_duration = vad_ms_min;
  s.gpu_device = gpu_device;
  s.max_batch = max_batch;
  s.batch_window_us = batch_window_us;
  s.stream_buffer_samples = stream_buffer_samples;
  try {
    return new SttEngine(s);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "SttEngine: %s\n", e.what());
    return nullptr;
  }
}

// StreamSession over an engine: feed one chunk (len 0 = end of speech);
// returns the events as JSON (strings hex-encoded) like mwx_stt_transcribe_pcm16.
// If `cap` is too small the chunk is still consumed: the events are kept and
// -(needed + 2) is returned; mwx_stt_stream_drain then delivers them (never
// feed the chunk again). While such events are undelivered, a feed returns
// -3 (MWX_STT_PENDING) WITHOUT consuming its chunk: drain, then feed the same
// chunk again. -1 = error, -2 = EngineBusyException.
struct StreamHandle {
  explicit StreamHandle(SttEngine& e) : session(e) {}
  StreamSession session;
  std::string pending;  // undelivered events JSON
};
void* mwx_stt_stream_new(void* eng) { return new StreamHandle(*static_cast<SttEngine*>(eng)); }
void mwx_stt_stream_free(void* s) { delete static_cast<StreamHandle*>(s); }

int mwx_stt_stream_drain(void* s, char* out, int cap) {
  StreamHandle* h = static_cast<StreamHandle*>(s);
  const int r = emit(h->pending.empty() ? std::string("[]") : h->pending, out, cap);
  if (r >= 0) h->pending.clear();
  return r < -1 ? r - 2 : r;
}

int mwx_stt_stream_feed(void* s, const uint8_t* data, int len, char* out, int cap) {
  StreamHandle* h = static_cast<StreamHandle*>(s);
  if (!h->pending.empty()) return -3;  // MWX_STT_PENDING: drain first, chunk not consumed
  try {
    const auto evs = h->session.feed(data, len > 0 ? (size_t)len : 0);
    std::string o = "[";
    char buf[512];
    for (size_t i = 0; i < evs.size(); ++i) {
      const StreamEvent& e = evs[i];
      std::snprintf(buf, sizeof buf,
                    "%s{\"final\":%d,\"arousal\":%.9g,\"valence\":%.9g,\"pitch_mean\":%.9g,"
                    "\"pitch_std\":%.9g,\"energy_mean\":%.9g,\"energy_std\":%.9g,"
                    "\"spectral_centroid\":%.9g,\"zero_crossing_rate\":%.9g,",
                    i ? "," : "", (int)e.is_final, e.arousal, e.valence, e.pitch_mean, e.pitch_std,
                    e.energy_mean, e.energy_std, e.spectral_centroid, e.zero_crossing_rate);
      o += buf;
      o += "\"text\":\"" + hex(e.transcription) + "\",\"gender\":\"" + e.gender_proxy +
           "\",\"emotion\":\"" + e.emotion_proxy + "\",\"speaker\":\"" + e.speaker_id +
           "\",\"speaker_vec\":[";
      for (size_t j = 0; j < e.speaker_vec.size(); ++j) {
        std::snprintf(buf, sizeof buf, "%s%.9g", j ? "," : "", e.speaker_vec[j]);
        o += buf;
      }
      o += "],\"words\":[";
      for (size_t j = 0; j < e.words.size(); ++j) {
        const StreamWord& w = e.words[j];
        std::snprintf(buf, sizeof buf, "%s{\"start\":%.9g,\"end\":%.9g,\"p\":%.9g,\"word\":\"",
                      j ? "," : "", w.start, w.end, w.probability);
        o += buf;
        o += hex(w.word) + "\"}";
      }
      o += "]}";
    }
    o += "]";
    const int r = emit(o, out, cap);
    if (r < -1) h->pending = o;
    return r < -1 ? r - 2 : r;
  } catch (const EngineBusyException&) {
    return -2;
  } catch (...) {
    return -1;
  }
}

long mwx_stt_batches(void* eng) { return static_cast<SttEngine*>(eng)->batches_run(); }

void mwx_stt_free(void* eng) { delete static_cast<SttEngine*>(eng); }

// 0.. = JSON length written; -1 = error; -2 = EngineBusyException;
// < -2 = -(needed capacity). abort_after >= 0: RequestOptions::should_abort
// answers true from its (abort_after + 1)-th call on (the service's abort
// hook, src/stt_engine.cpp:17-23,215-219); < 0: no abort callback.
static int transcribe_any(void* eng, const int16_t* pcm16, const float* pcmf, int n,
                          int sample_rate, const char* language, int beam_size, float temperature,
                          char* out, int cap, double* metrics3, int abort_after, int* abort_calls);

int mwx_stt_transcribe_pcm16_ex(void* eng, const int16_t* pcm, int n, int sample_rate,
                                const char* language, int beam_size, float temperature, char* out,
                                int cap, double* metrics3, int abort_after, int* abort_calls) {
  return transcribe_any(eng, pcm, nullptr, n, sample_rate, language, beam_size, temperature, out,
                        cap, metrics3, abort_after, abort_calls);
}

// As mwx_stt_transcribe_pcm16_ex over f32 PCM (SttEngine::transcribe).
int mwx_stt_transcribe_f32_ex(void* eng, const float* pcm, int n, int sample_rate,
                              const char* language, int beam_size, float temperature, char* out,
                              int cap, double* metrics3, int abort_after, int* abort_calls) {
  return transcribe_any(eng, nullptr, pcm, n, sample_rate, language, beam_size, temperature, out,
                        cap, metrics3, abort_after, abort_calls);
}

static int transcribe_any(void* eng, const int16_t* pcm16, const float* pcmf, int n,
                          int sample_rate, const char* language, int beam_size, float temperature,
                          char* out, int cap, double* metrics3, int abort_after, int* abort_calls) {
  RequestOptions o;
  o.language = language ? language : "";
  o.beam_size = beam_size;
  o.temperature = temperature;
  auto calls = std::make_shared<int>(0);
  if (abort_after >= 0)
    o.should_abort = [calls, abort_after] { return (*calls)++ >= abort_after; };
  SttEngine::PerformanceMetrics m{0, 0, 0};
  try {
    SttEngine* e = static_cast<SttEngine*>(eng);
    const auto rs = pcm16 ? e->transcribe_pcm16(std::vector<int16_t>(pcm16, pcm16 + n), sample_rate, o, &m)
                          : e->transcribe(std::vector<float>(pcmf, pcmf + n), sample_rate, o, &m);
    if (metrics3) {
      metrics3[0] = m.queue_time_ms;
      metrics3[1] = m.processing_time_ms;
      metrics3[2] = m.token_count;
    }
    if (abort_calls) *abort_calls = *calls;
    const int r = emit(to_json(rs), out, cap);
    return r < -1 ? r - 2 : r;
  } catch (const EngineBusyException&) {
    return -2;
  } catch (...) {
    return -1;
  }
}

int mwx_stt_transcribe_pcm16(void* eng, const int16_t* pcm, int n, int sample_rate,
                             const char* language, int beam_size, float temperature, char* out,
                             int cap, double* metrics3) {
  RequestOptions o;
  o.language = language ? language : "";
  o.beam_size = beam_size;
  o.temperature = temperature;
  SttEngine::PerformanceMetrics m{0, 0, 0};
  try {
    const auto rs = static_cast<SttEngine*>(eng)->transcribe_pcm16(
        std::vector<int16_t>(pcm, pcm + n), sample_rate, o, &m);
    if (metrics3) {
      metrics3[0] = m.queue_time_ms;
      metrics3[1] = m.processing_time_ms;
      metrics3[2] = m.token_count;
    }
    const int r = emit(to_json(rs), out, cap);
    return r < -1 ? r - 2 : r;
  } catch (const EngineBusyException&) {
    return -2;
  } catch (...) {
    return -1;
  }
}

}  // extern "C"
