// StreamSession: see stt_stream.h (src/grpc_server.cpp:98-309 semantics).
#include "stt_stream.h"

#include <cstdio>
#include <cstring>

namespace mwx_host {

namespace {

bool is_wav(const uint8_t* p, size_t n) {  // src/utils.h:101-105
  return n >= 12 && std::memcmp(p, "RIFF", 4) == 0 && std::memcmp(p + 8, "WAVE", 4) == 0;
}

void set_affect(StreamEvent& ev, const TranscriptionResult& r, bool detail) {
  const AffectiveTags& a = r.affective;
  ev.gender_proxy = a.gender_proxy;
  ev.emotion_proxy = a.emotion_proxy;
  ev.arousal = a.arousal;
  ev.valence = a.valence;
  if (detail) {
    ev.pitch_mean = a.pitch_mean;
    ev.pitch_std = a.pitch_std;
    ev.energy_mean = a.energy_mean;
    ev.energy_std = a.energy_std;
    ev.spectral_centroid = a.spectral_centroid;
    ev.zero_crossing_rate = a.zero_crossing_rate;
  }
  ev.speaker_vec = a.speaker_vec;
  ev.speaker_id = r.speaker_id;
}

}  // namespace

StreamSession::StreamSession(SttEngine& engine)
    : engine_(engine), step_((size_t)engine.get_settings().stream_buffer_samples) {}

std::vector<StreamEvent> StreamSession::feed(const uint8_t* data, size_t len) {
  std::vector<StreamEvent> out;
  RequestOptions options;  // the stream path uses default request options
  if (len == 0) {          // end of speech: finalize the buffered sentence
    if (!buffer_.empty()) {
      const auto results = engine_.transcribe_pcm16(buffer_, 16000, options);
      for (const auto& r : results) {
        if (r.text.empty()) continue;
        StreamEvent ev;
        ev.transcription = r.text;
        ev.is_final = true;
        set_affect(ev, r, true);
        for (const auto& t : r.tokens)
          ev.words.push_back({t.text, (float)t.t0 / 100.0f, (float)t.t1 / 100.0f, t.p});
        out.push_back(std::move(ev));
      }
      buffer_.clear();
      last_processed_ = 0;
    }
    return out;
  }
  if (first_chunk_) {
    if (is_wav(data, len)) {
      wav_container_ = true;
      if (len > 44) header_skip_ = 44;
    }
    first_chunk_ = false;
  }
  if (wav_container_ && header_skip_ > 0) {
    if (len >= header_skip_) {
      data += header_skip_;
      len -= header_skip_;
      header_skip_ = 0;
    } else {
      header_skip_ -= len;
      len = 0;
    }
  }
  if (len > 0) {
    const size_t samples = len / 2;
    const size_t cur = buffer_.size();
    buffer_.resize(cur + samples);
    std::memcpy(buffer_.data() + cur, data, samples * 2);
  }
  if (buffer_.size() - last_processed_ >= step_) {
    try {
      SttEngine::PerformanceMetrics perf;
      const auto results = engine_.transcribe_pcm16(buffer_, 16000, options, &perf);
      last_processed_ = buffer_.size();
      StreamEvent partial;
      bool any = false;
      for (const auto& r : results) {
        if (r.text.empty()) continue;
        partial.transcription += r.text + " ";
        set_affect(partial, r, true);  // the last non-empty segment's
        any = true;
      }
      if (any) out.push_back(std::move(partial));
      if (buffer_.size() > kMaxBufferSamples) {  // 30 s without a pause
        for (const auto& r : results) {
          if (r.text.empty()) continue;
          StreamEvent ev;
          ev.transcription = r.text;
          ev.is_final = true;
          set_affect(ev, r, false);
          out.push_back(std::move(ev));
        }
        buffer_.clear();
        last_processed_ = 0;
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "Streaming error: %s\n", e.what());
    }
  }
  return out;
}

}  // namespace mwx_host
