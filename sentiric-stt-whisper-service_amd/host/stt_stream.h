// Streaming re-transcription session: the reference's
// per-stream buffer loop of WhisperTranscribeStream (src/grpc_server.cpp:98-309)
// without the gRPC transport, over the GPU SttEngine.
//
// Kept from the reference, chunk by chunk:
//  * the first chunk may carry a WAV container: "RIFF"...."WAVE" at bytes 0-11
//    (src/utils.h:101-105); then 44 header bytes are skipped — only when that
//    first chunk is longer than 44 bytes, as the reference does (:195-212);
//  * chunk bytes are appended as little-endian int16 (an odd trailing byte is
//    dropped, :214-219);
//  * every `stream_buffer_samples` new samples (Settings, default 8000 =
//    0.5 s) the WHOLE buffer is re-transcribed and one partial event carries
//    the non-empty segment texts joined with trailing spaces plus the affect
//    fields and speaker of the last such segment (:222-262);
//  * past 30 s of buffer the segments of that transcription are forced final
//    (text, gender, emotion, arousal, valence, speaker, speaker vector) and the
//    buffer restarts (:264-290); a transcription error on this path is
//    swallowed, as the reference logs it and carries on (:292-295);
//  * an empty chunk is the end-of-speech signal: a non-empty buffer is
//    transcribed once more and every non-empty segment becomes a final event
//    with all affect fields and its words (token text, t0 / 100, t1 / 100, p),
//    then the buffer restarts (:150-190).
//
// GPU-side, concurrent sessions of an engine built with Settings::max_batch > 1
// have their re-transcriptions gathered into shared mwx_full_batch calls by
// the engine's request batcher: many live streams, one decode loop.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "stt_engine.h"

namespace mwx_host {

// The fields of one WhisperTranscribeStreamResponse; fields the reference
// leaves unset in a given message keep their protobuf defaults (0 / empty).
struct StreamWord {
  std::string word;
  float start = 0.0f;  // seconds
  float end = 0.0f;
  float probability = 0.0f;
};

struct StreamEvent {
  std::string transcription;
  bool is_final = false;
  std::string gender_proxy;
  std::string emotion_proxy;
  float arousal = 0.0f;
  float valence = 0.0f;
  float pitch_mean = 0.0f;
  float pitch_std = 0.0f;
  float energy_mean = 0.0f;
  float energy_std = 0.0f;
  float spectral_centroid = 0.0f;
  float zero_crossing_rate = 0.0f;
  std::vector<float> speaker_vec;
  std::string speaker_id;
  std::vector<StreamWord> words;
};

class StreamSession {
 public:
  explicit StreamSession(SttEngine& engine);

  // One received audio chunk (bytes as sent by the client); an empty chunk is
  // the end-of-speech signal. Returns the events the reference would write.
  std::vector<StreamEvent> feed(const uint8_t* data, size_t len);

  size_t buffered_samples() const { return buffer_.size(); }

  static constexpr size_t kMaxBufferSamples = 16000 * 30;  // src/grpc_server.cpp:132

 private:
  SttEngine& engine_;
  std::vector<int16_t> buffer_;
  size_t last_processed_ = 0;
  size_t step_;  // Settings::stream_buffer_samples
  bool first_chunk_ = true;
  bool wav_container_ = false;
  size_t header_skip_ = 0;
};

}  // namespace mwx_host
