// SttEngine on the mwx C ABI — the drop-in for the reference's
// src/stt_engine.h:16-115 (same class, method names, argument meaning, result
// types and error behaviour), with whisper.h replaced by include/mwx.h.
//
// Kept from the reference: the state pool with a queue timeout that throws
// EngineBusyException (src/stt_engine.cpp:63-85), the request-option defaults
// (:204-212), the whisper_full parameter mapping (:214-243), the too-short
// audio gate (:153-167), and the result post-filters (:261-311: hallucination
// phrases, tokens with id >= eot skipped, average token p < 0.40 drops the
// segment), per-segment prosody (src/stt_engine.cpp:313-337: computed on the
// GPU by mwx_prosody_batch, bit-identical to src/prosody_extractor.cpp) and
// speaker clustering (src/speaker_cluster.cpp, restated below), and
// resampling of non-16 kHz input (resample_audio, :87-106, :138-145: on the
// GPU by mwx_resample; the input is kept when resampling yields nothing, as
// the reference keeps it when libsamplerate fails, :141). Out of scope
// (SURVEY.md §8): VAD.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mwx.h"

namespace mwx_host {

// The Settings fields SttEngine reads (reference src/config.h:10-80 defaults).
struct Settings {
  std::string model_dir = "/models";
  std::string model_filename = "ggml-medium.bin";
  bool enable_vad = false;  // VAD is out of scope: must stay false
  int vad_ms_min_duration = 500;
  int n_threads = 4;
  int parallel_requests = 2;
  int request_queue_timeout_ms = 5000;
  std::string language = "auto";
  bool no_timestamps = false;
  int beam_size = 5;
  float temperature = 0.0f;
  int best_of = 5;
  float logprob_threshold = -0.7f;
  float no_speech_threshold = 0.85f;
  bool flash_attn = true;
  bool suppress_nst = true;
  int gpu_device = 0;
  int stream_buffer_samples = 8000;
  float cluster_threshold = 0.88f;  // src/config.h:71
  // Engine extension (no reference counterpart): dynamic request batching.
  // max_batch > 1: concurrent transcribe() calls with the same decoding
  // options are gathered (up to max_batch, waiting at most batch_window_us
  // for more) and run as one mwx_full_batch by one of parallel_requests
  // batcher threads. max_batch = 1 keeps the reference's one-request-per-
  // state path.
  int max_batch = 1;
  int batch_window_us = 2000;
};

struct TokenData {
  std::string text;
  float p;
  int64_t t0;
  int64_t t1;
};

// src/prosody_extractor.h:6-27
struct AffectiveTags {
  std::string gender_proxy;   // "M" / "F" / "?"
  std::string emotion_proxy;  // "excited" | "neutral" | "sad" | "angry"
  float arousal = 0.0f;
  float valence = 0.0f;
  float pitch_mean = 0.0f;
  float pitch_std = 0.0f;
  float energy_mean = 0.0f;
  float energy_std = 0.0f;
  float spectral_centroid = 0.0f;
  float zero_crossing_rate = 0.0f;
  std::vector<float> speaker_vec;  // 8-D
};

struct ProsodyOptions {
  float lpf_alpha = 0.07f;
  float gender_threshold = 170.0f;
  float min_pitch = 60.0f;
  float max_pitch = 500.0f;
};

// Online speaker clustering of segment speaker vectors (the reference's
// SpeakerClusterer, src/speaker_cluster.h:45-66 / .cpp:5-40): each vector
// joins the cluster of highest cosine similarity if that is >= threshold
// (running-mean centroid), else opens "spk_<n>". Clusters live in an
// std::unordered_map keyed by id, scanned in the map's order with ties kept
// by the first — the same container as the reference, hence the same order.
class SpeakerClusterer {
 public:
  explicit SpeakerClusterer(float threshold = 0.88f) : threshold_(threshold) {}
  std::string assign_or_add(const std::vector<float>& vec);

 private:
  struct Cluster {
    std::string id;
    std::vector<float> centroid;
    size_t count = 0;
  };
  float threshold_;
  std::unordered_map<std::string, Cluster> clusters_;
  int next_id_ = 0;
};

struct RequestOptions {
  std::string language;
  std::string prompt;
  bool translate = false;
  bool enable_diarization = false;
  float temperature = -1.0f;
  int beam_size = -1;
  int best_of = -1;
  ProsodyOptions prosody_opts;
  std::function<bool()> should_abort = nullptr;
};

struct TranscriptionResult {
  std::string text;
  std::string language;
  float prob;
  int64_t t0;
  int64_t t1;
  bool speaker_turn_next;
  std::vector<TokenData> tokens;
  int token_count = 0;
  std::string gender_proxy;
  std::string emotion_proxy;
  float arousal = 0.0f;
  float valence = 0.0f;
  AffectiveTags affective;
  std::string speaker_id;
};

class EngineBusyException : public std::runtime_error {
 public:
  explicit EngineBusyException(const std::string& msg) : std::runtime_error(msg) {}
};

class SttEngine {
 public:
  explicit SttEngine(const Settings& settings);  // throws std::runtime_error on load failure
  ~SttEngine();
  SttEngine(const SttEngine&) = delete;
  SttEngine& operator=(const SttEngine&) = delete;

  bool is_ready() const { return ctx_ != nullptr; }
  const Settings& get_settings() const { return settings_; }

  struct PerformanceMetrics {
    double queue_time_ms;
    double processing_time_ms;
    int token_count;
  };

  std::vector<TranscriptionResult> transcribe(const std::vector<float>& pcmf32,
                                              int input_sample_rate,
                                              const RequestOptions& options,
                                              PerformanceMetrics* out_metrics = nullptr);
  std::vector<TranscriptionResult> transcribe_pcm16(const std::vector<int16_t>& pcm16,
                                                    int input_sample_rate,
                                                    const RequestOptions& options,
                                                    PerformanceMetrics* out_metrics = nullptr);

  // Batched entry (no reference counterpart): B independent 16 kHz clips in
  // one GPU pass, each result list filtered exactly as transcribe() filters
  // it. Runs on states kept for batch calls (grown on demand, reused; one
  // batch call at a time).
  std::vector<std::vector<TranscriptionResult>> transcribe_batch(
      const std::vector<std::vector<float>>& clips, const RequestOptions& options);

  // SttEngine::resample_audio (src/stt_engine.cpp:87-106) on the GPU
  // (mwx_resample): empty when src_rate == target_rate, the input is empty or
  // resampling fails — the caller then keeps its input, as the reference does.
  std::vector<float> resample_audio(const float* input, size_t input_size, int src_rate,
                                    int target_rate);

  // Batches run by the request batcher so far (max_batch > 1).
  long batches_run() const { return batches_run_.load(); }

 private:
  // ---- dynamic request batching (Settings::max_batch > 1) ----
  struct Pending {
    const std::vector<float>* pcm;
    RequestOptions options;
    std::string key;  // requests with equal keys share mwx_full_params
    std::chrono::steady_clock::time_point t_enq;
    bool started = false, done = false, cancelled = false;
    int ret = 0;
    double t_start_ms = 0.0, t_proc_ms = 0.0;
    int token_count = 0;
    std::vector<TranscriptionResult> results;
  };
  std::vector<TranscriptionResult> transcribe_batched(const std::vector<float>& pcmf32,
                                                      const RequestOptions& options,
                                                      PerformanceMetrics* out_metrics);
  void batcher_loop(std::vector<mwx_state*> states);
  std::string options_key(const RequestOptions& o) const;
  std::deque<std::shared_ptr<Pending>> queue_;
  std::mutex q_mutex_;
  std::condition_variable q_cv_;     // batcher: new work / stop
  std::condition_variable done_cv_;  // callers: started / done
  std::vector<std::thread> batchers_;
  bool stop_ = false;
  std::atomic<long> batches_run_{0};

  mwx_state* acquire_state();
  void release_state(mwx_state* state);
  mwx_full_params make_params(const RequestOptions& options, std::string& target_lang,
                              std::function<bool()>& abort_fn) const;
  std::vector<TranscriptionResult> collect(mwx_state* state, const std::string& lang,
                                           const float* pcm, size_t pcm_size,
                                           const ProsodyOptions& popts, int* token_count) const;

  Settings settings_;
  mwx_context* ctx_ = nullptr;
  std::queue<mwx_state*> state_pool_;
  std::mutex pool_mutex_;
  std::condition_variable pool_cv_;
  std::vector<mwx_state*> all_states_;
  mwx_state* aux_state_ = nullptr;  // resampling (its own stream)
  std::mutex aux_mutex_;
  std::vector<mwx_state*> batch_states_;  // transcribe_batch
  std::mutex batch_mutex_;

  struct StateGuard {
    SttEngine& engine;
    mwx_state* state;
    explicit StateGuard(SttEngine& e) : engine(e) { state = engine.acquire_state(); }
    ~StateGuard() {
      if (state) engine.release_state(state);
    }
    mwx_state* get() { return state; }
  };
};

}  // namespace mwx_host
