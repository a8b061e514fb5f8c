// SttEngine over the mwx C ABI. See stt_engine.h for what is kept from the
// reference (file:line citations there and below).
#include "stt_engine.h"

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "text_filters.h"

namespace mwx_host {

namespace {

bool abort_trampoline(void* user_data) {
  auto* fn = static_cast<std::function<bool()>*>(user_data);
  return fn && *fn && (*fn)();
}

double ms_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

constexpr float kMinAvgTokenProb = 0.40f;  // src/stt_engine.cpp:264

}  // namespace

SttEngine::SttEngine(const Settings& settings) : settings_(settings) {
  const std::string path = settings_.model_dir + "/" + settings_.model_filename;
  mwx_context_params cp = mwx_context_default_params();
  cp.use_gpu = true;
  cp.flash_attn = settings_.flash_attn;
  cp.gpu_device = settings_.gpu_device;
  ctx_ = mwx_init_from_file_with_params(path.c_str(), cp);
  if (!ctx_) throw std::runtime_error("Whisper model initialization failed");
  const int pool = std::max(1, settings_.parallel_requests);
  for (int i = 0; i < pool; ++i) {
    mwx_state* st = mwx_init_state(ctx_);
    if (!st) throw std::runtime_error("Whisper state initialization failed");
    state_pool_.push(st);
    all_states_.push_back(st);
  }
}

SttEngine::~SttEngine() {
  for (mwx_state* st : all_states_) mwx_free_state(st);
  if (ctx_) mwx_free(ctx_);
}

mwx_state* SttEngine::acquire_state() {
  std::unique_lock<std::mutex> lock(pool_mutex_);
  const bool ok = pool_cv_.wait_for(lock,
                                    std::chrono::milliseconds(settings_.request_queue_timeout_ms),
                                    [this] { return !state_pool_.empty(); });
  if (!ok) throw EngineBusyException("Server is busy (Queue timeout)");
  mwx_state* st = state_pool_.front();
  state_pool_.pop();
  return st;
}

void SttEngine::release_state(mwx_state* state) {
  std::lock_guard<std::mutex> lock(pool_mutex_);
  state_pool_.push(state);
  pool_cv_.notify_one();
}

std::vector<TranscriptionResult> SttEngine::transcribe_pcm16(const std::vector<int16_t>& pcm16,
                                                             int input_sample_rate,
                                                             const RequestOptions& options,
                                                             PerformanceMetrics* out_metrics) {
  std::vector<float> f(pcm16.size());
  for (size_t i = 0; i < pcm16.size(); ++i) f[i] = static_cast<float>(pcm16[i]) / 32768.0f;
  return transcribe(f, input_sample_rate, options, out_metrics);
}

// Parameter mapping of src/stt_engine.cpp:204-243.
mwx_full_params SttEngine::make_params(const RequestOptions& options, std::string& target_lang,
                                       std::function<bool()>& abort_fn) const {
  const int beam = options.beam_size >= 0 ? options.beam_size : settings_.beam_size;
  const float temp = options.temperature >= 0.0f ? options.temperature : settings_.temperature;
  const int best_of = options.best_of >= 0 ? options.best_of : settings_.best_of;
  const int strategy = beam > 1 ? MWX_SAMPLING_BEAM_SEARCH : MWX_SAMPLING_GREEDY;
  mwx_full_params p = mwx_full_default_params(strategy);
  if (abort_fn) {
    p.abort_callback = abort_trampoline;
    p.abort_callback_user_data = &abort_fn;
  }
  p.print_realtime = false;
  p.print_progress = false;
  p.print_timestamps = !settings_.no_timestamps;
  p.print_special = false;
  p.token_timestamps = true;
  p.suppress_nst = settings_.suppress_nst;
  p.no_speech_thold = settings_.no_speech_threshold;
  p.translate = options.translate;
  p.tdrz_enable = options.enable_diarization;
  target_lang = options.language.empty() ? settings_.language : options.language;
  p.language = target_lang.c_str();
  if (!options.prompt.empty()) p.initial_prompt = options.prompt.c_str();
  p.temperature = temp;
  if (strategy == MWX_SAMPLING_BEAM_SEARCH)
    p.beam_search.beam_size = beam;
  else
    p.greedy.best_of = best_of;
  p.entropy_thold = 2.40f;
  p.logprob_thold = settings_.logprob_threshold;
  p.n_threads = settings_.n_threads;
  return p;
}

// Segment / token extraction and post-filters of src/stt_engine.cpp:258-337.
std::vector<TranscriptionResult> SttEngine::collect(mwx_state* state, const std::string& lang,
                                                    size_t pcm_size, int* token_count) const {
  std::vector<TranscriptionResult> results;
  const int eot = mwx_token_eot(ctx_);
  const int n_seg = mwx_full_n_segments_from_state(state);
  for (int i = 0; i < n_seg; ++i) {
    const char* tc = mwx_full_get_segment_text_from_state(state, i);
    std::string text = tc ? std::string(tc) : "";
    if (is_hallucination(text)) continue;
    const int64_t t0 = mwx_full_get_segment_t0_from_state(state, i);
    const int64_t t1 = mwx_full_get_segment_t1_from_state(state, i);
    const bool turn = mwx_full_get_segment_speaker_turn_next_from_state(state, i);
    std::vector<TokenData> tokens;
    double total_p = 0.0;
    int valid = 0;
    const int nt = mwx_full_n_tokens_from_state(state, i);
    for (int j = 0; j < nt; ++j) {
      const mwx_token_data d = mwx_full_get_token_data_from_state(state, i, j);
      if (d.id >= eot) continue;
      const char* ts = mwx_token_to_str(ctx_, d.id);
      tokens.push_back({std::string(ts ? ts : ""), d.p, d.t0, d.t1});
      total_p += d.p;
      ++valid;
    }
    if (token_count) *token_count += valid;
    const float avg = valid > 0 ? static_cast<float>(total_p / valid) : 0.0f;
    if (avg < kMinAvgTokenProb && valid > 0) continue;
    // segment sample range (src/stt_engine.cpp:313-321): consumed by the
    // prosody stage, which is out of scope; kept for the bounds behaviour
    int64_t s0 = static_cast<int64_t>((static_cast<double>(t0) / 100.0) * 16000.0);
    int64_t s1 = static_cast<int64_t>((static_cast<double>(t1) / 100.0) * 16000.0);
    s0 = std::max<int64_t>(0, std::min<int64_t>(s0, (int64_t)pcm_size));
    s1 = std::max<int64_t>(s0, std::min<int64_t>(s1, (int64_t)pcm_size));
    (void)s1;
    TranscriptionResult r;
    r.text = text;
    r.language = lang;
    r.prob = avg;
    r.t0 = t0;
    r.t1 = t1;
    r.speaker_turn_next = turn;
    r.tokens = std::move(tokens);
    r.token_count = valid;
    r.gender_proxy = "unknown";
    r.emotion_proxy = "neutral";
    r.speaker_id = "?";
    results.push_back(std::move(r));
  }
  return results;
}

std::vector<TranscriptionResult> SttEngine::transcribe(const std::vector<float>& pcmf32,
                                                       int input_sample_rate,
                                                       const RequestOptions& options,
                                                       PerformanceMetrics* out_metrics) {
  const auto t_start = std::chrono::steady_clock::now();
  if (!ctx_) return {};
  if (options.should_abort && options.should_abort()) return {};
  (void)input_sample_rate;  // non-16 kHz input is passed through (see header)
  const size_t pcm_size = pcmf32.size();
  const size_t min_samples = static_cast<size_t>((settings_.vad_ms_min_duration * 16000) / 1000);
  if (pcm_size < min_samples) {
    if (out_metrics) *out_metrics = {0.0, 0.0, 0};
    return {};
  }
  StateGuard guard(*this);
  mwx_state* state = guard.get();
  const auto t_acq = std::chrono::steady_clock::now();
  std::string lang;
  std::function<bool()> abort_fn = options.should_abort;
  const mwx_full_params p = make_params(options, lang, abort_fn);
  const int ret = mwx_full_with_state(ctx_, state, p, pcmf32.data(), static_cast<int>(pcm_size));
  const auto t_end = std::chrono::steady_clock::now();
  if (out_metrics) *out_metrics = {ms_between(t_start, t_acq), ms_between(t_acq, t_end), 0};
  if (ret != 0) {
    std::fprintf(stderr, options.should_abort && options.should_abort()
                             ? "Whisper processing aborted.\n"
                             : "Whisper processing failed: %d\n",
                 ret);
    return {};
  }
  return collect(state, lang, pcm_size, out_metrics ? &out_metrics->token_count : nullptr);
}

std::vector<std::vector<TranscriptionResult>> SttEngine::transcribe_batch(
    const std::vector<std::vector<float>>& clips, const RequestOptions& options) {
  std::vector<std::vector<TranscriptionResult>> out(clips.size());
  if (!ctx_ || clips.empty()) return out;
  std::vector<mwx_state*> states;
  std::vector<const float*> ptrs;
  std::vector<int> lens;
  for (const auto& c : clips) {
    mwx_state* st = mwx_init_state(ctx_);
    if (!st) {
      for (mwx_state* s : states) mwx_free_state(s);
      return out;
    }
    states.push_back(st);
    ptrs.push_back(c.data());
    lens.push_back(static_cast<int>(c.size()));
  }
  std::string lang;
  std::function<bool()> abort_fn = options.should_abort;
  const mwx_full_params p = make_params(options, lang, abort_fn);
  const int ret = mwx_full_batch(ctx_, states.data(), p, ptrs.data(), lens.data(),
                                 static_cast<int>(clips.size()));
  if (ret == 0) {
    const size_t min_samples = static_cast<size_t>((settings_.vad_ms_min_duration * 16000) / 1000);
    for (size_t b = 0; b < clips.size(); ++b)
      if (clips[b].size() >= min_samples) out[b] = collect(states[b], lang, clips[b].size(), nullptr);
  }
  for (mwx_state* s : states) mwx_free_state(s);
  return out;
}

}  // namespace mwx_host
