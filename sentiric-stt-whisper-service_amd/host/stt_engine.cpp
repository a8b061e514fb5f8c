// SttEngine over the mwx C ABI. See stt_engine.h for what is kept from the
// reference (file:line citations there and below).
#include "stt_engine.h"

#include <algorithm>
#include <chrono>
#include <cmath>
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

float cosine_sim(const std::vector<float>& a, const std::vector<float>& b) {
  float dot = 0.0f, na = 0.0f, nb = 0.0f;  // one pass, in index order
  for (size_t i = 0; i < a.size(); ++i) {
    dot += a[i] * b[i];
    na += a[i] * a[i];
    nb += b[i] * b[i];
  }
  if (na == 0.0f || nb == 0.0f) return 0.0f;
  return dot / (std::sqrt(na) * std::sqrt(nb));
}

AffectiveTags to_tags(const mwx_prosody& p) {
  static const char* kGender[] = {"?", "M", "F"};
  static const char* kEmotion[] = {"neutral", "excited", "angry", "sad"};
  AffectiveTags t;
  t.gender_proxy = kGender[p.gender];
  t.emotion_proxy = kEmotion[p.emotion];
  t.arousal = p.arousal;
  t.valence = p.valence;
  t.pitch_mean = p.pitch_mean;
  t.pitch_std = p.pitch_std;
  t.energy_mean = p.energy_mean;
  t.energy_std = p.energy_std;
  t.spectral_centroid = p.spectral_centroid;
  t.zero_crossing_rate = p.zero_crossing_rate;
  t.speaker_vec.assign(p.speaker_vec, p.speaker_vec + 8);
  return t;
}

}  // namespace

std::string SpeakerClusterer::assign_or_add(const std::vector<float>& vec) {
  const Cluster* best = nullptr;
  float best_sim = 0.0f;
  for (const auto& kv : clusters_) {
    const float sim = cosine_sim(vec, kv.second.centroid);
    if (sim > best_sim) {
      best_sim = sim;
      best = &kv.second;
    }
  }
  if (best && best_sim >= threshold_) {
    Cluster& c = clusters_[best->id];
    const size_t n = c.count;
    for (size_t i = 0; i < c.centroid.size(); ++i)
      c.centroid[i] = (c.centroid[i] * n + vec[i]) / (n + 1);
    c.count = n + 1;
    return c.id;
  }
  Cluster fresh;
  fresh.id = "spk_" + std::to_string(next_id_++);
  fresh.centroid = vec;
  fresh.count = 1;
  const std::string id = fresh.id;
  clusters_[id] = std::move(fresh);
  return id;
}

SttEngine::SttEngine(const Settings& settings) : settings_(settings) {
  const std::string path = settings_.model_dir + "/" + settings_.model_filename;
  mwx_context_params cp = mwx_context_default_params();
  cp.use_gpu = true;
  cp.flash_attn = settings_.flash_attn;
  cp.gpu_device = settings_.gpu_device;
  ctx_ = mwx_init_from_file_with_params(path.c_str(), cp);
  if (!ctx_) throw std::runtime_error("Whisper model initialization failed");
  aux_state_ = mwx_init_state(ctx_);
  if (!aux_state_) throw std::runtime_error("Whisper state initialization failed");
  all_states_.push_back(aux_state_);
  const int pool = std::max(1, settings_.parallel_requests);
  if (settings_.max_batch > 1) {
    // one batcher thread per pool slot, each with its own max_batch states
    for (int i = 0; i < pool; ++i) {
      std::vector<mwx_state*> sts;
      for (int b = 0; b < settings_.max_batch; ++b) {
        mwx_state* st = mwx_init_state(ctx_);
        if (!st) throw std::runtime_error("Whisper state initialization failed");
        sts.push_back(st);
        all_states_.push_back(st);
      }
      batchers_.emplace_back(&SttEngine::batcher_loop, this, sts);
    }
    return;
  }
  for (int i = 0; i < pool; ++i) {
    mwx_state* st = mwx_init_state(ctx_);
    if (!st) throw std::runtime_error("Whisper state initialization failed");
    state_pool_.push(st);
    all_states_.push_back(st);
  }
}

SttEngine::~SttEngine() {
  {
    std::lock_guard<std::mutex> lock(q_mutex_);
    stop_ = true;
  }
  q_cv_.notify_all();
  for (auto& t : batchers_) t.join();
  for (mwx_state* st : all_states_) mwx_free_state(st);
  if (ctx_) mwx_free(ctx_);
}

// Everything make_params reads from the request: equal keys -> identical
// mwx_full_params, so those requests can share one mwx_full_batch.
std::string SttEngine::options_key(const RequestOptions& o) const {
  const int beam = o.beam_size >= 0 ? o.beam_size : settings_.beam_size;
  const float temp = o.temperature >= 0.0f ? o.temperature : settings_.temperature;
  const int best_of = o.best_of >= 0 ? o.best_of : settings_.best_of;
  const std::string lang = o.language.empty() ? settings_.language : o.language;
  char buf[96];
  std::snprintf(buf, sizeof buf, "%d|%.9g|%d|%d|%d|", beam, temp, best_of, (int)o.translate,
                (int)o.enable_diarization);
  return std::string(buf) + lang + "|" + o.prompt;
}

std::vector<TranscriptionResult> SttEngine::transcribe_batched(const std::vector<float>& pcmf32,
                                                               const RequestOptions& options,
                                                               PerformanceMetrics* out_metrics) {
  auto req = std::make_shared<Pending>();
  req->pcm = &pcmf32;
  req->options = options;
  req->key = options_key(options);
  req->t_enq = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lock(q_mutex_);
  queue_.push_back(req);
  // every batcher: one already gathering another key would swallow a single
  // wakeup while an idle batcher sleeps
  q_cv_.notify_all();
  // EngineBusyException when no batcher picks the request up in time
  // (the state-pool queue timeout of src/stt_engine.cpp:63-85)
  if (!done_cv_.wait_for(lock, std::chrono::milliseconds(settings_.request_queue_timeout_ms),
                         [&] { return req->started; })) {
    req->cancelled = true;
    for (auto it = queue_.begin(); it != queue_.end(); ++it)
      if (*it == req) {
        queue_.erase(it);
        break;
      }
    throw EngineBusyException("Server is busy (Queue timeout)");
  }
  done_cv_.wait(lock, [&] { return req->done; });
  if (out_metrics) *out_metrics = {req->t_start_ms, req->t_proc_ms, req->token_count};
  if (req->ret != 0) {
    std::fprintf(stderr, "Whisper processing failed: %d\n", req->ret);
    return {};
  }
  return std::move(req->results);
}

void SttEngine::batcher_loop(std::vector<mwx_state*> states) {
  const int max_b = (int)states.size();
  while (true) {
    std::vector<std::shared_ptr<Pending>> batch;
    {
      std::unique_lock<std::mutex> lock(q_mutex_);
      q_cv_.wait(lock, [&] { return stop_ || !queue_.empty(); });
      if (stop_) return;
      // gather: wait up to batch_window_us for more requests of this key
      const auto deadline = queue_.front()->t_enq +
                            std::chrono::microseconds(settings_.batch_window_us);
      const std::string key = queue_.front()->key;
      auto count = [&] {
        int c = 0;
        for (auto& r : queue_) c += r->key == key;
        return c;
      };
      while (!stop_ && count() < max_b &&
             q_cv_.wait_until(lock, deadline) != std::cv_status::timeout) {
      }
      if (stop_) return;
      for (auto it = queue_.begin(); it != queue_.end() && (int)batch.size() < max_b;) {
        if ((*it)->key == key) {
          (*it)->started = true;
          batch.push_back(*it);
          it = queue_.erase(it);
        } else {
          ++it;
        }
      }
      // requests left behind (other keys, or beyond max_batch) go to an idle
      // batcher now rather than after this batch
      if (!queue_.empty()) q_cv_.notify_all();
    }
    done_cv_.notify_all();
    if (batch.empty()) continue;
    const auto t0 = std::chrono::steady_clock::now();
    std::string lang;
    // the batch is aborted only when every request in it asks to abort
    std::function<bool()> abort_fn = nullptr;
    bool any_abort = false;
    for (auto& r : batch) any_abort |= (bool)r->options.should_abort;
    if (any_abort)
      abort_fn = [&batch] {
        for (auto& r : batch)
          if (!r->options.should_abort || !r->options.should_abort()) return false;
        return true;
      };
    const mwx_full_params p = make_params(batch[0]->options, lang, abort_fn);
    std::vector<const float*> ptrs;
    std::vector<int> lens;
    for (auto& r : batch) {
      ptrs.push_back(r->pcm->data());
      lens.push_back((int)r->pcm->size());
    }
    const int ret = mwx_full_batch(ctx_, states.data(), p, ptrs.data(), lens.data(), (int)batch.size());
    const auto t1 = std::chrono::steady_clock::now();
    batches_run_++;
    for (size_t b = 0; b < batch.size(); ++b) {
      auto& r = *batch[b];
      r.ret = ret;
      r.t_start_ms = ms_between(r.t_enq, t0);
      r.t_proc_ms = ms_between(t0, t1);
      if (ret == 0) {
        try {
          r.results = collect(states[b], lang, r.pcm->data(), r.pcm->size(),
                              r.options.prosody_opts, &r.token_count);
        } catch (const std::exception& e) {
          std::fprintf(stderr, "SttEngine: %s\n", e.what());
          r.ret = -100;
        }
      }
    }
    {
      std::lock_guard<std::mutex> lock(q_mutex_);
      for (auto& r : batch) r->done = true;
    }
    done_cv_.notify_all();
  }
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
                                                    const float* pcm, size_t pcm_size,
                                                    const ProsodyOptions& popts,
                                                    int* token_count) const {
  std::vector<TranscriptionResult> results;
  std::vector<int64_t> seg_start, seg_len;
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
    // segment sample range (src/stt_engine.cpp:313-321)
    int64_t s0 = static_cast<int64_t>((static_cast<double>(t0) / 100.0) * 16000.0);
    int64_t s1 = static_cast<int64_t>((static_cast<double>(t1) / 100.0) * 16000.0);
    s0 = std::max<int64_t>(0, std::min<int64_t>(s0, (int64_t)pcm_size));
    s1 = std::max<int64_t>(s0, std::min<int64_t>(s1, (int64_t)pcm_size));
    seg_start.push_back(s0);
    seg_len.push_back(s1 - s0);
    TranscriptionResult r;
    r.text = text;
    r.language = lang;
    r.prob = avg;
    r.t0 = t0;
    r.t1 = t1;
    r.speaker_turn_next = turn;
    r.tokens = std::move(tokens);
    r.token_count = valid;
    results.push_back(std::move(r));
  }
  // prosody of every kept segment in one GPU launch, then speaker clustering
  // in segment order (src/stt_engine.cpp:323-337); segments shorter than 160
  // samples get the empty-input tags and speaker "?"
  std::vector<mwx_prosody> pros(results.size());
  if (!results.empty()) {
    mwx_prosody_params pp;
    pp.lpf_alpha = popts.lpf_alpha;
    pp.gender_threshold = popts.gender_threshold;
    pp.min_pitch = popts.min_pitch;
    pp.max_pitch = popts.max_pitch;
    const int rc = mwx_prosody_batch(ctx_, state, pcm, (int64_t)pcm_size, seg_start.data(),
                                     seg_len.data(), (int)results.size(), 16000, &pp, pros.data());
    if (rc != 0) throw std::runtime_error("mwx_prosody_batch failed");
  }
  SpeakerClusterer clusterer(settings_.cluster_threshold);
  for (size_t i = 0; i < results.size(); ++i) {
    TranscriptionResult& r = results[i];
    r.affective = to_tags(pros[i]);
    r.gender_proxy = r.affective.gender_proxy;
    r.emotion_proxy = r.affective.emotion_proxy;
    r.arousal = r.affective.arousal;
    r.valence = r.affective.valence;
    r.speaker_id = seg_len[i] < 160 ? "?" : clusterer.assign_or_add(r.affective.speaker_vec);
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
  // src/stt_engine.cpp:136-145: non-16 kHz input is resampled; an empty
  // result (failure) keeps the original buffer. One pass, as the reference
  // swaps its pcm pointer: the abort callback is polled once above and
  // processing_time_ms includes the resampling.
  std::vector<float> resampled;
  if (input_sample_rate != 16000)
    resampled = resample_audio(pcmf32.data(), pcmf32.size(), input_sample_rate, 16000);
  const std::vector<float>& pcm = resampled.empty() ? pcmf32 : resampled;
  const size_t pcm_size = pcm.size();
  const size_t min_samples = static_cast<size_t>((settings_.vad_ms_min_duration * 16000) / 1000);
  if (pcm_size < min_samples) {
    if (out_metrics) *out_metrics = {0.0, 0.0, 0};
    return {};
  }
  if (settings_.max_batch > 1) return transcribe_batched(pcm, options, out_metrics);
  StateGuard guard(*this);
  mwx_state* state = guard.get();
  const auto t_acq = std::chrono::steady_clock::now();
  std::string lang;
  std::function<bool()> abort_fn = options.should_abort;
  const mwx_full_params p = make_params(options, lang, abort_fn);
  const int ret = mwx_full_with_state(ctx_, state, p, pcm.data(), static_cast<int>(pcm_size));
  const auto t_end = std::chrono::steady_clock::now();
  if (out_metrics) *out_metrics = {ms_between(t_start, t_acq), ms_between(t_acq, t_end), 0};
  if (ret != 0) {
    std::fprintf(stderr, options.should_abort && options.should_abort()
                             ? "Whisper processing aborted.\n"
                             : "Whisper processing failed: %d\n",
                 ret);
    return {};
  }
  return collect(state, lang, pcm.data(), pcm_size, options.prosody_opts,
                 out_metrics ? &out_metrics->token_count : nullptr);
}

std::vector<float> SttEngine::resample_audio(const float* input, size_t input_size, int src_rate,
                                             int target_rate) {
  if (src_rate == target_rate || input_size == 0) return {};
  const long cap = mwx_resample_max_frames(static_cast<int>(input_size), src_rate, target_rate);
  if (cap <= 0) return {};
  std::vector<float> out(static_cast<size_t>(cap));
  int n = 0;
  {
    std::lock_guard<std::mutex> lock(aux_mutex_);
    n = mwx_resample(ctx_, aux_state_, input, static_cast<int>(input_size), src_rate, target_rate,
                     out.data(), static_cast<int>(cap));
  }
  if (n <= 0) {
    std::fprintf(stderr, "SttEngine: resampling %d -> %d Hz failed (%d)\n", src_rate, target_rate, n);
    return {};
  }
  out.resize(static_cast<size_t>(n));
  return out;
}

std::vector<std::vector<TranscriptionResult>> SttEngine::transcribe_batch(
    const std::vector<std::vector<float>>& clips, const RequestOptions& options) {
  std::vector<std::vector<TranscriptionResult>> out(clips.size());
  if (!ctx_ || clips.empty()) return out;
  std::lock_guard<std::mutex> batch_lock(batch_mutex_);
  while (batch_states_.size() < clips.size()) {
    mwx_state* st = mwx_init_state(ctx_);
    if (!st) return out;
    batch_states_.push_back(st);
    all_states_.push_back(st);
  }
  std::vector<mwx_state*> states(batch_states_.begin(), batch_states_.begin() + clips.size());
  std::vector<const float*> ptrs;
  std::vector<int> lens;
  for (const auto& c : clips) {
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
      if (clips[b].size() >= min_samples)
        out[b] = collect(states[b], lang, clips[b].data(), clips[b].size(), options.prosody_opts,
                         nullptr);
  }
  return out;
}

}  // namespace mwx_host
