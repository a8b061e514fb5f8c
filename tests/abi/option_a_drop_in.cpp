// Compile-and-link check of INTEGRATION.md Option A: every whisper.h call the
// reference SttEngine makes (src/stt_engine.cpp:28-58 init / state pool,
// :210-246 parameter mapping and the whisper_full_with_state call, :258-293
// result extraction, src/main.cpp:71 log hook), written against mwx.h with
// the symbol map of INTEGRATION.md and the same parameter field names. Built by
// tests/test_abi.py (g++, linked against libmwx.so, not run: no GPU needed).
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "mwx.h"

namespace {

bool abort_wrapper(void* user_data) {  // src/stt_engine.cpp:17-23
  auto* fn = static_cast<std::function<bool()>*>(user_data);
  return fn && *fn && (*fn)();
}

void log_hook(enum mwx_log_level level, const char* text, void*) {  // src/main.cpp:37-55
  if (level <= MWX_LOG_LEVEL_WARN) std::fputs(text, stderr);
}

struct Word {
  std::string text;
  float p;
  int64_t t0, t1;
};
struct Result {
  std::string text;
  int64_t t0, t1;
  bool speaker_turn_next;
  std::vector<Word> words;
};

}  // namespace

int transcribe_like_reference(const char* model_path, const std::vector<float>& pcm,
                              int beam_size, float temperature, int best_of,
                              const std::string& language, const std::string& prompt,
                              bool translate, bool diarize, int n_threads,
                              std::function<bool()> should_abort, std::vector<Result>& out) {
  mwx_log_set(log_hook, nullptr);
  mwx_context_params cparams = mwx_context_default_params();
  cparams.use_gpu = true;
  cparams.gpu_device = 0;
  mwx_context* ctx = mwx_init_from_file_with_params(model_path, cparams);
  if (!ctx) return -1;
  mwx_state* state = mwx_init_state(ctx);
  if (!state) {
    mwx_free(ctx);
    return -1;
  }
  const int strategy = beam_size > 1 ? MWX_SAMPLING_BEAM_SEARCH : MWX_SAMPLING_GREEDY;
  mwx_full_params wparams = mwx_full_default_params(strategy);
  if (should_abort) {
    wparams.abort_callback = abort_wrapper;
    wparams.abort_callback_user_data = &should_abort;
  }
  wparams.print_realtime = false;
  wparams.print_progress = false;
  wparams.print_timestamps = true;
  wparams.print_special = false;
  wparams.token_timestamps = true;
  wparams.suppress_nst = true;
  wparams.no_speech_thold = 0.85f;
  wparams.translate = translate;
  wparams.tdrz_enable = diarize;
  wparams.language = language.c_str();
  if (!prompt.empty()) wparams.initial_prompt = prompt.c_str();
  wparams.temperature = temperature;
  if (strategy == MWX_SAMPLING_BEAM_SEARCH)
    wparams.beam_search.beam_size = beam_size;
  else
    wparams.greedy.best_of = best_of;
  wparams.entropy_thold = 2.40f;
  wparams.logprob_thold = -0.7f;
  wparams.n_threads = n_threads;
  const int ret = mwx_full_with_state(ctx, state, wparams, pcm.data(), (int)pcm.size());
  if (ret == 0) {
    const int n_seg = mwx_full_n_segments_from_state(state);
    for (int i = 0; i < n_seg; ++i) {
      Result r;
      r.text = mwx_full_get_segment_text_from_state(state, i);
      r.t0 = mwx_full_get_segment_t0_from_state(state, i);
      r.t1 = mwx_full_get_segment_t1_from_state(state, i);
      r.speaker_turn_next = mwx_full_get_segment_speaker_turn_next_from_state(state, i);
      const int n_tok = mwx_full_n_tokens_from_state(state, i);
      for (int j = 0; j < n_tok; ++j) {
        const mwx_token_data td = mwx_full_get_token_data_from_state(state, i, j);
        if (td.id >= mwx_token_eot(ctx)) continue;  // src/stt_engine.cpp:292
        r.words.push_back({mwx_token_to_str(ctx, td.id), td.p, td.t0, td.t1});
      }
      out.push_back(r);
    }
  }
  mwx_free_state(state);
  mwx_free(ctx);
  return ret;
}

// (linked, not run: the check is that it compiles and every symbol resolves)
int main(int argc, char** argv) {
  if (argc < 99) return 0;
  std::vector<Result> out;
  return transcribe_like_reference(argv[1], std::vector<float>(16000), 5, 0.0f, 5, "auto", "",
                                   false, false, 4, nullptr, out);
}
