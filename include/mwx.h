/*
 * mwx.h — C ABI of the MI355X-native Whisper engine.
 *
 * This is the drop-in boundary for the hot path of sentiric-stt-whisper-service.
 * The service's SttEngine (src/stt_engine.cpp) binds the whisper.h subset listed
 * below; every entry point here replaces exactly one of those symbols with the
 * same argument meaning, ownership and error behaviour. Reference call sites
 * (paths relative to the reference repository):
 *
 *   mwx_context_default_params            <- whisper_context_default_params      src/stt_engine.cpp:28
 *   mwx_init_from_file_with_params        <- whisper_init_from_file_with_params  src/stt_engine.cpp:33
 *   mwx_init_state                        <- whisper_init_state                  src/stt_engine.cpp:39
 *   mwx_free_state / mwx_free             <- whisper_free_state / whisper_free   src/stt_engine.cpp:56-57
 *   mwx_full_default_params               <- whisper_full_default_params         src/stt_engine.cpp:214
 *   mwx_full_with_state                   <- whisper_full_with_state             src/stt_engine.cpp:245-246
 *   mwx_full_n_segments_from_state        <- whisper_full_n_segments_from_state  src/stt_engine.cpp:261
 *   mwx_full_get_segment_text_from_state  <- whisper_full_get_segment_text_from_state   :267
 *   mwx_full_get_segment_t0/t1_from_state <- whisper_full_get_segment_t0/t1_from_state  :278-279
 *   mwx_full_get_segment_speaker_turn_next_from_state <- whisper_..._speaker_turn_next  :280-281
 *   mwx_full_n_tokens_from_state          <- whisper_full_n_tokens_from_state    src/stt_engine.cpp:284
 *   mwx_full_get_token_data_from_state    <- whisper_full_get_token_data_from_state :288
 *   mwx_token_to_str                      <- whisper_token_to_str                src/stt_engine.cpp:289
 *   mwx_token_eot                         <- whisper_token_eot                   src/stt_engine.cpp:290
 *   mwx_log_set                           <- whisper_log_set                     src/main.cpp:71
 *   mwx_resample                          <- SttEngine::resample_audio (libsamplerate
 *                                            src_simple, SRC_SINC_FASTEST) src/stt_engine.cpp:87-106
 *
 * New (no whisper.h counterpart): mwx_full_batch runs B independent clips in one
 * batched GPU pass (the data-parallel unit of this engine), and
 * mwx_write_synthetic_model writes a seeded model in the ggml .bin layout that
 * src/model_manager.cpp provisions (no real checkpoints exist offline).
 *
 * Conventions: plain C, no exceptions cross this boundary, all functions return
 * NULL / negative on failure (0 = success), strings returned by getters stay
 * valid until the next mwx_full* call on the same state.
 */
#ifndef MWX_H
#define MWX_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MWX_SAMPLE_RATE 16000
#define MWX_N_FFT 400
#define MWX_HOP_LENGTH 160
#define MWX_CHUNK_SIZE 30
#define MWX_MAX_DECODERS 8

typedef int32_t mwx_token;
struct mwx_context;
struct mwx_state;

/* ggml_log_level-compatible levels (src/main.cpp:37-55 switches on these). */
enum mwx_log_level {
  MWX_LOG_LEVEL_NONE = 0,
  MWX_LOG_LEVEL_DEBUG = 1,
  MWX_LOG_LEVEL_INFO = 2,
  MWX_LOG_LEVEL_WARN = 3,
  MWX_LOG_LEVEL_ERROR = 4,
  MWX_LOG_LEVEL_CONT = 5,
};
typedef void (*mwx_log_callback)(enum mwx_log_level level, const char* text,
                                 void* user_data);

struct mwx_context_params {
  bool use_gpu;     /* must be true: the engine has no CPU path */
  bool flash_attn;  /* accepted for API parity; attention is always fused */
  int gpu_device;   /* HIP device ordinal */
  /* Engine extension: MWX_COMPUTE_MXFP8 runs the encoder and cross-K/V GEMMs
   * on MX-fp8 operands (e4m3 + one E8M0 scale per 32 k; weights quantized at
   * load, activations by the producer step) with gfx950's block-scaled fp8
   * MFMA. MWX_COMPUTE_MODEL (default) computes in the model's 16-bit type. */
  int compute;
};
enum mwx_compute {
  MWX_COMPUTE_MODEL = 0,
  MWX_COMPUTE_MXFP8 = 1,
};

enum mwx_sampling_strategy {
  MWX_SAMPLING_GREEDY = 0,
  MWX_SAMPLING_BEAM_SEARCH = 1,
};

typedef bool (*mwx_abort_callback)(void* user_data);

/* Same fields and meaning as whisper_token_data. */
typedef struct mwx_token_data {
  mwx_token id;  /* token id */
  mwx_token tid; /* forced timestamp token id */
  float p;       /* probability of the token */
  float plog;    /* log probability of the token */
  float pt;      /* probability of the timestamp token */
  float ptsum;   /* sum of probabilities of all timestamp tokens */
  int64_t t0;    /* token-level timestamps (10 ms units), -1 if unset */
  int64_t t1;
  int64_t t_dtw;
  float vlen; /* voice length of the token */
} mwx_token_data;

/* Mirrors the whisper_full_params fields the service sets or relies on
 * (src/stt_engine.cpp:214-243) plus the upstream defaults it inherits. */
struct mwx_full_params {
  int strategy;
  int n_threads;
  int n_max_text_ctx;
  int offset_ms;
  int duration_ms;

  bool translate;
  bool no_context;
  bool no_timestamps;
  bool single_segment;
  bool print_special;
  bool print_progress;
  bool print_realtime;
  bool print_timestamps;

  bool token_timestamps;
  float thold_pt;
  float thold_ptsum;
  int max_len;
  bool split_on_word;
  int max_tokens;

  int audio_ctx;
  bool tdrz_enable;

  const char* initial_prompt;
  const mwx_token* prompt_tokens;
  int prompt_n_tokens;

  const char* language;
  bool detect_language;

  bool suppress_blank;
  bool suppress_nst;

  float temperature;
  float max_initial_ts;
  float length_penalty;
  float temperature_inc;
  float entropy_thold;
  float logprob_thold;
  float no_speech_thold;

  struct {
    int best_of;
  } greedy;
  struct {
    int beam_size;
    float patience;
  } beam_search;

  mwx_abort_callback abort_callback;
  void* abort_callback_user_data;

  /* Engine extension (benchmark workload only): when > 0 every 30-s window of
   * every clip is decoded for exactly this many steps (greedy or beam) with EOT
   * and timestamp tokens suppressed, and the clip then advances by a whole
   * window, so each window costs the same fixed number of decode steps and a
   * long clip runs window after window. */
  int bench_fixed_steps;
};

/* --- lifecycle --------------------------------------------------------- */
struct mwx_context_params mwx_context_default_params(void);
struct mwx_context* mwx_init_from_file_with_params(
    const char* path_model, struct mwx_context_params params);
struct mwx_state* mwx_init_state(struct mwx_context* ctx);
void mwx_free_state(struct mwx_state* state);
void mwx_free(struct mwx_context* ctx);

/* --- inference --------------------------------------------------------- */
struct mwx_full_params mwx_full_default_params(int strategy);

/* Returns 0 on success, <0 on failure (same codes as whisper_full_with_state). */
int mwx_full_with_state(struct mwx_context* ctx, struct mwx_state* state,
                        struct mwx_full_params params, const float* samples,
                        int n_samples);

/* Batched variant: clip b (f32 PCM @16 kHz, n_samples[b] samples) is decoded
 * into states[b]. All clips share params. Returns 0 or the first error.
 * samples[b] may be host memory or device memory of the context's GPU
 * (HBM-resident input: copied device-to-device, no PCIe transfer). */
int mwx_full_batch(struct mwx_context* ctx, struct mwx_state* const* states,
                   struct mwx_full_params params,
                   const float* const* samples, const int* n_samples,
                   int n_clips);

/* As mwx_full_batch with 16-bit PCM (host or device memory), converted on
 * the device exactly as SttEngine::transcribe_pcm16 converts it (x / 32768,
 * src/stt_engine.cpp:123): half the bytes over PCIe. */
int mwx_full_batch_pcm16(struct mwx_context* ctx, struct mwx_state* const* states,
                         struct mwx_full_params params, const int16_t* const* samples,
                         const int* n_samples, int n_clips);

/* Device input buffers on the context's GPU (for mwx_full_batch over
 * HBM-resident PCM): allocate n floats, upload n floats from host memory
 * (synchronous), free. NULL / <0 on failure. */
float* mwx_device_buffer(struct mwx_context* ctx, size_t n);
int mwx_device_upload(struct mwx_context* ctx, float* dst, const float* src, size_t n);
void mwx_device_buffer_free(struct mwx_context* ctx, float* p);

/* --- results ------------------------------------------------------------ */
int mwx_full_n_segments_from_state(struct mwx_state* state);
const char* mwx_full_get_segment_text_from_state(struct mwx_state* state,
                                                 int i_segment);
int64_t mwx_full_get_segment_t0_from_state(struct mwx_state* state,
                                           int i_segment);
int64_t mwx_full_get_segment_t1_from_state(struct mwx_state* state,
                                           int i_segment);
bool mwx_full_get_segment_speaker_turn_next_from_state(struct mwx_state* state,
                                                       int i_segment);
float mwx_full_get_segment_no_speech_prob_from_state(struct mwx_state* state,
                                                     int i_segment);
int mwx_full_n_tokens_from_state(struct mwx_state* state, int i_segment);
mwx_token_data mwx_full_get_token_data_from_state(struct mwx_state* state,
                                                  int i_segment, int i_token);
int mwx_full_lang_id_from_state(struct mwx_state* state);

/* --- segment prosody -----------------------------------------------------
 * The reference's per-segment affect / speaker features
 * (src/prosody_extractor.h:6-31 AffectiveTags, ProsodyOptions; computed by
 * extract_prosody for every kept segment, src/stt_engine.cpp:313-337) on the
 * GPU, bit-identical to the reference's CPU build. */
typedef struct mwx_prosody_params { /* ProsodyOptions, same defaults */
  float lpf_alpha;                  /* 0.07 */
  float gender_threshold;           /* 170 Hz */
  float min_pitch;                  /* 60 Hz */
  float max_pitch;                  /* 500 Hz */
} mwx_prosody_params;

enum mwx_gender { MWX_GENDER_UNKNOWN = 0 /* "?" */, MWX_GENDER_M = 1, MWX_GENDER_F = 2 };
enum mwx_emotion {
  MWX_EMOTION_NEUTRAL = 0,
  MWX_EMOTION_EXCITED = 1,
  MWX_EMOTION_ANGRY = 2,
  MWX_EMOTION_SAD = 3
};

typedef struct mwx_prosody { /* AffectiveTags */
  float pitch_mean, pitch_std, energy_mean, energy_std, spectral_centroid,
      zero_crossing_rate, arousal, valence;
  float speaker_vec[8];
  int gender;      /* enum mwx_gender (gender_proxy) */
  int emotion;     /* enum mwx_emotion (emotion_proxy) */
  int serial_runs; /* diagnostics: filter runs recomputed serially */
  int reserved;
} mwx_prosody;

mwx_prosody_params mwx_prosody_default_params(void);

/* Prosody of n_seg segments [seg_start[i], seg_start[i] + seg_len[i]) of one
 * PCM buffer (host or device memory, n_pcm samples at sample_rate, 100 <=
 * sample_rate <= 160000). A segment shorter than 160 samples gets the
 * reference's empty-input result (extract_prosody(nullptr, 0, ...)). Runs on
 * the state's stream; synchronous. 0 on success, <0 on bad arguments or a
 * device error. */
int mwx_prosody_batch(struct mwx_context* ctx, struct mwx_state* state, const float* pcm,
                      int64_t n_pcm, const int64_t* seg_start, const int64_t* seg_len,
                      int n_seg, int sample_rate, const mwx_prosody_params* params,
                      mwx_prosody* out);

/* As mwx_prosody_batch with every array in device memory (no host copies, no
 * synchronization: the results are ready when the state's stream is). For
 * throughput measurement over HBM-resident inputs. d_desc holds n_seg int64
 * triples {start, len, frame_offset}: frame_offset = the sum of
 * len / (sample_rate / 100) over the segments before it; total_frames = that
 * sum over all n_seg. */
int mwx_prosody_batch_device(struct mwx_context* ctx, struct mwx_state* state,
                             const float* d_pcm, const int64_t* d_desc, int n_seg,
                             int64_t total_frames, int sample_rate,
                             const mwx_prosody_params* params, mwx_prosody* d_out);

/* --- resampling -------------------------------------------------------------
 * SttEngine::resample_audio (src/stt_engine.cpp:87-106, called for every
 * request whose sample rate is not 16 kHz, :138-145): libsamplerate's
 * src_simple(SRC_SINC_FASTEST, mono, end_of_input = 0) restated on the GPU —
 * the same output count (the converter holds back the last filter half-width
 * of input) and alignment; the coefficient table is a reconstruction of the
 * "fastest" table's geometry (libsamplerate is absent, parity unpinned).
 * `in` / `out` may be host or device memory of the context's GPU. Returns the
 * frames generated (the reference's output_frames_gen; 0 when
 * src_rate == dst_rate or n_in == 0, where the reference keeps the input), or
 * < 0 on bad arguments / a ratio outside libsamplerate's [1/256, 256] / a
 * device error. Runs on the state's stream; synchronous. */
long mwx_resample_max_frames(int n_in, int src_rate, int dst_rate); /* (long)(n_in*ratio)+100 */
int mwx_resample(struct mwx_context* ctx, struct mwx_state* state, const float* in, int n_in,
                 int src_rate, int dst_rate, float* out, int out_cap);

/* --- vocabulary / model ------------------------------------------------- */
const char* mwx_token_to_str(struct mwx_context* ctx, mwx_token token);
mwx_token mwx_token_eot(struct mwx_context* ctx);
mwx_token mwx_token_sot(struct mwx_context* ctx);
mwx_token mwx_token_beg(struct mwx_context* ctx);
mwx_token mwx_token_not(struct mwx_context* ctx);
mwx_token mwx_token_nosp(struct mwx_context* ctx);
mwx_token mwx_token_transcribe(struct mwx_context* ctx);
mwx_token mwx_token_translate(struct mwx_context* ctx);
mwx_token mwx_token_lang(struct mwx_context* ctx, int lang_id);
int mwx_n_vocab(struct mwx_context* ctx);
int mwx_n_text_ctx(struct mwx_context* ctx);
int mwx_n_audio_ctx(struct mwx_context* ctx);
int mwx_n_mels(struct mwx_context* ctx);
int mwx_is_multilingual(struct mwx_context* ctx);
int mwx_model_wtype(struct mwx_context* ctx); /* 1 = f16, 30 = bf16 */
int mwx_lang_id(const char* lang);
const char* mwx_lang_str(int id);
int mwx_lang_max_id(void);
/* Greedy longest-match tokenizer (whisper_tokenize semantics). Returns the
 * number of tokens, or -(needed) if n_max_tokens is too small. */
int mwx_tokenize(struct mwx_context* ctx, const char* text, mwx_token* tokens,
                 int n_max_tokens);

void mwx_log_set(mwx_log_callback log_callback, void* user_data);

/* --- measurement ------------------------------------------------------------
 * Times every launch of one kernel class with a pair of HIP events recorded on
 * the state's stream (the stream the kernels run on). Classes: "mel",
 * "enc_gemm", "enc_attn", "cross_gemm", "dec_gemm", "dec_attn_self",
 * "dec_attn_cross", "logits_gemm", "logits_proc", "prosody". NULL disables.
 * mwx_perf_read synchronizes, returns the summed milliseconds and the launch
 * count since the last read, and resets them. */
void mwx_perf_enable(struct mwx_state* state, const char* kernel_class);
int mwx_perf_read(struct mwx_state* state, double* total_ms, int* launches);
/* Several classes may be enabled at once as a comma-separated list;
 * mwx_perf_read reads the first, mwx_perf_read_class any of them. Launches
 * inside the decode-step graph are timed on every 8th step (MWX_PERF_PERIOD). */
int mwx_perf_read_class(struct mwx_state* state, const char* kernel_class, double* total_ms,
                        int* launches);

/* --- model tooling --------------------------------------------------------
 * Writes a model in the ggml .bin layout read by whisper.cpp and by
 * mwx_init_from_file_with_params: magic, 11 hparams, mel filterbank, vocab,
 * tensors. Weights are splitmix64-seeded; wtype 1 = f16, 30 = bf16 for the 2-D
 * tensors (1-D tensors, conv biases and positional embeddings are f32, as in
 * the upstream converter). arch: "tiny.en", "tiny", "base.en", "base",
 * "small", "medium", "large-v3", or "micro" (test-sized).
 * Returns 0 on success. */
int mwx_write_synthetic_model(const char* path, const char* arch, int wtype,
                              uint64_t seed);

/* Quantizes a whisper ggml .bin (f32 / f16 / bf16) into a ggml block type
 * (q4_0 = 2, q4_1 = 3, q5_0 = 6, q5_1 = 7, q8_0 = 8; the 256-element K types
 * q2_K = 10, q3_K = 11, q4_K = 12, q5_K = 13, q6_K = 14) with the rules of
 * whisper.cpp's `quantize` tool: 2-D tensors except the positional
 * embeddings are quantized, everything else is copied; ftype becomes
 * 2000 + ftype. Legacy blocks are ggml's quantize_row_q*_ref bit for bit; K
 * blocks come from a plain min/max encoder (valid blocks, not ggml's scale
 * search). A row length that is not a multiple of the block (tiny's 384 for
 * K types) fails with -8, as ggml's quantizer does. Returns 0 on success. */
int mwx_model_quantize(const char* in_path, const char* out_path, int type);

#ifdef __cplusplus
}
#endif

#endif /* MWX_H */
