/*
 * mwx_test.h — per-stage entry points of the mwx engine used by the parity
 * tests (tests/test_gpu_parity.py). They run one stage of the device hot path
 * for a single clip and copy the result back to the host as f32, so each stage
 * can be compared with the CPU oracle (oracle/) in isolation. Not used by the
 * service path.
 */
#ifndef MWX_TEST_H
#define MWX_TEST_H

#include "mwx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device log-mel of one clip. out receives [n_mels][n_len] (if out_cap is
 * large enough); returns n_len, or <0 on error. */
int mwx_test_mel(struct mwx_context* ctx, struct mwx_state* state, const float* pcm, int n,
                 float* out, long out_cap);

/* mel + conv stem + encoder + cross K/V of one clip at `seek`. enc_out:
 * [n_audio_ctx][n_audio_state] (encoder output after ln_post, as stored on the
 * device); k_out / v_out (nullable): [n_text_layer][n_audio_ctx][n_text_state]
 * cross K/V. The cross K/V stay resident in `state` for mwx_test_decode. */
int mwx_test_encode(struct mwx_context* ctx, struct mwx_state* state, const float* pcm, int n,
                    int seek, float* enc_out, float* k_out, float* v_out);

/* Teacher-forced decoder run against the cross K/V left by mwx_test_encode:
 * token i at position i, logits_out [n][n_vocab] (raw logits). */
/* The encoder of one clip window with its intermediates copied out: x_out
 * [n_audio_layer + 1][n_audio_ctx][n_audio_state] f32 = the residual stream
 * after the conv stem and after each layer; a_out[0..3] = per layer the four
 * GEMM A operands as the model's 16-bit type (raw bits), before any MX-fp8
 * quantization: attention LayerNorm out, attention out, MLP LayerNorm out
 * ([L][n_ctx][d] each) and GELU out ([L][n_ctx][4 d]). */
int mwx_test_encode_dump(struct mwx_context* ctx, struct mwx_state* state, const float* pcm,
                         int n, int seek, float* x_out, uint16_t* const* a_out);

int mwx_test_decode(struct mwx_context* ctx, struct mwx_state* state, const int* tokens, int n,
                    float* logits_out);

/* As mwx_test_decode_last, with tokens 0 .. n-2 run by the batched prompt
 * prefill (one pass of the layer stack) and only token n-1 as a decode step. */
int mwx_test_decode_last_prefill(struct mwx_context* ctx, struct mwx_state* state,
                                 const int* tokens, int n, float* logits_last);

/* Self-attention K / V cache of row 0 of a state for one decoder layer,
 * positions 0 .. n_pos-1, as f32 [n_pos][n_text_head][64] each. */
int mwx_test_self_kv(struct mwx_state* state, int layer, int n_pos, float* k_out, float* v_out);

/* The engine's load-time dequantizer (host code, no device work): n values
 * of ggml block type `type` (legacy q4_0 .. q8_0 or K q2_K .. q6_K; n a
 * multiple of the block) from src into dst as f32, before the f16 rounding
 * of the upload. Returns 0, or -1 for an unsupported type / length. */
int mwx_test_dequantize(int type, const void* src, long n, float* dst);

/* Decode work counters of a state (the first state of a batch drives it):
 * decode steps launched and prompt positions run by the batched prompt
 * prefill since the last reset. reset != 0 zeroes them after reading. */
int mwx_test_decode_counters(struct mwx_state* state, long* steps, long* prefill_positions,
                             int reset);

/* Window counters of a state (the first state of a batch drives it): clip
 * windows decoded, decode attempts run (one per window and temperature
 * tried, so attempts - windows = temperature-fallback re-runs) and decode
 * steps summed over the clips live in each (each such clip-step reads the
 * clip's cross K/V once per layer) since the last reset. reset != 0 zeroes
 * them after reading. */
int mwx_test_window_counters(struct mwx_state* state, long* windows, long* attempts,
                             long* clip_steps, int reset);

/* Run-ahead decode attempts a state redid on the host-driven token loop
 * because the device's advance and the host's replay disagreed (or
 * MWX_TEST_RA_MISMATCH=k forced it at step k). reset != 0 zeroes it. */
long mwx_test_runahead_fallbacks(struct mwx_state* state, int reset);

/* As mwx_test_decode, but only the logits of the last token are copied out
 * (logits_last [n_vocab]). */
int mwx_test_decode_last(struct mwx_context* ctx, struct mwx_state* state, const int* tokens,
                         int n, float* logits_last);

/* One MX-fp8 GEMM as the fp8 compute mode runs it: a [M][K] is rounded to
 * bf16 and quantized by the device kernel, w [N][K] by the load-time host
 * quantizer, c [M][N] = the block-scaled fp8 MFMA product (f32). K % 128 == 0.
 * Returns 0 or <0. */
int mwx_test_gemm_mx(struct mwx_context* ctx, int M, int N, int K, const float* a,
                     const float* w, float* c);

/* The encoder FFN1 GEMM with its GELU epilogue on given data: a [M][K] and
 * w [N][K] rounded to bf16 (bf16 != 0) or f16, bias [N]; out [M][N] =
 * gelu_ggml(a.w + bias) in that type, widened to f32. use_table: the f16 GELU
 * table looked up from LDS (the engine's path) or tanhf per output. N % 64 ==
 * 0, K % 64 == 0. Returns 0 or <0. */
int mwx_test_gemm_gelu(struct mwx_context* ctx, int M, int N, int K, const float* a,
                       const float* w, const float* bias, int bf16, int use_table, float* out);

/* std::discrete_distribution draws on the device (k_misc.hip sample_draws):
 * probs / logprobs [R][V], u [R][KD] (generate_canonical<double, 53> values),
 * ndraw [R] (<= KD <= 16); ids [R][KD] out. exact != 0 runs only the
 * sequential-order kernel. reps > 1 repeats the launch and returns the mean
 * microseconds per launch in *us (HIP events). Returns 0 or <0. */
int mwx_test_sample_draws(struct mwx_context* ctx, const float* probs, const float* logprobs,
                          int R, int V, const double* u, const int* ndraw, int KD, int exact,
                          int reps, int* ids, double* us);

/* MX-fp8 grouped cross-attention scores and P.V on MFMA (1, the default) or
 * the v_dot2 kernel (0); -1 restores the MWX_XATTN_MFS default. Returns the
 * previous setting. */
int mwx_test_set_xattn_mfs(int on);

/* Decode GEMMs at more than 64 rows (beam / best-of decoders of many clips):
 * the shared-A kernels (1, the default) or the per-strip grids (0); -1
 * restores the MWX_DEC_SHARED default. Returns the previous setting. */
int mwx_test_set_dec_shared(int on);

/* The encoder GEMM's 8-phase main loop (bit-identical to the default 2-stage
 * ring) on (1) / off (0) / back to the MWX_GEMM_8PH environment default (-1).
 * Returns the previous mode. */
int mwx_test_set_gemm_8ph(int on);

/* The decode LayerNorms before the QKV and cross-Q projections folded into
 * those split-K GEMMs at one row (gemm_splitk_ln, bit-identical to the
 * separate LayerNorm launch) on (1) / off (0) / back to the MWX_LN_FOLD
 * environment default, on (-1). Read when a decode step is captured. Returns
 * the previous mode. */
int mwx_test_set_ln_fold(int on);


/* The MX-fp8 cross K/V cache's widening of e4m3 codes to f16 as the
 * cross-attention kernels run it: n8 groups of 8 codes (codes[8 n8]), each
 * group with one E8M0 exponent (e8[n8]); out[8 n8] = f16 bits. */
int mwx_test_mx_widen(struct mwx_context* ctx, const uint8_t* codes, const uint8_t* e8, int n8,
                      uint16_t* out);

/* Fault injection of the run-ahead safety net: run-ahead step `step` of every
 * later attempt is treated as a device/host disagreement (-1: none; -2: back
 * to the MWX_TEST_RA_MISMATCH environment default). Returns the previous
 * setting. */
long mwx_test_set_ra_mismatch(long step);

/* The MX-fp8 grouped cross-attention kernel on given data: q [R][H*64] f32
 * queries (rounded to f16 by the kernel), K / V as e4m3 codes [R/nq][H][n][64]
 * with E8M0 scales [R/nq][H][n][2] (one per 32-element half), rows
 * g*nq .. g*nq+nq-1 reading slot g; o [R][H*64] f32 = the kernel's 16-bit
 * output (the context's weight type). Scores / P.V on MFMA or v_dot2 per
 * mwx_test_set_xattn_mfs. Returns 0 or <0. */
int mwx_test_xattn_mx(struct mwx_context* ctx, int R, int H, int n, int nq, const float* q,
                      const uint8_t* k8, const uint8_t* ks, const uint8_t* v8, const uint8_t* vs,
                      float* o);

#ifdef __cplusplus
}
#endif

#endif /* MWX_TEST_H */
