// Host-visible launcher declarations for the gfx950 kernels of the mwx engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mwx {

// launch span stamp slots (kcommon.h span_start; engine.cpp span_slot): a slot
// is SPAN_SHARDS (start, end) pairs 128 B apart
constexpr int SPAN_SHARDS = 8, SPAN_SLOT_U64 = SPAN_SHARDS * 16;

// GEMM epilogues. Every GEMM computes acc[m][n] = sum_k A[m][k] * W[n][k]
// (W stored [N][K] as in ggml), accumulating in f32 on MFMA, and then applies
// exactly the ops ggml applies after the matmul, at the same rounding points.
enum Epi : int {
  EPI_ENC_QKV = 0,  // encoder Q/K/V (+bias) -> f16 head-major Q, K and V^T
  EPI_GELU = 1,     // out_T = gelu_ggml(acc + bias)       (FFN1, conv1)
  EPI_RES = 2,      // out32 = (acc + bias) + res32         (out-proj, FFN2)
  EPI_CONV2 = 3,    // out32 = pe + gelu_ggml(acc + bias)   (conv2 + pos emb)
  EPI_F32 = 4,      // out32 = acc                          (logits)
  EPI_CROSS_KV = 5, // cross K = f16(acc*kscale), V = f16(acc + b), all layers
  EPI_DEC_QKV = 6,  // decoder Q (scaled) -> f16, K/V -> self KV cache at pos
  EPI_STORE16 = 7,  // out16 = f16(acc + bias)              (cross-attn Q)
};

struct EpiParams {
  const float* bias = nullptr;
  float* c32 = nullptr;
  void* c16 = nullptr;
  long ldc = 0;
  long c_bstride = 0;  // per grid.z batch stride of the output (elements)
  const float* r32 = nullptr;
  const float* pe = nullptr;
  _Float16* q = nullptr;
  _Float16* k = nullptr;
  _Float16* v = nullptr;
  int L = 0;     // sequence length (encoder / cross) or text ctx (decoder cache)
  int H = 0;     // heads
  int d = 0;     // model width
  int ncap = 0;  // slots in the cross / self cache
  int ldv = 0;   // encoder V^T row stride (padded L)
  const int* pos = nullptr;     // decoder: position per row
  const int* active = nullptr;  // decoder: row active flag
  const int* slot = nullptr;    // cross: cache slot per encoder batch index
  float kscale = 1.0f;
  float qscale = 1.0f;
  bool pack_out = false;  // EPI_GELU: write the output as decode-GEMM A tiles (pack_index, K = ldc)
  // MX-fp8 GEMMs: E8M0 scales [rows][K/32] of A (per grid.z batch stride) and W
  unsigned long long* span = nullptr;  // launch span stamps (perf; kcommon.h span_start)
  const uint8_t* sa = nullptr;
  long sa_bstride = 0;
  const uint8_t* sw = nullptr;
  bool xcd_remap = true;  // gemm_big: XCD-aware tile order
  int group_m = 0;        // gemm_big: row tiles per group of the grouped tile order (0: row-major)
  int mt = 0;             // gemm_decode: rows per block = 16 * mt (0: the default rule)
  int nw = 0;             // gemm_decode (skinny): waves splitting K (0: the default rule)
  // EPI_CROSS_KV with an MX-fp8 cache: k / v hold e4m3 codes, ks8 / vs8 the
  // E8M0 scales (two per (time, head) row of 64)
  uint8_t* ks8 = nullptr;
  uint8_t* vs8 = nullptr;
  // EPI_GELU in gemm_big's staged epilogue: the f16 GELU table
  // (gelu_table_build), copied to LDS after the main loop and looked up
  // instead of evaluating tanhf per output (the same values)
  const uint16_t* gelu_tab = nullptr;
};

// f16 GELU table: entry i < GELU_TAB_HALF holds f16(gelu_f32(h)) (kcommon.h,
// the expression gelu_ggml evaluates) for the f16 value h with bits i
// (0 <= h <= 10), entry GELU_TAB_HALF + i the same for bits 0x8000 | i; padded
// to a multiple of 8 entries
constexpr int GELU_TAB_HALF = 0x4901;
constexpr int GELU_TAB_N = (2 * GELU_TAB_HALF + 7) / 8 * 8;
void gelu_table_build(uint16_t* tab, hipStream_t st);

// The encoder GEMMs on MX-fp8 operands (e4m3 bytes + E8M0 scale per 32 k,
// P.sa / P.sw): EPI_ENC_QKV, EPI_GELU (16-bit T output), EPI_RES, EPI_CROSS_KV.
template <typename T>
void gemm_mx(int epi, const uint8_t* A, long lda, long a_bstride, const uint8_t* W, long ldw,
             int M, int N, int K, int batch, const EpiParams& P, hipStream_t st);
// Rows of a 16-bit matrix [M][K] (row stride ld) -> MX-fp8: q [M][K] e4m3,
// s [M][K/32] E8M0 (quant.cpp: mx_quantize_block semantics).
template <typename T>
void mx_quantize(const T* x, long ld, int M, int K, uint8_t* q, uint8_t* s, hipStream_t st);

// Decode weights live in HBM as MFMA fragment tiles: for each 16-column strip
// nt and 32-deep k-step kt, the 16x32 block is 1 KB contiguous in the order the
// 64 lanes of a wave consume it (lane = (k%32/8)*16 + n%16, 8 elements per
// lane), so one wave-wide 16-B-per-lane load is one fully used 1-KB burst.
// Rows are zero-padded to a multiple of 16.
__host__ __device__ inline long pack_index(long n, long k, long K) {
  const long nt = n >> 4, c = n & 15, kt = k >> 5, kk = k & 31;
  return ((nt * (K >> 5) + kt) * 64 + (kk >> 3) * 16 + c) * 8 + (kk & 7);
}

// T = _Float16 or __bf16 (model weight type). `OutT16` selects the 16-bit
// output type of EPI_GELU (f16 for conv1, T for FFN1).
template <typename T>
void gemm(int epi, bool out_f16, const T* A, long lda, long a_bstride, const T* W, long ldw,
          int M, int N, int K, int batch, const EpiParams& P, hipStream_t st);

// Decode GEMMs take both operands as fragment tiles: Ap = activations
// [ceil64(M) rows] packed with pack_index(m, k, K) by their producer kernel
// (decode LayerNorm, decode attention, FFN1 epilogue), Wp = weights.
//
// Decode split-K GEMM over fragment-tiled weights Wp (pack_index): writes KS
// f32 partial slabs P[KS][M][N] (no epilogue) and returns KS (0 if the shape is
// unsupported). The consumer kernel sums the slabs and applies the epilogue.
int splitk_factor(int K);
// A decode weight in fragment tiles: 16-bit (w) or MX-fp8 (q codes in
// pack_index order + s, one E8M0 scale per (column, 32-deep k-step) at
// s[(strip * K/32 + kt) * 16 + column % 16]; MWX_COMPUTE_MXFP8, bf16 models).
template <typename T>
struct DecW {
  const T* w = nullptr;
  const uint8_t* q = nullptr;
  const uint8_t* s = nullptr;
  DecW() = default;
  DecW(const T* w_) : w(w_) {}
  DecW(const uint8_t* q_, const uint8_t* s_) : q(q_), s(s_) {}
};
template <typename T>
int gemm_splitk_partials(const T* Ap, const DecW<T>& W, int M, int N, int K, float* P,
                         hipStream_t st);
// The decode LayerNorm folded into the split-K GEMM that consumes it, at one
// row (M = 1: C2, the service's single-clip requests): every workgroup forms
// the row's residual x_in + (sum P + pbias) and its LayerNorm as its A operand
// (ln_core.h: ln_dec_kernel's arithmetic, bit-identical) instead of reading a
// packed LayerNorm output, so the LayerNorm costs no launch of its own.
// Workgroup (0, 0) writes the residual to x_out, a buffer other than x_in (the
// other workgroups still read x_in); an inactive row's x_in is copied.
struct LnFuse {
  const float* x_in = nullptr;
  float* x_out = nullptr;
  const float* P = nullptr;  // the producer's KS split-K slabs (nullptr: none)
  int KS = 0;
  long pstride = 0;
  const float* pbias = nullptr;
  const float* w = nullptr;  // LayerNorm weight / bias
  const float* b = nullptr;
  const int* active = nullptr;
};
template <typename T>
int gemm_splitk_ln(const LnFuse& ln, const DecW<T>& W, int N, int K, float* P, hipStream_t st);
// The same fold into a full-K decode GEMM with its epilogue (FFN1 + GELU at one
// row); false if the shape is unsupported (the caller launches the two kernels).
template <typename T>
bool gemm_decode_ln(int epi, const LnFuse& ln, const DecW<T>& W, int N, int K, const EpiParams& P,
                    hipStream_t st);
// Decode full-K GEMM over fragment-tiled weights with a fused epilogue
// (EPI_GELU / EPI_RES / EPI_F32 / EPI_STORE16 / EPI_DEC_QKV), rows in blocks of
// 64 so a row's arithmetic does not depend on the batch. Returns false if K is
// unsupported.
template <typename T>
bool gemm_decode(int epi, const T* Ap, const DecW<T>& W, int M, int N, int K, const EpiParams& P,
                 hipStream_t st);
// Log-mel of a batch of clips in one pass (three launches): clip c's samples
// at pcm_base + desc[c].pcm_off (n), its mel [n_mels][n_len] at mel_base +
// desc[c].mel_off, normalised in place; mx[c] = the clip's raw max; part:
// n_clips * 16 floats of scratch.
// Incremental log-mel (streaming re-transcription): with prev_pcm set, a tile
// of frames whose input samples equal the previous call's (and were real
// samples then) copies its raw log-mel from prev_raw instead of recomputing
// it; save_pcm / save_raw (the other slot of the state's ping-pong cache)
// receive this call's samples and raw log-mel for the next call.
struct MelClip {
  long pcm_off, mel_off;
  int n, n_len, n_fft;
  int n_prev;    // samples of the previous call on this state (0: no cache)
  int len_prev;  // its n_len (stride of prev_raw)
  int pad;
  const float* prev_pcm;  // [n_prev]
  const float* prev_raw;  // [n_mels][len_prev], before normalisation
  float* save_pcm;        // [n] or nullptr
  float* save_raw;        // [n_mels][n_len] or nullptr
};
void launch_mel_batch(const float* pcm_base, const MelClip* desc, int n_clips, int max_n_len,
                      const float* filters, int n_mels, const float* tables, float* mel_base,
                      float* part, float* mx, hipStream_t st);
void launch_mel_window(const float* mel, long mel_clip_stride, const int* clip_of_slot,
                       const int* seek_of_slot, const int* n_len_of_slot, int n_mels, int T,
                       int cpad, _Float16* melT, int n_slots, hipStream_t st);
void launch_signal_energy(const float* x, int n, float* out, hipStream_t st);
// pcm16 / 32768 -> f32 (in and out 8- / 16-byte aligned)
void launch_pcm16_to_f32(const int16_t* in, long n, float* out, hipStream_t st);

// LayerNorm of x rows into y. With P != nullptr, x is first completed from
// the KS split-K partial slabs P[KS][M][N]: x = (sum P + pbias) + x.
template <typename T>
void layer_norm(const float* x, const float* w, const float* b, T* y, int M, int N,
                const int* active, hipStream_t st, const float* P = nullptr, int KS = 0,
                const float* pbias = nullptr);
// Decode LayerNorm: as above, but y is written as decode-GEMM A tiles
// (pack_index) and each thread owns 8 consecutive elements (N % 8 == 0,
// N <= 2048).
// EmbedIn (the first LayerNorm of a step): x is first formed as the token +
// position embedding, x = te[tok[row]] + pe[pos[row]] (embed's arithmetic),
// and written, so no separate embed launch precedes the layer stack.
template <typename T>
struct EmbedIn {
  const T* te = nullptr;
  const float* pe = nullptr;
  const int* tok = nullptr;
  const int* pos = nullptr;
  // rows of te / pe: the gather runs before the inactive-row exit, so its
  // indices are clamped (an inactive row may carry any token / position)
  int n_tok = 1, n_pos = 1;
};
template <typename T>
void layer_norm_dec(float* x, const float* w, const float* b, T* y, int M, int N,
                    const int* active, hipStream_t st, const float* P, int KS,
                    const float* pbias, const EmbedIn<T>& emb = EmbedIn<T>());


// encoder self-attention: q,k [B][H][L][64], vt [B][H][64][L] f16 -> o [B*L][H*64] (T)
template <typename T>
void enc_attention(const _Float16* q, const _Float16* k, const _Float16* vt, T* o, int B,
                   int H, int L, float scale, hipStream_t st);

// decode attention for R rows: q [R][H*64] f16; K/V rows [n_keys][64] per
// (row, head). self: K = kbase + ((row*H + h)*kstride_rows)*64, n_keys =
// pos[row] + 1. cross: K = kbase + ((clip[row]*H + h)*L)*64, n_keys = L.
// o is written as decode-GEMM A tiles (pack_index, K = H*64).
// The query of (row, head) is reduced from the producing split-K GEMM's
// slabs P[KS][R][pcols] (q = f16((sum P + bias) * qscale), columns h*64..).
// self (fixed_len == 0): the slabs hold Q|K|V (pcols = 3d); the kernel also
// forms k = f16(sum * kscale), v = f16(sum + bias) for the row's position and
// appends them to the KV cache before attending over positions 0..pos.
// self (beam search): with own_from != nullptr, position j < own_from[row] of
// row `row` is read from the cache of row kvmap[row * kv_len_cap + j] - map_row0.
// cross: nq > 1 = rows come in groups of nq sharing one slot (beam / best-of
// decoders of a clip); their workgroups are co-scheduled on one XCD.
template <typename T>
void dec_attention(const float* P, int KS, int pcols, const float* bias, float qscale,
                   float kscale, _Float16* kbase, _Float16* vbase, const int* kv_index,
                   const int* pos, const int* active, int fixed_len, int kv_len_cap, T* o, int R,
                   int H, float scale, hipStream_t st, const int* kvmap = nullptr,
                   const int* own_from = nullptr, int map_row0 = 0, int nq = 1,
                   int write_new = 1, unsigned long long* span = nullptr);

// Prompt prefill: K / V of every row (reduced from the QKV slabs exactly as
// dec_attention's self kernel reduces its own position) appended to cache row
// crow[row] (nullptr: row) at position pos[row].
template <typename T>
void kv_append(const float* P, int KS, int pcols, const float* bias, float kscale,
               _Float16* kbase, _Float16* vbase, const int* crow, const int* pos,
               const int* active, int cap, int R, int H, hipStream_t st);

// Cross-attention for groups of nq consecutive rows that share one cross
// slot (beam-search / best-of decoders of a clip; kv_index[row] equal within a
// group): K/V of the slot are streamed once per group. Same per-row results as
// dec_attention. Returns false if nq is not supported (1..8; f16 caches: 2..8).
// kscale8 / vscale8 != nullptr: the cache is MX-fp8 (kbase / vbase hold e4m3
// codes [slot][H][cap][64], the scales [slot][H][cap][2] E8M0), any nq >= 1.
// MX-fp8 grouped cross-attention on MFMA (1, default) or v_dot2 (0); -1:
// MWX_XATTN_MFS. Returns the previous setting (the A/B tests).
int xattn_mfs_set(int on);
// decode GEMMs at M > 64 rows: shared-A kernels (1) or per-strip grids (0);
// -1 restores the MWX_DEC_SHARED default. Returns the previous setting.
int dec_shared_set(int on);
// the encoder GEMM's 8-phase main loop on / off (-1: back to MWX_GEMM_8PH)
int gemm_8ph_set(int on);
// test hook: the MX-fp8 cache's code widening (8 codes per E8M0 exponent) to f16 bits
void mx_widen_test(const uint8_t* codes, const uint8_t* e8, int n8, uint16_t* out, hipStream_t st);
template <typename T>
bool dec_cross_attention_grouped(const float* P, int KS, int pcols, const float* bias,
                                 const void* kbase, const void* vbase, const int* kv_index,
                                 const int* active, int n_keys, int cap, T* o, int R, int H,
                                 float scale, int nq, hipStream_t st,
                                 const uint8_t* kscale8 = nullptr,
                                 const uint8_t* vscale8 = nullptr,
                                 unsigned long long* span = nullptr);

struct RowCtl {
  int active;        // row participates in this step
  int sample;        // logits of this step are processed (last prompt token or generated)
  int is_initial;    // no tokens generated yet
  int last_ts;       // last generated token is a timestamp
  int penult_ts;     // penultimate generated token is a timestamp (or < 2 tokens)
  int has_ts;        // decoder.has_ts
  int seek_delta;    // decoder.seek_delta
  int want_probs;    // write probs/logprobs rows (sampling path)
  float temperature; // > 0: logits /= temperature
  int want_nosp;     // compute no_speech probability from the raw logits
  int pad[2];
};
struct TokOut {
  int id;
  int tid;
  float p;
  float plog;
  float pt;
  float ptsum;
  float nosp;
  int pad;
};
// Run-ahead greedy decoding: the per-row stop / next-input rules of the
// whisper_full token loop (driver.inc, the host restatement of whisper.cpp
// v1.8.2's decoder loop) applied on the device after every step, so the next
// step's inputs (stepin, RowCtl) are ready without a host round trip and the
// host processes step k while step k+1 runs.
struct RowRun {
  int fed;          // positions fed so far (the next step feeds position `fed`)
  int p_len;        // prompt length
  int ntok;         // tokens generated
  int last_id;      // last / penultimate generated token ids
  int penult_id;
  int has_ts;       // decoder.has_ts / seek_delta / result_len
  int seek_delta;
  int result_len;
  int stopped;
  int seek, seek_end;  // the clip's window position and end (centiseconds)
  int cls;          // beam: token-sequence class (equal sequences <=> equal cls)
  int used;         // beam: uniforms of the row's RNG consumed so far
  int pad;
  double sum;       // beam: sum_logprobs_all
};
struct RunConst {
  int beg, eot, max_tokens, n_max, delta_min, R, nslot, prompt_stride;
  float temperature;
  int want_probs;
  int pad[2];
};
// what the host reads back per row and step (written straight into pinned
// host memory by the advance kernel: no copy launch per step)
struct RunReport {
  TokOut out;        // the step's token record
  int tok, pos, act, pad;  // the next step's inputs as the device set them
  RowCtl next;
};
// empty one-wave kernel (timing-event overhead calibration, bench.py)
void launch_perf_empty(hipStream_t st);
struct LPPart;
struct LPRes;
struct LogitsConst {
  int n_vocab;
  int eot;
  int beg;
  int space_id;       // token id of " " (suppress_blank)
  int suppress_blank;
  int max_initial_tid;  // timestamps > beg + tid0 suppressed at the first step (-1: off)
  int nosp_id;
};
// The step's logits-processing phase 3 (lp_pick) run inside the advance
// kernel (parts != nullptr: logits_process was launched with pick = false)
struct PickIn {
  const float* logits = nullptr;
  const float* flt = nullptr;
  const LPPart* parts = nullptr;
  const LPRes* res = nullptr;
  LogitsConst C{};
};
struct Draw;
// Run-ahead beam search: per clip (n decoders = rows r0 .. r0+n-1), the
// beam step of whisper.cpp's decoder loop on the device (driver.inc
// beam_step: candidate ranking, dedup, hand-over of state and KV maps), then
// the token rules as row_advance, the next step's inputs and its uniforms
// (from the host-filled ring uring[R][ring_n], the rows' RNG streams).
struct BeamReport {
  int src;      // decoder (row) whose candidate this row took (itself: no move)
  int nd;       // uniforms the row's next step draws
  int pad[2];
};
struct BeamRun {
  const Draw* draws;  // [R][KD] this step's draws
  int KD;             // = beam size
  int n;              // decoders per clip
  double* du;         // [R][KD] next step's uniforms
  int* dnd;           // [R]
  const double* uring;  // [R][ring_n] host-filled
  int ring_n;
  int* kvmap;         // [R][Tctx]
  int* kvown;         // [R]
  int Tctx;
  BeamReport* brep;   // [nslot][R]
  Draw* drep;         // [nslot][R][KD] the step's draws, for the host replay
};
void beam_advance(RowRun* run, int* run_step, const int* prompt, int* stepin, RowCtl* ctl,
                  TokOut* out, RunReport* rep, const RunConst& C, const BeamRun& B,
                  const PickIn& pk, hipStream_t st);
// Run-ahead greedy decoding and temperature sampling (best-of): B.draws ==
// nullptr: the step's argmax; else each sampling row takes its draw
// B.draws[r][0] and the next step's uniform comes from the ring as in
// beam_advance (B.n, kvmap, kvown, Tctx and brep unused)
void row_advance(RowRun* run, int* run_step, const int* prompt, int* stepin, RowCtl* ctl,
                 TokOut* out, RunReport* rep, const RunConst& C, const BeamRun& B,
                 const PickIn& pk, hipStream_t st);

// Logits processing is split over LP_G chunks of LP_CHUNK vocabulary entries
// per row (LP_G * LP_CHUNK >= n_vocab for every Whisper vocabulary).
constexpr int LP_G = 16;
constexpr int LP_CHUNK = 3328;  // 13 x 256
struct LPPart {  // per-chunk statistics of the filtered (and raw) logits
  float m, s, mtext, mts, sts, rm, rs, pad;
};
struct LPRes {  // per-chunk argmax / timestamp argmax / timestamp prob sum
  float best;
  int best_i;
  float tbest;
  int tbest_i;
  double sum_ts;
};
struct LPScratch {
  float* flt;     // [R][n_vocab] filtered logits
  LPPart* parts;  // [R][LP_G]
  LPRes* res;     // [R][LP_G]
};
// pick = false: phase 3 (lp_pick) is left to the run-ahead advance kernel
// (PickIn)
void logits_process(float* logits, const float* static_mask, const RowCtl* ctl, TokOut* out,
                    float* probs, float* logprobs, const LogitsConst& C, int R, LPScratch ws,
                    hipStream_t st, bool pick = true);

// std::discrete_distribution draws from the probs rows (k_misc.hip):
// out[row][d] for d < ndraw[row] (<= KD <= 16), u[row][d] =
// generate_canonical<double, 53> of the row's RNG.
struct Draw {
  int id;
  float p;
  float plog;
  int pad;
};
// need: [R] scratch (rows whose fast-path draw lies within the rounding
// margin and is redone by the sequential libstdc++-order kernel).
// MWX_DRAW_EXACT=1 runs the sequential kernel for every row.
// force_exact: -1 = MWX_DRAW_EXACT env, 0 = fast path + fallback, 1 = exact only.
void sample_draws(const float* probs, const float* logprobs, int V, const double* u,
                  const int* ndraw, int KD, Draw* out, int* need, int R, hipStream_t st,
                  int force_exact = -1);

// Sinc resampler (k_resample.hip): libsamplerate SRC_SINC_FASTEST's filter
// sum per output sample; fixed-point filter indices with 12 fractional bits
// (src_sinc.c SHIFT_BITS).
constexpr int RS_SHIFT = 12;
constexpr int RS_FRAC_MASK = (1 << RS_SHIFT) - 1;
constexpr double RS_INV_FP_ONE = 1.0 / (double)(1 << RS_SHIFT);
void resample_launch(const float* in, int half, const float* coeffs, int coeff_half_len,
                     int increment, double scale, const int2* pos, int n_out, float* out,
                     hipStream_t st);

// Segment prosody (k_prosody.hip): reference extract_prosody per segment.
struct ProsodySeg {
  long start;      // first sample in the clip
  long len;        // samples
  long frame_off;  // offset of the segment's frames in the scratch arrays
};
// same layout as mwx_prosody (include/mwx.h)
struct ProsodyOut {
  float pitch_mean, pitch_std, energy_mean, energy_std, spectral_centroid, zero_crossing_rate,
      arousal, valence;
  float speaker_vec[8];
  int gender;   // 0 '?', 1 'M', 2 'F'
  int emotion;  // 0 neutral, 1 excited, 2 angry, 3 sad
  int serial_runs;
  int pad;
};
// fstate: [sum frames] floats, feat: [sum frames] float4, fcyc: [sum frames]
// ints (frames = len / frame)
void prosody_launch(const float* pcm, const ProsodySeg* seg, int n_seg, float* fstate,
                    float4* feat, int* fcyc, ProsodyOut* out, int frame, int sample_rate, float alpha,
                    float gender_thr, float min_pitch, float max_pitch, hipStream_t st);

}  // namespace mwx
