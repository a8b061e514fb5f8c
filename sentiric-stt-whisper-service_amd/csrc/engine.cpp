// mwx engine: context / state lifecycle, weight upload and the batched
// whisper_full driver (the reference's L1 hot path), exposed
// through the C ABI of include/mwx.h.
//
// Work split:
//   device (HIP, gfx950): log-mel, conv stem, encoder, cross K/V, every decoder
//     step (embedding -> layers -> logits -> logits processing + greedy pick);
//   host: the whisper_full control flow — seek windows, prompt handling,
//     temperature fallback, decoder state machine, sequence scoring, segment
//     and token-timestamp construction — restated from whisper.cpp v1.8.2.
//     Per decode step only a 32-byte record per row comes back to the host.
//
// Batching: mwx_full_batch runs B clips through every device stage together
// (rows = clips x decoders); each clip keeps its own host state machine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "common.h"
#include "kernels.h"

#define HIPC(x)                                                                        \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      MWX_LOG_ERROR("mwx: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                         \
      throw std::runtime_error("hip");                                                 \
    }                                                                                  \
  } while (0)

namespace mwx {

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// LayerNorm folded into the next split-K GEMM at one row (gemm_splitk_ln):
// env MWX_LN_FOLD (default on) read once; mwx_test_set_ln_fold switches it
// (read when a decode step is captured)
inline std::atomic<int>& ln_fold_mode() {
  static std::atomic<int> m{-1};
  return m;
}
inline bool ln_fold_on() {
  int v = ln_fold_mode().load();
  if (v < 0) {
    v = (getenv("MWX_LN_FOLD") && atoi(getenv("MWX_LN_FOLD")) == 0) ? 0 : 1;
    ln_fold_mode().store(v);
  }
  return v != 0;
}

// Process-wide order between graph capture and (de)allocation: while any
// thread captures a stream, HIP rejects legacy-stream operations such as
// hipMemset ("would make the legacy stream depend on a capturing stream") and
// hipFree / hipHostFree synchronize the device. Concurrent batches (the
// SttEngine's parallel_requests batchers) capture their decode graphs while
// another batch may be growing its buffers, so both hold this lock
// (recursive: a capture may grow a buffer of its own).
inline std::recursive_mutex& capture_mutex() {
  static std::recursive_mutex m;
  return m;
}

// grow-only device buffer
struct DBuf {
  void* p = nullptr;
  size_t n = 0;
  void* get(size_t bytes, bool zero = false) {
    if (bytes > n) {
      std::lock_guard<std::recursive_mutex> lock(capture_mutex());
      if (p) (void)hipFree(p);
      p = nullptr;
      n = 0;
      HIPC(hipMalloc(&p, bytes));
      n = bytes;
      if (zero) {
        // the fill is queued on the null stream, which the states' non-blocking
        // streams do not wait for: wait for it here, or the first kernels on a
        // fresh buffer can run before (or under) it -- seen as run-to-run
        // differences of a fresh context's first batch with another process
        // on the GPU (zero-padded encoder inputs overwritten after the
        // producer wrote them)
        HIPC(hipMemset(p, 0, bytes));
        HIPC(hipStreamSynchronize(nullptr));
      }
    }
    return p;
  }
  void release() {
    std::lock_guard<std::recursive_mutex> lock(capture_mutex());
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// MX-fp8 weight: e4m3 codes [N][K] + E8M0 scales [N][K/32]
struct MxW {
  const uint8_t* q = nullptr;
  const uint8_t* s = nullptr;
};
struct EncLayerW {
  const float *ln1_w, *ln1_b, *ln2_w, *ln2_b;
  const void *qkv_w, *o_w, *fc1_w, *fc2_w;
  const float *qkv_b, *o_b, *fc1_b, *fc2_b;
  MxW qkv_x, o_x, fc1_x, fc2_x;  // compute = MXFP8
};
// decode-GEMM weight: 16-bit fragment tiles (w) or MX-fp8 fragment tiles
// (q codes + s scales; MWX_COMPUTE_MXFP8 with a bf16 model)
struct DecWeight {
  const void* w = nullptr;
  const uint8_t* q = nullptr;
  const uint8_t* s = nullptr;
};
struct DecLayerW {
  const float *ln1_w, *ln1_b, *lnc_w, *lnc_b, *ln2_w, *ln2_b;
  DecWeight qkv, o, cq, co, fc1, fc2;
  const float *qkv_b, *o_b, *cq_b, *co_b, *fc1_b, *fc2_b;
};

struct Context {
  Hparams hp;
  Vocab vocab;
  std::vector<float> filters;
  int wtype = GGML_F16;
  int device = 0;
  int cpad = 128;  // conv1 input channels padded (3*cpad % 64 == 0)
  void* arena = nullptr;
  uint16_t* gelu_tab = nullptr;  // f16 GELU table (gelu_table_build), read by the encoder GELU GEMMs
  const float* d_filters = nullptr;
  const float* d_tables = nullptr;  // hann[400], cos[400], sin[400]
  const _Float16* conv1_w = nullptr;
  const float* conv1_b = nullptr;
  const _Float16* conv2_w = nullptr;
  const float* conv2_b = nullptr;
  const float* enc_pe = nullptr;
  std::vector<EncLayerW> enc;
  const float *enc_ln_w = nullptr, *enc_ln_b = nullptr;
  const void* tok_emb = nullptr;  // [n_vocab][d] rows (embedding gather)
  DecWeight tok_p;                // fragment-tiled copy (logits GEMM)
  const float* dec_pe = nullptr;
  std::vector<DecLayerW> dec;
  const void* cross_w = nullptr;
  const float* cross_b = nullptr;
  bool mx = false;  // MX-fp8 encoder / cross-K/V GEMMs
  bool dec8 = false;  // MX-fp8 decoder weights (mx with a bf16 model)
  bool kv8 = false;   // MX-fp8 cross K/V cache (mx)
  MxW cross_x;
  const float *dec_ln_w = nullptr, *dec_ln_b = nullptr;
  int space_id = -1;
  std::vector<int> nst_ids;  // suppress_nst token ids
};

struct Segment {
  int64_t t0, t1;
  std::string text;
  float no_speech_prob;
  std::vector<mwx_token_data> tokens;
  bool speaker_turn_next;
};

struct State {
  Context* ctx = nullptr;
  hipStream_t stream = nullptr;
  // encoder stream (MWX_STREAM_PRIO=enc_low / both): the encoder of a batch runs
  // on a low-priority stream, ordered after / before `stream` by two events,
  // so a concurrent batch's latency-bound decode chain is dispatched first
  hipStream_t estream = nullptr;
  hipEvent_t ev_e0 = nullptr, ev_e1 = nullptr;
  // encoder workspace (clip-batched)
  DBuf pcm, mel, melmax, melT, h1p, x, h, q, k, vt, o, ff, enc, cross_k, cross_v;
  DBuf cross_ks, cross_vs;  // MX-fp8 cross cache: E8M0 scales (kv8)
  bool cross_kv8 = false;   // layout of cross_k / cross_v
  DBuf energy, pcm16;
  DBuf meld, melpart;  // batched log-mel: per-clip descriptors, partial maxima
  // incremental log-mel (streaming re-transcription of a growing buffer):
  // ping-pong slots of this state's previous samples and raw log-mel
  DBuf melc_pcm[2], melc_raw[2];
  int melc_slot = 0;  // slot holding the previous call's data
  int melc_n = 0;     // its samples (0: nothing cached)
  int melc_len = 0;   // its n_len
  DBuf aq, as;  // MX-fp8 activations (codes [rows][K], scales [rows][K/32])
  DBuf ibuf;  // small int arrays (slot maps)
  DBuf pro_pcm, pro_desc, pro_fs, pro_ft, pro_fc, pro_out;  // segment prosody
  DBuf rs_in, rs_out, rs_pos, rs_coef;                      // resampler
  // pinned host staging of the per-step decode control / result records
  // (DMA straight from / to page-locked memory: no runtime bounce buffer)
  void* pin = nullptr;
  size_t pin_n = 0;
  void* pinned(size_t bytes) {
    if (bytes > pin_n) {
      std::lock_guard<std::recursive_mutex> lock(capture_mutex());
      if (pin) (void)hipHostFree(pin);
      pin = nullptr;
      pin_n = 0;
      HIPC(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
      pin_n = bytes;
    }
    return pin;
  }
  // run-ahead greedy decode: device row states [R] + step counter, prompts
  // [R][Tctx], and a pinned ring of per-step reports the advance kernel
  // writes (RUN_SLOTS slots of R rows), one event per slot
  static constexpr int RUN_SLOTS = 4;
  DBuf rrun, rprompt;
  void* rep_pin = nullptr;
  size_t rep_n = 0;
  hipEvent_t ev_step[RUN_SLOTS] = {};
  RunReport* report_ring(size_t bytes) {
    if (bytes > rep_n) {
      std::lock_guard<std::recursive_mutex> lock(capture_mutex());
      if (rep_pin) (void)hipHostFree(rep_pin);
      rep_pin = nullptr;
      rep_n = 0;
      HIPC(hipHostMalloc(&rep_pin, bytes, hipHostMallocMapped | hipHostMallocCoherent));
      rep_n = bytes;
    }
    return (RunReport*)rep_pin;
  }
  // decoder workspace (row-batched)
  DBuf xd, xd2, hd, qd, od, ffd, logits, kself, vself, stepin, ctl, tokout, probs, logprobs, smask;
  DBuf pqkv, pres, pq;  // split-K partial slabs of the decode GEMMs
  // batched prompt prefill: virtual-row inputs [tok|pos|act|xidx|crow] and the
  // layer stack's activations / slabs for up to MWX_PREFILL_ROWS virtual rows
  DBuf pf_in, pf_x, pf_h, pf_o, pf_ff, pf_pqkv, pf_pres, pf_pq;
  // the prefill's host-side inputs of all chunks: read by its stream-ordered
  // uploads, rewritten only by the next prefill (after that window's step
  // synchronizes)
  std::vector<int> pf_hin;
  // counters (mwx_test_decode_counters): decode steps launched, prompt
  // positions prefilled
  long n_steps = 0, n_prefill = 0;
  // (mwx_test_window_counters): clip windows decoded, decode attempts run
  // (one per window and temperature tried: attempts - windows = fallbacks)
  long n_windows = 0, n_attempts = 0;
  // decode steps x clips with a live row in them (a clip's cross K/V is read
  // once per step by the grouped / per-row cross-attention): the bench's
  // bytes-per-launch model for legs whose clips finish at different steps
  long n_clip_steps = 0;
  // run-ahead attempts redone on the host loop (mwx_test_runahead_fallbacks)
  long n_ra_fallback = 0;
  DBuf lpflt, lpparts, lpres;  // logits-processing scratch
  // beam search KV hand-over without copies: per row, positions below
  // kvown[row] are read from row kvmap[row][pos] (host copies in kvmap_h/kvown_h)
  DBuf kvmap, kvown;
  std::vector<int> kvmap_h, kvown_h;
  // pinned mirrors of kvmap_h / kvown_h: the map uploads of a beam step are
  // asynchronous DMAs (a pageable 287-KB upload per step blocked the host)
  int* kvmap_pin = nullptr;
  size_t kvmap_pin_n = 0;
  // pinned host staging of the batch's signal energy (token timestamps): the
  // per-clip D2H copies are async DMAs, not pageable copies that block the
  // host before the encoder is queued
  float* energy_pin = nullptr;
  size_t energy_pin_n = 0;
  int cross_cap = 0;  // cross cache slots
  int row_cap = 0;    // self cache rows
  std::vector<Segment> result_all;
  int lang_id = 0;
  std::mt19937 rng0 = std::mt19937(0);  // decoders[0].rng persists per state
  // sampling / beam search: u of every draw (host RNG) in, draws out
  DBuf du, dnd, ddraw, dneed;
  int draw_k = 1;  // draws per row slot (KD)
  std::vector<Draw> draws_h;
  // perf: event pairs around launches of one kernel class. Eager launches
  // use perf_ev; launches captured into a decode-step graph use perf_gev (the
  // graph re-records them on every replay; harvested after each replay).
  // Several classes may be enabled at once (comma-separated): every pair is
  // tagged with its class and accumulated per class.
  std::string perf_class;                 // the enabled list ("" = off)
  std::vector<std::string> perf_classes;  // parsed
  std::vector<hipEvent_t> perf_ev, perf_gev;
  std::vector<int> perf_tag, perf_gtag;   // class of each event pair
  size_t perf_used = 0, perf_gused = 0;
  bool capturing = false;
  bool capture_perf = true;  // false while capturing the uninstrumented step graph
  std::vector<double> perf_acc_ms;
  std::vector<long> perf_acc_n;
  // launch spans (classes "<class>.span", kcommon.h span_start): device stamp
  // pairs [SPAN_SLOTS][2], graph slots first (zeroed by one memset node at the
  // head of each instrumented graph), eager slots after them (zeroed per
  // launch); the class of each slot; a pinned host copy and its stream
  static constexpr int SPAN_G = 256, SPAN_E = 2048;  // slots of SPAN_SLOT_U64 u64 (1 KB)
  DBuf perf_span;
  unsigned long long* span_host = nullptr;
  hipStream_t span_stream = nullptr;
  std::vector<int> span_gtag, span_etag;
  size_t span_gused = 0, span_eused = 0;
  double span_tick_ms = 0.0;  // ms per s_memrealtime tick
};

static void harvest_events(std::vector<hipEvent_t>& ev, const std::vector<int>& tag, size_t used,
                           State& S) {
  for (size_t i = 0; i + 1 < used; i += 2) {
    float ms = 0.0f;
    HIPC(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    const int c = tag[i / 2];
    S.perf_acc_ms[c] += ms;
    S.perf_acc_n[c] += 1;
  }
}

static int perf_class_index(const State& S, const char* cls);

// Launch spans: accumulate the (end - start) of the used slots of one region
// into their classes (graph: after an instrumented replay has completed;
// eager: after the state's stream has drained)
static void harvest_spans(State& S, bool graph, hipStream_t zs = nullptr) {
  const size_t n = graph ? S.span_gused : S.span_eused;
  if (n == 0 || !S.span_host || !S.span_stream) return;
  const size_t base = graph ? 0 : State::SPAN_G;
  const size_t su = SPAN_SLOT_U64;
  HIPC(hipMemcpyAsync(S.span_host, (unsigned long long*)S.perf_span.p + su * base, n * su * 8,
                      hipMemcpyDeviceToHost, S.span_stream));
  HIPC(hipStreamSynchronize(S.span_stream));
  const std::vector<int>& tag = graph ? S.span_gtag : S.span_etag;
  for (size_t i = 0; i < n; ++i) {
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int sh = 0; sh < SPAN_SHARDS; ++sh) {
      const unsigned long long a = S.span_host[su * i + 16 * sh], b = S.span_host[su * i + 16 * sh + 1];
      if (a) t0 = std::min(t0, ~a);
      t1 = std::max(t1, b);
    }
    if (t0 == ~0ull || t1 < t0) continue;  // (not launched)
    const int c = tag[i];
    S.perf_acc_ms[c] += (double)(t1 - t0) * S.span_tick_ms;
    S.perf_acc_n[c] += 1;
  }
  // re-zeroed for the next launches, ordered before them on the state's
  // stream (graph slots: the next instrumented replay is queued after this)
  HIPC(hipMemsetAsync((unsigned long long*)S.perf_span.p + su * base, 0, n * su * 8,
                      zs ? zs : S.stream));
  if (!graph) S.span_eused = 0;
}

static int perf_class_index(const State& S, const char* cls) {
  for (size_t i = 0; i < S.perf_classes.size(); ++i)
    if (S.perf_classes[i] == cls) return (int)i;
  return -1;
}

// True when a PerfScope of class `cls` would record events right now.
static bool perf_on(const State& s, const char* cls) {
  if (s.perf_class.empty() || (s.capturing && !s.capture_perf)) return false;
  return perf_class_index(s, cls) >= 0;
}

// The stamp pair a launch of class `cls` writes its span to (kcommon.h
// span_start / span_end) when "<cls>.span" is an enabled perf class, else
// nullptr. Slots are used once between two harvests, which re-zero them on
// the state's stream (no memset node in the instrumented graph: a blit node
// there lengthened the instrumented replays).
static unsigned long long* span_slot(State& S, const char* cls, hipStream_t s) {
  if (S.perf_class.empty() || (S.capturing && !S.capture_perf) || !S.perf_span.p) return nullptr;
  const int ci = perf_class_index(S, (std::string(cls) + ".span").c_str());
  if (ci < 0) return nullptr;
  unsigned long long* base = (unsigned long long*)S.perf_span.p;
  if (S.capturing) {
    // (graph slots are zero when the instrumented graph replays: zeroed at
    // allocation and re-zeroed on the state's stream by each harvest, which
    // follows every instrumented replay)
    if (S.span_gused >= (size_t)State::SPAN_G) return nullptr;
    if (S.span_gtag.size() <= S.span_gused) S.span_gtag.resize(S.span_gused + 1);
    S.span_gtag[S.span_gused] = ci;
    return base + SPAN_SLOT_U64 * S.span_gused++;
  }
  if (S.span_eused >= (size_t)State::SPAN_E) {
    HIPC(hipStreamSynchronize(s));
    harvest_spans(S, false, s);
  }
  // (eager slots are zero: allocated zeroed, re-zeroed by each harvest)
  unsigned long long* p = base + SPAN_SLOT_U64 * (State::SPAN_G + S.span_eused);
  if (S.span_etag.size() <= S.span_eused) S.span_etag.resize(S.span_eused + 1);
  S.span_etag[S.span_eused++] = ci;
  return p;
}

// Records a start/stop HIP event pair around a launch when `cls` is the
// state's enabled perf class.
struct PerfScope {
  State& S;
  bool on;
  hipEvent_t stop = nullptr;
  hipStream_t stream;
  PerfScope(State& s, const char* cls, hipStream_t strm = nullptr)
      : S(s), on(false), stream(strm ? strm : s.stream) {
    if (s.perf_class.empty() || (s.capturing && !s.capture_perf)) return;
    const int ci = perf_class_index(s, cls);
    if (ci < 0) return;
    on = true;
    std::vector<hipEvent_t>& ev = S.capturing ? S.perf_gev : S.perf_ev;
    std::vector<int>& tag = S.capturing ? S.perf_gtag : S.perf_tag;
    size_t& used = S.capturing ? S.perf_gused : S.perf_used;
    while (ev.size() < used + 2) {
      hipEvent_t e;
      HIPC(hipEventCreate(&e));
      ev.push_back(e);
    }
    if (tag.size() < used / 2 + 1) tag.resize(used / 2 + 1);
    tag[used / 2] = ci;
    record(ev[used]);
    stop = ev[used + 1];
    used += 2;
  }
  // Eager: hipEventRecord. While the stream is being captured, an explicit
  // event-record node is appended to the capturing graph instead (HIP 7.2
  // cannot time events recorded *through* capture; explicit nodes time fine).
  void record(hipEvent_t e) {
    if (!S.capturing) {
      HIPC(hipEventRecord(e, stream));
      return;
    }
    hipStreamCaptureStatus cs;
    unsigned long long cid = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    HIPC(hipStreamGetCaptureInfo_v2(stream, &cs, &cid, &g, &deps, &ndeps));
    hipGraphNode_t node;
    HIPC(hipGraphAddEventRecordNode(&node, g, deps, ndeps, e));
    HIPC(hipStreamUpdateCaptureDependencies(stream, &node, 1, hipStreamSetCaptureDependencies));
  }
  ~PerfScope() {
    if (!on) return;
    try {
      record(stop);
    } catch (...) {
    }
  }
};

// ---------------------------------------------------------------------------
// model upload
// ---------------------------------------------------------------------------
static const FileTensor* find_t(const ModelFile& mf, const std::string& n) {
  auto it = mf.tensors.find(n);
  return it == mf.tensors.end() ? nullptr : &it->second;
}

// f32 values of a whole tensor: f32 / f16 / bf16 exactly, block-quantized
// types through ggml's dequantize_row_q* (quant.cpp)
static std::vector<float> tensor_f32(const FileTensor& t) {
  const int64_t n = t.nelements();
  std::vector<float> v(n);
  switch (t.type) {
    case GGML_F32: memcpy(v.data(), t.data.data(), n * 4); break;
    case GGML_F16:
    case GGML_BF16:
      for (int64_t i = 0; i < n; ++i) {
        uint16_t h;
        memcpy(&h, t.data.data() + i * 2, 2);
        v[i] = t.type == GGML_F16 ? f16_to_f32(h) : bf16_to_f32(h);
      }
      break;
    default: ggml_dequantize(t.type, t.data.data(), v.data(), n); break;
  }
  return v;
}

namespace {
struct Arena {
  std::vector<uint8_t> host;
  std::vector<std::pair<size_t, const void**>> fixups;
  size_t add(const void* src, size_t bytes, const void** slot) {
    const size_t off = align_up(host.size(), 256);
    host.resize(off + bytes);
    if (src) memcpy(host.data() + off, src, bytes);
    fixups.emplace_back(off, slot);
    return off;
  }
  uint8_t* at(size_t off) { return host.data() + off; }
};
}  // namespace

static bool upload_model(Context& C, const ModelFile& mf) {
  const Hparams& hp = C.hp;
  const int d = hp.n_audio_state, dt = hp.n_text_state;
  if (d != dt || d % 128 != 0 || d / hp.n_audio_head != 64 || dt / hp.n_text_head != 64) {
    MWX_LOG_ERROR("mwx: unsupported dims (state %d/%d heads %d/%d)\n", d, dt, hp.n_audio_head,
                  hp.n_text_head);
    return false;
  }
  const FileTensor* te = find_t(mf, "decoder.token_embedding.weight");
  if (!te) return false;
  C.wtype = te->type == GGML_BF16 ? GGML_BF16 : GGML_F16;
  const bool bf = C.wtype == GGML_BF16;
  C.cpad = hp.n_mels <= 64 ? 64 : 128;
  if (hp.n_mels > 128) return false;
  Arena A;
  bool ok = true;
  auto need = [&](const std::string& n) -> const FileTensor* {
    const FileTensor* t = find_t(mf, n);
    if (!t) {
      MWX_LOG_ERROR("mwx: missing tensor '%s'\n", n.c_str());
      ok = false;
    }
    return t;
  };
  auto f32v = [&](const std::string& n, const float** slot, int64_t expect) {
    const FileTensor* t = need(n);
    if (!t) return;
    if (t->nelements() != expect) {
      MWX_LOG_ERROR("mwx: tensor '%s' has %lld elements, expected %lld\n", n.c_str(),
                    (long long)t->nelements(), (long long)expect);
      ok = false;
      return;
    }
    const std::vector<float> v = tensor_f32(*t);
    A.add(v.data(), v.size() * 4, (const void**)slot);
  };
  // 16-bit weight rows in the model type, concatenated from several tensors
  auto rows16 = [&](const std::vector<std::string>& names, int64_t K, std::vector<uint16_t>& out,
                    int64_t& rows) -> bool {
    std::vector<const FileTensor*> ts;
    rows = 0;
    for (const auto& n : names) {
      const FileTensor* t = need(n);
      if (!t) return false;
      if (t->ne[0] != K) {
        MWX_LOG_ERROR("mwx: tensor '%s' inner dim %lld != %lld\n", n.c_str(), (long long)t->ne[0],
                      (long long)K);
        ok = false;
        return false;
      }
      ts.push_back(t);
      rows += t->nelements() / K;
    }
    out.resize((size_t)rows * K);
    uint16_t* dst = out.data();
    for (const FileTensor* t : ts) {
      const int64_t n = t->nelements();
      const int want = bf ? GGML_BF16 : GGML_F16;
      if (t->type == want) {
        memcpy(dst, t->data.data(), n * 2);
      } else {  // (quantized files: dequantized once, computed in f16)
        const std::vector<float> f = tensor_f32(*t);
        for (int64_t i = 0; i < n; ++i) dst[i] = bf ? f32_to_bf16(f[i]) : f32_to_f16(f[i]);
      }
      dst += n;
    }
    return true;
  };
  // row layout [N][K] (encoder GEMMs, embedding gather); with `mx`, also the
  // MX-fp8 quantization of the same 16-bit values (fp8 compute mode)
  auto w16 = [&](const std::vector<std::string>& names, int64_t K, const void** slot,
                 MxW* mx = nullptr) {
    std::vector<uint16_t> w;
    int64_t rows = 0;
    if (!rows16(names, K, w, rows)) return;
    A.add(w.data(), w.size() * 2, slot);
    if (!mx || !C.mx) return;
    if (K % 128) {
      MWX_LOG_ERROR("mwx: MX-fp8 compute needs inner dims that are multiples of 128\n");
      ok = false;
      return;
    }
    std::vector<uint8_t> q((size_t)rows * K), sc((size_t)rows * (K / 32));
    std::vector<float> row(K);
    for (int64_t n = 0; n < rows; ++n) {
      for (int64_t k = 0; k < K; ++k)
        row[k] = bf ? bf16_to_f32(w[(size_t)n * K + k]) : f16_to_f32(w[(size_t)n * K + k]);
      mx_quantize_row(row.data(), (int)K, q.data() + (size_t)n * K, sc.data() + (size_t)n * (K / 32));
    }
    A.add(q.data(), q.size(), (const void**)&mx->q);
    A.add(sc.data(), sc.size(), (const void**)&mx->s);
  };
  // decode-GEMM fragment tiles (see kernels.h: pack_index); with dec8 the
  // MX-fp8 form instead: codes in the same order (1 byte per element) and the
  // E8M0 scale of each (row, 32-deep k-step) at [(strip * K/32 + kt) * 16 +
  // row % 16]. `rounded` (optional) receives the MX-rounded values in the
  // model type (exact in bf16), for the embedding gather copy.
  auto w16p = [&](const std::vector<std::string>& names, int64_t K, DecWeight* slot,
                  std::vector<uint16_t>* rounded = nullptr) {
    std::vector<uint16_t> w;
    int64_t rows = 0;
    if (!rows16(names, K, w, rows)) return;
    if (K % 32) {
      MWX_LOG_ERROR("mwx: decoder weight inner dim %lld is not a multiple of 32\n", (long long)K);
      ok = false;
      return;
    }
    const int64_t np = (rows + 15) / 16 * 16;
    if (!C.dec8) {
      std::vector<uint16_t> p((size_t)np * K, 0);
      for (int64_t n = 0; n < rows; ++n)
        for (int64_t k = 0; k < K; ++k) p[pack_index(n, k, K)] = w[(size_t)n * K + k];
      A.add(p.data(), p.size() * 2, &slot->w);
      return;
    }
    const int64_t KT = K / 32;
    std::vector<uint8_t> q((size_t)np * K, 0), sc((size_t)(np / 16) * KT * 16, 127);
    std::vector<float> row(K);
    std::vector<uint8_t> rq(K), rs(KT);
    if (rounded) rounded->assign(w.size(), 0);
    for (int64_t n = 0; n < rows; ++n) {
      for (int64_t k = 0; k < K; ++k) row[k] = bf16_to_f32(w[(size_t)n * K + k]);
      mx_quantize_row(row.data(), (int)K, rq.data(), rs.data());
      for (int64_t k = 0; k < K; ++k) q[pack_index(n, k, K)] = rq[k];
      for (int64_t kt = 0; kt < KT; ++kt) sc[((n >> 4) * KT + kt) * 16 + (n & 15)] = rs[kt];
      if (rounded)
        for (int64_t k = 0; k < K; ++k)
          (*rounded)[(size_t)n * K + k] = f32_to_bf16(mx_dequant(rq[k], rs[k / 32]));
    }
    A.add(q.data(), q.size(), (const void**)&slot->q);
    A.add(sc.data(), sc.size(), (const void**)&slot->s);
  };
  // filters + mel tables
  A.add(mf.filters.data(), mf.filters.size() * 4, (const void**)&C.d_filters);
  {
    std::vector<float> tab(1200);
    for (int i = 0; i < 400; ++i) {
      tab[i] = (float)(0.5 * (1.0 - cosf((float)((2.0 * M_PI * i) / 400))));
      const double theta = (2 * M_PI * i) / 400;
      tab[400 + i] = cosf((float)theta);
      tab[800 + i] = sinf((float)theta);
    }
    A.add(tab.data(), tab.size() * 4, (const void**)&C.d_tables);
  }
  // conv stem: repack [D][C][3] -> [D][3][Cpad] / [D][3][D], always f16 (im2col type)
  {
    const FileTensor* c1 = need("encoder.conv1.weight");
    const FileTensor* c2 = need("encoder.conv2.weight");
    if (!c1 || !c2) return false;
    const int nm = hp.n_mels, cp = C.cpad;
    const std::vector<float> f1 = tensor_f32(*c1), f2 = tensor_f32(*c2);
    std::vector<uint16_t> w1((size_t)d * 3 * cp, 0), w2((size_t)d * 3 * d);
    for (int o = 0; o < d; ++o)
      for (int c = 0; c < nm; ++c)
        for (int kk = 0; kk < 3; ++kk)
          w1[((size_t)o * 3 + kk) * cp + c] = f32_to_f16(f1[((size_t)o * nm + c) * 3 + kk]);
    for (int o = 0; o < d; ++o)
      for (int c = 0; c < d; ++c)
        for (int kk = 0; kk < 3; ++kk)
          w2[((size_t)o * 3 + kk) * d + c] = f32_to_f16(f2[((size_t)o * d + c) * 3 + kk]);
    A.add(w1.data(), w1.size() * 2, (const void**)&C.conv1_w);
    A.add(w2.data(), w2.size() * 2, (const void**)&C.conv2_w);
  }
  f32v("encoder.conv1.bias", &C.conv1_b, d);
  f32v("encoder.conv2.bias", &C.conv2_b, d);
  f32v("encoder.positional_embedding", &C.enc_pe, (int64_t)hp.n_audio_ctx * d);
  C.enc.resize(hp.n_audio_layer);
  for (int l = 0; l < hp.n_audio_layer; ++l) {
    const std::string p = "encoder.blocks." + std::to_string(l);
    EncLayerW& L = C.enc[l];
    f32v(p + ".attn_ln.weight", &L.ln1_w, d);
    f32v(p + ".attn_ln.bias", &L.ln1_b, d);
    f32v(p + ".mlp_ln.weight", &L.ln2_w, d);
    f32v(p + ".mlp_ln.bias", &L.ln2_b, d);
    w16({p + ".attn.query.weight", p + ".attn.key.weight", p + ".attn.value.weight"}, d, &L.qkv_w,
        &L.qkv_x);
    {
      const FileTensor* qb = need(p + ".attn.query.bias");
      const FileTensor* vb = need(p + ".attn.value.bias");
      if (!qb || !vb) return false;
      std::vector<float> b(3 * d, 0.0f);
      const std::vector<float> fq = tensor_f32(*qb), fv = tensor_f32(*vb);
      for (int i = 0; i < d; ++i) {
        b[i] = fq[i];
        b[2 * d + i] = fv[i];
      }
      A.add(b.data(), b.size() * 4, (const void**)&L.qkv_b);
    }
    w16({p + ".attn.out.weight"}, d, &L.o_w, &L.o_x);
    f32v(p + ".attn.out.bias", &L.o_b, d);
    w16({p + ".mlp.0.weight"}, d, &L.fc1_w, &L.fc1_x);
    f32v(p + ".mlp.0.bias", &L.fc1_b, 4 * d);
    w16({p + ".mlp.2.weight"}, 4 * d, &L.fc2_w, &L.fc2_x);
    f32v(p + ".mlp.2.bias", &L.fc2_b, d);
  }
  f32v("encoder.ln_post.weight", &C.enc_ln_w, d);
  f32v("encoder.ln_post.bias", &C.enc_ln_b, d);
  C.dec8 = C.mx && bf;
  C.kv8 = C.mx;
  if (C.dec8) {
    // the gather rows hold the same MX-rounded values as the logits tiles
    std::vector<uint16_t> r;
    w16p({"decoder.token_embedding.weight"}, dt, &C.tok_p, &r);
    if (ok) A.add(r.data(), r.size() * 2, &C.tok_emb);
  } else {
    w16({"decoder.token_embedding.weight"}, dt, &C.tok_emb);
    w16p({"decoder.token_embedding.weight"}, dt, &C.tok_p);
  }
  f32v("decoder.positional_embedding", &C.dec_pe, (int64_t)hp.n_text_ctx * dt);
  C.dec.resize(hp.n_text_layer);
  std::vector<std::string> cross_names;
  std::vector<float> cross_b;
  for (int l = 0; l < hp.n_text_layer; ++l) {
    const std::string p = "decoder.blocks." + std::to_string(l);
    DecLayerW& L = C.dec[l];
    f32v(p + ".attn_ln.weight", &L.ln1_w, dt);
    f32v(p + ".attn_ln.bias", &L.ln1_b, dt);
    f32v(p + ".cross_attn_ln.weight", &L.lnc_w, dt);
    f32v(p + ".cross_attn_ln.bias", &L.lnc_b, dt);
    f32v(p + ".mlp_ln.weight", &L.ln2_w, dt);
    f32v(p + ".mlp_ln.bias", &L.ln2_b, dt);
    w16p({p + ".attn.query.weight", p + ".attn.key.weight", p + ".attn.value.weight"}, dt, &L.qkv);
    {
      const FileTensor* qb = need(p + ".attn.query.bias");
      const FileTensor* vb = need(p + ".attn.value.bias");
      if (!qb || !vb) return false;
      std::vector<float> b(3 * dt, 0.0f);
      const std::vector<float> fq = tensor_f32(*qb), fv = tensor_f32(*vb);
      for (int i = 0; i < dt; ++i) {
        b[i] = fq[i];
        b[2 * dt + i] = fv[i];
      }
      A.add(b.data(), b.size() * 4, (const void**)&L.qkv_b);
    }
    w16p({p + ".attn.out.weight"}, dt, &L.o);
    f32v(p + ".attn.out.bias", &L.o_b, dt);
    w16p({p + ".cross_attn.query.weight"}, dt, &L.cq);
    f32v(p + ".cross_attn.query.bias", &L.cq_b, dt);
    w16p({p + ".cross_attn.out.weight"}, dt, &L.co);
    f32v(p + ".cross_attn.out.bias", &L.co_b, dt);
    w16p({p + ".mlp.0.weight"}, dt, &L.fc1);
    f32v(p + ".mlp.0.bias", &L.fc1_b, 4 * dt);
    w16p({p + ".mlp.2.weight"}, 4 * dt, &L.fc2);
    f32v(p + ".mlp.2.bias", &L.fc2_b, dt);
    cross_names.push_back(p + ".cross_attn.key.weight");
    cross_names.push_back(p + ".cross_attn.value.weight");
    const FileTensor* vb = need(p + ".cross_attn.value.bias");
    if (!vb) return false;
    for (int i = 0; i < dt; ++i) cross_b.push_back(0.0f);
    const std::vector<float> fv = tensor_f32(*vb);
    for (int i = 0; i < dt; ++i) cross_b.push_back(fv[i]);
  }
  w16(cross_names, d, &C.cross_w, &C.cross_x);
  A.add(cross_b.data(), cross_b.size() * 4, (const void**)&C.cross_b);
  f32v("decoder.ln.weight", &C.dec_ln_w, dt);
  f32v("decoder.ln.bias", &C.dec_ln_b, dt);
  if (!ok) return false;
  HIPC(hipMalloc(&C.arena, A.host.size()));
  HIPC(hipMemcpy(C.arena, A.host.data(), A.host.size(), hipMemcpyHostToDevice));
  for (auto& f : A.fixups) *f.second = (const uint8_t*)C.arena + f.first;
  HIPC(hipMalloc(&C.gelu_tab, GELU_TAB_N * sizeof(uint16_t)));
  gelu_table_build(C.gelu_tab, nullptr);
  HIPC(hipDeviceSynchronize());
  MWX_LOG_INFO("mwx: uploaded %.1f MB of weights to device %d\n", A.host.size() / 1048576.0,
               C.device);
  return true;
}

static const std::vector<std::string>& non_speech_tokens() {
  static const std::vector<std::string> v = {
      "\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^",
      "_", "`", "{", "|", "}", "~", "「", "」", "『", "』", "<<", ">>", "<<<", ">>>", "--",
      "---", "-(", "-[", "('", "(\"", "((", "))", "(((", ")))", "[[", "]]", "{{", "}}", "♪♪",
      "♪♪♪", "♩", "♪", "♫", "♬", "♭", "♮", "♯"};
  return v;
}

// ---------------------------------------------------------------------------
// batched driver
// ---------------------------------------------------------------------------
struct TsState {
  int64_t t_beg = 0, t_last = 0;
  int tid_last = 0;
  // the clip's signal energy (get_signal_energy), in the batch state's pinned
  // staging (State::energy_pin): written by an async copy queued before the
  // decode steps, read after them
  const float* energy = nullptr;
  int n_energy = 0;
};

struct ClipRun {
  State* st = nullptr;
  const void* pcm = nullptr;
  size_t pcm_off = 0;  // element offset in the device PCM staging
  int n = 0;
  int n_len = 0, n_len_org = 0, n_fft_frames = 0;
  size_t mel_off = 0;  // element offset of this clip's mel
  int seek = 0, seek_start = 0, seek_end = 0;
  bool finished = false;
  std::vector<int> prompt_past, prompt_init, prompt;
  int lang_id = 0;
  TsState ts;
  int enc_seek = -1;
  std::vector<std::mt19937> rng;  // per decoder j (j = 0 aliases st->rng0)
  float no_speech_prob = 0.0f;
};

struct Row {
  int clip = 0, dec = 0;
  int fed = 0;
  bool stopped = false, failed = false, completed = false, has_ts = false;
  int seek_delta = 3000, result_len = 0;
  double sum_logprobs_all = 0.0, sum_logprobs = -INFINITY, avg_logprobs = -INFINITY,
         entropy = 0.0, score = -INFINITY;
  std::vector<mwx_token_data> tokens;
};

template <typename T>
struct Driver {
  Context& C;
  State& S;
  hipStream_t st;
  const mwx_full_params& P;
  const Hparams& hp;
  int d, H, L_enc, L_dec, V, Tctx, Lp;
  LogitsConst LC;
  // run-ahead: the step's lp_pick runs inside the advance kernel (pick_in())
  bool pick_in_advance = false;
  PickIn pick_in() const {
    PickIn p;
    p.logits = (const float*)S.logits.p;
    p.flt = (const float*)S.lpflt.p;
    p.parts = (const LPPart*)S.lpparts.p;
    p.res = (const LPRes*)S.lpres.p;
    p.C = LC;
    return p;
  }
  // rows per clip in the current decode run (beam_size / best_of decoders are
  // consecutive rows of one clip); decode groups never split such a run
  int xgroup = 1;
  // test hook (mwx_test_encode_dump, one clip): host copies of the residual
  // stream after the stem and after every layer, and every layer's four GEMM
  // A operands before any MX quantization (attn LN out, attention out, mlp LN
  // out, GELU out; 16-bit bits)
  struct EncDump {
    float* x;        // [L_enc + 1][n_ctx][d]
    uint16_t* a[4];  // [L_enc][n_ctx][d] (a[3]: [L_enc][n_ctx][4d])
  };
  const EncDump* dump = nullptr;
  void dump_copy(void* dst, const void* src, size_t bytes) {
    HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
  }

  Driver(Context& c, State& s, const mwx_full_params& p)
      : C(c), S(s), st(s.stream), P(p), hp(c.hp) {
    d = hp.n_audio_state;
    H = hp.n_audio_head;
    L_enc = hp.n_audio_layer;
    L_dec = hp.n_text_layer;
    V = hp.n_vocab;
    Tctx = hp.n_text_ctx;
    Lp = (hp.n_audio_ctx + 7) & ~7;
    LC.n_vocab = V;
    LC.eot = C.vocab.token_eot;
    LC.beg = C.vocab.token_beg;
    LC.space_id = C.space_id;
    LC.suppress_blank = P.suppress_blank ? 1 : 0;
    LC.nosp_id = C.vocab.token_nosp;
    if (P.max_initial_ts > 0.0f) {
      const float precision = float(MWX_CHUNK_SIZE) / hp.n_audio_ctx;
      LC.max_initial_tid = C.vocab.token_beg + (int)std::round(P.max_initial_ts / precision);
    } else {
      LC.max_initial_tid = -1;
    }
  }

  const T* Wt(const void* p) const { return (const T*)p; }
  DecW<T> Dw(const DecWeight& x) const {
    return x.q ? DecW<T>(x.q, x.s) : DecW<T>((const T*)x.w);
  }

  // static suppression mask for this call's params
  void build_static_mask() {
    std::vector<float> m(V, 0.0f);
    const Vocab& vb = C.vocab;
    const float NI = -INFINITY;
    m[vb.token_not] = NI;
    if (P.no_timestamps)
      for (int i = vb.token_beg; i < V; ++i) m[i] = NI;
    m[vb.token_sot] = NI;
    m[vb.token_nosp] = NI;
    if (!P.tdrz_enable) m[vb.token_solm] = NI;
    m[vb.token_translate] = NI;
    m[vb.token_transcribe] = NI;
    m[vb.token_prev] = NI;
    for (int i = 0; i <= lang_max_id(); ++i) {
      const int tok = vb.token_sot + 1 + i;
      if (tok < V) m[tok] = NI;
    }
    if (P.suppress_nst)
      for (int id : C.nst_ids) m[id] = NI;
    if (P.bench_fixed_steps > 0) {
      m[vb.token_eot] = NI;
      for (int i = vb.token_beg; i < V; ++i) m[i] = NI;
    }
    float* dm = (float*)S.smask.get((size_t)V * 4);
    HIPC(hipMemcpyAsync(dm, m.data(), (size_t)V * 4, hipMemcpyHostToDevice, st));
  }

  // ---------------- encoder: nb windows -> cross K/V slots ----------------
  void encode(const std::vector<int>& clip_of_slot, const std::vector<int>& seek_of_slot,
              const std::vector<int>& nlen_of_slot, const std::vector<int>& cross_slot,
              long mel_clip_stride) {
    const int nb = (int)clip_of_slot.size();
    const int Lc = hp.n_audio_ctx, T2 = 2 * Lc, cp = C.cpad;
    const int M = nb * Lc;
    int* ib = (int*)S.ibuf.get(sizeof(int) * 4 * 4096);
    std::vector<int> hb(4 * 4096, 0);
    for (int i = 0; i < nb; ++i) {
      hb[i] = clip_of_slot[i];
      hb[4096 + i] = seek_of_slot[i];
      hb[2 * 4096 + i] = nlen_of_slot[i];
      hb[3 * 4096 + i] = cross_slot[i];
    }
    HIPC(hipMemcpyAsync(ib, hb.data(), hb.size() * 4, hipMemcpyHostToDevice, st));
    _Float16* melT = (_Float16*)S.melT.get((size_t)nb * (T2 + 2) * cp * 2, true);
    _Float16* h1p = (_Float16*)S.h1p.get((size_t)nb * (T2 + 2) * d * 2, true);
    float* x = (float*)S.x.get((size_t)M * d * 4);
    T* h = (T*)S.h.get((size_t)M * d * sizeof(T));
    _Float16* q = (_Float16*)S.q.get((size_t)M * d * 2);
    _Float16* k = (_Float16*)S.k.get((size_t)M * d * 2);
    _Float16* vt = (_Float16*)S.vt.get((size_t)nb * H * 64 * Lp * 2, true);
    T* o = (T*)S.o.get((size_t)M * d * sizeof(T));
    T* ff = (T*)S.ff.get((size_t)M * 4 * d * sizeof(T));
    T* enc = (T*)S.enc.get((size_t)M * d * sizeof(T));
    { PerfScope ps(S, "mel", st);
    launch_mel_window((const float*)S.mel.p, mel_clip_stride, ib, ib + 4096, ib + 2 * 4096,
                      hp.n_mels, T2, cp, melT, nb, st); }
    EpiParams e;
    // conv1 (k3 s1 p1) as a GEMM over overlapping rows of the padded window
    e.bias = C.conv1_b;
    e.gelu_tab = C.gelu_tab;
    e.c16 = h1p + d;
    e.ldc = d;
    e.c_bstride = (long)(T2 + 2) * d;
    { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
    gemm<_Float16>(EPI_GELU, true, melT, cp, (long)(T2 + 2) * cp, C.conv1_w, 3 * cp, T2, d,
                   3 * cp, nb, e, st); }
    // conv2 (k3 s2 p1) + GELU + positional embedding -> residual stream x
    e = EpiParams();
    e.bias = C.conv2_b;
    e.c32 = x;
    e.ldc = d;
    e.c_bstride = (long)Lc * d;
    e.pe = C.enc_pe;
    { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
    gemm<_Float16>(EPI_CONV2, false, h1p, 2 * d, (long)(T2 + 2) * d, C.conv2_w, 3 * d, Lc, d,
                   3 * d, nb, e, st); }
    const size_t md = (size_t)Lc * d;  // (dump: one clip)
    if (dump) dump_copy(dump->x, x, md * 4);
    const float kq_scale = 1.0f / sqrtf(64.0f);
    // fp8 compute: the A operand of every encoder / cross GEMM is the 16-bit
    // activation quantized to MX-fp8 (as the oracle's ORC_MXFP8 mode)
    uint8_t* aq = C.mx ? (uint8_t*)S.aq.get((size_t)M * 4 * d) : nullptr;
    uint8_t* as = C.mx ? (uint8_t*)S.as.get((size_t)M * 4 * d / 32) : nullptr;
    auto mgemm = [&](int epi, const T* a, int Kd, const MxW& w, const void* w16, int N,
                     EpiParams ep, bool out_f16 = false) {
      if (C.mx) {
        mx_quantize<T>(a, Kd, M, Kd, aq, as, st);
        ep.sa = as;
        ep.sw = w.s;
        gemm_mx<T>(epi, aq, Kd, 0, w.q, Kd, M, N, Kd, 1, ep, st);
      } else {
        gemm<T>(epi, out_f16, a, Kd, 0, Wt(w16), Kd, M, N, Kd, 1, ep, st);
      }
    };
    for (int l = 0; l < L_enc; ++l) {
      const EncLayerW& W = C.enc[l];
      layer_norm<T>(x, W.ln1_w, W.ln1_b, h, M, d, nullptr, st);
      e = EpiParams();
      e.bias = W.qkv_b;
      e.q = q;
      e.k = k;
      e.v = vt;
      e.L = Lc;
      e.H = H;
      e.d = d;
      e.ldv = Lp;  // V^T rows are padded to Lp (16-B aligned tile loads)
      { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
      mgemm(EPI_ENC_QKV, h, d, W.qkv_x, W.qkv_w, 3 * d, e); }
      if (dump) dump_copy(dump->a[0] + l * md, h, md * 2);
      { PerfScope ps(S, "enc_attn", st);
      enc_attention<T>(q, k, vt, o, nb, H, Lc, kq_scale, st); }
      if (dump) dump_copy(dump->a[1] + l * md, o, md * 2);
      e = EpiParams();
      e.bias = W.o_b;
      e.c32 = x;
      e.r32 = x;
      e.ldc = d;
      { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
      mgemm(EPI_RES, o, d, W.o_x, W.o_w, d, e); }
      layer_norm<T>(x, W.ln2_w, W.ln2_b, h, M, d, nullptr, st);
      e = EpiParams();
      e.bias = W.fc1_b;
      e.gelu_tab = C.gelu_tab;
      e.c16 = ff;
      e.ldc = 4 * d;
      { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
      mgemm(EPI_GELU, h, d, W.fc1_x, W.fc1_w, 4 * d, e); }
      if (dump) {
        dump_copy(dump->a[2] + l * md, h, md * 2);
        dump_copy(dump->a[3] + l * 4 * md, ff, 4 * md * 2);
      }
      e = EpiParams();
      e.bias = W.fc2_b;
      e.c32 = x;
      e.r32 = x;
      e.ldc = d;
      { PerfScope ps(S, "enc_gemm", st);
      e.span = span_slot(S, "enc_gemm", st);
      mgemm(EPI_RES, ff, 4 * d, W.fc2_x, W.fc2_w, d, e); }
      if (dump) dump_copy(dump->x + (l + 1) * md, x, md * 4);
    }
    layer_norm<T>(x, C.enc_ln_w, C.enc_ln_b, enc, M, d, nullptr, st);
    // cross K/V of every decoder layer in one GEMM
    e = EpiParams();
    e.bias = C.cross_b;
    e.k = (_Float16*)S.cross_k.p;
    e.v = (_Float16*)S.cross_v.p;
    if (C.kv8) {  // codes in cross_k / cross_v, scales beside them
      e.ks8 = (uint8_t*)S.cross_ks.p;
      e.vs8 = (uint8_t*)S.cross_vs.p;
    }
    e.L = Lc;
    e.H = H;
    e.d = d;
    e.ncap = S.cross_cap;
    e.slot = ib + 3 * 4096;
    e.kscale = powf(64.0f, -0.25f);
    PerfScope ps(S, "cross_gemm", st);
    mgemm(EPI_CROSS_KV, enc, d, C.cross_x, C.cross_w, L_dec * 2 * d, e);
  }

  void ensure_cross(int n_slots) {
    // f16 cache: 2 B per element; MX-fp8 cache: 1-B codes + 2 scale bytes per
    // (time, head) row of 64
    const size_t per = (size_t)L_dec * hp.n_audio_ctx * d * (C.kv8 ? 1 : 2);
    if (S.cross_cap < n_slots || S.cross_kv8 != C.kv8) {
      S.cross_k.release();
      S.cross_v.release();
      S.cross_ks.release();
      S.cross_vs.release();
      S.cross_k.get(per * n_slots);
      S.cross_v.get(per * n_slots);
      if (C.kv8) {
        const size_t ps = (size_t)L_dec * hp.n_audio_ctx * H * 2;
        S.cross_ks.get(ps * n_slots);
        S.cross_vs.get(ps * n_slots);
      }
      S.cross_cap = n_slots;
      S.cross_kv8 = C.kv8;
    }
  }

  void ensure_rows(int R) {
    if (S.row_cap < R) {
      S.kself.release();
      S.vself.release();
      const size_t per = (size_t)L_dec * H * Tctx * 64 * 2;
      S.kself.get(per * R);
      S.vself.get(per * R);
      S.row_cap = R;
    }
    S.pqkv.get((size_t)ks_d() * R * 3 * d * 4);
    S.pres.get((size_t)ks_res() * R * d * 4);
    S.pq.get((size_t)ks_d() * R * d * 4);
    S.xd.get((size_t)R * d * 4, true);
    S.xd2.get((size_t)R * d * 4, true);  // (the residual's other buffer: LayerNorm folded at R = 1)
    // decode-GEMM A operands (fragment tiles), rows padded to the 64-row block
    const size_t R64 = (size_t)(R + 63) / 64 * 64;
    S.hd.get(R64 * d * sizeof(T), true);
    S.od.get(R64 * d * sizeof(T), true);
    S.ffd.get(R64 * 4 * d * sizeof(T), true);
    S.logits.get((size_t)R * V * 4);
    S.lpflt.get((size_t)R * V * 4);
    S.lpparts.get((size_t)R * LP_G * sizeof(LPPart));
    S.lpres.get((size_t)R * LP_G * sizeof(LPRes));
    S.stepin.get((size_t)R * 4 * 4);
    S.kvmap.get((size_t)R * Tctx * 4, true);
    S.kvown.get((size_t)R * 4);
    // no taken-over histories: every row reads only its own cache
    HIPC(hipMemsetAsync(S.kvown.p, 0, (size_t)R * 4, st));
    S.ctl.get((size_t)R * sizeof(RowCtl));
    S.tokout.get((size_t)R * sizeof(TokOut));
  }

  // beam search: rows take over other rows' self-attention histories
  // (triples dst, src, npos; whisper.cpp copies the KV cells). Histories are
  // immutable, so the hand-over only rewrites the destination's position map:
  // kvmap[dst][0..npos) = where src reads those positions (pre-move state,
  // so any permutation is safe), kvown[dst] = npos.
  void reset_kv_maps(int R) {
    HIPC(hipStreamSynchronize(st));  // no map upload may still read the host arrays
    S.kvmap_h.assign((size_t)R * Tctx, 0);
    S.kvown_h.assign(R, 0);
    const size_t need = (size_t)R * Tctx + R;  // [kvmap | kvown]
    if (S.kvmap_pin_n < need) {
      std::lock_guard<std::recursive_mutex> lock(capture_mutex());
      if (S.kvmap_pin) (void)hipHostFree(S.kvmap_pin);
      S.kvmap_pin = nullptr;
      S.kvmap_pin_n = 0;
      HIPC(hipHostMalloc((void**)&S.kvmap_pin, need * 4, hipHostMallocDefault));
      S.kvmap_pin_n = need;
    }
    memset(S.kvmap_pin, 0, need * 4);
    HIPC(hipMemsetAsync(S.kvown.p, 0, (size_t)R * 4, st));
  }
  void copy_kv_rows(const std::vector<int>& triples) {
    const int n = (int)triples.size() / 3;
    if (n == 0) return;
    // pre-move state of the source rows (any permutation of moves is safe)
    std::vector<int> srow(S.kvown_h.size(), -1), snap;
    std::vector<int> own_src;
    for (int i = 0; i < n; ++i) {
      const int src = triples[3 * i + 1];
      if (srow[src] >= 0) continue;
      srow[src] = (int)own_src.size();
      own_src.push_back(S.kvown_h[src]);
      snap.insert(snap.end(), S.kvmap_h.begin() + (size_t)src * Tctx,
                  S.kvmap_h.begin() + (size_t)(src + 1) * Tctx);
    }
    int lo = 1 << 30, hi = -1;
    const size_t R = S.kvown_h.size();
    int* pmap = S.kvmap_pin;
    int* pown = S.kvmap_pin + R * Tctx;
    for (int i = 0; i < n; ++i) {
      const int dst = triples[3 * i], src = triples[3 * i + 1], npos = triples[3 * i + 2];
      const int si = srow[src];
      int* row = S.kvmap_h.data() + (size_t)dst * Tctx;
      for (int j = 0; j < npos; ++j) row[j] = j < own_src[si] ? snap[(size_t)si * Tctx + j] : src;
      S.kvown_h[dst] = npos;
      memcpy(pmap + (size_t)dst * Tctx, row, (size_t)Tctx * 4);
      pown[dst] = npos;
      lo = std::min(lo, dst);
      hi = std::max(hi, dst);
    }
    HIPC(hipMemcpyAsync((int*)S.kvmap.p + (size_t)lo * Tctx, pmap + (size_t)lo * Tctx,
                        (size_t)(hi - lo + 1) * Tctx * 4, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync((int*)S.kvown.p + lo, pown + lo, (size_t)(hi - lo + 1) * 4,
                        hipMemcpyHostToDevice, st));
    // (ordered before the next step on this stream; the host arrays are next
    // written after that step's synchronize, or in reset_kv_maps)
  }

  // one decoder step for all R rows on the state's stream; inputs already in
  // S.stepin / S.ctl
  void decode_step(int R, bool want_probs) { decode_rows(R, want_probs, st); }

  // The rows one pass of the decoder layer stack runs on: a decode step's
  // rows (one position each), or the virtual rows of a prompt prefill (one
  // per (row, prompt position)).
  struct LayerRows {
    int n = 0;
    const int *tok = nullptr, *pos = nullptr, *act = nullptr, *xidx = nullptr;
    // prefill: the self-cache row of each virtual row (nullptr: row = its own)
    const int* crow = nullptr;
    float* xd = nullptr;
    float* xd2 = nullptr;  // the residual's second buffer (nullptr: no LayerNorm folding)
    T *hd = nullptr, *od = nullptr, *ffd = nullptr;
    float *Pqkv = nullptr, *Pres = nullptr, *Pq = nullptr;
    _Float16 *kself = nullptr, *vself = nullptr;  // layer-0 self cache of row 0
    const int *kvmap = nullptr, *kvown = nullptr;
    int map_row0 = 0;
    int xgroup = 1;
    // prefill: the K/V of every virtual row are appended to the self cache
    // before the self-attention (a position reads the prompt positions before
    // it, which other virtual rows of the same launch produce), and the
    // cross-attention runs in groups of 8 virtual rows of one clip (one K/V
    // stream per group; every row's arithmetic is the single-row kernel's)
    bool prefill = false;
  };

  // One pass of the decoder layer stack over a set of rows, in parts: the
  // embedding, and per layer the chain up to the cross-attention's query
  // projection (pre), the cross-attention (cross) and the chain after it
  // (post); run_layers runs them in order on one stream.
  struct LayerRun {
    float* xd = nullptr;  // the residual stream's buffer
    int k1 = 0, k2 = 0, k3 = 0, k4 = 0;
    bool k5 = false;
    int ks_prev = 0;  // the last FFN2's split-K factor and bias (folded into
    const float* bias_prev = nullptr;  // the next consumer)
    bool embed = false;  // the first LayerNorm forms x from the embeddings
  };
  void layers_begin(const LayerRows& rw, LayerRun& c, hipStream_t) {
    c = LayerRun{};
    c.xd = rw.xd;
    c.embed = true;  // (no launch: layer 0's LN1 embeds, ln_dec EmbedIn)
  }
  // The d- and 3d-wide projections run as split-K GEMMs writing f32 partial
  // slabs; each consumer (LN: bias + residual, attention: bias/scale/f16 and
  // the KV-cache append) folds the slabs in, so no launch is added.
  // the LayerNorm fold at one row (layer_pre): x = the residual now (c.xd),
  // moving to the other buffer; P / KS / pbias the producer's slabs and bias
  bool ln_folds(const LayerRows& rw) const {
    return rw.n == 1 && rw.xd2 && !rw.prefill && ln_fold_on();
  }
  LnFuse ln_fuse(const LayerRows& rw, const LayerRun& c, const float* P, int KS,
                 const float* pbias, const float* w, const float* b) const {
    LnFuse f;
    f.x_in = c.xd;
    f.x_out = c.xd == rw.xd ? rw.xd2 : rw.xd;
    f.P = P;
    f.KS = KS;
    f.pstride = (long)rw.n * d;
    f.pbias = pbias;
    f.w = w;
    f.b = b;
    f.active = rw.act;
    return f;
  }
  void layer_pre(const LayerRows& rw, LayerRun& c, int l, hipStream_t s) {
    const int n = rw.n;
    const float kqs = powf(64.0f, -0.25f);
    const size_t layer_self = (size_t)S.row_cap * H * Tctx * 64;
    const DecLayerW& W = C.dec[l];
    _Float16* ks = rw.kself + l * layer_self;
    _Float16* vs = rw.vself + l * layer_self;
    T* hd = rw.hd;
    EmbedIn<T> emb;
    if (c.embed) {
      emb.te = Wt(C.tok_emb);
      emb.pe = C.dec_pe;
      emb.tok = rw.tok;
      emb.pos = rw.pos;
      emb.n_tok = V;
      emb.n_pos = Tctx;
      c.embed = false;
    }
    // one row (C2, single-clip requests): the LayerNorms before the QKV,
    // cross-Q and FFN1 projections are folded into those GEMMs
    // (gemm_splitk_ln / gemm_decode_ln: the same arithmetic, no launch of
    // their own); the residual moves to the other buffer at each.
    // MWX_LN_FOLD=0 keeps the separate launches (A/B).
    const bool fold = ln_folds(rw);
    c.k1 = 0;
    if (fold && !emb.te) {
      const LnFuse f = ln_fuse(rw, c, c.ks_prev ? rw.Pres : nullptr, c.ks_prev, c.bias_prev,
                               W.ln1_w, W.ln1_b);
      PerfScope ps(S, "dec_gemm", s);
      c.k1 = gemm_splitk_ln<T>(f, Dw(W.qkv), 3 * d, d, rw.Pqkv, s);
      if (c.k1) c.xd = f.x_out;
    }
    if (!c.k1) {
      layer_norm_dec<T>(c.xd, W.ln1_w, W.ln1_b, hd, n, d, rw.act, s, c.ks_prev ? rw.Pres : nullptr,
                        c.ks_prev, c.bias_prev, emb);
      PerfScope ps(S, "dec_gemm", s);
      c.k1 = gemm_splitk_partials<T>(hd, Dw(W.qkv), n, 3 * d, d, rw.Pqkv, s);
    }
    static const int pf_selfwrite =
        getenv("MWX_PREFILL_SELFWRITE") ? atoi(getenv("MWX_PREFILL_SELFWRITE")) : 0;
    if (rw.prefill)
      kv_append<T>(rw.Pqkv, c.k1, 3 * d, W.qkv_b, kqs, ks, vs, rw.crow, rw.pos, rw.act, Tctx, n, H,
                   s);
    { PerfScope ps(S, "dec_attn_self", s);
      dec_attention<T>(rw.Pqkv, c.k1, 3 * d, W.qkv_b, kqs, kqs, ks, vs, rw.crow, rw.pos, rw.act, 0,
                       Tctx, rw.od, n, H, 1.0f, s, rw.kvmap, rw.kvown, rw.map_row0,
                       rw.prefill ? 1 : rw.xgroup, pf_selfwrite || !rw.prefill); }
    { PerfScope ps(S, "dec_gemm", s);
      c.k2 = gemm_splitk_partials<T>(rw.od, Dw(W.o), n, d, d, rw.Pres, s); }
    c.k3 = 0;
    if (fold) {
      const LnFuse f = ln_fuse(rw, c, rw.Pres, c.k2, W.o_b, W.lnc_w, W.lnc_b);
      PerfScope ps(S, "dec_gemm", s);
      c.k3 = gemm_splitk_ln<T>(f, Dw(W.cq), d, d, rw.Pq, s);
      if (c.k3) c.xd = f.x_out;
    }
    if (!c.k3) {
      layer_norm_dec<T>(c.xd, W.lnc_w, W.lnc_b, hd, n, d, rw.act, s, rw.Pres, c.k2, W.o_b);
      PerfScope ps(S, "dec_gemm", s);
      c.k3 = gemm_splitk_partials<T>(hd, Dw(W.cq), n, d, d, rw.Pq, s);
    }
  }
  void layer_cross(const LayerRows& rw, LayerRun& c, int l, hipStream_t s) {
    const int n = rw.n;
    const float kqs = powf(64.0f, -0.25f);
    const size_t layer_cross = (size_t)S.cross_cap * H * hp.n_audio_ctx * 64;  // elements
    const size_t layer_xs = (size_t)S.cross_cap * H * hp.n_audio_ctx * 2;      // kv8 scales
    const DecLayerW& W = C.dec[l];
    if (!rw.prefill && perf_on(S, "event_bracket")) {
      // calibration: the same event pair around an empty kernel at the same
      // point of the chain (bench.py subtracts its average from the
      // cross-attention brackets: the two event nodes' own cost)
      PerfScope ps(S, "event_bracket", s);
      launch_perf_empty(s);
    }
    PerfScope ps(S, rw.prefill ? "prefill_cross" : "dec_attn_cross", s);
    // the decoders of a beam / best-of group share their clip's cross K/V:
    // stream it once per group; an MX-fp8 cache is read by the grouped
    // kernel for any group size
    const int nq = std::max(1, rw.xgroup);  // (prefill: Driver::prefill's q)
    unsigned long long* sp = rw.prefill ? nullptr : span_slot(S, "dec_attn_cross", s);
    if (C.kv8) {
      if (!dec_cross_attention_grouped<T>(
              rw.Pq, c.k3, d, W.cq_b, (const uint8_t*)S.cross_k.p + l * layer_cross,
              (const uint8_t*)S.cross_v.p + l * layer_cross, rw.xidx, rw.act, hp.n_audio_ctx,
              hp.n_audio_ctx, rw.od, n, H, kqs, nq, s,
              (const uint8_t*)S.cross_ks.p + l * layer_xs,
              (const uint8_t*)S.cross_vs.p + l * layer_xs, sp))
        throw std::runtime_error("mwx: unsupported fp8 cross-attention group");
    } else if (nq < 2 ||
               !dec_cross_attention_grouped<T>(rw.Pq, c.k3, d, W.cq_b,
                                               (const _Float16*)S.cross_k.p + l * layer_cross,
                                               (const _Float16*)S.cross_v.p + l * layer_cross,
                                               rw.xidx, rw.act, hp.n_audio_ctx, hp.n_audio_ctx,
                                               rw.od, n, H, kqs, nq, s, nullptr, nullptr, sp)) {
      dec_attention<T>(rw.Pq, c.k3, d, W.cq_b, 1.0f, 1.0f,
                       (_Float16*)S.cross_k.p + l * layer_cross,
                       (_Float16*)S.cross_v.p + l * layer_cross, rw.xidx, rw.pos, rw.act,
                       hp.n_audio_ctx, hp.n_audio_ctx, rw.od, n, H, kqs, s, nullptr, nullptr, 0,
                       nq, 1, sp);
    }
  }
  void layer_post(const LayerRows& rw, LayerRun& c, int l, hipStream_t s) {
    const int n = rw.n;
    const DecLayerW& W = C.dec[l];
    { PerfScope ps(S, "dec_gemm", s);
      c.k4 = gemm_splitk_partials<T>(rw.od, Dw(W.co), n, d, d, rw.Pres, s); }
    EpiParams e;
    e.bias = W.fc1_b;
    e.c16 = rw.ffd;
    e.ldc = 4 * d;
    e.pack_out = true;
    c.k5 = false;
    if (ln_folds(rw)) {  // (as layer_pre)
      const LnFuse f = ln_fuse(rw, c, rw.Pres, c.k4, W.co_b, W.ln2_w, W.ln2_b);
      PerfScope ps(S, "dec_gemm", s);
      c.k5 = gemm_decode_ln<T>(EPI_GELU, f, Dw(W.fc1), 4 * d, d, e, s);
      if (c.k5) c.xd = f.x_out;
    }
    if (!c.k5) {
      layer_norm_dec<T>(c.xd, W.ln2_w, W.ln2_b, rw.hd, n, d, rw.act, s, rw.Pres, c.k4, W.co_b);
      PerfScope ps(S, "dec_gemm", s);
      c.k5 = gemm_decode<T>(EPI_GELU, rw.hd, Dw(W.fc1), n, 4 * d, d, e, s);
    }
    { PerfScope ps(S, "dec_gemm", s);
      c.ks_prev = gemm_splitk_partials<T>(rw.ffd, Dw(W.fc2), n, d, 4 * d, rw.Pres, s); }
    c.bias_prev = W.fc2_b;
    if (!c.k1 || !c.k2 || !c.k3 || !c.k4 || !c.k5 || !c.ks_prev)
      throw std::runtime_error("mwx: unsupported split-K shape");
  }

  // embedding + all decoder layers; returns the last FFN2's split-K factor
  // and bias (folded into the consumer: the final LayerNorm)
  void run_layers(const LayerRows& rw, hipStream_t s, int& ks_prev, const float*& bias_prev,
                  float** xd_out = nullptr) {
    LayerRun c;
    layers_begin(rw, c, s);
    for (int l = 0; l < L_dec; ++l) {
      layer_pre(rw, c, l, s);
      layer_cross(rw, c, l, s);
      layer_post(rw, c, l, s);
    }
    ks_prev = c.ks_prev;
    bias_prev = c.bias_prev;
    if (xd_out) *xd_out = c.xd;  // (the buffer holding the residual after the last layer)
  }

  // Batched prompt prefill (whisper.cpp decodes a window's prompt in one
  // whisper_decode call, src/stt_engine.cpp:233 passes initial_prompt and
  // long-form windows carry prompt_past): positions 0 .. n_i - 1 of row i's
  // prompt run through the layer stack as virtual rows (one per position)
  // instead of one decode step each. Only the K / V they leave in the self
  // cache are kept (no logits: the prompt's last position is the first
  // sampling step of the decode loop). Every virtual row's arithmetic is a
  // decode step's for that row and position (row-blocked GEMMs, the same
  // attention kernels), so the cache holds the same bits as step by step.
  // Rows in chunks of <= MWX_PREFILL_ROWS virtual rows (default 2048), each
  // row's positions padded to a multiple of the cross-attention group q
  // (min(8, prompt length)). Queued without a host synchronize.
  // split-K slabs of the d-deep projections (QKV, out, cross Q, cross out)
  // and of the residual-producing ones (out, cross out, FFN2: 4d deep)
  int ks_d() const { return std::max(1, splitk_factor(d)); }
  int ks_res() const { return std::max(ks_d(), splitk_factor(4 * d)); }
  struct PrefillRow {
    int row;                 // self-cache row
    int clip;                // cross slot
    const int* tokens;       // prompt tokens
    int n;                   // positions to prefill (0 .. n-1)
  };
  void prefill(const std::vector<PrefillRow>& prs) {
    static const int vcap = std::max(64, getenv("MWX_PREFILL_ROWS")
                                             ? atoi(getenv("MWX_PREFILL_ROWS")) : 2048);
    int nmax = 0, nrows = 0;
    for (const auto& r : prs)
      if (r.n > 0) {
        nmax = std::max(nmax, r.n);
        ++nrows;
      }
    if (nrows == 0) return;
    for (const auto& r : prs) S.n_prefill += std::max(0, r.n);
    // positions per chunk: every row with work gets the same span (x 8)
    static const int span_env = getenv("MWX_PREFILL_SPAN") ? atoi(getenv("MWX_PREFILL_SPAN")) : 0;
    const int span = span_env > 0 ? span_env : std::max(8, (vcap / nrows) / 8 * 8);
    // cross-attention group: q consecutive virtual rows of one clip share one
    // K/V stream (MWX_PREFILL_XNQ caps it, default 8); each row's positions are
    // padded to a multiple of q (short prompts: q = their length, no padding)
    static const int xnq_cap =
        getenv("MWX_PREFILL_XNQ") ? std::max(1, std::min(8, atoi(getenv("MWX_PREFILL_XNQ")))) : 8;
    const int q = std::max(1, std::min(xnq_cap, std::min(span, nmax)));
    const size_t mcap = (size_t)nrows * ((std::min(span, nmax) + q - 1) / q * q);
    const size_t m64 = (mcap + 63) / 64 * 64;
    int* din = (int*)S.pf_in.get(mcap * 5 * 4);
    LayerRows rw;
    rw.xd = (float*)S.pf_x.get(mcap * d * 4);
    rw.hd = (T*)S.pf_h.get(m64 * d * sizeof(T), true);
    rw.od = (T*)S.pf_o.get(m64 * d * sizeof(T), true);
    rw.ffd = (T*)S.pf_ff.get(m64 * 4 * d * sizeof(T), true);
    // (large-v3, 2048 virtual rows: slabs 5 x 31.5 + 8 x 10.5 + 5 x 10.5 MB,
    // with the activations ~0.33 GB per state, held until mwx_free_state)
    rw.Pqkv = (float*)S.pf_pqkv.get((size_t)ks_d() * mcap * 3 * d * 4);
    rw.Pres = (float*)S.pf_pres.get((size_t)ks_res() * mcap * d * 4);
    rw.Pq = (float*)S.pf_pq.get((size_t)ks_d() * mcap * d * 4);
    rw.kself = (_Float16*)S.kself.p;
    rw.vself = (_Float16*)S.vself.p;
    rw.prefill = true;
    rw.xgroup = q;
    // host inputs of every chunk in one array (no reallocation while its
    // uploads are queued): the pass is queued without a synchronize, so the
    // host goes on to capture / launch the decode steps behind it
    size_t chunks = 0;
    for (int p0 = 0; p0 < nmax; p0 += span) ++chunks;
    S.pf_hin.clear();
    S.pf_hin.reserve(chunks * mcap * 5);
    // MWX_PREFILL_TIME=1: device time of the pass (events) and host time of
    // the call on stderr (diagnostic)
    static const bool timing = getenv("MWX_PREFILL_TIME") && atoi(getenv("MWX_PREFILL_TIME")) != 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    const auto th0 = std::chrono::steady_clock::now();
    if (timing) {
      HIPC(hipEventCreate(&ev0));
      HIPC(hipEventCreate(&ev1));
      HIPC(hipEventRecord(ev0, st));
    }
    for (int p0 = 0; p0 < nmax; p0 += span) {
      std::vector<int> tok, pos, act, xidx, crow;
      for (const auto& r : prs) {
        const int len = std::min(r.n, p0 + span) - p0;
        if (len <= 0) continue;
        const int padded = (len + q - 1) / q * q;
        for (int j = 0; j < padded; ++j) {
          const bool a = j < len;
          tok.push_back(a ? r.tokens[p0 + j] : 0);
          pos.push_back(a ? p0 + j : 0);
          act.push_back(a ? 1 : 0);
          xidx.push_back(r.clip);
          crow.push_back(r.row);
        }
      }
      const int M = (int)tok.size();
      if (M == 0) continue;
      if ((size_t)M > mcap) throw std::runtime_error("mwx: prefill chunk exceeds its buffers");
      const size_t h0 = S.pf_hin.size();
      for (auto* v : {&tok, &pos, &act, &xidx, &crow})
        S.pf_hin.insert(S.pf_hin.end(), v->begin(), v->end());
      // (din is reused by the next chunk: its upload is ordered after this
      // chunk's kernels on the same stream)
      HIPC(hipMemcpyAsync(din, S.pf_hin.data() + h0, (S.pf_hin.size() - h0) * 4,
                          hipMemcpyHostToDevice, st));
      rw.n = M;
      rw.tok = din;
      rw.pos = din + M;
      rw.act = din + 2 * M;
      rw.xidx = din + 3 * M;
      rw.crow = din + 4 * M;
      int ks_prev = 0;
      const float* bias_prev = nullptr;
      run_layers(rw, st, ks_prev, bias_prev);
    }
    if (timing) {
      HIPC(hipEventRecord(ev1, st));
      HIPC(hipStreamSynchronize(st));
      float ms = 0.0f;
      HIPC(hipEventElapsedTime(&ms, ev0, ev1));
      const double host_ms = std::chrono::duration<double, std::milli>(
                                 std::chrono::steady_clock::now() - th0).count();
      fprintf(stderr, "mwx prefill: %d rows, %d positions max, span %d, %zu virtual rows per chunk: "
              "device %.3f ms, host call %.3f ms\n", nrows, nmax, span, mcap, ms, host_ms);
      HIPC(hipEventDestroy(ev0));
      HIPC(hipEventDestroy(ev1));
    }
  }

  // the decode-step rows (all R) and their buffers
  LayerRows step_rows(int R) {
    int* si = (int*)S.stepin.p;
    LayerRows rw;
    rw.n = R;
    rw.tok = si;
    rw.pos = si + R;
    rw.act = si + 2 * R;
    rw.xidx = si + 3 * R;
    rw.xd = (float*)S.xd.p;
    rw.xd2 = (float*)S.xd2.p;
    rw.hd = (T*)S.hd.p;
    rw.od = (T*)S.od.p;
    rw.ffd = (T*)S.ffd.p;
    rw.Pqkv = (float*)S.pqkv.p;
    rw.Pres = (float*)S.pres.p;
    rw.Pq = (float*)S.pq.p;
    rw.kself = (_Float16*)S.kself.p;
    rw.vself = (_Float16*)S.vself.p;
    rw.kvmap = (const int*)S.kvmap.p;
    rw.kvown = (const int*)S.kvown.p;
    rw.map_row0 = 0;
    rw.xgroup = xgroup;
    return rw;
  }

  // one decode step of all R rows on stream s
  void decode_rows(int R, bool want_probs, hipStream_t s) {
    LayerRows rw = step_rows(R);
    int ks_prev = 0;
    const float* bias_prev = nullptr;
    float* xd = rw.xd;
    run_layers(rw, s, ks_prev, bias_prev, &xd);
    rw.xd = xd;
    step_tail(R, rw, ks_prev, bias_prev, want_probs, s);
  }

  // final LayerNorm, logits and logits processing of a step's row set
  void step_tail(int R, const LayerRows& rw, int ks_prev, const float* bias_prev, bool want_probs,
                 hipStream_t s) {
    const int n = rw.n;
    const int r0 = rw.map_row0;
    const int* act = rw.act;
    float* xd = rw.xd;
    T* hd = rw.hd;
    float* Pres = rw.Pres;
    layer_norm_dec<T>(xd, C.dec_ln_w, C.dec_ln_b, hd, n, d, act, s, Pres, ks_prev, bias_prev);
    EpiParams e;
    e.c32 = (float*)S.logits.p + (size_t)r0 * V;
    e.ldc = V;
    // tied-embedding logits: the 133-MB (large-v3) weight exceeds every L2,
    // so all rows of a block share one read of it: 32-row blocks (up to 64
    // rows: ceil(n/16) tiles per block). Per-row arithmetic is the same MFMA
    // chain in any block, so the logits are bit-identical (38.2 -> 23.0 us per
    // launch at 32 rows, scripts/probe/dec_chain_probe.hip).
    e.mt = n <= 64 ? std::max(1, (n + 15) / 16) : 2;
    { PerfScope ps(S, "logits_gemm", s);
    if (!gemm_decode<T>(EPI_F32, hd, Dw(C.tok_p), n, V, d, e, s))
      throw std::runtime_error("mwx: unsupported logits GEMM shape"); }
    float* pr = nullptr;
    float* lp = nullptr;
    if (want_probs) {
      pr = (float*)S.probs.get((size_t)R * V * 4) + (size_t)r0 * V;
      lp = (float*)S.logprobs.get((size_t)R * V * 4) + (size_t)r0 * V;
    }
    PerfScope ps(S, "logits_proc", s);
    logits_process((float*)S.logits.p + (size_t)r0 * V, (const float*)S.smask.p,
                   (const RowCtl*)S.ctl.p + r0, (TokOut*)S.tokout.p + r0, pr, lp, LC, n,
                   LPScratch{(float*)S.lpflt.p + (size_t)r0 * V, (LPPart*)S.lpparts.p + r0 * LP_G,
                             (LPRes*)S.lpres.p + r0 * LP_G},
                   s, !pick_in_advance);
    if (want_probs) {  // std::discrete_distribution draws of the sampling rows
      const int KD = S.draw_k;
      sample_draws(pr, lp, V, (const double*)S.du.p + (size_t)r0 * KD, (const int*)S.dnd.p + r0,
                   KD, (Draw*)S.ddraw.p + (size_t)r0 * KD, (int*)S.dneed.p + r0, n, s);
    }
  }
};

}  // namespace mwx

struct mwx_context {
  mwx::Context c;
};
struct mwx_state {
  mwx::State s;
};

// The decode-loop / window logic lives in driver.cpp (same TU via include to
// keep templates local).
#include "driver.inc"
