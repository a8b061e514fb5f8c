// TEST INFRASTRUCTURE ONLY — drives the host SttEngine through its C shim
// (host/stt_capi.cpp) from many threads, linked against tests/san/mwx_stub.cpp,
// in an AddressSanitizer + UBSan build and a ThreadSanitizer build
// (tests/san/Makefile; run by tests/test_sanitizers.py). A sanitizer report
// aborts the process; the checks below only assert the host logic's own
// contracts (EngineBusy under an exhausted pool, abort before/after start,
// batching of equal-option requests, the stream's undelivered-events drain).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int mwx_stt_is_hallucination(const char* text);
void* mwx_stt_new(const char* dir, const char* file, int parallel, int timeout_ms, int beam,
                  const char* lang, int vad_ms, int gpu);
void* mwx_stt_new_ex(const char* dir, const char* file, int parallel, int timeout_ms, int beam,
                     const char* lang, int vad_ms, int gpu, int max_batch, int window_us,
                     int stream_buffer_samples);
void mwx_stt_free(void* eng);
long mwx_stt_batches(void* eng);
int mwx_stt_cluster_ids(const float* vecs, int n, float threshold, char* out, int cap);
int mwx_stt_transcribe_pcm16_ex(void* eng, const int16_t* pcm, int n, int sr, const char* lang,
                                int beam, float temperature, char* out, int cap, double* m3,
                                int abort_after, int* abort_calls);
int mwx_stt_transcribe_f32_ex(void* eng, const float* pcm, int n, int sr, const char* lang,
                              int beam, float temperature, char* out, int cap, double* m3,
                              int abort_after, int* abort_calls);
void* mwx_stt_stream_new(void* eng);
void mwx_stt_stream_free(void* s);
int mwx_stt_stream_feed(void* s, const uint8_t* data, int len, char* out, int cap);
int mwx_stt_stream_drain(void* s, char* out, int cap);
}

namespace {

int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

std::vector<int16_t> clip(int seed, int n) {
  std::vector<int16_t> x(n);
  uint32_t s = 0x9e3779b9u * (seed + 1);
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    x[i] = (int16_t)((int)(s >> 16) % 12000 - 6000);
  }
  return x;
}

int transcribe(void* eng, const std::vector<int16_t>& x, int sr, int beam, int abort_after,
               int* calls, std::string* json) {
  std::vector<char> buf(1 << 16);
  double m[3];
  int c = 0;
  const int r = mwx_stt_transcribe_pcm16_ex(eng, x.data(), (int)x.size(), sr, "en", beam, -1.0f,
                                            buf.data(), (int)buf.size(), m, abort_after, &c);
  if (calls) *calls = c;
  if (json && r >= 0) *json = buf.data();
  return r;
}

void filters() {
  const char* drop[] = {"", " ", "a", " ... ", "[Music]", "(laughs)", " Thank you.",
                        "Hmm!", "Okay.", "ご視聴ありがとう"};
  const char* keep[] = {"hello world", "the engine runs", "ab"};
  for (const char* t : drop)
    if (mwx_stt_is_hallucination(t) != 1) std::fprintf(stderr, "kept: '%s'\n", t), ++failures;
  for (const char* t : keep)
    if (mwx_stt_is_hallucination(t) != 0) std::fprintf(stderr, "dropped: '%s'\n", t), ++failures;
  CHECK(mwx_stt_is_hallucination(nullptr) == 1);
  std::vector<float> v(8 * 6);
  for (int i = 0; i < 48; ++i) v[i] = (float)((i / 8) % 2 ? i % 8 : 7 - i % 8) + 0.5f;
  char out[256];
  CHECK(mwx_stt_cluster_ids(v.data(), 6, 0.88f, out, sizeof out) > 0);
  CHECK(std::strncmp(out, "spk_0\nspk_1\nspk_0\n", 18) == 0);
  CHECK(mwx_stt_cluster_ids(v.data(), 6, 0.88f, out, 4) < 0);  // too small: needed size
}

// reference mode (max_batch 1): state pool of 2, 8 concurrent requesters;
// some get EngineBusy (-2) with a short queue timeout
void pool(const char* dir) {
  void* eng = mwx_stt_new(dir, "model.bin", 2, 3, 1, "en", 500, 0);
  CHECK(eng != nullptr);
  std::atomic<int> ok{0}, busy{0}, other{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < 6; ++k) {
        const int r = transcribe(eng, clip(t * 16 + k, 16000 * (2 + (t + k) % 5)), 16000, 1, -1,
                                 nullptr, nullptr);
        (r >= 0 ? ok : r == -2 ? busy : other)++;
      }
    });
  for (auto& x : th) x.join();
  CHECK(ok > 0 && other == 0 && ok + busy == 48);
  std::string a, b;
  CHECK(transcribe(eng, clip(1, 16000 * 7), 16000, 1, -1, nullptr, &a) >= 0);
  CHECK(transcribe(eng, clip(1, 16000 * 7), 16000, 1, -1, nullptr, &b) >= 0);
  CHECK(a == b && a.size() > 2);
  int calls = 0;
  CHECK(transcribe(eng, clip(2, 16000 * 9), 16000, 1, 0, &calls, &a) >= 0);
  CHECK(a == "[]" && calls == 1);  // aborted at entry
  CHECK(transcribe(eng, clip(2, 16000 * 9), 16000, 1, 2, &calls, &a) >= 0);
  CHECK(a == "[]" && calls >= 3);  // aborted inside the run
  CHECK(transcribe(eng, clip(3, 4000), 16000, 1, -1, nullptr, &a) >= 0);
  CHECK(a == "[]");  // shorter than vad_ms_min_duration
  CHECK(transcribe(eng, clip(4, 48000 * 4), 48000, 1, -1, nullptr, &a) >= 0);  // resampled
  CHECK(a.size() > 2);
  std::vector<float> f(16000 * 3, 0.25f);
  std::vector<char> buf(1 << 15);
  double m[3];
  int c = 0;
  CHECK(mwx_stt_transcribe_f32_ex(eng, f.data(), (int)f.size(), 16000, "en", 1, -1.0f, buf.data(),
                                  (int)buf.size(), m, -1, &c) >= 0);
  CHECK(mwx_stt_transcribe_f32_ex(eng, f.data(), (int)f.size(), 16000, "en", 1, -1.0f, buf.data(),
                                  8, m, -1, &c) < -2);  // needed capacity
  mwx_stt_free(eng);
}

// batched mode: 2 batchers x 4 states, 12 requesters, two option keys
void batched(const char* dir) {
  void* eng = mwx_stt_new_ex(dir, "model.bin", 2, 5000, 1, "en", 500, 0, 4, 3000, 8000);
  CHECK(eng != nullptr);
  std::vector<std::string> solo(12);
  for (int t = 0; t < 12; ++t)
    CHECK(transcribe(eng, clip(100 + t, 16000 * (3 + t % 4)), 16000, t % 2 ? 5 : 1, -1, nullptr,
                     &solo[t]) >= 0);
  const long before = mwx_stt_batches(eng);
  std::vector<std::string> got(12);
  std::vector<int> rc(12);
  std::vector<std::thread> th;
  // inputs made first and the requests released together, so they arrive
  // within the batching window even on a loaded host (sanitizer builds)
  std::vector<std::vector<int16_t>> pcm;
  for (int t = 0; t < 12; ++t) pcm.push_back(clip(100 + t, 16000 * (3 + t % 4)));
  std::atomic<int> ready{0};
  for (int t = 0; t < 12; ++t)
    th.emplace_back([&, t] {
      ready.fetch_add(1);
      while (ready.load() < 12) std::this_thread::yield();
      rc[t] = transcribe(eng, pcm[t], 16000, t % 2 ? 5 : 1, t == 5 ? 1 : -1, nullptr, &got[t]);
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < 12; ++t) {
    CHECK(rc[t] >= 0);
    if (t != 5) CHECK(got[t] == solo[t]);  // batching does not change a request's result
  }
  CHECK(mwx_stt_batches(eng) - before < 12);  // some requests shared a batch
  mwx_stt_free(eng);
}

// streaming: WAV header skip, partials every stream_buffer_samples, end of
// speech final; a too-small buffer keeps the events for drain
void stream(const char* dir) {
  void* eng = mwx_stt_new_ex(dir, "model.bin", 2, 5000, 1, "en", 500, 0, 1, 0, 8000);
  CHECK(eng != nullptr);
  for (int pass = 0; pass < 2; ++pass) {
    void* s = mwx_stt_stream_new(eng);
    std::vector<int16_t> x = clip(7 + pass, 16000 * 6);
    std::vector<uint8_t> bytes(44, 0);
    std::memcpy(bytes.data(), "RIFF", 4);
    std::memcpy(bytes.data() + 8, "WAVE", 4);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(x.data());
    bytes.insert(bytes.end(), p, p + x.size() * 2);
    std::vector<char> out(1 << 16);
    size_t off = 0;
    int events = 0;
    while (off < bytes.size()) {
      const int len = (int)std::min<size_t>(3201, bytes.size() - off);  // odd: split samples
      const int cap = pass == 1 && off > 40000 ? 16 : (int)out.size();
      int r = mwx_stt_stream_feed(s, bytes.data() + off, len, out.data(), cap);
      off += len;
      if (r < -2) {
        CHECK(mwx_stt_stream_feed(s, bytes.data(), 2, out.data(), (int)out.size()) == -3);  // pending
        r = mwx_stt_stream_drain(s, out.data(), (int)out.size());
      }
      CHECK(r >= 0);
      events += std::strstr(out.data(), "\"final\"") != nullptr;
    }
    CHECK(mwx_stt_stream_feed(s, nullptr, 0, out.data(), (int)out.size()) >= 0);
    CHECK(events > 0);
    mwx_stt_stream_free(s);
  }
  // concurrent sessions on one engine
  std::vector<std::thread> th;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      void* s = mwx_stt_stream_new(eng);
      std::vector<int16_t> x = clip(50 + t, 16000 * 4);
      std::vector<char> out(1 << 16);
      for (size_t i = 0; i < x.size(); i += 1600)
        if (mwx_stt_stream_feed(s, reinterpret_cast<const uint8_t*>(x.data() + i), 3200,
                                out.data(), (int)out.size()) < 0)
          bad++;
      if (mwx_stt_stream_feed(s, nullptr, 0, out.data(), (int)out.size()) < 0) bad++;
      mwx_stt_stream_free(s);
    });
  for (auto& x : th) x.join();
  CHECK(bad == 0);
  mwx_stt_free(eng);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* dir = argv[1];
  std::string path = std::string(dir) + "/model.bin";
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return 2;
  std::fputs("stub", f);
  std::fclose(f);
  CHECK(mwx_stt_new(dir, "missing.bin", 1, 100, 1, "en", 500, 0) == nullptr);
  filters();
  pool(dir);
  batched(dir);
  stream(dir);
  std::printf("host_check: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
