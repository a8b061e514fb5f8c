// TEST INFRASTRUCTURE ONLY (linked into liborc.so): CPU restatement of the
// reference's segment prosody and speaker clustering, the checker for the
// engine's GPU prosody (mwx_prosody_batch, k_prosody.hip) and the host
// SttEngine's clusterer. Pinned bit-exactly against the reference's own build
// (oracle/_ref/libref_prosody.so, see ref_prosody_shim.cpp) and against the
// golden vectors generated from it (tests/golden/prosody_ref.json,
// tests/golden/make_prosody_golden.py).
//
// Follows src/prosody_extractor.cpp:9-224 and src/speaker_cluster.cpp:5-40.
// Compiled with -ffp-contract=off: plain IEEE single precision, as the
// reference's -O3 x86-64 (SSE, no FMA) build computes it.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct OrcProsody {  // layout of mwx_prosody (include/mwx.h)
  float pitch_mean, pitch_std, energy_mean, energy_std, spectral_centroid, zero_crossing_rate,
      arousal, valence;
  float speaker_vec[8];
  int gender, emotion, serial_runs, reserved;
};

float mean_of(const std::vector<float>& v) {  // :9-12
  if (v.empty()) return 0.0f;
  float s = 0.0f;
  for (float x : v) s += x;
  return s / (float)v.size();
}

float dev_of(const std::vector<float>& v, float m) {  // :13-18
  if (v.empty()) return 0.0f;
  float a = 0.0f;
  for (float x : v) a += (x - m) * (x - m);
  return std::sqrt(a / (float)v.size());
}

float median_of(std::vector<float> v) {  // :19-24 (nth_element at n/2)
  if (v.empty()) return 0.0f;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

float norm01(float v, float lo, float hi) {  // :25-28
  const float n = (v - lo) / (hi - lo);
  return std::max(0.0f, std::min(1.0f, n));
}

void prosody(const float* x, size_t n, int sr, float alpha, float gthr, float pmin, float pmax,
             OrcProsody* o) {
  std::memset(o, 0, sizeof *o);
  if (n < 160 || !x) return;  // :35-48: zeros, "?", "neutral"
  const int F = sr / 100;
  const int W = std::min(F, 1600);
  std::vector<float> f0, rms_v, zcr_v, sc_v;
  std::vector<float> filt(W);
  int peaks = 0;
  float prev_rms = 0.0f, y = 0.0f;
  for (size_t i = 0; i + F <= n; i += F) {  // :63-128
    float e = 0.0f;
    for (int k = 0; k < W; ++k) {
      const float v = x[i + k];
      e += v * v;
      y += alpha * (v - y);
      filt[k] = y;
    }
    const float r = std::sqrt(e / W);
    rms_v.push_back(r);
    if (r > 0.05f && prev_rms <= 0.05f) ++peaks;
    prev_rms = r;
    const float clip = std::max(0.002f, r * 0.15f);
    int cyc = 0, zc = 0;
    int sign = 0;  // 0: not yet, 1: positive, -1: negative
    for (int k = 1; k < W; ++k) {
      const float v = filt[k];
      if ((v >= 0) != (filt[k - 1] >= 0)) ++zc;
      if (sign == 0) {
        if (v > clip) sign = 1;
        else if (v < -clip) sign = -1;
      } else if (sign == 1 && v < -clip) {
        sign = -1;
        ++cyc;
      } else if (sign == -1 && v > clip) {
        sign = 1;
      }
    }
    zcr_v.push_back((float)zc / W);
    if (r > 0.015f && cyc > 0) {
      const float est = cyc / ((float)F / sr);
      if (est >= pmin && est <= pmax) f0.push_back(est);
    }
    float pw = 0.0f, wt = 0.0f;
    for (int k = 1; k < W; ++k) {
      const float d = std::fabs(x[i + k] - x[i + k - 1]);
      wt += d * k;
      pw += d;
    }
    sc_v.push_back(pw > 0 ? wt / pw : 0.0f);
  }
  float pitch = median_of(f0);  // :130-135
  o->pitch_std = f0.empty() ? 0.0f : dev_of(f0, mean_of(f0));
  o->energy_mean = rms_v.empty() ? 0.01f : mean_of(rms_v);
  o->energy_std = rms_v.empty() ? 0.0f : dev_of(rms_v, o->energy_mean);
  o->spectral_centroid = sc_v.empty() ? 50.0f : mean_of(sc_v);
  o->zero_crossing_rate = zcr_v.empty() ? 0.1f : mean_of(zcr_v);
  if (pitch > gthr && o->zero_crossing_rate < 0.024f)  // :140-148
    pitch *= 0.5f;
  else if (o->energy_mean > 0.12f && pitch < 240.0f && o->spectral_centroid < 90.0f)
    pitch *= 0.5f;
  o->pitch_mean = pitch;
  const float dur = (float)n / sr;  // :150-152
  const float rate = dur > 0 ? (float)peaks / dur : 0.0f;
  if (pitch == 0.0f || o->energy_mean < 0.018f)  // :155-163
    o->gender = 0;
  else if (o->zero_crossing_rate < 0.030f)
    o->gender = 1;
  else
    o->gender = pitch > gthr ? 2 : 1;
  const float np = o->gender == 1 ? norm01(pitch, 60.0f, 180.0f) : norm01(pitch, 160.0f, 350.0f);
  const float nb = norm01(o->spectral_centroid, 40.0f, 150.0f);  // :166-175
  o->valence = ((np * 0.4f) + (nb * 0.6f)) * 2.0f - 1.0f;
  o->valence += 0.35f;
  o->arousal = (norm01(o->energy_mean, 0.02f, 0.20f) * 0.7f) + (norm01(rate, 2.0f, 9.0f) * 0.3f);
  if (o->arousal > 0.65f)  // :181-186
    o->emotion = o->valence > 0.1f ? 1 : 2;
  else if (o->arousal < 0.30f)
    o->emotion = o->valence < -0.4f ? 3 : 0;
  else
    o->emotion = 0;
  float* sv = o->speaker_vec;  // :191-221
  sv[0] = o->gender == 1   ? norm01(pitch, 60.0f, 200.0f) * 0.4f
          : o->gender == 2 ? 0.6f + (norm01(pitch, 160.0f, 350.0f) * 0.4f)
                           : 0.5f;
  sv[1] = norm01(o->spectral_centroid, 40.0f, 250.0f);
  sv[4] = norm01(o->zero_crossing_rate, 0.0f, 0.5f) * 0.8f;
  sv[2] = norm01(o->pitch_std, 5.0f, 100.0f) * 0.1f;
  sv[3] = norm01(o->energy_mean, 0.0f, 0.3f) * 0.1f;
  sv[5] = norm01(rate, 1.0f, 12.0f) * 0.1f;
  sv[6] = o->arousal * 0.05f;
  sv[7] = ((o->valence + 1.0f) / 2.0f) * 0.05f;
}

// src/speaker_cluster.cpp: running-mean centroids keyed "spk_<n>", best
// cosine over the map's iteration order (ties keep the first), threshold >=
struct Clusterer {
  struct C {
    std::string id;
    std::vector<float> c;
    size_t count;
  };
  float thr;
  int next = 0;
  std::unordered_map<std::string, C> m;
  static float cos(const std::vector<float>& a, const std::vector<float>& b) {
    float d = 0, na = 0, nb = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      d += a[i] * b[i];
      na += a[i] * a[i];
      nb += b[i] * b[i];
    }
    if (na == 0 || nb == 0) return 0;
    return d / (std::sqrt(na) * std::sqrt(nb));
  }
  std::string assign(const std::vector<float>& v) {
    std::string best;
    float bs = 0.0f;
    for (auto& kv : m) {
      const float s = cos(v, kv.second.c);
      if (s > bs) {
        bs = s;
        best = kv.first;
      }
    }
    if (!best.empty() && bs >= thr) {
      C& c = m[best];
      for (size_t i = 0; i < c.c.size(); ++i) c.c[i] = (c.c[i] * c.count + v[i]) / (c.count + 1);
      ++c.count;
      return best;
    }
    const std::string id = "spk_" + std::to_string(next++);
    m[id] = C{id, v, 1};
    return id;
  }
};

}  // namespace

extern "C" {

void orc_prosody(const float* pcm, int64_t n, int sample_rate, float lpf_alpha,
                 float gender_threshold, float min_pitch, float max_pitch, void* out) {
  prosody(pcm, (size_t)n, sample_rate, lpf_alpha, gender_threshold, min_pitch, max_pitch,
          static_cast<OrcProsody*>(out));
}

void* orc_clusterer_new(float threshold) { return new Clusterer{threshold}; }
void orc_clusterer_free(void* c) { delete static_cast<Clusterer*>(c); }
int orc_clusterer_assign(void* c, const float* vec, int n, char* id, int cap) {
  const std::string s = static_cast<Clusterer*>(c)->assign(std::vector<float>(vec, vec + n));
  std::snprintf(id, cap, "%s", s.c_str());
  return (int)s.size();
}

}  // extern "C"
