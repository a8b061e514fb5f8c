// TEST INFRASTRUCTURE ONLY — C entry points over the reference's own
// prosody / speaker-clustering code. oracle/Makefile compiles this shim
// together with /root/reference/src/prosody_extractor.cpp and
// speaker_cluster.cpp (the reference's sources, where they lie; not copied)
// into oracle/_ref/libref_prosody.so with the reference's Release flags
// (-O3 -DNDEBUG, no -march: CMakeLists.txt:16, Dockerfile:35). Only tests/
// load it, as the checker of the engine's GPU prosody (mwx_prosody_batch) and
// of the host SttEngine's clusterer.
#include <cstring>
#include <string>
#include <vector>

#include "prosody_extractor.h"
#include "speaker_cluster.h"

extern "C" {

struct RefProsody {
  float pitch_mean, pitch_std, energy_mean, energy_std, spectral_centroid, zero_crossing_rate,
      arousal, valence;
  float speaker_vec[8];
  int n_vec;
  char gender[8];
  char emotion[16];
};

// extract_prosody(pcm, n, sr, opts); pcm may be NULL (the reference's
// "segment shorter than 160 samples" call, src/stt_engine.cpp:327)
int ref_extract_prosody(const float* pcm, long n, int sample_rate, float lpf_alpha,
                        float gender_threshold, float min_pitch, float max_pitch,
                        RefProsody* out) {
  ProsodyOptions o;
  o.lpf_alpha = lpf_alpha;
  o.gender_threshold = gender_threshold;
  o.min_pitch = min_pitch;
  o.max_pitch = max_pitch;
  const AffectiveTags t = extract_prosody(pcm, (size_t)n, sample_rate, o);
  out->pitch_mean = t.pitch_mean;
  out->pitch_std = t.pitch_std;
  out->energy_mean = t.energy_mean;
  out->energy_std = t.energy_std;
  out->spectral_centroid = t.spectral_centroid;
  out->zero_crossing_rate = t.zero_crossing_rate;
  out->arousal = t.arousal;
  out->valence = t.valence;
  out->n_vec = (int)t.speaker_vec.size();
  for (int i = 0; i < 8; ++i) out->speaker_vec[i] = i < out->n_vec ? t.speaker_vec[i] : 0.0f;
  std::strncpy(out->gender, t.gender_proxy.c_str(), sizeof out->gender - 1);
  out->gender[sizeof out->gender - 1] = 0;
  std::strncpy(out->emotion, t.emotion_proxy.c_str(), sizeof out->emotion - 1);
  out->emotion[sizeof out->emotion - 1] = 0;
  return 0;
}

void* ref_clusterer_new(float threshold) { return new SpeakerClusterer(threshold); }
void ref_clusterer_free(void* c) { delete static_cast<SpeakerClusterer*>(c); }
// assign_or_add(vec[0..n)); writes the speaker id
int ref_clusterer_assign(void* c, const float* vec, int n, char* id, int cap) {
  const std::string s = static_cast<SpeakerClusterer*>(c)->assign_or_add(std::vector<float>(vec, vec + n));
  std::strncpy(id, s.c_str(), cap - 1);
  id[cap - 1] = 0;
  return (int)s.size();
}

}  // extern "C"
