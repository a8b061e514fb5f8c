// Segment prosody on the GPU: the reference's extract_prosody
// (src/prosody_extractor.cpp:31-224), run for every kept segment of a clip
// (src/stt_engine.cpp:313-337) — one 256-thread workgroup per segment,
// results bit-identical to the reference's x86-64 build (-O3, no -march: plain
// IEEE single precision, no contraction — this file is built with
// -ffp-contract=off, and every division below is the correctly rounded one and
// sqrt_rn restores the correctly rounded square root).
//
// The reference is one sequential loop per segment; three of its parts are
// order-dependent in float and are restated so the GPU can run them wide
// without changing a bit:
//  * the one-pole low-pass y += a * (x - y) runs across the whole segment.
//    Each thread takes a run of frames, warms the filter up over the W samples
//    before its run from a guessed state, and records the state it reaches at
//    each of its frame starts. The filter is a contraction, so the guessed and
//    true trajectories meet exactly (same float) within the warm-up; whether
//    they met is CHECKED — thread t's state at its first frame must equal
//    thread t-1's exact end state, bit for bit — and a run that fails the
//    check is recomputed serially from the exact state. The serial pass is
//    therefore the fallback, never an approximation.
//  * per-frame sums (energy, spectral centroid, crossings) are sequential
//    over the frame's samples, one thread per frame — as the reference.
//  * segment means / deviations accumulate over frames in frame order: one
//    wave per statistic, a wave-uniform chain fed 64 frames at a time by
//    v_readlane (coalesced loads, the adds stay in the reference's order).
//  * the pitch median (std::nth_element) is the (n/2)-th smallest f0; every f0
//    is cycles / frame duration, monotone in the integer cycle count, so a
//    cycle-count histogram gives it exactly.
#include "kcommon.h"
#include "kernels.h"

namespace mwx {

namespace {

constexpr int PT = 256;        // threads per segment
constexpr int PMAX_HALF = 801; // cycle-count bins: a frame of <= 1600 samples has < 800 cycles

__device__ __forceinline__ float fmin_ref(float a, float b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ float fmax_ref(float a, float b) { return (a < b) ? b : a; }  // std::max

// soft_norm (src/prosody_extractor.cpp:25-28)
__device__ __forceinline__ float soft_norm(float v, float lo, float hi) {
  const float n = __fdiv_rn(v - lo, hi - lo);
  return fmax_ref(0.0f, fmin_ref(1.0f, n));
}

// correctly rounded sqrt (std::sqrt on the reference's SSE build): v_sqrt_f32
// is within 1 ulp, so the answer is the candidate among its neighbours whose
// rounding interval holds x — decided exactly in double (a midpoint of two
// adjacent floats has 25 significant bits, its square 50)
__device__ __forceinline__ float sqrt_rn(float x) {
  float s = __builtin_sqrtf(x);
  if (!(x > 0.0f) || __builtin_isinf(x)) return s;
  const double d = x;
  for (int it = 0; it < 2; ++it) {
    const float up = __int_as_float(__float_as_int(s) + 1);
    const double mu = ((double)s + (double)up) * 0.5;
    if (mu * mu < d) {
      s = up;
      continue;
    }
    const float dn = __int_as_float(__float_as_int(s) - 1);
    const double md = ((double)s + (double)dn) * 0.5;
    if (md * md > d) s = dn;
  }
  return s;
}

__device__ __forceinline__ float lpf_step(float y, float x, float a) { return y + a * (x - y); }

// Streams p[0..n) through registers in blocks of 32 (eight 16-byte loads in
// flight per lane, each lane on its own run of samples) and calls fn on every
// sample in order: a lane's 128-byte lines are consumed whole from registers
// instead of being re-fetched sample by sample through L1.
template <class Fn>
__device__ __forceinline__ void stream(const float* __restrict__ p, long n, Fn&& fn) {
  long i = 0;
  for (; i + 32 <= n; i += 32) {
    float v[32];
#pragma unroll
    for (int q = 0; q < 32; q += 4) {
      float4 t;
      __builtin_memcpy(&t, p + i + q, 16);
      v[q] = t.x;
      v[q + 1] = t.y;
      v[q + 2] = t.z;
      v[q + 3] = t.w;
    }
#pragma unroll
    for (int q = 0; q < 32; ++q) fn(v[q]);
  }
  for (; i < n; ++i) fn(p[i]);
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

}  // namespace

// pcm: the clip; seg: [n_seg] descriptors; fstate / feat: scratch of
// sum(frames) floats / float4; out: [n_seg] results.
__global__ __launch_bounds__(PT) void prosody_kernel(const float* __restrict__ pcm,
                                                     const ProsodySeg* __restrict__ seg,
                                                     float* __restrict__ fstate,
                                                     float4* __restrict__ feat, ProsodyOut* out,
                                                     int F, int sample_rate, float alpha,
                                                     float gender_thr, float min_pitch,
                                                     float max_pitch, int warm) {
  __shared__ float s_spec[PT], s_end[PT];
  __shared__ int s_hist[PMAX_HALF];
  __shared__ float s_stat[8];
  __shared__ int s_cnt[2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const ProsodySeg sg = seg[blockIdx.x];
  ProsodyOut& o = out[blockIdx.x];
  const long n = sg.len;
  if (n < 160) {  // src/prosody_extractor.cpp:35-48
    if (t == 0) {
      o = ProsodyOut{};
      o.gender = 0;
      o.emotion = 0;
    }
    return;
  }
  const float* x = pcm + sg.start;
  const long nfr = (long)((unsigned)n / (unsigned)F);  // frames i + F <= n (n < 2^31: host-checked)
  float* fs = fstate + sg.frame_off;
  float4* ft = feat + sg.frame_off;
  // phase-1 silence flags live in the feature slots until phase 2 fills them
  int* zf = reinterpret_cast<int*>(ft);

  // ---- 1. low-pass states at every frame start (speculative, checked) ----
  const long fpt = (nfr + PT - 1) / PT;
  const long f0 = (long)t * fpt, f1 = f0 + fpt < nfr ? f0 + fpt : nfr;
  float y_end = 0.0f, y_spec = 0.0f;
  if (f0 < f1) {
    const long j0 = f0 * F;
    long w0 = j0 - warm;
    if (w0 < 0) w0 = 0;
    float y = t == 0 ? 0.0f : x[w0];  // thread 0 starts from the true state
    stream(x + w0, j0 - w0, [&](float v) { y = lpf_step(y, v, alpha); });
    y_spec = y;
    for (long f = f0; f < f1; ++f) {
      fs[f] = y;
      unsigned any = 0;
      stream(x + f * F, F, [&](float v) {
        any |= __float_as_uint(v);
        y = lpf_step(y, v, alpha);
      });
      zf[f] = any == 0;  // digital-silence frame (all +0.0)
    }
    y_end = y;
  }
  s_spec[t] = y_spec;
  s_end[t] = y_end;
  __syncthreads();
  int redo = 0;
  if (t == 0) {
    float prev = s_end[0];
    for (int u = 1; u < PT; ++u) {
      const long g0 = (long)u * fpt, g1 = g0 + fpt < nfr ? g0 + fpt : nfr;
      if (g0 >= g1) break;
      if (__float_as_uint(s_spec[u]) == __float_as_uint(prev)) {
        prev = s_end[u];
        continue;
      }
      // serial recomputation from the exact state. It stops as soon as it
      // meets the run's own trajectory at a frame start (the rest of the run
      // is then exact already), and steps over digital-silence frames once
      // the state is a fixed point of y += a * (0 - y) — the case where the
      // check fails for good: a decayed state stuck at a denormal never
      // meets a guessed 0.
      ++redo;
      float y = prev;
      bool met = false;
      for (long f = g0; f < g1; ++f) {
        if (f > g0 && __float_as_uint(fs[f]) == __float_as_uint(y)) {
          met = true;
          break;
        }
        fs[f] = y;
        if (zf[f] && __float_as_uint(lpf_step(y, 0.0f, alpha)) == __float_as_uint(y)) continue;
        const float* xf = x + f * F;
        for (int k = 0; k < F; ++k) y = lpf_step(y, xf[k], alpha);
      }
      prev = met ? s_end[u] : y;
    }
  }
  for (int i = t; i < PMAX_HALF; i += PT) s_hist[i] = 0;
  __syncthreads();

  // ---- 2. per-frame features (src/prosody_extractor.cpp:63-128) ----
  const float duration = __fdiv_rn((float)F, (float)sample_rate);
  for (long f = t; f < nfr; f += PT) {
    const float* xf = x + f * F;
    // energy and spectral-centroid sums (raw samples), in sample order
    float r0 = 0.0f, power = 0.0f, weighted = 0.0f, prev = 0.0f;
    int k = 0;
    stream(xf, F, [&](float v) {
      r0 += v * v;
      if (k > 0) {
        const float d = fabsf(v - prev);
        weighted += d * (float)k;
        power += d;
      }
      prev = v;
      ++k;
    });
    const float rms = sqrt_rn(__fdiv_rn(r0, (float)F));
    const float clip = fmax_ref(0.002f, rms * 0.15f);
    // low-passed crossings and the hysteresis cycle counter (state 0: not
    // yet armed, 1: positive, 2: negative; a 1 -> 2 move is one cycle)
    float y = fs[f], yp = 0.0f;
    int cycles = 0, zc = 0, sm = 0;
    k = 0;
    stream(xf, F, [&](float v) {
      y = lpf_step(y, v, alpha);
      if (k > 0) {
        zc += (y >= 0.0f) != (yp >= 0.0f);
        const bool up = y > clip, dn = y < -clip;
        cycles += (sm == 1) & dn;
        sm = up ? 1 : (dn ? 2 : sm);
      }
      yp = y;
      ++k;
    });
    float f0v = -1.0f;
    if (rms > 0.015f && cycles > 0) {
      const float e = __fdiv_rn((float)cycles, duration);
      if (e >= min_pitch && e <= max_pitch) {
        f0v = e;
        atomicAdd(&s_hist[cycles], 1);
      }
    }
    ft[f] = make_float4(rms, __fdiv_rn((float)zc, (float)F),
                        power > 0.0f ? __fdiv_rn(weighted, power) : 0.0f, f0v);
  }
  __syncthreads();

  // ---- 3. segment statistics, each in frame order (one wave per chain) ----
  if (wave == 0) {  // f0: mean and deviation over the voiced frames
    float s = 0.0f;
    int cnt = 0;
    for (long b = 0; b < nfr; b += 64) {
      const float v = b + lane < nfr ? ft[b + lane].w : -1.0f;
      const int m = (int)(nfr - b < 64 ? nfr - b : 64);
      for (int i = 0; i < m; ++i) {
        const float e = readlane_f(v, i);
        if (e >= 0.0f) {
          s += e;
          ++cnt;
        }
      }
    }
    float acc = 0.0f, mean = 0.0f;
    if (cnt > 0) {
      mean = __fdiv_rn(s, (float)cnt);
      for (long b = 0; b < nfr; b += 64) {
        const float v = b + lane < nfr ? ft[b + lane].w : -1.0f;
        const int m = (int)(nfr - b < 64 ? nfr - b : 64);
        for (int i = 0; i < m; ++i) {
          const float e = readlane_f(v, i);
          if (e >= 0.0f) acc += (e - mean) * (e - mean);
        }
      }
    }
    if (lane == 0) {
      s_stat[0] = cnt > 0 ? sqrt_rn(__fdiv_rn(acc, (float)cnt)) : 0.0f;  // pitch_std
      s_cnt[0] = cnt;
    }
  } else if (wave == 1) {  // energy: mean, deviation, onsets
    float s = 0.0f, last = 0.0f;
    int peaks = 0;
    for (long b = 0; b < nfr; b += 64) {
      const float v = b + lane < nfr ? ft[b + lane].x : 0.0f;
      const int m = (int)(nfr - b < 64 ? nfr - b : 64);
      for (int i = 0; i < m; ++i) {
        const float r = readlane_f(v, i);
        s += r;
        if (r > 0.05f && last <= 0.05f) ++peaks;
        last = r;
      }
    }
    const float mean = __fdiv_rn(s, (float)nfr);
    float acc = 0.0f;
    for (long b = 0; b < nfr; b += 64) {
      const float v = b + lane < nfr ? ft[b + lane].x : 0.0f;
      const int m = (int)(nfr - b < 64 ? nfr - b : 64);
      for (int i = 0; i < m; ++i) {
        const float r = readlane_f(v, i);
        acc += (r - mean) * (r - mean);
      }
    }
    if (lane == 0) {
      s_stat[1] = mean;
      s_stat[2] = sqrt_rn(__fdiv_rn(acc, (float)nfr));
      s_cnt[1] = peaks;
    }
  } else {  // waves 2 / 3: spectral centroid / zero-crossing-rate means
    float s = 0.0f;
    for (long b = 0; b < nfr; b += 64) {
      const float4 q = b + lane < nfr ? ft[b + lane] : make_float4(0, 0, 0, 0);
      const float v = wave == 2 ? q.z : q.y;
      const int m = (int)(nfr - b < 64 ? nfr - b : 64);
      for (int i = 0; i < m; ++i) s += readlane_f(v, i);
    }
    if (lane == 0) s_stat[wave + 1] = nfr > 0 ? __fdiv_rn(s, (float)nfr) : 0.0f;
  }
  __syncthreads();
  if (t != 0) return;

  // ---- 4. heuristics (src/prosody_extractor.cpp:130-221) ----
  ProsodyOut r{};
  const int nf0 = s_cnt[0];
  float pitch = 0.0f;  // vector_median: the (n/2)-th smallest f0
  if (nf0 > 0) {
    const int k = nf0 / 2;
    int cum = 0;
    for (int c = 0; c < PMAX_HALF; ++c) {
      cum += s_hist[c];
      if (cum > k) {
        pitch = __fdiv_rn((float)c, duration);
        break;
      }
    }
  }
  r.pitch_std = s_stat[0];
  if (nfr > 0) {
    r.energy_mean = s_stat[1];
    r.energy_std = s_stat[2];
    r.spectral_centroid = s_stat[3];
    r.zero_crossing_rate = s_stat[4];
  } else {
    r.energy_mean = 0.01f;
    r.energy_std = 0.0f;
    r.spectral_centroid = 50.0f;
    r.zero_crossing_rate = 0.1f;
  }
  const int peaks = nfr > 0 ? s_cnt[1] : 0;
  if (pitch > gender_thr && r.zero_crossing_rate < 0.024f)
    pitch *= 0.5f;
  else if (r.energy_mean > 0.12f && pitch < 240.0f && r.spectral_centroid < 90.0f)
    pitch *= 0.5f;
  r.pitch_mean = pitch;
  const float dur_s = __fdiv_rn((float)n, (float)sample_rate);
  const float rate = dur_s > 0.0f ? __fdiv_rn((float)peaks, dur_s) : 0.0f;
  int g;  // 0 '?', 1 'M', 2 'F'
  if (pitch == 0.0f || r.energy_mean < 0.018f)
    g = 0;
  else if (r.zero_crossing_rate < 0.030f)
    g = 1;
  else
    g = pitch > gender_thr ? 2 : 1;
  const float np = g == 1 ? soft_norm(pitch, 60.0f, 180.0f) : soft_norm(pitch, 160.0f, 350.0f);
  const float nb = soft_norm(r.spectral_centroid, 40.0f, 150.0f);
  float val = ((np * 0.4f) + (nb * 0.6f)) * 2.0f - 1.0f;
  val += 0.35f;
  const float ne = soft_norm(r.energy_mean, 0.02f, 0.20f);
  const float nr = soft_norm(rate, 2.0f, 9.0f);
  const float ar = (ne * 0.7f) + (nr * 0.3f);
  int em;  // 0 neutral, 1 excited, 2 angry, 3 sad
  if (ar > 0.65f)
    em = val > 0.1f ? 1 : 2;
  else if (ar < 0.30f)
    em = val < -0.4f ? 3 : 0;
  else
    em = 0;
  r.arousal = ar;
  r.valence = val;
  r.gender = g;
  r.emotion = em;
  float base;
  if (g == 1)
    base = soft_norm(pitch, 60.0f, 200.0f) * 0.4f;
  else if (g == 2)
    base = 0.6f + (soft_norm(pitch, 160.0f, 350.0f) * 0.4f);
  else
    base = 0.5f;
  r.speaker_vec[0] = base;
  r.speaker_vec[1] = soft_norm(r.spectral_centroid, 40.0f, 250.0f);
  r.speaker_vec[4] = soft_norm(r.zero_crossing_rate, 0.0f, 0.5f) * 0.8f;
  r.speaker_vec[2] = soft_norm(r.pitch_std, 5.0f, 100.0f) * 0.1f;
  r.speaker_vec[3] = soft_norm(r.energy_mean, 0.0f, 0.3f) * 0.1f;
  r.speaker_vec[5] = soft_norm(rate, 1.0f, 12.0f) * 0.1f;
  r.speaker_vec[6] = ar * 0.05f;
  r.speaker_vec[7] = __fdiv_rn(val + 1.0f, 2.0f) * 0.05f;
  r.serial_runs = redo;
  o = r;
}

void prosody_launch(const float* pcm, const ProsodySeg* seg, int n_seg, float* fstate,
                    float4* feat, ProsodyOut* out, int frame, int sample_rate, float alpha,
                    float gender_thr, float min_pitch, float max_pitch, hipStream_t st) {
  if (n_seg <= 0) return;
  // warm-up: |1 - alpha|^W below e^-40 (~2^-58), then 64 steps for the two
  // trajectories to settle on the same float (0.07 -> 615 samples); other
  // alphas just take the checked serial pass more often
  int warm = 640;
  if (alpha > 0.0f && alpha < 1.0f) {
    const float w = 40.0f / -log1pf(-alpha);
    warm = w > 4096.0f ? 4096 : (int)w + 64;
  }
  prosody_kernel<<<n_seg, PT, 0, st>>>(pcm, seg, fstate, feat, out, frame, sample_rate, alpha,
                                        gender_thr, min_pitch, max_pitch, warm);
}

}  // namespace mwx
