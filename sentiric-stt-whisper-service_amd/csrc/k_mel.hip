// Log-mel front end on gfx950 (replaces whisper.cpp log_mel_spectrogram +
// log_mel_spectrogram_worker_thread, which run on the HOST CPU even in the
// reference's CUDA build — SURVEY.md §2.2 first row).
//
// Semantics followed (whisper.cpp v1.8.2, restated in oracle/mwx_oracle.cpp
// log_mel()):
//   * 200-sample reflect pad at the start (samples[200..1]), zeros after the
//     clip (30 s of zero padding + 200), periodic Hann(400), hop 160;
//   * |X_k|^2 for k = 0..200 in f32; mel energy accumulated in double;
//     log10(max(e, 1e-10)); frames past n_samples/160 + 1 are log10(1e-10);
//   * global max over the whole spectrogram, clamp at max - 8, (x + 4) / 4.
// The DFT is evaluated directly per bin (the upstream radix-2 recursion + 25-
// point DFT gives the same sums up to f32 rounding; tolerance 1e-4 on log-mel).
//
// Layout in HBM: mel[clip][n_mels][n_len] f32 (mel-bin major, time contiguous,
// as upstream), plus the encoder's f16 time-major input window
// melT[clip][1 + 3000 + 1][CPAD] (zero rows for the conv's t = -1 / 3000 taps).
#include "kcommon.h"
#include "kernels.h"

namespace mwx {

constexpr int MEL_FRAMES_PER_WG = 16;

// tables: hann[400], cosT[400], sinT[400] (whisper.cpp global cache values).
// All clips of a batch in one launch: grid (frame tiles of the longest clip,
// clips); clip c's samples / mel rows are at the offsets of desc[c].
__global__ __launch_bounds__(256) void mel_frames_kernel(
    const float* __restrict__ pcm_base, const MelClip* __restrict__ desc,
    const float* __restrict__ filters, int n_mels, const float* __restrict__ tables,
    float* __restrict__ out_base) {
  __shared__ float xs[MEL_FRAMES_PER_WG][400];
  __shared__ float tc[400], ts[400];
  __shared__ float pw[MEL_FRAMES_PER_WG][204];
  const MelClip dc = desc[blockIdx.y];
  const int n = dc.n, n_len = dc.n_len, n_fft_frames = dc.n_fft;
  const float* __restrict__ pcm = pcm_base + dc.pcm_off;
  float* __restrict__ out = out_base + dc.mel_off;
  float* __restrict__ save_raw = dc.save_raw;
  const int tid = threadIdx.x;
  const int i0 = blockIdx.x * MEL_FRAMES_PER_WG;
  if (i0 >= n_len) return;
  if (dc.save_pcm) {  // this tile's hop range of samples, for the next call
    const int j1 = min(n, (i0 + MEL_FRAMES_PER_WG) * 160);
    for (int j = i0 * 160 + tid; j < j1; j += 256) dc.save_pcm[j] = pcm[j];
  }
  const float floor_v = -10.0f;  // log10(1e-10)
  if (i0 >= n_fft_frames) {
    // constant frames (no signal): whole tile is log10(1e-10)
    for (int idx = tid; idx < MEL_FRAMES_PER_WG * n_mels; idx += 256) {
      const int f = idx % MEL_FRAMES_PER_WG, m = idx / MEL_FRAMES_PER_WG;
      const int i = i0 + f;
      if (i < n_len) {
        out[(size_t)m * n_len + i] = floor_v;
        if (save_raw) save_raw[(size_t)m * n_len + i] = floor_v;
      }
    }
    return;
  }
  // incremental: frame i reads padded samples [160 i, 160 i + 400), i.e.
  // samples [160 i - 200, 160 i + 200) (and samples 1..200 reflected for the
  // first frames). If every sample the tile reads is bit-identical to the
  // previous call's and lay inside that call's clip, the tile's raw log-mel
  // is the previous call's (same inputs, same arithmetic).
  if (dc.n_prev > 0) {
    const int last = min(i0 + MEL_FRAMES_PER_WG, n_fft_frames) - 1;
    const int lo = max(0, i0 * 160 - 200), hi = last * 160 + 200;
    bool same = hi <= n && hi <= dc.n_prev && last < dc.len_prev;
    if (same) {
      for (int j = lo + tid; j < hi; j += 256)
        same &= __float_as_uint(pcm[j]) == __float_as_uint(dc.prev_pcm[j]);
    }
    if (__syncthreads_and(same)) {
      for (int idx = tid; idx < MEL_FRAMES_PER_WG * n_mels; idx += 256) {
        const int f = idx % MEL_FRAMES_PER_WG, m = idx / MEL_FRAMES_PER_WG;
        const int i = i0 + f;
        if (i > last) continue;
        const float r = dc.prev_raw[(size_t)m * dc.len_prev + i];
        out[(size_t)m * n_len + i] = r;
        if (save_raw) save_raw[(size_t)m * n_len + i] = r;
      }
      // frames of the tile past n_fft_frames (the last tile): log10(1e-10)
      for (int idx = tid; idx < MEL_FRAMES_PER_WG * n_mels; idx += 256) {
        const int f = idx % MEL_FRAMES_PER_WG, m = idx / MEL_FRAMES_PER_WG;
        const int i = i0 + f;
        if (i <= last || i >= n_len) continue;
        out[(size_t)m * n_len + i] = floor_v;
        if (save_raw) save_raw[(size_t)m * n_len + i] = floor_v;
      }
      return;
    }
  }
  for (int j = tid; j < 400; j += 256) {
    tc[j] = tables[400 + j];
    ts[j] = tables[800 + j];
  }
  for (int idx = tid; idx < MEL_FRAMES_PER_WG * 400; idx += 256) {
    const int f = idx / 400, j = idx % 400;
    const int i = i0 + f;
    float v = 0.0f;
    if (i < n_fft_frames) {
      const int p = i * 160 + j;  // index into the padded signal
      float s = 0.0f;
      if (p < 200) {
        const int q = 200 - p;
        s = q < n ? pcm[q] : 0.0f;
      } else if (p - 200 < n) {
        s = pcm[p - 200];
      }
      v = tables[j] * s;
    }
    xs[f][j] = v;
  }
  __syncthreads();
  // DFT: thread k computes bin k for all frames of the tile
  if (tid < 201) {
    const int k = tid;
    float re[MEL_FRAMES_PER_WG], im[MEL_FRAMES_PER_WG];
#pragma unroll
    for (int f = 0; f < MEL_FRAMES_PER_WG; ++f) re[f] = im[f] = 0.0f;
    int idx = 0;
    for (int j = 0; j < 400; ++j) {
      const float c = tc[idx], s = ts[idx];
#pragma unroll
      for (int f = 0; f < MEL_FRAMES_PER_WG; ++f) {
        re[f] = fmaf(xs[f][j], c, re[f]);
        im[f] = fmaf(-xs[f][j], s, im[f]);
      }
      idx += k;
      if (idx >= 400) idx -= 400;
    }
#pragma unroll
    for (int f = 0; f < MEL_FRAMES_PER_WG; ++f) pw[f][k] = re[f] * re[f] + im[f] * im[f];
  }
  __syncthreads();
  for (int idx = tid; idx < MEL_FRAMES_PER_WG * n_mels; idx += 256) {
    const int f = idx % MEL_FRAMES_PER_WG, m = idx / MEL_FRAMES_PER_WG;
    const int i = i0 + f;
    if (i >= n_len) continue;
    float r;
    if (i < n_fft_frames) {
      const float* fl = filters + (size_t)m * 201;
      double sum = 0.0;
      for (int k = 0; k < 201; ++k) sum += (double)(pw[f][k] * fl[k]);
      r = (float)log10(fmax(sum, 1e-10));
    } else {
      r = floor_v;
    }
    out[(size_t)m * n_len + i] = r;
    if (save_raw) save_raw[(size_t)m * n_len + i] = r;
  }
}

// per-clip global max of the raw log-mel: MEL_MAX_PARTS workgroups per clip
// each reduce a slice into part[clip][p]; the normalisation takes the max of
// the parts (max is exact, so the result does not depend on the split)
constexpr int MEL_MAX_PARTS = 16;
__global__ __launch_bounds__(1024) void mel_max_kernel(const float* __restrict__ mel_base,
                                                       const MelClip* __restrict__ desc, int n_mels,
                                                       float* __restrict__ part) {
  const MelClip dc = desc[blockIdx.y];
  const long count = (long)n_mels * dc.n_len;
  const float* p = mel_base + dc.mel_off;
  const long per = (count + MEL_MAX_PARTS - 1) / MEL_MAX_PARTS;
  const long b = blockIdx.x * per, e = min(count, b + per);
  float v = -INFINITY;
  for (long i = b + threadIdx.x; i < e; i += 1024) v = fmaxf(v, p[i]);
  v = wave_max(v);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    float w = threadIdx.x < 16 ? red[threadIdx.x] : -INFINITY;
    w = wave_max(w);
    if (threadIdx.x == 0) part[blockIdx.y * MEL_MAX_PARTS + blockIdx.x] = w;
  }
}

// clamp at max - 8 and rescale: x = (max(x, mx - 8) + 4) / 4; mx[clip] keeps
// the clip's max
__global__ __launch_bounds__(256) void mel_norm_kernel(float* __restrict__ mel_base,
                                                       const MelClip* __restrict__ desc, int n_mels,
                                                       const float* __restrict__ part,
                                                       float* __restrict__ mx) {
  const MelClip dc = desc[blockIdx.y];
  const long count = (long)n_mels * dc.n_len;
  float m = part[blockIdx.y * MEL_MAX_PARTS];
#pragma unroll
  for (int q = 1; q < MEL_MAX_PARTS; ++q) m = fmaxf(m, part[blockIdx.y * MEL_MAX_PARTS + q]);
  if (blockIdx.x == 0 && threadIdx.x == 0) mx[blockIdx.y] = m;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  float* p = mel_base + dc.mel_off;
  const float lo = m - 8.0f;
  float x = p[i];
  if (x < lo) x = lo;
  p[i] = (x + 4.0f) / 4.0f;
}

// encoder input window: melT[slot][1 + t][c] = f16(mel[c][seek + t]) for
// t < 2*n_ctx, c < n_mels (0 beyond), rows 0 and 2*n_ctx + 1 stay zero.
// 64x64 tiles transposed through LDS (coalesced on both sides).
__global__ __launch_bounds__(256) void mel_window_kernel(
    const float* __restrict__ mel, long mel_clip_stride, const int* __restrict__ clip_of_slot,
    const int* __restrict__ seek_of_slot, const int* __restrict__ n_len_of_slot, int n_mels,
    int T, int cpad, _Float16* __restrict__ melT) {
  __shared__ float tile[64][65];
  const int slot = blockIdx.z;
  const int t0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* src = mel + (long)clip_of_slot[slot] * mel_clip_stride;
  const int seek = seek_of_slot[slot], n_len = n_len_of_slot[slot];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, t = t0 + tx;
    float v = 0.0f;
    if (c < n_mels && t < T && seek + t < n_len) v = src[(long)c * n_len + seek + t];
    tile[r][tx] = v;
  }
  __syncthreads();
  _Float16* dst = melT + (long)slot * (T + 2) * cpad;
  for (int r = ty; r < 64; r += 4) {
    const int t = t0 + r, c = c0 + tx;
    if (t < T && c < cpad) dst[(long)(1 + t) * cpad + c] = (_Float16)tile[tx][r];
  }
}

// whisper.cpp get_signal_energy(signal, n, 32): mean |x| over a 65-sample
// window, summed in the same sequential f32 order (bit-exact with the host).
__global__ __launch_bounds__(256) void signal_energy_kernel(const float* __restrict__ x, int n,
                                                            float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float sum = 0.0f;
  for (int j = -32; j <= 32; ++j) {
    const int k = i + j;
    if (k >= 0 && k < n) sum += fabsf(x[k]);
  }
  out[i] = sum / 65.0f;
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
void launch_mel_batch(const float* pcm_base, const MelClip* desc, int n_clips, int max_n_len,
                      const float* filters, int n_mels, const float* tables, float* mel_base,
                      float* part, float* mx, hipStream_t st) {
  if (n_clips <= 0 || max_n_len <= 0) return;
  const dim3 gf((max_n_len + MEL_FRAMES_PER_WG - 1) / MEL_FRAMES_PER_WG, n_clips);
  mel_frames_kernel<<<gf, 256, 0, st>>>(pcm_base, desc, filters, n_mels, tables, mel_base);
  mel_max_kernel<<<dim3(MEL_MAX_PARTS, n_clips), 1024, 0, st>>>(mel_base, desc, n_mels, part);
  const long count = (long)n_mels * max_n_len;
  const dim3 gn((unsigned)((count + 255) / 256), n_clips);
  mel_norm_kernel<<<gn, 256, 0, st>>>(mel_base, desc, n_mels, part, mx);
}
void launch_mel_window(const float* mel, long mel_clip_stride, const int* clip_of_slot,
                       const int* seek_of_slot, const int* n_len_of_slot, int n_mels, int T,
                       int cpad, _Float16* melT, int n_slots, hipStream_t st) {
  dim3 g((T + 63) / 64, (cpad + 63) / 64, n_slots);
  mel_window_kernel<<<g, 256, 0, st>>>(mel, mel_clip_stride, clip_of_slot, seek_of_slot,
                                       n_len_of_slot, n_mels, T, cpad, melT);
}
// pcm16 -> f32 as SttEngine::transcribe_pcm16 converts (x / 32768, exact)
__global__ void pcm16_to_f32_kernel(const int16_t* __restrict__ in, long n, float* __restrict__ out) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const short4 v = *reinterpret_cast<const short4*>(in + i);
    *reinterpret_cast<float4*>(out + i) =
        make_float4((float)v.x / 32768.0f, (float)v.y / 32768.0f, (float)v.z / 32768.0f,
                    (float)v.w / 32768.0f);
  } else {
    for (long j = i; j < n; ++j) out[j] = (float)in[j] / 32768.0f;
  }
}

void launch_pcm16_to_f32(const int16_t* in, long n, float* out, hipStream_t st) {
  if (n <= 0) return;
  const long th = (n + 3) / 4;
  pcm16_to_f32_kernel<<<(unsigned)((th + 255) / 256), 256, 0, st>>>(in, n, out);
}

void launch_signal_energy(const float* x, int n, float* out, hipStream_t st) {
  signal_energy_kernel<<<(n + 255) / 256, 256, 0, st>>>(x, n, out);
}

}  // namespace mwx
