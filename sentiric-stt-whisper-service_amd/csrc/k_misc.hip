// LayerNorm, decoder embedding and on-device logits processing for gfx950.
//
// logits_process_kernel restates whisper.cpp's whisper_process_logits +
// whisper_sample_token(best = true) (host code in the reference, run on every
// decode step over all n_vocab logits — SURVEY.md §8 a10/a11) so only a
// 32-byte token record per row crosses PCIe per step. One 1024-thread
// workgroup per row keeps the row in registers (51 values per thread) and
// does every pass with wave-shuffle + LDS reductions.
#include "kcommon.h"
#include "kernels.h"

namespace mwx {

// ggml_norm (eps 1e-5, double accumulation) followed by *w + b. One 256-thread
// workgroup per row; every element of the row is loaded once, all loads of a
// thread are issued back to back (NPT = ceil(N / 256) registers per thread).
//
// With P != nullptr the row is first completed from the KS split-K partial
// slabs of the producing GEMM: x = (sum_ks P[ks] + pbias) + x (ggml: the
// matmul + bias, then the residual add), written back to x.
template <typename T, int NPT>
__global__ __launch_bounds__(256) void ln_kernel(float* __restrict__ x,
                                                 const float* __restrict__ w,
                                                 const float* __restrict__ b, T* __restrict__ y,
                                                 int N, const int* __restrict__ active,
                                                 const float* __restrict__ P, int KS,
                                                 long pstride, const float* __restrict__ pbias) {
  __shared__ double red[2][4];
  const int row = blockIdx.x;
  if (active && !active[row]) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* xr = x + (long)row * N;
  float v[NPT], wv[NPT], bv[NPT];
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int i = tid + 256 * j;
    v[j] = i < N ? xr[i] : 0.0f;
    wv[j] = i < N ? w[i] : 0.0f;
    bv[j] = i < N ? b[i] : 0.0f;
  }
  if (P) {
    // all KS (<= 8) partials of all NPT elements are loaded before summing
    float pk[NPT][8];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = min(tid + 256 * j, N - 1);
      const float* pp = P + (long)row * N + i;
#pragma unroll
      for (int k = 0; k < 8; ++k) pk[j][k] = k < KS ? pp[k * pstride] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = tid + 256 * j;
      float acc = pk[j][0];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (k < KS) acc += pk[j][k];
      if (i < N) {
        v[j] = (acc + pbias[i]) + v[j];
        xr[i] = v[j];
      }
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NPT; ++j) s += (double)v[j];
  s = wave_sum_d(s);
  if (lane == 0) red[0][wid] = s;
  __syncthreads();
  s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const float mean = (float)(s / N);
  double s2 = 0.0;
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int i = tid + 256 * j;
    const float d = v[j] - mean;
    if (i < N) s2 += (double)(d * d);
  }
  s2 = wave_sum_d(s2);
  if (lane == 0) red[1][wid] = s2;
  __syncthreads();
  s2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const float variance = (float)(s2 / N);
  const float scale = 1.0f / sqrtf(variance + 1e-5f);
  T* yr = y + (long)row * N;
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int i = tid + 256 * j;
    if (i < N) yr[i] = to_t<T>(((v[j] - mean) * scale) * wv[j] + bv[j]);
  }
}

template <typename T>
void layer_norm(const float* x, const float* w, const float* b, T* y, int M, int N,
                const int* active, hipStream_t st, const float* P, int KS, const float* pbias) {
  const int npt = (N + 255) / 256;
  const long pstride = (long)M * N;
  switch (npt) {
#define LNC(K)                                                                               \
  case K:                                                                                    \
    ln_kernel<T, K><<<M, 256, 0, st>>>((float*)x, w, b, y, N, active, P, KS, pstride, pbias); \
    break;
    LNC(1) LNC(2) LNC(3) LNC(4) LNC(5) LNC(6) LNC(7) LNC(8)
#undef LNC
    default: break;
  }
}

// x[r] = te[tok[r]] + pe[pos[r]]   (ggml_get_rows(d_te) + ggml_get_rows(d_pe))
template <typename T>
__global__ __launch_bounds__(256) void embed_kernel(const T* __restrict__ te,
                                                    const float* __restrict__ pe,
                                                    const int* __restrict__ tok,
                                                    const int* __restrict__ pos,
                                                    const int* __restrict__ active,
                                                    float* __restrict__ x, int d) {
  const int r = blockIdx.x;
  if (!active[r]) return;
  const T* er = te + (long)tok[r] * d;
  const float* pr = pe + (long)pos[r] * d;
  for (int i = threadIdx.x; i < d; i += 256) x[(long)r * d + i] = to_f<T>(er[i]) + pr[i];
}

template <typename T>
void embed(const T* te, const float* pe, const int* tok, const int* pos, const int* active,
           float* x, int R, int d, hipStream_t st) {
  embed_kernel<T><<<R, 256, 0, st>>>(te, pe, tok, pos, active, x, d);
}

template void layer_norm<_Float16>(const float*, const float*, const float*, _Float16*, int, int,
                                   const int*, hipStream_t, const float*, int, const float*);
template void layer_norm<__bf16>(const float*, const float*, const float*, __bf16*, int, int,
                                 const int*, hipStream_t, const float*, int, const float*);
template void embed<_Float16>(const _Float16*, const float*, const int*, const int*, const int*,
                              float*, int, int, hipStream_t);
template void embed<__bf16>(const __bf16*, const float*, const int*, const int*, const int*, float*,
                            int, int, hipStream_t);

// ---------------------------------------------------------------------------
// logits processing + greedy sampling
// ---------------------------------------------------------------------------
constexpr int LP_T = 1024;
constexpr int LP_NPT = 51;  // 51 * 1024 = 52224 >= 51866

struct BlockRed {
  float f[16];
  double d[16];
  int i[16];
};

__device__ __forceinline__ float bmax(float v, BlockRed& R) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) R.f[wid] = v;
  __syncthreads();
  float r = R.f[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) r = fmaxf(r, R.f[k]);
  return r;
}
__device__ __forceinline__ float bsum(float v, BlockRed& R) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) R.f[wid] = v;
  __syncthreads();
  float r = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) r += R.f[k];
  return r;
}
__device__ __forceinline__ double bsumd(double v, BlockRed& R) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) R.d[wid] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) r += R.d[k];
  return r;
}
// argmax with lowest-index tie break; entries with v <= floor never win
__device__ __forceinline__ void bargmax(float& v, int& idx, BlockRed& R) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    R.f[wid] = v;
    R.i[wid] = idx;
  }
  __syncthreads();
  v = R.f[0];
  idx = R.i[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    if (R.f[k] > v || (R.f[k] == v && R.i[k] < idx)) {
      v = R.f[k];
      idx = R.i[k];
    }
  }
}

__global__ __launch_bounds__(LP_T) void logits_process_kernel(
    const float* __restrict__ logits, const float* __restrict__ smask,
    const RowCtl* __restrict__ ctl, TokOut* __restrict__ out, float* __restrict__ probs_out,
    float* __restrict__ logprobs_out, LogitsConst C, int nosp_id) {
  __shared__ BlockRed R;
  const int row = blockIdx.x;
  const RowCtl c = ctl[row];
  if (!c.active || !c.sample) return;
  const int V = C.n_vocab;
  const int tid = threadIdx.x;
  const float* L = logits + (long)row * V;
  float x[LP_NPT];
  float rmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k) {
    const int i = tid + k * LP_T;
    x[k] = i < V ? L[i] : -INFINITY;
    rmax = fmaxf(rmax, x[k]);
  }
  float nosp = 0.0f;
  if (c.want_nosp) {
    // no_speech_prob from the raw logits (before any filtering)
    rmax = bmax(rmax, R);
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < LP_NPT; ++k) {
      const int i = tid + k * LP_T;
      if (i < V && x[k] > -INFINITY) s += expf(x[k] - rmax);
    }
    s = bsum(s, R);
    const float lse = logf(s) + rmax;
    nosp = expf(L[nosp_id] - lse);
  }
  const int tid0_init = C.max_initial_tid;
  const int ts_lo = C.beg + c.seek_delta / 2;
  float vmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k) {
    const int i = tid + k * LP_T;
    if (i >= V) continue;
    float v = x[k];
    if (c.temperature > 0.0f) v = v / c.temperature;
    bool kill = smask[i] < 0.0f;
    if (c.is_initial && C.suppress_blank && (i == C.eot || i == C.space_id)) kill = true;
    if (c.last_ts) {
      if (c.penult_ts) {
        if (i >= C.beg) kill = true;
      } else {
        if (i < C.eot) kill = true;
      }
    }
    if (c.is_initial && tid0_init >= 0 && i > tid0_init) kill = true;
    if (c.has_ts && i >= C.beg && i < ts_lo) kill = true;
    if (kill) v = -INFINITY;
    x[k] = v;
    vmax = fmaxf(vmax, v);
  }
  vmax = bmax(vmax, R);
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k) {
    const int i = tid + k * LP_T;
    if (i < V && x[k] > -INFINITY) s += expf(x[k] - vmax);
  }
  s = bsum(s, R);
  const float lse = logf(s) + vmax;
  // x -> logprobs
  float tsmax = -INFINITY, txmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k) {
    const int i = tid + k * LP_T;
    if (i >= V) continue;
    x[k] = x[k] > -INFINITY ? x[k] - lse : -INFINITY;
    if (i >= C.beg)
      tsmax = fmaxf(tsmax, x[k]);
    else
      txmax = fmaxf(txmax, x[k]);
  }
  tsmax = bmax(tsmax, R);
  txmax = bmax(txmax, R);
  float ss = 0.0f;
  if (tsmax > -INFINITY) {
#pragma unroll
    for (int k = 0; k < LP_NPT; ++k) {
      const int i = tid + k * LP_T;
      if (i < V && i >= C.beg && x[k] > -INFINITY) ss += expf(x[k] - tsmax);
    }
  }
  ss = bsum(ss, R);
  const float ts_logprob = ss > 0.0f ? logf(ss) + tsmax : -INFINITY;
  const bool kill_text = ts_logprob > txmax;
  // probs, greedy argmax, timestamp stats
  float best = 0.0f;
  int best_i = 0x7fffffff;
  float tbest = 0.0f;
  int tbest_i = 0x7fffffff;
  double sum_ts = 0.0;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k) {
    const int i = tid + k * LP_T;
    if (i >= V) continue;
    if (kill_text && i < C.beg) x[k] = -INFINITY;
    const float p = x[k] == -INFINITY ? 0.0f : expf(x[k]);
    if (c.want_probs) {
      probs_out[(long)row * V + i] = p;
      logprobs_out[(long)row * V + i] = x[k];
    }
    if (p > best) {
      best = p;
      best_i = i;
    }
    if (i >= C.beg) {
      sum_ts += (double)p;
      if (p > tbest) {
        tbest = p;
        tbest_i = i;
      }
    }
  }
  bargmax(best, best_i, R);
  bargmax(tbest, tbest_i, R);
  sum_ts = bsumd(sum_ts, R);
  // plog = logprobs[id]: the owning thread publishes it through LDS
  const int id = best > 0.0f ? best_i : 0;
  __shared__ float plog_sh;
#pragma unroll
  for (int k = 0; k < LP_NPT; ++k)
    if (tid + k * LP_T == id) plog_sh = x[k];
  __syncthreads();
  if (tid == 0) {
    TokOut t;
    t.tid = tbest > 0.0f ? tbest_i : 0;
    t.pt = (float)((double)tbest / (sum_ts + 1e-10));
    t.ptsum = (float)sum_ts;
    t.id = id;
    t.p = best;
    t.plog = plog_sh;  // (host applies the id >= beg -> tid/pt override)
    t.nosp = nosp;
    t.pad = 0;
    out[row] = t;
  }
}

void logits_process(float* logits, const float* static_mask, const RowCtl* ctl, TokOut* out,
                    float* probs, float* logprobs, const LogitsConst& C, int R, hipStream_t st) {
  logits_process_kernel<<<R, LP_T, 0, st>>>(logits, static_mask, ctl, out, probs, logprobs, C,
                                            C.nosp_id);
}

}  // namespace mwx
