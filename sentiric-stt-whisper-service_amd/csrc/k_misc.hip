// LayerNorm, decoder embedding and on-device logits processing for gfx950.
//
// logits_process_kernel restates whisper.cpp's whisper_process_logits +
// whisper_sample_token(best = true) (host code in the reference, run on every
// decode step over all n_vocab logits — SURVEY.md §8 a10/a11) so only a
// 32-byte token record per row crosses PCIe per step. One 1024-thread
// workgroup per row keeps the row in registers (51 values per thread) and
// does every pass with wave-shuffle + LDS reductions.
#include <type_traits>

#include <cstdlib>

#include "kcommon.h"
#include "kernels.h"
#include "ln_core.h"

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

// Decode LayerNorm (same arithmetic as ln_kernel) for the few rows of a
// decode step: each thread owns 8 consecutive elements, so all loads are
// 16-B vectors, and the normalised row is stored as 16-B pieces of the
// decode-GEMM A tiles (pack_index).
template <typename T>
__global__ __launch_bounds__(256) void ln_dec_kernel(float* __restrict__ x,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ b,
                                                     T* __restrict__ y, int N,
                                                     const int* __restrict__ active,
                                                     const float* __restrict__ P, int KS,
                                                     long pstride,
                                                     const float* __restrict__ pbias,
                                                     EmbedIn<T> emb) {
  __shared__ double red[2][4];
  const int row = blockIdx.x;
  // the row, its split-K slabs and the activity flag are all requested before
  // the inactive-row exit waits on the flag (one round trip, not two)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool own = tid * 8 < N;
  const int i0 = own ? tid * 8 : 0;
  float* xr = x + (long)row * N + i0;
  f32x4 xa, xc;
  if (emb.te) {
    // x = te[tok] + pe[pos] (ggml_get_rows(d_te) + ggml_get_rows(d_pe)), the ids first.
    // The clamp keeps inactive rows' stale ids / positions in bounds (they
    // are requested before the activity flag); active rows' ids are in range
    // by construction (sampled ids, host-validated prompts: driver.inc
    // tokens_valid) and positions < n_text_ctx (the token loop's cap)
    const int tk = min(max(emb.tok[row], 0), emb.n_tok - 1);
    const int ps = min(max(emb.pos[row], 0), emb.n_pos - 1);
    const typename Elt<T>::v8 er =
        *reinterpret_cast<const typename Elt<T>::v8*>(emb.te + (long)tk * N + i0);
    const float* pr = emb.pe + (long)ps * N + i0;
    const f32x4 pa = *reinterpret_cast<const f32x4*>(pr);
    const f32x4 pc = *reinterpret_cast<const f32x4*>(pr + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xa[e] = to_f<T>(er[e]) + pa[e];
      xc[e] = to_f<T>(er[4 + e]) + pc[e];
    }
  } else {
    xa = *reinterpret_cast<const f32x4*>(xr);
    xc = *reinterpret_cast<const f32x4*>(xr + 4);
  }
  f32x4 pk[8][2];
  f32x4 pb0, pb1;
  if (P) {
    const float* pp = P + (long)row * N + i0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < KS) {
        pk[k][0] = *reinterpret_cast<const f32x4*>(pp + k * pstride);
        pk[k][1] = *reinterpret_cast<const f32x4*>(pp + k * pstride + 4);
      }
    pb0 = *reinterpret_cast<const f32x4*>(pbias + i0);
    pb1 = *reinterpret_cast<const f32x4*>(pbias + i0 + 4);
  }
  // the LayerNorm weights too: no load is left behind the two reductions
  const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + i0);
  const f32x4 w1 = *reinterpret_cast<const f32x4*>(w + i0 + 4);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + i0);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(b + i0 + 4);
  __builtin_amdgcn_sched_barrier(0);
  const int act_r = active ? active[row] : 1;
  if (!act_r) {
    asm volatile("" ::"v"(xa[0]), "v"(xc[0]));  // (the loads stay above the exit)
    return;
  }
  float v[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = xa[e];
    v[4 + e] = xc[e];
  }
  if (P) ln_fold8(v, pk, KS, pb0, pb1);
  if (P || emb.te) {
    if (own) {
      *reinterpret_cast<f32x4*>(xr) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(xr + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
  float mean, scale;
  ln_stats(v, own, N, red, lane, wid, mean, scale);
  if (!own) return;
  *reinterpret_cast<typename Elt<T>::v8*>(y + pack_index(row, i0, N)) =
      ln_out8<T>(v, mean, scale, w0, w1, b0, b1);
}

template <typename T>
void layer_norm_dec(float* x, const float* w, const float* b, T* y, int M, int N,
                    const int* active, hipStream_t st, const float* P, int KS,
                    const float* pbias, const EmbedIn<T>& emb) {
  ln_dec_kernel<T><<<M, 256, 0, st>>>(x, w, b, y, N, active, P, KS, (long)M * N, pbias, emb);
}

template void layer_norm<_Float16>(const float*, const float*, const float*, _Float16*, int, int,
                                   const int*, hipStream_t, const float*, int, const float*);
template void layer_norm<__bf16>(const float*, const float*, const float*, __bf16*, int, int,
                                 const int*, hipStream_t, const float*, int, const float*);
template void layer_norm_dec<_Float16>(float*, const float*, const float*, _Float16*, int, int,
                                       const int*, hipStream_t, const float*, int, const float*,
                                       const EmbedIn<_Float16>&);
template void layer_norm_dec<__bf16>(float*, const float*, const float*, __bf16*, int, int,
                                     const int*, hipStream_t, const float*, int, const float*,
                                     const EmbedIn<__bf16>&);

// ---------------------------------------------------------------------------
// logits processing + greedy sampling
//
// Each row is split over LP_G chunk workgroups so the exp/compare passes run
// on LP_G x rows CUs instead of one CU per row:
//   phase 1: filter (temperature, suppression, timestamp rules) -> flt, and
//            per-chunk max / sum-exp statistics;
//   phase 2: combine the chunk statistics (lse, timestamp log-prob, text max
//            -> the "force timestamp" rule), probs = expf(logprob), per-chunk
//            argmax / timestamp argmax / timestamp prob sum;
//   phase 3: combine the chunks in index order (lowest-index tie break).
// ---------------------------------------------------------------------------
constexpr int LP_T = 256;
constexpr int LP_NPT = (LP_CHUNK + LP_T - 1) / LP_T;

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

__device__ __forceinline__ float bmax256(float v, float* red) {
  v = wave_max_dpp(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ float bsum256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ double bsum256d(double v, double* red) {
  v = wave_sum_d_dpp(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
// several workgroup reductions through one barrier pair: each value is
// reduced exactly as by its single-value form (wave reduction, then the four
// wave results in the same order), so results are bit-identical
__device__ __forceinline__ void bmax3_256(float& a, float& b, float& c, float (*red)[4]) {
  a = wave_max_dpp(a);
  b = wave_max_dpp(b);
  c = wave_max_dpp(c);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    red[0][wid] = a;
    red[1][wid] = b;
    red[2][wid] = c;
  }
  __syncthreads();
  a = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  b = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  c = fmaxf(fmaxf(red[2][0], red[2][1]), fmaxf(red[2][2], red[2][3]));
}
__device__ __forceinline__ void bsum2_256(float& a, float& b, float (*red)[4]) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    red[0][wid] = a;
    red[1][wid] = b;
  }
  __syncthreads();
  a = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  b = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
}
// argmax with lowest-index tie break
__device__ __forceinline__ void better(float& v, int& idx, float ov, int oi) {
  if (ov > v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}
__device__ __forceinline__ void bargmax256(float& v, int& idx, float* redf, int* redi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) better(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    redf[wid] = v;
    redi[wid] = idx;
  }
  __syncthreads();
  v = redf[0];
  idx = redi[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) better(v, idx, redf[k], redi[k]);
}

__global__ __launch_bounds__(LP_T) void lp_filter_kernel(const float* __restrict__ logits,
                                                         const float* __restrict__ smask,
                                                         const RowCtl* __restrict__ ctl,
                                                         float* __restrict__ flt,
                                                         LPPart* __restrict__ parts,
                                                         LogitsConst C) {
  __shared__ float red[4];
  __shared__ float red3[3][4];
  const int row = blockIdx.y, ch = blockIdx.x;
  const RowCtl c = ctl[row];
  if (!c.active || !c.sample) return;
  const int V = C.n_vocab, tid = threadIdx.x;
  const int base = ch * LP_CHUNK;
  const float* L = logits + (long)row * V;
  float* F = flt + (long)row * V;
  const int tid0_init = C.max_initial_tid;
  const int ts_lo = C.beg + c.seek_delta / 2;
  float x[LP_NPT], v[LP_NPT];
  float rmax = -INFINITY, m = -INFINITY, mtext = -INFINITY, mts = -INFINITY;
  sfor<0, LP_NPT>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int off = tid + k * LP_T;
    const int i = min(base + off, V - 1);
    const bool in = off < LP_CHUNK && base + off < V;
    x[k] = in ? L[i] : -INFINITY;
    float y = x[k];
    if (c.temperature > 0.0f) y = y / c.temperature;
    bool kill = !in || smask[i] < 0.0f;
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
    v[k] = kill ? -INFINITY : y;
    if (in) F[i] = v[k];
    rmax = fmaxf(rmax, x[k]);
    m = fmaxf(m, v[k]);
    if (i >= C.beg)
      mts = fmaxf(mts, v[k]);
    else
      mtext = fmaxf(mtext, v[k]);
  });
  bmax3_256(m, mts, mtext, red3);
  float s = 0.0f, sts = 0.0f, rs = 0.0f;
  sfor<0, LP_NPT>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int i = base + tid + k * LP_T;
    if (v[k] > -INFINITY) {
      s += expf(v[k] - m);
      if (i >= C.beg) sts += expf(v[k] - mts);
    }
  });
  bsum2_256(s, sts, red3);
  if (c.want_nosp) {
    rmax = bmax256(rmax, red);
    sfor<0, LP_NPT>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if (x[k] > -INFINITY) rs += expf(x[k] - rmax);
    });
    rs = bsum256(rs, red);
  }
  if (tid == 0) {
    LPPart P;
    P.m = m;
    P.s = s;
    P.mtext = mtext;
    P.mts = mts;
    P.sts = sts;
    P.rm = rmax;
    P.rs = rs;
    P.pad = 0.0f;
    parts[row * LP_G + ch] = P;
  }
}

struct LPStats {
  float lse, rlse;
  bool kill_text;
};
__device__ __forceinline__ LPStats lp_combine(const LPPart* P, bool want_nosp) {
  float M = -INFINITY, Mts = -INFINITY, Mtext = -INFINITY, RM = -INFINITY;
  for (int g = 0; g < LP_G; ++g) {
    M = fmaxf(M, P[g].m);
    Mts = fmaxf(Mts, P[g].mts);
    Mtext = fmaxf(Mtext, P[g].mtext);
    RM = fmaxf(RM, P[g].rm);
  }
  float S = 0.0f, Sts = 0.0f, RS = 0.0f;
  for (int g = 0; g < LP_G; ++g) {
    if (P[g].m > -INFINITY) S += P[g].s * expf(P[g].m - M);
    if (P[g].mts > -INFINITY) Sts += P[g].sts * expf(P[g].mts - Mts);
    if (want_nosp && P[g].rm > -INFINITY) RS += P[g].rs * expf(P[g].rm - RM);
  }
  LPStats st;
  st.lse = logf(S) + M;
  st.rlse = want_nosp ? logf(RS) + RM : 0.0f;
  // whisper_process_logits: timestamp log-prob = logsumexp of the timestamp
  // log-probs; max text log-prob = max(text logits) - lse
  const float ts_logprob = Sts > 0.0f ? (logf(Sts) + Mts) - st.lse : -INFINITY;
  const float txmax = Mtext > -INFINITY ? Mtext - st.lse : -INFINITY;
  st.kill_text = ts_logprob > txmax;
  return st;
}

__global__ __launch_bounds__(LP_T) void lp_probs_kernel(float* __restrict__ flt,
                                                        const LPPart* __restrict__ parts,
                                                        const RowCtl* __restrict__ ctl,
                                                        LPRes* __restrict__ res,
                                                        float* __restrict__ probs_out,
                                                        float* __restrict__ logprobs_out,
                                                        LogitsConst C) {
  __shared__ float redf2[2][4];
  __shared__ int redi2[2][4];
  __shared__ double redd[4];
  const int row = blockIdx.y, ch = blockIdx.x;
  const RowCtl c = ctl[row];
  if (!c.active || !c.sample) return;
  const int V = C.n_vocab, tid = threadIdx.x;
  const int base = ch * LP_CHUNK;
  const LPStats st = lp_combine(parts + row * LP_G, c.want_nosp);
  const float* F = flt + (long)row * V;
  float best = 0.0f, tbest = 0.0f;
  int best_i = 0x7fffffff, tbest_i = 0x7fffffff;
  double sum_ts = 0.0;
  sfor<0, LP_NPT>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int off = tid + k * LP_T;
    const int i = base + off;
    if (off < LP_CHUNK && i < V) {
      const float v = F[i];
      const float lp = (v == -INFINITY || (st.kill_text && i < C.beg)) ? -INFINITY : v - st.lse;
      const float p = lp == -INFINITY ? 0.0f : expf(lp);
      if (c.want_probs) {
        probs_out[(long)row * V + i] = p;
        logprobs_out[(long)row * V + i] = lp;
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
  });
  {  // (bargmax256 x 2 + bsum256d through one barrier pair, same orders)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      better(best, best_i, __shfl_xor(best, o, 64), __shfl_xor(best_i, o, 64));
      better(tbest, tbest_i, __shfl_xor(tbest, o, 64), __shfl_xor(tbest_i, o, 64));
    }
    sum_ts = wave_sum_d_dpp(sum_ts);
    const int lane = tid & 63, wid = tid >> 6;
    __syncthreads();
    if (lane == 0) {
      redf2[0][wid] = best;
      redi2[0][wid] = best_i;
      redf2[1][wid] = tbest;
      redi2[1][wid] = tbest_i;
      redd[wid] = sum_ts;
    }
    __syncthreads();
    best = redf2[0][0];
    best_i = redi2[0][0];
    tbest = redf2[1][0];
    tbest_i = redi2[1][0];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      better(best, best_i, redf2[0][k], redi2[0][k]);
      better(tbest, tbest_i, redf2[1][k], redi2[1][k]);
    }
    sum_ts = (redd[0] + redd[1]) + (redd[2] + redd[3]);
  }
  if (tid == 0) {
    LPRes r;
    r.best = best;
    r.best_i = best_i;
    r.tbest = tbest;
    r.tbest_i = tbest_i;
    r.sum_ts = sum_ts;
    res[row * LP_G + ch] = r;
  }
}

// phase 3 for one row (sampling rows only): lp_pick_kernel, or the run-ahead
// advance kernels directly (no launch of its own)
__device__ TokOut lp_pick_row(int row, const RowCtl& c, const float* __restrict__ logits,
                              const float* __restrict__ flt, const LPPart* __restrict__ parts,
                              const LPRes* __restrict__ res, const LogitsConst& C) {
  const int V = C.n_vocab;
  const LPStats st = lp_combine(parts + row * LP_G, c.want_nosp);
  const LPRes* R = res + row * LP_G;
  float best = 0.0f, tbest = 0.0f;
  int best_i = 0x7fffffff, tbest_i = 0x7fffffff;
  double sum_ts = 0.0;
  for (int g = 0; g < LP_G; ++g) {
    better(best, best_i, R[g].best, R[g].best_i);
    better(tbest, tbest_i, R[g].tbest, R[g].tbest_i);
    sum_ts += R[g].sum_ts;
  }
  const int id = best > 0.0f ? best_i : 0;
  const float v = flt[(long)row * V + id];
  const float plog =
      (v == -INFINITY || (st.kill_text && id < C.beg)) ? -INFINITY : v - st.lse;
  TokOut t;
  t.tid = tbest > 0.0f ? tbest_i : 0;
  t.pt = (float)((double)tbest / (sum_ts + 1e-10));
  t.ptsum = (float)sum_ts;
  t.id = id;
  t.p = best;
  t.plog = plog;  // (host applies the id >= beg -> tid/pt override)
  t.nosp = c.want_nosp ? expf(logits[(long)row * V + C.nosp_id] - st.rlse) : 0.0f;
  t.pad = 0;
  return t;
}

__global__ __launch_bounds__(64) void lp_pick_kernel(const float* __restrict__ logits,
                                                     const float* __restrict__ flt,
                                                     const LPPart* __restrict__ parts,
                                                     const LPRes* __restrict__ res,
                                                     const RowCtl* __restrict__ ctl,
                                                     TokOut* __restrict__ out, LogitsConst C) {
  const int row = blockIdx.x;
  const RowCtl c = ctl[row];
  if (!c.active || !c.sample || threadIdx.x != 0) return;
  out[row] = lp_pick_row(row, c, logits, flt, parts, res, C);
}

void logits_process(float* logits, const float* static_mask, const RowCtl* ctl, TokOut* out,
                    float* probs, float* logprobs, const LogitsConst& C, int R, LPScratch ws,
                    hipStream_t st, bool pick) {
  const dim3 g(LP_G, R);
  lp_filter_kernel<<<g, LP_T, 0, st>>>(logits, static_mask, ctl, ws.flt, ws.parts, C);
  lp_probs_kernel<<<g, LP_T, 0, st>>>(ws.flt, ws.parts, ctl, ws.res, probs, logprobs, C);
  if (pick) lp_pick_kernel<<<R, 64, 0, st>>>(logits, ws.flt, ws.parts, ws.res, ctl, out, C);
}

// The token loop's per-row rules on the token a row generated this step
// (whisper.cpp v1.8.2 whisper_full_with_state, its decoder loop after
// sampling; host restatement driver.inc process_step, same order of tests).
__device__ __forceinline__ void token_rules(RowRun& w, int id, const RunConst& C) {
  const int i = w.ntok;
  w.penult_id = w.last_id;
  w.last_id = id;
  w.ntok = i + 1;
  bool stop = false;
  if (id > C.beg) {
    const int sd_new = 2 * (id - C.beg);
    if (w.has_ts && w.seek_delta > sd_new && w.result_len < i) {
      stop = true;  // (failed)
    } else {
      w.seek_delta = sd_new;
      w.result_len = i + 1;
      w.has_ts = 1;
    }
  }
  if (!stop) {
    if (id == C.eot || (C.max_tokens > 0 && i >= C.max_tokens) ||
        (w.has_ts && w.seek + w.seek_delta + C.delta_min >= w.seek_end))
      stop = true;
    else if (i == C.n_max - 1)
      stop = true;
  }
  if (stop) w.stopped = 1;
}

// The next step's inputs of a row (driver.inc fill_inputs).
__device__ __forceinline__ RowCtl next_inputs(const RowRun& w, const RunConst& C,
                                              const int* prompt_row, int& tok) {
  tok = w.fed < w.p_len ? prompt_row[w.fed] : (w.ntok > 0 ? w.last_id : 0);
  RowCtl n;
  n.active = w.stopped ? 0 : 1;
  n.sample = (!w.stopped && w.fed >= w.p_len - 1) ? 1 : 0;
  n.is_initial = w.ntok == 0 ? 1 : 0;
  n.last_ts = (w.ntok > 0 && w.last_id >= C.beg) ? 1 : 0;
  n.penult_ts = (w.ntok < 2 || w.penult_id >= C.beg) ? 1 : 0;
  n.has_ts = w.has_ts;
  n.seek_delta = w.seek_delta;
  n.want_probs = C.want_probs;
  n.temperature = C.temperature;
  n.want_nosp = (n.sample && n.is_initial) ? 1 : 0;
  n.pad[0] = n.pad[1] = 0;
  return n;
}

// Run-ahead greedy decoding and temperature sampling: applies the token rules
// to the step just run and writes the next step's inputs. One workgroup; every
// row is independent. The step's token records and the inputs chosen for the
// next step go straight to the pinned host ring slot `*run_step % nslot`.
// Sampling (B.draws set): a sampling row's token is its std::discrete_distribution
// draw of this step (sample_draws, earlier in the same graph); the next step's
// uniform is the row's next one in the host-filled ring, and the step's draws
// are reported for the host replay.
__global__ __launch_bounds__(256) void row_advance_kernel(RowRun* __restrict__ run,
                                                          int* __restrict__ run_step,
                                                          const int* __restrict__ prompt,
                                                          int* __restrict__ si,
                                                          RowCtl* __restrict__ ctl,
                                                          TokOut* __restrict__ out,
                                                          RunReport* __restrict__ rep, RunConst C,
                                                          BeamRun B, PickIn pk) {
  const int step = *run_step;
  const int R = C.R;
  const int sl = step % C.nslot;
  RunReport* slot = rep + (long)sl * R;
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    RowRun w = run[r];
    const RowCtl k = ctl[r];
    TokOut t = out[r];
    if (pk.parts && k.active && k.sample) {  // (the step's lp_pick, here)
      t = lp_pick_row(r, k, pk.logits, pk.flt, pk.parts, pk.res, pk.C);
      out[r] = t;
    }
    if (!w.stopped) {
      if (k.sample) token_rules(w, B.draws ? B.draws[(long)r * B.KD].id : t.id, C);
      if (!w.stopped) w.fed++;
    }
    int tok;
    const RowCtl n = next_inputs(w, C, prompt + (long)r * C.prompt_stride, tok);
    if (B.draws) {
      const int nd = (!w.stopped && n.sample) ? B.KD : 0;
      for (int d = 0; d < nd; ++d)
        B.du[(long)r * B.KD + d] = B.uring[(long)r * B.ring_n + (w.used + d) % B.ring_n];
      w.used += nd;
      B.dnd[r] = nd;
      for (int d = 0; d < B.KD; ++d)
        B.drep[((long)sl * R + r) * B.KD + d] = B.draws[(long)r * B.KD + d];
    }
    si[r] = tok;
    si[R + r] = w.fed;
    si[2 * R + r] = n.active;
    ctl[r] = n;
    run[r] = w;
    RunReport o;
    o.out = t;
    o.tok = tok;
    o.pos = w.fed;
    o.act = n.active;
    o.pad = 0;
    o.next = n;
    slot[r] = o;
  }
  __syncthreads();
  if (threadIdx.x == 0) *run_step = step + 1;
}

// Run-ahead beam search, one workgroup per clip (its n decoders are rows
// r0 .. r0+n-1, stepping in lockstep). The beam step of driver.inc beam_step
// (whisper.cpp v1.8.2 WHISPER_SAMPLING_BEAM_SEARCH):
//  * candidates: beam_size draws per live decoder, sum = decoder's
//    sum_logprobs_all + plog;
//  * ranking: by sum (desc), then decoder, then draw index — each candidate's
//    rank counted in parallel against all others (a total order: the same
//    permutation std::stable_sort gives the host);
//  * hand-over: decoders in order take candidates in rank order, skipping the
//    run of candidates equal to the one just taken (from the second token on).
//    Equal token sequences are tracked as classes (cls): two candidates are
//    equal iff their parents' classes and their tokens are equal, and a
//    decoder's new class is the first decoder holding an equal sequence;
//  * a decoder taking another decoder's candidate takes its state and its KV
//    position map (the parent's maps as they were before the step).
// Then the token rules and the next step's inputs as row_advance_kernel, and
// the next step's uniforms copied from the host-filled ring.
constexpr int BA_T = 256;
constexpr int BA_MAXN = 16;
__global__ __launch_bounds__(BA_T) void beam_advance_kernel(RowRun* __restrict__ run,
                                                            int* __restrict__ run_step,
                                                            const int* __restrict__ prompt,
                                                            int* __restrict__ si,
                                                            RowCtl* __restrict__ ctl,
                                                            TokOut* __restrict__ out,
                                                            RunReport* __restrict__ rep, RunConst C,
                                                            BeamRun B, PickIn pk) {
  extern __shared__ int smap[];  // [n][Tctx]: maps of the decoders others take over
  __shared__ RowRun sw[BA_MAXN];
  __shared__ RowCtl s_ctl[BA_MAXN];  // this step's controls (ctl is rewritten below)
  __shared__ int s_smp[BA_MAXN], s_src[BA_MAXN], s_tok[BA_MAXN], s_need[BA_MAXN],
      s_own[BA_MAXN];
  __shared__ double s_csum[BA_MAXN];
  __shared__ double c_sum[BA_MAXN * 16];
  __shared__ int c_id[BA_MAXN * 16], c_ord[BA_MAXN * 16], c_eq[BA_MAXN * 16];
  const int n = B.n, KD = B.KD, tid = threadIdx.x;
  const int r0 = blockIdx.x * n, R = C.R;
  const int step = run_step[blockIdx.x];
  if (tid < n) {
    sw[tid] = run[r0 + tid];
    s_ctl[tid] = ctl[r0 + tid];
    s_smp[tid] = s_ctl[tid].sample;
    s_src[tid] = tid;
    s_need[tid] = 0;
  }
  __syncthreads();
  int live = -1, nlive = 0;
  for (int j = 0; j < n; ++j) {
    if (sw[j].stopped) continue;
    ++nlive;
    if (live < 0 && s_smp[j]) live = j;
  }
  if (live >= 0) {
    const int nc = n * KD;
    for (int c = tid; c < nc; c += BA_T) {
      const Draw dr = B.draws[(long)(r0 + c / KD) * KD + c % KD];
      c_sum[c] = sw[c / KD].sum + (double)dr.plog;
      c_id[c] = dr.id;
    }
    __syncthreads();
    for (int c = tid; c < nc; c += BA_T) {
      if (sw[c / KD].stopped) continue;
      const double s = c_sum[c];
      int rank = 0;
      for (int u = 0; u < nc; ++u) {
        if (sw[u / KD].stopped) continue;
        const double t = c_sum[u];
        rank += (t > s || (t == s && u < c)) ? 1 : 0;
      }
      c_ord[rank] = c;
    }
    __syncthreads();
    const int ncand = nlive * KD;
    for (int p = tid; p < ncand; p += BA_T) {
      int eq = 0;
      if (p > 0) {
        const int a = c_ord[p], b = c_ord[p - 1];
        eq = (c_id[a] == c_id[b] && sw[a / KD].cls == sw[b / KD].cls) ? 1 : 0;
      }
      c_eq[p] = eq;
    }
    __syncthreads();
    if (tid == 0) {
      const int i_step = sw[live].ntok;
      int cur = 0;
      for (int j = 0; j < n; ++j) {
        if (sw[j].stopped) continue;
        if (cur >= ncand) cur = 0;
        const int c = c_ord[cur++];
        while (cur < ncand && c_eq[cur] && i_step > 0) ++cur;
        s_src[j] = c / KD;
        s_tok[j] = c_id[c];
        s_csum[j] = c_sum[c];
        if (c / KD != j) s_need[c / KD] = 1;
      }
    }
    __syncthreads();
  }
  // the decoders' new states (from their parents' pre-step states)
  RowRun w;
  if (tid < n) {
    w = sw[tid];
    if (!w.stopped) {
      if (live >= 0) {
        const RowRun& p = sw[s_src[tid]];
        int cls = tid;  // the first decoder holding an equal sequence
        for (int j = 0; j < tid; ++j)
          if (!sw[j].stopped && sw[s_src[j]].cls == p.cls && s_tok[j] == s_tok[tid]) {
            cls = j;
            break;
          }
        w.ntok = p.ntok;
        w.last_id = p.last_id;
        w.penult_id = p.penult_id;
        w.has_ts = p.has_ts;
        w.seek_delta = p.seek_delta;
        w.result_len = p.result_len;
        w.cls = cls;
        w.sum = s_csum[tid];
        token_rules(w, s_tok[tid], C);
      }
      // (w.fed: the positions 0..fed of this window hold KV after this step)
    }
  }
  // KV position maps: snapshot the taken-over decoders' maps, then rewrite
  // the takers' (kvmap[dst][0..npos) = where src reads them, kvown = npos)
  const int npos = live >= 0 ? sw[live].fed + 1 : 0;
  if (live >= 0) {
    if (tid < n && s_need[tid]) s_own[tid] = B.kvown[r0 + tid];
    __syncthreads();
    for (int j = 0; j < n; ++j) {
      if (!s_need[j]) continue;
      const int lim = min(s_own[j], npos);
      for (int p = tid; p < lim; p += BA_T) smap[j * B.Tctx + p] = B.kvmap[(long)(r0 + j) * B.Tctx + p];
    }
    __syncthreads();
    for (int j = 0; j < n; ++j) {
      const int src = s_src[j];
      if (src == j || sw[j].stopped) continue;
      int* dm = B.kvmap + (long)(r0 + j) * B.Tctx;
      for (int p = tid; p < npos; p += BA_T) dm[p] = p < s_own[src] ? smap[src * B.Tctx + p] : r0 + src;
      if (tid == 0) B.kvown[r0 + j] = npos;
    }
  }
  if (tid < n) {
    const int r = r0 + tid;
    if (!w.stopped) w.fed++;
    int tok;
    const RowCtl nx = next_inputs(w, C, prompt + (long)r * C.prompt_stride, tok);
    const int nd = (!w.stopped && nx.sample) ? KD : 0;
    for (int k = 0; k < nd; ++k) B.du[(long)r * KD + k] = B.uring[(long)r * B.ring_n + (w.used + k) % B.ring_n];
    w.used += nd;
    B.dnd[r] = nd;
    si[r] = tok;
    si[R + r] = w.fed;
    si[2 * R + r] = nx.active;
    ctl[r] = nx;
    run[r] = w;
    const int sl = step % C.nslot;
    RunReport o;
    const RowCtl k0 = s_ctl[tid];
    if (pk.parts && k0.active && k0.sample) {  // (the step's lp_pick, here)
      o.out = lp_pick_row(r, k0, pk.logits, pk.flt, pk.parts, pk.res, pk.C);
      out[r] = o.out;
    } else {
      o.out = out[r];
    }
    o.tok = tok;
    o.pos = w.fed;
    o.act = nx.active;
    o.pad = 0;
    o.next = nx;
    rep[(long)sl * R + r] = o;
    BeamReport b;
    b.src = r0 + s_src[tid];
    b.nd = nd;
    b.pad[0] = b.pad[1] = 0;
    B.brep[(long)sl * R + r] = b;
    for (int k = 0; k < KD; ++k)
      B.drep[((long)sl * R + r) * KD + k] = B.draws[(long)r * KD + k];
    if (tid == 0) run_step[blockIdx.x] = step + 1;
  }
}

// Event-bracket calibration (bench.py roofline): an empty kernel launched
// between two timing events in the instrumented decode-step graph, so the
// event nodes' own cost can be measured and removed from the kernel brackets.
__global__ __launch_bounds__(64) void perf_empty_kernel() {}
void launch_perf_empty(hipStream_t st) { perf_empty_kernel<<<1, 64, 0, st>>>(); }

void row_advance(RowRun* run, int* run_step, const int* prompt, int* stepin, RowCtl* ctl,
                 TokOut* out, RunReport* rep, const RunConst& C, const BeamRun& B,
                 const PickIn& pk, hipStream_t st) {
  row_advance_kernel<<<1, 256, 0, st>>>(run, run_step, prompt, stepin, ctl, out, rep, C, B, pk);
}

void beam_advance(RowRun* run, int* run_step, const int* prompt, int* stepin, RowCtl* ctl,
                  TokOut* out, RunReport* rep, const RunConst& C, const BeamRun& B,
                  const PickIn& pk, hipStream_t st) {
  const size_t lds = (size_t)B.n * B.Tctx * 4;
  beam_advance_kernel<<<C.R / B.n, BA_T, lds, st>>>(run, run_step, prompt, stepin, ctl, out, rep,
                                                   C, B, pk);
}


// ---------------------------------------------------------------------------
// std::discrete_distribution draws on the device (whisper_sample_token with
// temperature > 0 and whisper_sample_token_topk: `std::discrete_distribution<>
// dist(probs.begin(), probs.end()); id = dist(rng)`), bit-exact to libstdc++:
//   param:  sum = accumulate(double(p_i)) (sequential), q_i = p_i / sum,
//           cp = partial_sum(q) (sequential), cp[V-1] = 1.0;
//   draw:   u = generate_canonical<double, 53>(rng), id = lower_bound(cp, u).
// The u of every draw are produced on the host from the row's std::mt19937
// (the RNG stream stays on the host, consumed in the same order). The two
// running sums are inherently sequential (their rounding is the result), so
// one lane performs the adds while the wave stages each chunk through LDS
// (converted / divided in parallel) and searches the chunk's cumulative
// values in parallel for the threshold crossings.
// ---------------------------------------------------------------------------
constexpr int DR_CH = 1024;  // elements per staged chunk

// s = (((s + q[0]) + q[1]) + ...) in index order (one lane); the LDS reads are
// issued 16 elements ahead of the dependent adds. cp (optional) receives
// every running value.
__device__ __forceinline__ double seq_sum(const double* q, int n, double s, double* cp) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* q2 = reinterpret_cast<const d2*>(q);
  d2* c2 = reinterpret_cast<d2*>(cp);
  int j = 0;
  for (; j + 16 <= n; j += 16) {
    d2 a[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) a[t] = q2[(j >> 1) + t];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const double s0 = s + a[t].x;
      s = s0 + a[t].y;
      if (cp) c2[(j >> 1) + t] = d2{s0, s};
    }
  }
  for (; j < n; ++j) {
    s += q[j];
    if (cp) cp[j] = s;
  }
  return s;
}

__global__ __launch_bounds__(64) void sample_draws_exact_kernel(const float* __restrict__ probs,
                                                                const float* __restrict__ logprobs,
                                                                int V, const double* __restrict__ u,
                                                                const int* __restrict__ ndraw, int KD,
                                                                Draw* __restrict__ out,
                                                                const int* __restrict__ need) {
  __shared__ double q[DR_CH];
  __shared__ double cp[DR_CH];
  const int row = blockIdx.x, lane = threadIdx.x;
  const int nd = ndraw[row];
  if (nd <= 0 || (need && !need[row])) return;
  const float* P = probs + (long)row * V;
  constexpr int PL = DR_CH / 64;  // elements per lane per chunk
  // pass 1: sum in index order
  double sum = 0.0;
  float nx[PL];
  auto load = [&](int c0) {
#pragma unroll
    for (int t = 0; t < PL; ++t) {
      const int i = c0 + t * 64 + lane;
      nx[t] = i < V ? P[i] : 0.0f;
    }
  };
  load(0);
  for (int c0 = 0; c0 < V; c0 += DR_CH) {
#pragma unroll
    for (int t = 0; t < PL; ++t) q[t * 64 + lane] = (double)nx[t];
    __syncthreads();
    if (c0 + DR_CH < V) load(c0 + DR_CH);  // in flight during the sequential adds
    if (lane == 0) sum = seq_sum(q, min(DR_CH, V - c0), sum, nullptr);
    __syncthreads();
  }
  sum = __shfl(sum, 0, 64);
  // pass 2: cumulative of p_i / sum; each draw takes the first index whose
  // cumulative value is >= u (cp[V-1] is 1.0, so a draw not taken earlier
  // takes V-1)
  double ud[16];
  int id[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    ud[d] = d < nd ? u[(long)row * KD + d] : 2.0;
    id[d] = d < nd ? -1 : 0;
  }
  double run = 0.0;
  load(0);
  for (int c0 = 0; c0 < V; c0 += DR_CH) {
#pragma unroll
    for (int t = 0; t < PL; ++t) q[t * 64 + lane] = (double)nx[t] / sum;
    __syncthreads();
    if (c0 + DR_CH < V) load(c0 + DR_CH);
    const int n = min(DR_CH, V - c0);
    if (lane == 0) {
      run = seq_sum(q, n, run, cp);
      if (c0 + n == V) cp[n - 1] = 1.0;
    }
    __syncthreads();
    // lane owns the contiguous slots [lane*PL, lane*PL + PL)
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      if (d >= nd) break;
      if (__shfl(id[d], 0, 64) >= 0) continue;  // taken in an earlier chunk
      int first = 0x7fffffff;
      for (int t = 0; t < PL; ++t) {
        const int j = lane * PL + t;
        if (j < n && cp[j] >= ud[d]) {
          first = j;
          break;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
      if (first != 0x7fffffff) id[d] = c0 + first;
    }
    run = __shfl(run, 0, 64);
    __syncthreads();
  }
  if (lane < nd) {
    int my = 0;
#pragma unroll
    for (int d = 0; d < 16; ++d)
      if (d == lane) my = id[d];
    Draw r;
    r.id = my;
    r.p = P[my];
    r.plog = logprobs[(long)row * V + my];
    r.pad = 0;
    out[(long)row * KD + lane] = r;
  }
}

// Fast path: the same draws from a parallel evaluation. S = sum p_i (any
// order), q_i = p_i * (1 / S); each of the 16 waves owns a contiguous 1/16 of the row
// and walks it in tiles of 512 (8 consecutive elements per lane, coalesced
// loads), cumulative values = wave base + lane scan + in-lane order.
// Sequential rounding (the exact kernel) and this evaluation differ by at most
// ~1e-11 in any cumulative value (V * 2^-53 for the running sums, plus the
// relative difference of the two S through q), so when u lies more than
// DR_MARGIN from the cumulative values on both sides of the crossing the
// exact kernel would pick the same index. Rows with a draw inside the margin
// — or not claimed by exactly one element, as rounding can leave a gap or an
// overlap at lane / tile / wave boundaries — are flagged and redone by
// sample_draws_exact_kernel.
constexpr double DR_MARGIN = 2e-10;
constexpr int DR_T = 1024;  // 16 waves per row: each walks ~1/16 of the vocabulary

__device__ __forceinline__ double wave_incl_scan_d(double x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  return x;
}

__global__ __launch_bounds__(DR_T) void sample_draws_kernel(const float* __restrict__ probs,
                                                            const float* __restrict__ logprobs,
                                                            int V, const double* __restrict__ u,
                                                            const int* __restrict__ ndraw, int KD,
                                                            Draw* __restrict__ out,
                                                            int* __restrict__ need) {
  __shared__ double red[DR_T / 64];
  __shared__ int ids[16];
  __shared__ int claims[16];
  __shared__ int bad;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nd = ndraw[row];
  if (nd <= 0) return;
  const float* P = probs + (long)row * V;
  if (tid < 16) {
    ids[tid] = -1;
    claims[tid] = 0;
  }
  if (tid == 0) bad = 0;
  // wave regions: contiguous, multiples of 8 elements (V is even: 8-byte loads)
  constexpr int NW = DR_T / 64;
  const int RW = ((V + NW - 1) / NW + 7) & ~7;
  const int r0 = min(V, wid * RW), r1 = min(V, r0 + RW);
  auto ld2 = [&](int i) {
    return i + 1 < r1 ? *reinterpret_cast<const float2*>(P + i)
                      : make_float2(i < r1 ? P[i] : 0.0f, 0.0f);
  };
  double s = 0.0;
  for (int i0 = r0 + 2 * lane; i0 < r1; i0 += 8 * 128) {
    float2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld2(i0 + k * 128);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += (double)v[k].x + (double)v[k].y;
  }
  s = wave_sum_d(s);
  if (lane == 0) red[wid] = s;
  __syncthreads();
  double S = 0.0;
  for (int w = 0; w < NW; ++w) S += red[w];
  const double iS = 1.0 / S;
  double carry = 0.0;
  for (int w = 0; w < wid; ++w) carry += red[w] * iS;
  double ud[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) ud[d] = d < nd ? u[(long)row * KD + d] : 2.0;
  // tiles double-buffered: the next tile's loads are in flight during the
  // scan of this one
  float2 nx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) nx[k] = ld2(r0 + 8 * lane + 2 * k);
  for (int t0 = r0; t0 < r1; t0 += 512) {
    const int e0 = t0 + 8 * lane;
    float v[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = nx[k].x;
      v[2 * k + 1] = nx[k].y;
    }
    if (t0 + 512 < r1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) nx[k] = ld2(e0 + 512 + 2 * k);
    }
    double loc = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) loc += (double)v[k] * iS;
    const double inc = wave_incl_scan_d(loc, lane);
    const double before = carry + (inc - loc), after = carry + inc;
    const double total = __shfl(inc, 63, 64);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      if (d >= nd) break;
      // a draw crosses this tile only if carry < u <= carry + total (+ margin)
      if (!(ud[d] > carry - DR_MARGIN) || ud[d] > carry + total + DR_MARGIN) continue;
      if (!(ud[d] > before && ud[d] <= after) && !(e0 + 8 > V - 1 && e0 <= V - 1 && ud[d] > before))
        continue;
      double prev = before, c = before;
      for (int k = 0; k < 8; ++k) {
        const int i = e0 + k;
        if (i >= r1) break;
        c = i == V - 1 ? 1.0 : c + (double)v[k] * iS;  // cp[V-1] = 1.0
        if (c >= ud[d]) {
          ids[d] = i;
          atomicAdd(&claims[d], 1);
          if (!(ud[d] - prev > DR_MARGIN && c - ud[d] > DR_MARGIN)) bad = 1;
          break;
        }
        prev = c;
      }
    }
    carry += total;
  }
  __syncthreads();
  if (tid < nd) {
    const int id = ids[tid];
    Draw r;
    r.id = id < 0 ? V - 1 : id;
    r.p = P[r.id];
    r.plog = logprobs[(long)row * V + r.id];
    r.pad = 0;
    out[(long)row * KD + tid] = r;
    if (id < 0 || claims[tid] != 1) bad = 1;  // unclaimed / doubly claimed -> exact path
  }
  __syncthreads();
  if (tid == 0) need[row] = bad;
}

void sample_draws(const float* probs, const float* logprobs, int V, const double* u,
                  const int* ndraw, int KD, Draw* out, int* need, int R, hipStream_t st,
                  int force_exact) {
  static const bool env_exact = getenv("MWX_DRAW_EXACT") != nullptr;
  const bool exact_only = force_exact < 0 ? env_exact : force_exact != 0;
  if (!exact_only)
    sample_draws_kernel<<<R, DR_T, 0, st>>>(probs, logprobs, V, u, ndraw, KD, out, need);
  sample_draws_exact_kernel<<<R, 64, 0, st>>>(probs, logprobs, V, u, ndraw, KD, out,
                                              exact_only ? nullptr : need);
}

}  // namespace mwx
