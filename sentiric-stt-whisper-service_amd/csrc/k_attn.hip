// Attention kernels for gfx950.
//
// enc_attn_kernel: encoder self-attention (whisper_build_graph_encoder,
//   softmax(Q K^T / 8) V over 1500 frames). Flash-style: one workgroup = 4
//   waves x 32 queries of one (clip, head); K and V^T tiles of 64 keys are
//   register-prefetched and staged through double-buffered LDS (K rows XOR-
//   swizzled, V^T rows padded to 144 B: conflict-free ds_read_b128 / _b64).
//   S^T = K Q^T is computed with the key on the MFMA row, so every lane owns
//   one query column: row max / row sum need two cross-lane shuffles, and the
//   f16 P^T registers are directly the B operand of O^T = V^T P^T.
//   Numerics: Q, K, V, P in f16 (ggml itype), f32 accumulation and softmax.
//
// dec_attn_kernel: one query per (row, head) against its KV rows — the
//   decoder self-attention over the KV cache and the cross-attention over the
//   1500 encoder frames (whisper_build_graph_decoder). Follows ggml's
//   non-flash path exactly: f32 scores of f16 q.k, scale, max, exp, double
//   sum, multiply by (float)(1/sum), round P to f16, then P.V in f32. K and V
//   rows are streamed with 8 lanes per 128-B row (fully coalesced).
#include <cstdlib>
#include <type_traits>

#include <atomic>

#include "kcommon.h"
#include "kernels.h"

namespace mwx {

constexpr int VSTR = 72;  // padded V^T tile row (elements)

template <typename T, int QW = 4>
__global__ __launch_bounds__(64 * QW) void enc_attn_kernel(const _Float16* __restrict__ q,
                                                       const _Float16* __restrict__ k,
                                                       const _Float16* __restrict__ vt, T* __restrict__ o,
                                                       int H, int L, int Lp, float scale_log2,
                                                       int nqb) {
  __shared__ __attribute__((aligned(16))) _Float16 ks[2][64 * 64];
  __shared__ __attribute__((aligned(16))) _Float16 vs[2][64 * VSTR];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  // 1-D grid, XCD-aware order: workgroups are placed round-robin over the 8
  // XCDs (id % 8); each XCD gets a contiguous range of (clip, head, query
  // block) ids, so the nqb query blocks of a (clip, head) run on one XCD and
  // its K / V^T (384 KB at large-v3) are fetched from HBM into that XCD's L2
  // once instead of once per XCD
  int wgid = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = wgid % 8, qq = nwg / 8, rr = nwg % 8;
    wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + wgid / 8;
  }
  const int bh = wgid / nqb;
  const int b = bh / H, h = bh - b * H;
  const int q0 = (wgid - bh * nqb) * (32 * QW) + wid * 32;
  const _Float16* Q = q + (long)bh * L * 64;
  const _Float16* Kh = k + (long)bh * L * 64;
  const _Float16* VT = vt + (long)bh * 64 * Lp;

  f16x8 qf[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int qr = min(q0 + u * 16 + c16, L - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
      qf[u][s] = *reinterpret_cast<const f16x8*>(Q + (long)qr * 64 + s * 32 + g * 8);
  }
  f32x4 oacc[4][2];
#pragma unroll
  for (int te = 0; te < 4; ++te)
#pragma unroll
    for (int u = 0; u < 2; ++u) oacc[te][u] = f32x4{0, 0, 0, 0};
  float mrow[2] = {-INFINITY, -INFINITY}, lrow[2] = {0.0f, 0.0f};

  // staging: thread t moves 16-B chunk (row = t/8 + (8 QW) i, ch = t%8) of the
  // K tile (64 keys x 64 dims) and of the V^T tile (64 dims x 64 keys); NP
  // passes of 8 QW rows
  constexpr int NP = 64 / (8 * QW), RS = 8 * QW;
  const int srow = tid >> 3, sch = tid & 7;
  const int kso0 = srow * 64 + ((sch ^ (srow & 7)) << 3);  // (row+RS)&7 == row&7
  const int vso0 = srow * VSTR + sch * 8;
#define GLOAD(kb)                                                                    \
  do {                                                                               \
    const int key0 = (kb) * 64 + sch * 8;                                            \
    _Pragma("unroll") for (int p_ = 0; p_ < NP; ++p_) {                              \
      const int kr = min((kb) * 64 + srow + RS * p_, L - 1);                         \
      rk[p_] = *reinterpret_cast<const uint4*>(Kh + (long)kr * 64 + sch * 8);        \
      rv[p_] = key0 < Lp ? *reinterpret_cast<const uint4*>(VT + (long)(srow + RS * p_) * Lp + key0) \
                         : uint4{0, 0, 0, 0};                                        \
    }                                                                                \
  } while (0)
#define SSTORE(buf)                                                          \
  do {                                                                       \
    _Pragma("unroll") for (int p_ = 0; p_ < NP; ++p_) {                      \
      *reinterpret_cast<uint4*>(&ks[buf][kso0 + RS * p_ * 64]) = rk[p_];     \
      *reinterpret_cast<uint4*>(&vs[buf][vso0 + RS * p_ * VSTR]) = rv[p_];   \
    }                                                                        \
  } while (0)

  const int nkb = (L + 63) / 64;
  {
    uint4 rk[NP], rv[NP];
    GLOAD(0);
    SSTORE(0);
  }
  __syncthreads();
  // one 64-key tile; MASKED: the last tile of a length that is not a multiple
  // of 64 (keys >= L get -inf); the full tiles run without the key test
  auto tile = [&](const int kb, auto masked) {
    constexpr bool MASKED = decltype(masked)::value;
    const int cur = kb & 1;
    uint4 rk[NP], rv[NP];  // tile kb+1 in flight (global -> registers -> LDS)
    if (kb + 1 < nkb) GLOAD(kb + 1);
    // S^T = K Q^T : sacc[t][u] rows = keys 16t + 4g + r, col = query c16
    f32x4 sacc[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int row = t * 16 + c16;
      f16x8 kf[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = s * 4 + g;
        kf[s] = *reinterpret_cast<const f16x8*>(&ks[cur][row * 64 + ((ch ^ (row & 7)) << 3)]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x4 a = f32x4{0, 0, 0, 0};
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[0], qf[u][0], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[1], qf[u][1], a, 0, 0, 0);
        sacc[t][u] = a;
      }
    }
    // mask keys beyond L
    if constexpr (MASKED) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * 64 + t * 16 + g * 4 + r;
          if (key >= L) {
            sacc[t][0][r] = -INFINITY;
            sacc[t][1][r] = -INFINITY;
          }
        }
    }
    // online softmax per query column
    f16x8 pf[2][2];  // [u][k-step]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sacc[t][u][r]);
      mx = max_xor16(mx);
      mx = max_xor32(mx);
      const float mnew = fmaxf(mrow[u], mx * scale_log2);
      // v_exp_f32 directly (exponents here are <= 0; the libm wrapper only
      // adds the denormal-range rescale, for results far below f16 resolution)
      const float alpha = __builtin_amdgcn_exp2f(mrow[u] - mnew);
      float ps[4][4];
      float rs = 0.0f;
      // s * scale - m rounded twice as before (packed: v_pk_mul_f32 +
      // v_pk_add_f32 on element pairs), then the sum in the same order
      // (a packed FMA and packed partial sums cut 81 VALU instructions and
      // 5 % of the kernel, 637.7 -> 605.8 us per layer, but moved the
      // full-depth greedy window off the oracle at a near-tie step (2 of
      // 220, within its 2 x err bound; r06f): not kept)
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      const f32x2 sc2 = f32x2{scale_log2, scale_log2}, mn2 = f32x2{-mnew, -mnew};
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 sv = f32x2{sacc[t][u][r], sacc[t][u][r + 1]};
          const f32x2 xv = sv * sc2 + mn2;
          ps[t][r] = __builtin_amdgcn_exp2f(xv[0]);
          ps[t][r + 1] = __builtin_amdgcn_exp2f(xv[1]);
          rs += ps[t][r];
          rs += ps[t][r + 1];
        }
      rs = add_xor16(rs);
      rs = add_xor32(rs);
      lrow[u] = lrow[u] * alpha + rs;
      mrow[u] = mnew;
      // (skipping this rescale when no query's running max moved -- alpha = 1
      // is exact -- measured slower: 685 vs 638 us per layer, r06g)
#pragma unroll
      for (int te = 0; te < 4; ++te) oacc[te][u] *= alpha;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f16x8 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = (_Float16)ps[2 * s2][r];
          v[4 + r] = (_Float16)ps[2 * s2 + 1][r];
        }
        pf[u][s2] = v;
      }
    }
    // O^T += V^T P^T
#pragma unroll
    for (int te = 0; te < 4; ++te) {
      const int e = te * 16 + c16;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const _Float16* vp = &vs[cur][e * VSTR + s2 * 32 + g * 4];
        const f16x4 lo = *reinterpret_cast<const f16x4*>(vp);
        const f16x4 hi = *reinterpret_cast<const f16x4*>(vp + 16);
        const f16x8 vf = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int u = 0; u < 2; ++u)
          oacc[te][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[u][s2], oacc[te][u], 0, 0, 0);
      }
    }
    if (kb + 1 < nkb) SSTORE(cur ^ 1);
    __syncthreads();
  };
  for (int kb = 0; kb < nkb - 1; ++kb) tile(kb, std::false_type{});
  if (L % 64)
    tile(nkb - 1, std::true_type{});
  else
    tile(nkb - 1, std::false_type{});
#undef GLOAD
#undef SSTORE
  const int D = H * 64;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int qi = q0 + u * 16 + c16;
    if (qi >= L) continue;
    const float inv = 1.0f / lrow[u];
    T* dst = o + ((long)b * L + qi) * D + h * 64;
#pragma unroll
    for (int te = 0; te < 4; ++te)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[te * 16 + g * 4 + r] = to_t<T>(oacc[te][u][r] * inv);
  }
}

template <typename T>
void enc_attention(const _Float16* q, const _Float16* k, const _Float16* vt, T* o, int B, int H,
                   int L, float scale, hipStream_t st) {
  const int Lp = (L + 7) & ~7;
  // (8 waves = 256 queries per workgroup, each K / V tile staged once for
  // twice the queries: measured slower, 704 vs 624 us per large-v3 layer,
  // profiles/r04_ab_regression_beam.md)
  const int nqb = (L + 127) / 128;
  enc_attn_kernel<T, 4><<<nqb * B * H, 256, 0, st>>>(q, k, vt, o, H, L, Lp,
                                                    scale * 1.4426950408889634f, nqb);
}

// ---------------------------------------------------------------------------
// decode attention
// ---------------------------------------------------------------------------
constexpr int DEC_MAX_KEYS = 1536;

__device__ __forceinline__ float block_max_256(float v, float* red) {
  v = wave_max_dpp(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ double block_sum_256d(double v, double* red) {
  v = wave_sum_d_dpp(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
// q.k over 8 f16 elements with v_dot2_f32_f16 (q, k exact f16 values; f32
// accumulation, pairs in index order): 4 instructions instead of 8 multiplies
// and 8 adds. Used by every decode attention kernel, so all of them score a
// row identically.
__device__ __forceinline__ float dot8(const h2* q, f16x8 k) {
  float d = __builtin_amdgcn_fdot2(q[0], __builtin_shufflevector(k, k, 0, 1), 0.0f, false);
  d = __builtin_amdgcn_fdot2(q[1], __builtin_shufflevector(k, k, 2, 3), d, false);
  d = __builtin_amdgcn_fdot2(q[2], __builtin_shufflevector(k, k, 4, 5), d, false);
  d = __builtin_amdgcn_fdot2(q[3], __builtin_shufflevector(k, k, 6, 7), d, false);
  return d;
}

// sum over the 8 lanes of an aligned lane group (DPP: xor 1, xor 2 within a
// quad, then the mirrored quad); every lane of the group gets the same value.
// update_dpp with bound_ctrl (all sources valid: the same values as mov_dpp)
// lets each step compile to one v_add_f32_dpp instead of a v_mov_b32_dpp and
// a v_add_f32
__device__ __forceinline__ float dpp_sum8(float d) {
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0xB1, 0xF, 0xF, true));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x4E, 0xF, 0xF, true));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x141, 0xF, 0xF, true));
  return d;
}

// One workgroup per (row, head). Key/value rows are streamed in batches: 8
// rows per 8-lane group (each lane 16 B of a 128-B row), 64 rows per wave,
// 256 per workgroup, double-buffered so batch b+1 is in flight while batch b
// is consumed. All loads are unconditional (indices clamped to the last key)
// so the compiler can keep exactly one batch outstanding across the loop.
// SELF: the row appended by this launch is formed here from the QKV slabs,
// written to the cache and taken from LDS (its cache line may be stale in L1).
// The loop body is straight-line (two batches per trip, no early exit), so the
// compiler keeps exactly one batch in flight with counted vmcnt waits.
template <typename T, bool SELF, int UBX = 8, bool NTL = !SELF, int NBC = 0>
__global__ __launch_bounds__(256) void dec_attn_kernel(
    const float* __restrict__ P, int KS, int pcols, const float* __restrict__ bias, float qscale,
    float kscale, _Float16* __restrict__ kbase, _Float16* __restrict__ vbase,
    const int* __restrict__ kv_index, const int* __restrict__ pos, const int* __restrict__ active,
    int fixed_len, int cap, T* __restrict__ o, int H, float scale,
    const int* __restrict__ kvmap, const int* __restrict__ own_from, int map_row0, int nq,
    int R, int write_new = 1, unsigned long long* span = nullptr) {
  __shared__ float sc[DEC_MAX_KEYS];
  __shared__ float redf[4];
  __shared__ double redd[4];
  __shared__ float pv[4][64][9];
  __shared__ float sq[64], snk[64], snv[64];
  span_start(span);
  int row = blockIdx.y, h = blockIdx.x;
  if (nq > 1) {
    // nq rows per clip (beam / best-of decoders: cross, the same K/V; self,
    // histories taken over from each other): 1-D grid where the nq
    // workgroups of one (clip, head) are dispatched within a window of 8*nq
    // ids with equal id % 8 -- one XCD under the round-robin placement, so
    // the rows they share are read from HBM about once and served to the
    // others from that XCD's L2
    const int L = blockIdx.x, W = 8 * nq;
    const int q = (L % W) / 8, g = (L / W) * 8 + L % 8;
    if (g >= (R / nq) * H) {
      span_end(span);
      return;
    }
    row = (g / H) * nq + q;
    h = g % H;
  }
  // the row's control words are fetched together (one round trip), then the
  // inactive-row exit
  const int act_r = active[row];
  const int p_row = SELF ? pos[row] : 0;
  const int slot = kv_index ? kv_index[row] : row;
  const int own0 = SELF && own_from ? own_from[row] : 0;
  // self: the position-map words of this lane's batch-0 rows are requested
  // with the control words, not after them (indices unclamped: a row past the
  // end is never read for its value, and only rows below own_from, all below
  // the new position, use their map word), so the batch-0 K / V addresses
  // wait for one memory round trip instead of two
  int mraw[SELF ? UBX : 1];
  if constexpr (SELF) {
    const int* mr = kvmap ? kvmap + (long)row * cap : nullptr;
    const int kgl = (threadIdx.x & 63) >> 3, wdl = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < UBX; ++u) mraw[u] = mr ? mr[min(wdl * (8 * UBX) + u * 8 + kgl, cap - 1)] : 0;
  }
  asm volatile("" ::"s"(act_r), "s"(p_row), "s"(slot), "s"(own0));
  if (!act_r) {
    span_end(span);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = lane >> 3, c = lane & 7;
  const int n = SELF ? p_row + 1 : fixed_len;
  const int jnew = SELF ? p_row : -1;
  const int D = H * 64;
  _Float16* K = kbase + (((long)slot * H + h) * cap) * 64;
  _Float16* V = vbase + (((long)slot * H + h) * cap) * 64;
  // self (beam search): positions below own_from[row] were taken over from
  // other rows' histories; kvmap[row][j] names the row (numbered from
  // -map_row0 relative to kbase) whose cache holds position j (histories are
  // never overwritten, so no KV is copied)
  const int* mrow = SELF && kvmap ? kvmap + (long)row * cap : nullptr;
  const long rstride = (long)H * cap * 64;
  // rows per 8-lane group per batch (cross: UBX, tunable), BR rows per batch
  constexpr int UB = UBX, BR = 32 * UB;
  // NBC > 0 (cross over the 1500 encoder frames): the batch count is a
  // compile-time constant, so the K / V stream below is fully unrolled
  const int nb = NBC > 0 ? NBC : (n + BR - 1) / BR;
  // rows past the end are clamped to the last OLD row (self: the new row is
  // being written by this workgroup and is taken from LDS instead)
  const int jmax = SELF ? max(n - 2, 0) : n - 1;
  const bool wave_busy = wid * (8 * UB) < n;  // self: waves past the last row idle (n <= 32 UB)
  f16x8 ka[UB], kb2[UB];
#define LOADROWS(buf, base, bidx)                                                  \
  _Pragma("unroll") for (int u = 0; u < UB; ++u) {                               \
    const int j = min((bidx) * BR + wid * (8 * UB) + u * 8 + kg, jmax);          \
    const _Float16* src = base + (long)j * 64 + c * 8;                            \
    if (SELF && j < own0)                                                         \
      src += ((long)mrow[j] - map_row0 - slot) * rstride;                         \
    buf[u] = ld_stream<NTL>(reinterpret_cast<const f16x8*>(src));                 \
  }
  // self (beam search): the history rows of batch 0 are resolved through the
  // position map once (its words requested with the control words, above),
  // and the row deltas are kept in registers for both the K and the V loads
  // of that batch
  int mdel[SELF ? UB : 1];
  if constexpr (SELF) {
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = wid * (8 * UB) + u * 8 + kg;
      mdel[u] = (mrow && idx < own0) ? mraw[u] - map_row0 - slot : 0;
    }
  }
#define LOADROWS0(buf, base)                                                      \
  _Pragma("unroll") for (int u = 0; u < UB; ++u) {                               \
    const int j = min(wid * (8 * UB) + u * 8 + kg, jmax);                        \
    const _Float16* src = base + (long)j * 64 + c * 8;                            \
    if (SELF) {                                                                   \
      int md = mdel[SELF ? u : 0];                                                \
      asm volatile("" : "+v"(md)); /* no hoisted 64-bit V addresses */            \
      src += (long)md * rstride;                                                  \
    }                                                                             \
    buf[u] = ld_stream<NTL>(reinterpret_cast<const f16x8*>(src));                 \
  }
  // reduce the projections of this head from the split-K slabs (KS <= 8):
  // the slab loads are issued first, then the first key batch, so the
  // reduction waits only for its own loads
  const long pstride = (long)R * pcols;
  const bool red = tid < (SELF ? 192 : 64);
  const int part = tid >> 6, e = tid & 63;
  const int col = part * D + h * 64 + e;
  float pk[8];
  float bcol = 0.0f;
  if (red) {
    const float* pp = P + (long)row * pcols + col;
#pragma unroll
    for (int k = 0; k < 8; ++k) pk[k] = pp[min(k, KS - 1) * pstride];
    // (requested with the slabs: a bias load issued after the key batches
    // would make the query wait for all of them)
    if (part != 1) bcol = bias[col];
  }
  LOADROWS0(ka, K)
  // NBC: the second key batch is requested before the query is formed too,
  // so two batches are in flight from the start
  if constexpr (NBC > 0) LOADROWS(kb2, K, 1)
  // Cross: the packed score stores and the register softmax with f16 P pairs
  // (below). Self keeps one score store per row and the LDS softmax: with
  // them (and with value batch 0 requested beside key batch 0) it was faster
  // alone but cost the two-lane bench ~1.2 % (A/B on one box, 4 runs each,
  // profiles/r04_ab_regression_beam.md)
  constexpr bool SPACK = !SELF, SREG = !SELF;
  if (red) {
    float acc = pk[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) acc += k < KS ? pk[k] : 0.0f;
    if (part == 0) {
      sq[e] = (float)f16r((acc + bcol) * qscale);
    } else if (part == 1) {
      const _Float16 kv = f16r(acc * kscale);
      snk[e] = (float)kv;
      if (write_new) K[(long)p_row * 64 + e] = kv;
    } else {
      const _Float16 vv = f16r(acc + bcol);
      snv[e] = (float)vv;
      if (write_new) V[(long)p_row * 64 + e] = vv;
    }
  }
  __syncthreads();
  float nv[8];
  h2 qh[4];
  f16x8 nkh;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    nkh[e] = SELF ? (_Float16)snk[c * 8 + e] : (_Float16)0.0f;
    nv[e] = SELF ? snv[c * 8 + e] : 0.0f;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    qh[e] = h2{(_Float16)sq[c * 8 + 2 * e], (_Float16)sq[c * 8 + 2 * e + 1]};
  // scores (q.k in f32 over the f16 rows)
  auto score_batch = [&](const f16x8* kk, int bidx) {
    __builtin_amdgcn_sched_barrier(0);  // keep exactly one batch of loads ahead
    // SPACK: every lane of an 8-lane group holds the row's sum (dpp_sum8's
    // steps are symmetric), so lane c stores row u = c: one LDS write per batch
    float du = 0.0f;
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int j = bidx * BR + wid * (8 * UB) + u * 8 + kg;
      // (j >= n lanes also take the LDS row: finite, and their score is dropped)
      const bool isnew = SELF && min(j, n - 1) == jnew;
      float d = dot8(qh, isnew ? nkh : kk[u]);
      d = dpp_sum8(d);
      if constexpr (SPACK)
        du = (u == 0 || c == u) ? d : du;
      else if (c == 0 && j < n)
        sc[j] = d * scale;
    }
    if constexpr (SPACK) {
      const int jc = bidx * BR + wid * (8 * UB) + c * 8 + kg;
      if (c < UB && jc < n) sc[jc] = du * scale;
    }
  };
  // softmax over the n scores in LDS (ggml order: f32 max, exp, double sum,
  // P = f16(e * (float)(1/sum))). SREG: thread tid owns scores j = tid + 256 i
  // (the order of its double sum), read once and kept in registers. P is written
  // over the scores as packed f16 pairs pp[(j >> 4) * 8 + (j & 7)] =
  // {P[j], P[j + 8]} (0 past n), the row pairs (u, u + 1) of pv_batch: key
  // j + 8 is owned by lane ^ 8 (DPP row_ror:8), and the pair's lane with bit 3
  // clear writes it (same f16 values as one read per row: bit-identical)
  auto softmax = [&]() {
    if constexpr (!SREG) {
      __syncthreads();
      float mx = -INFINITY;
      for (int j = tid; j < n; j += 256) mx = fmaxf(mx, sc[j]);
      mx = block_max_256(mx, redf);
      double sum = 0.0;
      for (int j = tid; j < n; j += 256) {
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        sum += (double)e;
      }
      sum = block_sum_256d(sum, redd);
      const float inv = (float)(1.0 / sum);
      for (int j = tid; j < n; j += 256) sc[j] = (float)f16r(sc[j] * inv);
      __syncthreads();
      return;
    }
    constexpr int NI = DEC_MAX_KEYS / 256;
    float sv[NI];
    __syncthreads();
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = tid + 256 * i;
      sv[i] = j < n ? sc[j] : -INFINITY;
      mx = fmaxf(mx, sv[i]);
    }
    mx = block_max_256(mx, redf);  // (its barriers order every score read before the P writes)
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (tid + 256 * i < n) {
        const float e = expf(sv[i] - mx);
        sv[i] = e;
        sum += (double)e;
      }
    }
    sum = block_sum_256d(sum, redd);
    const float inv = (float)(1.0 / sum);
    h2* pp = reinterpret_cast<h2*>(sc);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = tid + 256 * i;
      const _Float16 p = j < n ? f16r(sv[i] * inv) : (_Float16)0.0f;
      const uint32_t own = (uint32_t)__builtin_bit_cast(uint16_t, p);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)own, 0x128, 0xF, 0xF, true);
      if ((tid & 8) == 0) pp[(j >> 4) * 8 + (j & 7)] = __builtin_bit_cast(h2, own | (hi << 16));
    }
    __syncthreads();
  };
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
  f16x8 nvh;
#pragma unroll
  for (int e = 0; e < 8; ++e) nvh[e] = (_Float16)nv[e];
  // P.V with v_dot2_f32_f16 over the lane's row pairs (u, u+1) = keys
  // (j0, j0 + 8): acc[e] += p_u*v_u[e] + p_u1*v_u1[e] (P is f16 exact, as
  // ggml rounds it), the pair one LDS read (0 past n)
  static_assert(UB % 2 == 0, "row pairs");
  const h2* ppr = reinterpret_cast<const h2*>(sc);
  auto pv_batch = [&](const f16x8* vv, int bidx) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < UB; u += 2) {
      const int j0 = bidx * BR + wid * (8 * UB) + u * 8 + kg;
      // (pairs past DEC_MAX_KEYS / 2 are clamped: their rows are past n)
      h2 ph;
      if constexpr (SREG) {
        ph = ppr[min((j0 >> 4) * 8 + kg, DEC_MAX_KEYS / 2 - 1)];
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int j = j0 + 8 * t;
          float p = sc[min(j, n - 1)];
          if (j >= n) p = 0.0f;
          ph[t] = (_Float16)p;
        }
      }
      f16x8 r[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int j = j0 + 8 * t;
        const bool isnew = SELF && min(j, n - 1) == jnew;
        r[t] = isnew ? nvh : vv[u + t];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = __builtin_amdgcn_fdot2(ph, h2{r[0][e], r[1][e]}, acc[e], false);
    }
  };
  if constexpr (SELF) {
    // <= 4 batches of 128 rows at UB = 4 (n <= 448): latency-bound, one batch
    // per trip (loading V batch 0 together with K batch 0 measured 10% slower
    // at UB = 8, occupancy 4 -> 3, and 1.2 % slower on the two-lane bench at
    // UB = 4)
    for (int b = 0; wave_busy && b < nb; ++b) {
      if (b > 0) LOADROWS(ka, K, b)
      score_batch(ka, b);
    }
    LOADROWS0(ka, V)
    softmax();
    for (int b = 0; wave_busy && b < nb; ++b) {
      if (b > 0) LOADROWS(ka, V, b)
      pv_batch(ka, b);
    }
  } else if constexpr (NBC > 0) {
    // cross with a compile-time even batch count (n = 1500: 6): the K batches
    // and then the V batches form one load stream through the two register
    // buffers (loops of constant trip count, last trips peeled), no batch is loaded past the last one (the
    // runtime loop below loads a clamped K and V batch past the end, and its
    // K -> V hand-over drains every load), and V batches 0 and 1 are in
    // flight across the softmax
    static_assert(NBC % 2 == 0 && NBC >= 4, "even batch count");
#pragma unroll 1
    for (int b = 0; b < NBC - 2; b += 2) {
      score_batch(ka, b);
      LOADROWS(ka, K, b + 2)
      score_batch(kb2, b + 1);
      LOADROWS(kb2, K, b + 3)
    }
    score_batch(ka, NBC - 2);
    LOADROWS(ka, V, 0)
    score_batch(kb2, NBC - 1);
    LOADROWS(kb2, V, 1)
    softmax();
#pragma unroll 1
    for (int b = 0; b < NBC - 2; b += 2) {
      pv_batch(ka, b);
      LOADROWS(ka, V, b + 2)
      pv_batch(kb2, b + 1);
      LOADROWS(kb2, V, b + 3)
    }
    pv_batch(ka, NBC - 2);
    pv_batch(kb2, NBC - 1);
  } else {
    for (int b = 0; b < nb; b += 2) {  // (odd nb: one clamped batch extra)
      LOADROWS(kb2, K, b + 1)
      score_batch(ka, b);
      LOADROWS(ka, K, b + 2)
      score_batch(kb2, b + 1);
    }
    LOADROWS0(ka, V)
    softmax();
    for (int b = 0; b < nb; b += 2) {
      LOADROWS(kb2, V, b + 1)
      pv_batch(ka, b);
      LOADROWS(ka, V, b + 2)
      pv_batch(kb2, b + 1);
    }
  }
#undef LOADROWS
#undef LOADROWS0
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] = add_xor8(acc[e]);
    acc[e] = add_xor16(acc[e]);
    acc[e] = add_xor32(acc[e]);
  }
  if (kg == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) pv[wid][c][e] = acc[e];
  }
  __syncthreads();
  if (tid < 64) {
    const int cc = tid >> 3, e = tid & 7;
    const float r = (pv[0][cc][e] + pv[1][cc][e]) + (pv[2][cc][e] + pv[3][cc][e]);
    o[pack_index(row, h * 64 + cc * 8 + e, D)] = to_t<T>(r);
  }
  span_end(span);
}

// Cross-attention of NQ rows that share one clip's cross K/V (the decoders
// of a beam search / best-of group: rows g*NQ .. g*NQ+NQ-1): one workgroup per
// (group, head) streams the clip's K and V once for all NQ queries instead of
// once per row. Every row's arithmetic (scores, softmax, P.V reduction order)
// is exactly that of dec_attn_kernel<T, false>, so results do not depend on
// the grouping.
// KV8 (MWX_COMPUTE_MXFP8): the cross K/V cache holds MX-fp8 rows (64 e4m3
// codes per (time, head) and two E8M0 scales, one per 32-element half), half
// the bytes of the f16 cache. A lane's 8 codes lie in one half, so they are
// widened to f16 with that half's scale (v_cvt_scalef32_pk_f16_fp8: exact
// while code x scale is f16-representable — the cache's values are f16 values
// MX-rounded, so they are; measured: f16 RNE including subnormals, +-inf
// past f16's range, test_mx_cache_widening_pinned) and every score / P.V
// operation then runs
// on f16 exactly as for the f16 cache. Each lane loads the scale pair of one
// of its wave's 64 rows per batch; the pair a row needs is read from the lane
// that loaded it (__shfl).
#ifndef XATTN_VB
#define XATTN_VB 2
#endif
__device__ __forceinline__ f16x8 dequant_h8(uint2 raw, uint32_t e) {
  const float sc = e ? __uint_as_float(e << 23) : __uint_as_float(0x00400000u);
  const h2 a = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.x, sc, false);
  const h2 b = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.x, sc, true);
  const h2 c = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.y, sc, false);
  const h2 d = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.y, sc, true);
  return f16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// test hook (mwx_test_mx_widen): dequant_h8 itself on 8 codes per thread
__global__ void mx_widen_test_kernel(const uint2* __restrict__ codes, const uint8_t* __restrict__ e8,
                                     int n8, f16x8* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n8) out[i] = dequant_h8(codes[i], e8[i]);
}
void mx_widen_test(const uint8_t* codes, const uint8_t* e8, int n8, uint16_t* out, hipStream_t st) {
  mx_widen_test_kernel<<<(n8 + 255) / 256, 256, 0, st>>>(reinterpret_cast<const uint2*>(codes), e8,
                                                         n8, reinterpret_cast<f16x8*>(out));
}

// MFS (MX-fp8 cache only, MWX_XATTN_MFS): scores and P.V on MFMA instead of
// v_dot2 chains. Scores: a 16-key tile is the A operand of two chained
// v_mfma_f32_16x16x32_f16 (one per 32-element scale half; lane l holds key
// l&15's 8 codes at e = 8(l>>4) .. +7 of that half, widened to f16 with that
// key's half scale: exact while code x scale is f16-representable, as in the
// v_dot2 path), the queries (f16, rows
// >= NQ zero) the B operand; lane l receives query l&15's scores with keys
// 4(l>>4) .. +3. P.V: the V tile staged in LDS as exactly widened f16, the
// f16 P the A operand (below). A query's results depend only on its own row,
// so they do not depend on the group size NQ. Each wave streams its key tiles
// (wave w: w, w + 4, ...) four at a time, two groups in flight. Round 5: the
// per-key scale arithmetic after the MFMAs (scores) and on P (P.V) cost ~2/3
// of the kernel's VALU instructions (PMC, profiles/r05_pmc_xattn_raw.md).
template <typename T, int NQ, bool KV8 = false, bool NTL = true, int NBC = 0, bool MFS = false>
__global__ __launch_bounds__(256) void dec_xattn_kernel(
    const float* __restrict__ P, int KS, int pcols, const float* __restrict__ bias,
    const void* __restrict__ kbase, const void* __restrict__ vbase,
    const uint8_t* __restrict__ kscale8, const uint8_t* __restrict__ vscale8,
    const int* __restrict__ kv_index, const int* __restrict__ active, int n, int cap, int R,
    T* __restrict__ o, int H, float scale, unsigned long long* span = nullptr) {
  static_assert(!MFS || KV8, "MFS: MX-fp8 caches only");
  span_start(span);
  __shared__ __attribute__((aligned(16))) float sc[NQ][DEC_MAX_KEYS];
  __shared__ float redf[4][NQ];
  __shared__ double redd[4][NQ];
  // the waves' P.V partials: [4][64][9] (v_dot2 path) or [4][NQ][64] (MFS,
  // sized so three workgroups still fit a CU's LDS beside the f16 V tiles)
  constexpr int PVN = MFS ? 4 * NQ * 64 : 4 * 64 * 9;
  __shared__ float pvb[PVN];
  auto pv = reinterpret_cast<float(*)[64][9]>(pvb);
  __shared__ float sq[NQ][64];
  const int g = blockIdx.y, h = blockIdx.x, row0 = g * NQ;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = lane >> 3, c = lane & 7;
  bool act[NQ];
  bool any = false;
  // the group's control words and its K/V slot are fetched together (one
  // round trip), then the all-inactive exit
  const int slot = kv_index ? kv_index[row0] : row0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    act[q] = row0 + q < R && active[min(row0 + q, R - 1)];
    any |= act[q];
  }
  asm volatile("" ::"s"(slot));
  if (!any) {
    span_end(span);
    return;
  }
  const int D = H * 64;
  const long rbase = ((long)slot * H + h) * cap;  // first (time) row of this (slot, head)
  const _Float16* K = reinterpret_cast<const _Float16*>(kbase) + rbase * 64;
  const _Float16* V = reinterpret_cast<const _Float16*>(vbase) + rbase * 64;
  const uint8_t* K8 = reinterpret_cast<const uint8_t*>(kbase) + rbase * 64;
  const uint8_t* V8 = reinterpret_cast<const uint8_t*>(vbase) + rbase * 64;
  const uint8_t* KS8 = KV8 ? kscale8 + rbase * 2 : nullptr;
  const uint8_t* VS8 = KV8 ? vscale8 + rbase * 2 : nullptr;
  // the key/value rows of a batch are those of dec_attn_kernel (row
  // bidx*256 + wid*64 + u*8 + kg, u < 8) but are streamed in halves of 4 rows
  // per lane group (u = 4*half + uu), so fewer registers hold loads in flight
  constexpr int UH = 4;
  const int nb = NBC > 0 ? NBC : (n + 255) >> 8;
  const int jmax = n - 1;
  f16x8 ka[UH], kb2[UH];
  uint2 qa[KV8 ? UH : 1], qb[KV8 ? UH : 1];  // fp8 rows in flight
  uint32_t sa = 0, sb = 0;                   // scale pairs (lane: row wid*64 + lane)
#define LOADROWS16(buf, base, bidx, half)                                      \
  _Pragma("unroll") for (int uu = 0; uu < UH; ++uu) {                         \
    const int j = min((bidx) * 256 + wid * 64 + ((half) * UH + uu) * 8 + kg, jmax); \
    buf[uu] = ld_stream<NTL>(reinterpret_cast<const f16x8*>(base + (long)j * 64 + c * 8)); \
  }
#define LOADROWS8(qbuf, sreg, base8, sbase, bidx, half)                              \
  _Pragma("unroll") for (int uu = 0; uu < UH; ++uu) {                               \
    const int j = min((bidx) * 256 + wid * 64 + ((half) * UH + uu) * 8 + kg, jmax);   \
    const u32x2 q2_ = ld_stream<NTL>(reinterpret_cast<const u32x2*>(base8 + (long)j * 64 + c * 8)); \
    qbuf[uu] = uint2{q2_[0], q2_[1]};                                                 \
  }                                                                                 \
  sreg = *reinterpret_cast<const uint16_t*>(                                        \
      sbase + (long)min((bidx) * 256 + wid * 64 + lane, jmax) * 2);
#define WIDEN8(buf, qbuf, sreg, half)                                               \
  _Pragma("unroll") for (int uu = 0; uu < UH; ++uu) {                               \
    const uint32_t pr = (uint32_t)__shfl((int)(sreg), ((half) * UH + uu) * 8 + kg, 64); \
    buf[uu] = dequant_h8(qbuf[uu], (pr >> (8 * (c >> 2))) & 0xffu);                 \
  }
  // queries: q = f16(sum of the split-K slabs + bias), head h's 64 columns.
  // All slab loads (KS <= 8, clamped) are issued first, then the first key
  // batch, so the sums wait for one round trip and the keys are in flight
  const long pstride = (long)R * pcols;
  constexpr int QI = (NQ * 64 + 255) / 256;
  float pq[QI][8];
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int t = tid + 256 * i;
    const int q = min(t >> 6, NQ - 1), e = t & 63;
    const float* pp = P + (long)min(row0 + q, R - 1) * pcols + h * 64 + e;
#pragma unroll
    for (int k = 0; k < 8; ++k) pq[i][k] = pp[min(k, KS - 1) * pstride];
  }
  // the bias is requested with the slabs (after the key loads, the query
  // would wait for them)
  const float bq = bias[h * 64 + (tid & 63)];
  // MFS: key tiles in flight (TD tiles of 2 x 8 code bytes + the scale pair
  // of the lane's A-operand key)
  constexpr int TD = 4;
  const int ntile = (n + 15) >> 4;
  const int mrow = lane & 15, gq = lane >> 4;
  uint2 kr[MFS ? 2 : 1][MFS ? TD : 1][2];
  uint32_t ksr[MFS ? 2 : 1][MFS ? TD : 1];
  auto mfs_load = [&](int buf, int grp) {  // tiles wid + 4 * (TD * grp + i)
#pragma unroll
    for (int i = 0; i < TD; ++i) {
      const int t = min(wid + 4 * (TD * grp + i), ntile - 1);
      const int key = min(t * 16 + mrow, jmax);
      const uint8_t* row = K8 + (long)key * 64 + 8 * gq;
      const u32x2 a = ld_stream<NTL>(reinterpret_cast<const u32x2*>(row));
      const u32x2 b = ld_stream<NTL>(reinterpret_cast<const u32x2*>(row + 32));
      kr[buf][i][0] = uint2{a[0], a[1]};
      kr[buf][i][1] = uint2{b[0], b[1]};
      ksr[buf][i] = *reinterpret_cast<const uint16_t*>(KS8 + (long)key * 2);
    }
  };
  const int ngrp = ((ntile + 3) / 4 + TD - 1) / TD;  // (tile groups per wave, upper bound)
  if constexpr (MFS) {
    mfs_load(0, 0);
  } else if constexpr (KV8) {
    LOADROWS8(qa, sa, K8, KS8, 0, 0)
  } else {
    LOADROWS16(ka, K, 0, 0)
  }
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int t = tid + 256 * i;
    if (t < NQ * 64) {
      const int q = t >> 6, e = t & 63;
      float acc = pq[i][0];
#pragma unroll
      for (int k = 1; k < 8; ++k) acc += k < KS ? pq[i][k] : 0.0f;
      sq[q][e] = (float)f16r(acc + bq);  // (e == tid & 63)
    }
  }
  __syncthreads();
  h2 qh[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      qh[q][e] = h2{(_Float16)sq[q][c * 8 + 2 * e], (_Float16)sq[q][c * 8 + 2 * e + 1]};
  auto score_batch = [&](const f16x8* kk, int bidx, int half) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int uu = 0; uu < UH; ++uu) {
      const int u = half * UH + uu;
      const int j = bidx * 256 + wid * 64 + u * 8 + kg;
      // every lane of the 8-lane group holds each query's sum (dpp_sum8's
      // steps are symmetric), so lane c stores query c's score: one LDS
      // write per key row instead of NQ
      float dc = 0.0f;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        float d = dot8(qh[q], kk[uu]);
        d = dpp_sum8(d);
        dc = (q == 0 || c == q) ? d : dc;
      }
      if (c < NQ && j < n) sc[c][j] = dc * scale;
      __builtin_amdgcn_sched_barrier(0);  // one key row's conversions live at a time
    }
  };
  // NBC > 0 (n = 1500: 6 batches, a compile-time count): the last K trip
  // loads V batch 0 instead of a clamped K batch past the end (whose loads the
  // K -> V hand-over would otherwise drain), and the last V trip loads nothing
  auto k_trip = [&](int b, bool last) {
    if constexpr (KV8) {
      LOADROWS8(qb, sb, K8, KS8, b, 1)
      WIDEN8(ka, qa, sa, 0)
      score_batch(ka, b, 0);
      if (NBC > 0 && last) {
        LOADROWS8(qa, sa, V8, VS8, 0, 0)
      } else {
        LOADROWS8(qa, sa, K8, KS8, b + 1, 0)
      }
      WIDEN8(kb2, qb, sb, 1)
      score_batch(kb2, b, 1);
    } else {
      LOADROWS16(kb2, K, b, 1)
      score_batch(ka, b, 0);
      if (NBC > 0 && last) {
        LOADROWS16(ka, V, 0, 0)
      } else {
        LOADROWS16(ka, K, b + 1, 0)
      }
      score_batch(kb2, b, 1);
    }
  };
  // MFS: P.V on MFMA as well. Wave w stages its 32-key V tiles (w, w + 4, ...)
  // in LDS as f16, dequantized at staging: a lane's 32 codes are one half of
  // one key row, so one E8M0 scale widens them exactly while code x scale is
  // f16-representable, as in the v_dot2 path; the B operand (8 keys of one
  // column) is two transposed 16-bit reads (ds_read_b64_tr_b16), and the A
  // operand the query's f16 P itself (no per-key scale arithmetic). The
  // 32-B column blocks of a row are XOR-swizzled (vsw below) so that both
  // the staging stores and the transposed reads are bank-conflict free.
  // (256-B aligned: the block swizzle assumes a tile row starts at bank 0)
  __shared__ __attribute__((aligned(256))) _Float16 vtile[MFS ? 4 : 1][MFS ? 32 * 64 : 8];
  const int nt32 = (n + 31) >> 5;
  const int vrow = lane >> 1, vch = 2 * (lane & 1);
  // VB tiles in flight per wave (build constant XATTN_VB)
  constexpr int VB = MFS ? XATTN_VB : 1;
  u32x4 vr[VB][2];     // the next tiles' codes (row vrow, chunks vch, vch + 1)
  uint32_t vse[VB];    // their E8M0 scale (row vrow, half lane & 1)
  auto v_load = [&](int t, int b) {
    const int row = min(t * 32 + vrow, jmax);
    if constexpr (KV8) {
      const u32x4* src = reinterpret_cast<const u32x4*>(V8 + (long)row * 64) + vch;
      vr[b][0] = ld_stream<NTL>(src);
      vr[b][1] = ld_stream<NTL>(src + 1);
      vse[b] = VS8[(long)row * 2 + (lane & 1)];
    }
  };
  if constexpr (MFS) {
    // B operand: query l&15 at e = 8(l>>4) + j (half 0) and 32 + 8(l>>4) + j
    f16x8 qb0, qb1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      qb0[j] = mrow < NQ ? (_Float16)sq[min(mrow, NQ - 1)][8 * gq + j] : (_Float16)0.0f;
      qb1[j] = mrow < NQ ? (_Float16)sq[min(mrow, NQ - 1)][32 + 8 * gq + j] : (_Float16)0.0f;
    }
    // each lane widens its A-operand key's codes with that key's two
    // scales (one per 32-element half; exact while code x scale is
    // f16-representable, as the v_dot2 path widens them), and the two halves
    // chain in one accumulator
    auto score_tile = [&](int buf, int i, int t) {
      f32x4 out;
      {
        const uint32_t sp = ksr[buf][i];
        const f16x8 a0 = dequant_h8(kr[buf][i][0], sp & 0xffu);
        const f16x8 a1 = dequant_h8(kr[buf][i][1], sp >> 8);
        const f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
        f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, qb0, z, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, qb1, d, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = d[r] * scale;
      }
      if (mrow < NQ && t < ntile)
        *reinterpret_cast<f32x4*>(&sc[min(mrow, NQ - 1)][t * 16 + 4 * gq]) = out;
    };
#pragma unroll 1
    for (int grp = 0; grp < ngrp; grp += 2) {
      if (grp + 1 < ngrp) mfs_load(1, grp + 1);
#pragma unroll
      for (int i = 0; i < TD; ++i) score_tile(0, i, wid + 4 * (TD * grp + i));
      if (grp + 2 < ngrp) mfs_load(0, grp + 2);
      if (grp + 1 < ngrp) {
#pragma unroll
        for (int i = 0; i < TD; ++i) score_tile(1, i, wid + 4 * (TD * (grp + 1) + i));
      }
    }
#pragma unroll
    for (int b = 0; b < VB; ++b)  // (in flight across the softmax)
      if (wid + 4 * b < nt32) v_load(wid + 4 * b, b);
  } else if constexpr (NBC > 0) {
#pragma unroll 1
    for (int b = 0; b < NBC - 1; ++b) k_trip(b, false);
    k_trip(NBC - 1, true);
  } else {
    for (int b = 0; b < nb; ++b) k_trip(b, false);
    if constexpr (KV8) {
      LOADROWS8(qa, sa, V8, VS8, 0, 0)
    } else {
      LOADROWS16(ka, V, 0, 0)
    }
  }
  __syncthreads();
  // softmax per query (block_max_256 / block_sum_256d order). Thread tid owns
  // scores j = tid + 256 i (the order of its double sum); they are read from
  // LDS once and kept in registers through max, exp and P.
  constexpr int NI = DEC_MAX_KEYS / 256;
  float sv[NQ][NI];
  float mx[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = tid + 256 * i;
      sv[q][i] = j < n ? sc[q][j] : -INFINITY;
      m = fmaxf(m, sv[q][i]);
    }
    mx[q] = wave_max_dpp(m);
  }
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NQ; ++q) redf[wid][q] = mx[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    mx[q] = fmaxf(fmaxf(redf[0][q], redf[1][q]), fmaxf(redf[2][q], redf[3][q]));
  double sum[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    double sm = 0.0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (tid + 256 * i < n) {
        const float e = expf(sv[q][i] - mx[q]);
        sv[q][i] = e;
        sm += (double)e;
      }
    }
    sum[q] = wave_sum_d_dpp(sm);
  }
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < NQ; ++q) redd[wid][q] = sum[q];
  __syncthreads();
  // P = f16(e * (float)(1/sum)) (ggml order), written over the scores (no
  // thread reads a score after the barrier above). The v_dot2 P.V below takes
  // the weights of its row pairs (j, j + 8) as packed f16 pairs,
  // pp[q][(j >> 4) * 8 + (j & 7)] = {P[j], P[j + 8]} (0 past n), so each pair
  // is one LDS read instead of two reads and three conversions (the same f16
  // values: bit-identical). Key j + 8 is owned by lane ^ 8 (DPP row_ror:8),
  // and the lane of the pair with bit 3 clear writes it.
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const double t = (redd[0][q] + redd[1][q]) + (redd[2][q] + redd[3][q]);
    const float inv = (float)(1.0 / t);
    if constexpr (MFS) {
      // f16 P over the score row's storage (zeros past n: the A operand of
      // the last tile reads whole 8-key groups)
      _Float16* ph = reinterpret_cast<_Float16*>(&sc[q][0]);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = tid + 256 * i;
        ph[j] = j < n ? f16r(sv[q][i] * inv) : (_Float16)0.0f;
      }
    } else {
      h2* pp = reinterpret_cast<h2*>(&sc[q][0]);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = tid + 256 * i;
        const _Float16 p = j < n ? f16r(sv[q][i] * inv) : (_Float16)0.0f;
        const uint32_t own = (uint32_t)__builtin_bit_cast(uint16_t, p);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)own, 0x128, 0xF, 0xF, true);
        if ((tid & 8) == 0) pp[(j >> 4) * 8 + (j & 7)] = __builtin_bit_cast(h2, own | (hi << 16));
      }
    }
  }
  __syncthreads();
  if constexpr (MFS) {
    _Float16* vw = &vtile[0][0] + wid * (32 * 64);
    f32x4 oacc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) oacc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int qrow = min(mrow, NQ - 1);
    const _Float16* prow = reinterpret_cast<const _Float16*>(&sc[qrow][0]);
    // this lane's transposed-read slot: row q = (lane >> 2) & 3 of the
    // group's 4-row block, columns 4 (lane & 3) .. + 3 of the 16-column block
    const int trq = (lane >> 2) & 3, trp = lane & 3;
    // 32-B column-block swizzle of a V tile row: (row >> 1) & 3 spreads a
    // read group's rows 4 apart over the banks; row bit 3 (lanes 16-31 of a
    // transposed read: rows 8-15) flips the block pair too, so the two
    // 16-lane halves of a ds_read_b64_tr_b16 no longer meet on the same banks
    auto vsw = [](int row) { return ((row >> 1) & 3) ^ (((row >> 3) & 1) << 1); };
    auto pv_tile = [&](int t, int b) {
      {  // stage the tile as f16 (this wave's region only: in-order LDS, no barrier)
        const f16x8 d0 = dequant_h8(uint2{vr[b][0][0], vr[b][0][1]}, vse[b]);
        const f16x8 d1 = dequant_h8(uint2{vr[b][0][2], vr[b][0][3]}, vse[b]);
        const f16x8 d2 = dequant_h8(uint2{vr[b][1][0], vr[b][1][1]}, vse[b]);
        const f16x8 d3 = dequant_h8(uint2{vr[b][1][2], vr[b][1][3]}, vse[b]);
        const int sw = vsw(vrow), b0 = 2 * (lane & 1);  // the lane's two 16-column blocks
        _Float16* rw = vw + vrow * 64;
        // odd rows store their two 16-B halves in the other order, so each
        // store instruction's 8-lane groups cover 8 distinct 16-B bank slots
        // (same LDS image; in one order rows 2m and 2m + 1 collided)
        const bool odd = vrow & 1;
        *reinterpret_cast<f16x8*>(rw + ((b0 ^ sw) << 4) + (odd ? 8 : 0)) = odd ? d1 : d0;
        *reinterpret_cast<f16x8*>(rw + ((b0 ^ sw) << 4) + (odd ? 0 : 8)) = odd ? d0 : d1;
        *reinterpret_cast<f16x8*>(rw + (((b0 + 1) ^ sw) << 4) + (odd ? 8 : 0)) = odd ? d3 : d2;
        *reinterpret_cast<f16x8*>(rw + (((b0 + 1) ^ sw) << 4) + (odd ? 0 : 8)) = odd ? d2 : d3;
      }
      if (t + 4 * VB < nt32) v_load(t + 4 * VB, b);
      // A operand: P of query mrow (rows >= NQ zero) at keys t*32 + 8 gq .. + 7
      // (zero past n, written so by the softmax)
      const int kb = t * 32 + 8 * gq;
      f16x8 pa = *reinterpret_cast<const f16x8*>(prow + kb);
      if (mrow >= NQ) pa = f16x8{};
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        // B operand: column 16 nt + mrow of keys 8 gq .. 8 gq + 7, as two
        // 4-row transposed reads (rows 8 gq + 4 h + trq, this lane's 4 columns)
        typedef short v4s_t __attribute__((ext_vector_type(4)));
        u32x2 tw[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = 8 * gq + 4 * h + trq;
          const _Float16* src = vw + row * 64 + ((nt ^ vsw(row)) << 4) + 4 * trp;
          // (the whole 64-bit result reinterpreted at once: per-element
          // extraction of the v4i16 miscompiled here, only element 0 of each
          // read reached the operand)
          tw[h] = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                (__attribute__((address_space(3))) v4s_t*)(src)));
        }
        const f16x8 vb = __builtin_bit_cast(f16x8, u32x4{tw[0][0], tw[0][1], tw[1][0], tw[1][1]});
        oacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa, vb, oacc[nt], 0, 0, 0);
      }
    };
#pragma unroll 1
    for (int t = wid; t < nt32; t += 4 * VB) {
#pragma unroll
      for (int b = 0; b < VB; ++b)
        if (t + 4 * b < nt32) pv_tile(t + 4 * b, b);
    }
    // the four waves' partial sums: (w0 + w1) + (w2 + w3)
    float* op = pvb;  // [4][NQ][64] floats
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = 4 * gq + r;
        if (q < NQ) op[(wid * NQ + q) * 64 + 16 * nt + mrow] = oacc[nt][r];
      }
    __syncthreads();
    for (int i = tid; i < NQ * 64; i += 256) {
      const int q = i >> 6, e = i & 63;
      const float r = (op[q * 64 + e] + op[(NQ + q) * 64 + e]) +
                      (op[(2 * NQ + q) * 64 + e] + op[(3 * NQ + q) * 64 + e]);
      if (act[q]) o[pack_index(row0 + q, h * 64 + e, D)] = to_t<T>(r);
    }
    span_end(span);
    return;
  }
  float acc[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[q][e] = 0.0f;
  auto pv_batch = [&](const f16x8* vv, int bidx, int half) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int uu = 0; uu < UH; uu += 2) {  // row pairs (u, u+1) as in dec_attn_kernel
      const int j0 = bidx * 256 + wid * 64 + (half * UH + uu) * 8 + kg, j1 = j0 + 8;
      h2 vp[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) vp[e] = h2{vv[uu][e], vv[uu + 1][e]};
      (void)j1;
      const int pidx = (j0 >> 4) * 8 + (j0 & 7);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const h2 ph = reinterpret_cast<const h2*>(&sc[q][0])[pidx];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[q][e] = __builtin_amdgcn_fdot2(ph, vp[e], acc[q][e], false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto v_trip = [&](int b, bool last) {
    if constexpr (KV8) {
      LOADROWS8(qb, sb, V8, VS8, b, 1)
      WIDEN8(ka, qa, sa, 0)
      pv_batch(ka, b, 0);
      if (!(NBC > 0 && last)) {
        LOADROWS8(qa, sa, V8, VS8, b + 1, 0)
      }
      WIDEN8(kb2, qb, sb, 1)
      pv_batch(kb2, b, 1);
    } else {
      LOADROWS16(kb2, V, b, 1)
      pv_batch(ka, b, 0);
      if (!(NBC > 0 && last)) {
        LOADROWS16(ka, V, b + 1, 0)
      }
      pv_batch(kb2, b, 1);
    }
  };
  if constexpr (NBC > 0) {
#pragma unroll 1
    for (int b = 0; b < NBC - 1; ++b) v_trip(b, false);
    v_trip(NBC - 1, true);
  } else {
    for (int b = 0; b < nb; ++b) v_trip(b, false);
  }
#undef LOADROWS16
#undef LOADROWS8
#undef WIDEN8
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float a = acc[q][e];
      a = add_xor8(a);
      a = add_xor16(a);
      a = add_xor32(a);
      acc[q][e] = a;
    }
    if (kg == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) pv[wid][c][e] = acc[q][e];
    }
    __syncthreads();
    if (tid < 64 && act[q]) {
      const int cc = tid >> 3, e = tid & 7;
      const float r = (pv[0][cc][e] + pv[1][cc][e]) + (pv[2][cc][e] + pv[3][cc][e]);
      o[pack_index(row0 + q, h * 64 + cc * 8 + e, D)] = to_t<T>(r);
    }
    __syncthreads();
  }
  span_end(span);
}

static std::atomic<int>& xattn_mfs_mode() {
  static std::atomic<int> m{-1};
  return m;
}
static bool xattn_mfs_on() {
  int v = xattn_mfs_mode().load();
  if (v < 0) {
    v = (getenv("MWX_XATTN_MFS") && atoi(getenv("MWX_XATTN_MFS")) == 0) ? 0 : 1;
    xattn_mfs_mode().store(v);
  }
  return v != 0;
}
int xattn_mfs_set(int on) { return xattn_mfs_mode().exchange(on < 0 ? -1 : (on ? 1 : 0)); }

template <typename T>
bool dec_cross_attention_grouped(const float* P, int KS, int pcols, const float* bias,
                                 const void* kbase, const void* vbase, const int* kv_index,
                                 const int* active, int n_keys, int cap, T* o, int R, int H,
                                 float scale, int nq, hipStream_t st, const uint8_t* kscale8,
                                 const uint8_t* vscale8, unsigned long long* span) {
  if (n_keys > DEC_MAX_KEYS || KS > 8) return false;
  const dim3 g(H, (R + nq - 1) / nq);
  const bool kv8 = kscale8 != nullptr;
  if (!kv8 && nq == 1) return false;  // (f16 single rows: dec_attention)
  // MWX_XATTN_NT=0: default-policy K/V loads (A/B of the non-temporal stream)
  static const bool nt = !(getenv("MWX_XATTN_NT") && atoi(getenv("MWX_XATTN_NT")) == 0);
  // 1500 keys: the constant-batch-count load stream, opt-in (MWX_XATTN_NBC=1):
  // beam 5, same box, 770.6 / 775.7 against 778.9 / 778.8 audio-s/s for the
  // runtime count, so the grouped kernel keeps the runtime count by default
  static const bool nbc = getenv("MWX_XATTN_NBC") && atoi(getenv("MWX_XATTN_NBC")) == 1;
  const bool c6 = nbc && !kv8 && n_keys > 1280 && n_keys <= 1536;
#define XL(N, K8, NT)                                                                          \
  do {                                                                                         \
    if (c6)                                                                                    \
      dec_xattn_kernel<T, N, K8, NT, 6><<<g, 256, 0, st>>>(P, KS, pcols, bias, kbase, vbase,   \
                                                           kscale8, vscale8, kv_index, active, \
                                                           n_keys, cap, R, o, H, scale, span); \
    else                                                                                       \
      dec_xattn_kernel<T, N, K8, NT><<<g, 256, 0, st>>>(P, KS, pcols, bias, kbase, vbase,      \
                                                        kscale8, vscale8, kv_index, active,    \
                                                        n_keys, cap, R, o, H, scale, span);    \
  } while (0)
  // MX-fp8 cache: scores on MFMA (default; MWX_XATTN_MFS=0 or
  // xattn_mfs_set(0): the v_dot2 scores, the A/B: C5 one lane 735.8 -> 778.8
  // audio-s/s, 52.4 -> 44.6 us per launch)
  const bool mfs = xattn_mfs_on();
  switch (nq) {
#define XQ(N)                                  \
  case N:                                      \
    if (kv8 && mfs)                            \
      dec_xattn_kernel<T, N, true, true, 0, true><<<g, 256, 0, st>>>(P, KS, pcols, bias, kbase, \
          vbase, kscale8, vscale8, kv_index, active, n_keys, cap, R, o, H, scale, span);       \
    else if (kv8 && nt)                        \
      XL(N, true, true);                       \
    else if (kv8)                              \
      XL(N, true, false);                      \
    else if (nt)                               \
      XL(N, false, true);                      \
    else                                       \
      XL(N, false, false);                     \
    return true;
    XQ(1) XQ(2) XQ(3) XQ(4) XQ(5) XQ(6) XQ(7) XQ(8)
#undef XQ
#undef XL
    default: return false;
  }
}
template bool dec_cross_attention_grouped<_Float16>(const float*, int, int, const float*,
                                                    const void*, const void*, const int*,
                                                    const int*, int, int, _Float16*, int, int,
                                                    float, int, hipStream_t, const uint8_t*,
                                                    const uint8_t*, unsigned long long*);
template bool dec_cross_attention_grouped<__bf16>(const float*, int, int, const float*,
                                                  const void*, const void*, const int*,
                                                  const int*, int, int, __bf16*, int, int, float,
                                                  int, hipStream_t, const uint8_t*,
                                                  const uint8_t*, unsigned long long*);

// Prompt prefill: the self-attention K / V of every (virtual) row appended
// to its cache row crow[row] at position pos[row] before the self-attention
// launch of the same layer, so a prompt position can read the positions
// before it that other rows of the same launch produce. The values are those
// dec_attn_kernel<T, true> forms for its own position (same slab sum, same
// roundings), which it also writes again (the same bits).
__global__ __launch_bounds__(128) void kv_append_kernel(const float* __restrict__ P, int KS,
                                                       int pcols, const float* __restrict__ bias,
                                                       float kscale, _Float16* __restrict__ kbase,
                                                       _Float16* __restrict__ vbase,
                                                       const int* __restrict__ crow,
                                                       const int* __restrict__ pos,
                                                       const int* __restrict__ active, int cap,
                                                       int R, int H) {
  const int h = blockIdx.x, row = blockIdx.y;
  if (!active[row]) return;
  const int tid = threadIdx.x, part = 1 + (tid >> 6), e = tid & 63;
  const int D = H * 64;
  const int col = part * D + h * 64 + e;
  const long pstride = (long)R * pcols;
  const float* pp = P + (long)row * pcols + col;
  float pk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) pk[k] = pp[min(k, KS - 1) * pstride];
  float acc = pk[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) acc += k < KS ? pk[k] : 0.0f;
  const long dst = (((long)(crow ? crow[row] : row) * H + h) * cap + pos[row]) * 64 + e;
  if (part == 1)
    kbase[dst] = f16r(acc * kscale);
  else
    vbase[dst] = f16r(acc + bias[col]);
}

template <typename T>
void kv_append(const float* P, int KS, int pcols, const float* bias, float kscale,
               _Float16* kbase, _Float16* vbase, const int* crow, const int* pos,
               const int* active, int cap, int R, int H, hipStream_t st) {
  if (R <= 0) return;
  kv_append_kernel<<<dim3(H, R), 128, 0, st>>>(P, KS, pcols, bias, kscale, kbase, vbase, crow, pos,
                                              active, cap, R, H);
}
template void kv_append<_Float16>(const float*, int, int, const float*, float, _Float16*,
                                  _Float16*, const int*, const int*, const int*, int, int, int,
                                  hipStream_t);
template void kv_append<__bf16>(const float*, int, int, const float*, float, _Float16*, _Float16*,
                                const int*, const int*, const int*, int, int, int, hipStream_t);

template <typename T>
void dec_attention(const float* P, int KS, int pcols, const float* bias, float qscale,
                   float kscale, _Float16* kbase, _Float16* vbase, const int* kv_index,
                   const int* pos, const int* active, int fixed_len, int kv_len_cap, T* o, int R,
                   int H, float scale, hipStream_t st, const int* kvmap, const int* own_from,
                   int map_row0, int nq, int write_new, unsigned long long* span) {
  dim3 g(H, R);
  if (nq > 1 && R % nq == 0) {
    const int groups = (R / nq) * H;
    g = dim3((groups + 7) / 8 * 8 * nq, 1);
  } else {
    nq = 1;
  }
  // (cross rows per lane group per batch: 8 measured best; 12 -1.2%, 16 -5%)
  // (self rows per lane group per batch: 4 -- 66 VGPRs, 7 waves/SIMD: beam 5
  // 659 -> 687 audio-s/s; 8 with MWX_SELF_UB=8 for A/B)
  static const bool self_ub4 = !(getenv("MWX_SELF_UB") && atoi(getenv("MWX_SELF_UB")) == 8);
  // cross K/V streamed with non-temporal loads (MWX_XATTN_NT=0: default policy
  // always, 1: nt always). Default: nt unless the launch's cross K/V is small
  // (<= 4 MB: one base / small-model request), where the model's whole cross
  // cache stays resident in the 256-MB MALL across decode steps with the
  // default policy and nt would evict it every step
  static const int xattn_nt_env = getenv("MWX_XATTN_NT") ? atoi(getenv("MWX_XATTN_NT")) : -1;
  const bool xattn_nt =
      xattn_nt_env >= 0 ? xattn_nt_env != 0 : (long)R * H * fixed_len * 256 > (4l << 20);
  // MWX_XATTN_NBC=0: the runtime-batch-count cross kernel (A/B of the
  // constant-count load stream)
  static const bool xattn_nbc = !(getenv("MWX_XATTN_NBC") && atoi(getenv("MWX_XATTN_NBC")) == 0);
  if (fixed_len == 0 && self_ub4)
    dec_attn_kernel<T, true, 4><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale, kbase,
                                                   vbase, kv_index, pos, active, fixed_len,
                                                   kv_len_cap, o, H, scale, kvmap, own_from,
                                                   map_row0, nq, R, write_new, span);
  else if (fixed_len == 0)
    dec_attn_kernel<T, true><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale, kbase, vbase,
                                                kv_index, pos, active, fixed_len, kv_len_cap, o,
                                                H, scale, kvmap, own_from, map_row0, nq, R,
                                                write_new);
  else if (xattn_nt && fixed_len == 1500 && xattn_nbc)  // (every Whisper model: 1500 frames)
    dec_attn_kernel<T, false, 8, true, 6><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale,
                                                             kbase, vbase, kv_index, pos, active,
                                                             fixed_len, kv_len_cap, o, H, scale,
                                                             nullptr, nullptr, 0, nq, R, 1, span);
  else if (fixed_len == 1500 && xattn_nbc)
    dec_attn_kernel<T, false, 8, false, 6><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale,
                                                              kbase, vbase, kv_index, pos, active,
                                                              fixed_len, kv_len_cap, o, H, scale,
                                                              nullptr, nullptr, 0, nq, R, 1, span);
  else if (xattn_nt)
    dec_attn_kernel<T, false, 8, true><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale,
                                                          kbase, vbase, kv_index, pos, active,
                                                          fixed_len, kv_len_cap, o, H, scale,
                                                          nullptr, nullptr, 0, nq, R, 1, span);
  else
    dec_attn_kernel<T, false, 8, false><<<g, 256, 0, st>>>(P, KS, pcols, bias, qscale, kscale,
                                                           kbase, vbase, kv_index, pos, active,
                                                           fixed_len, kv_len_cap, o, H, scale,
                                                           nullptr, nullptr, 0, nq, R, 1, span);
}

template void enc_attention<_Float16>(const _Float16*, const _Float16*, const _Float16*, _Float16*,
                                      int, int, int, float, hipStream_t);
template void enc_attention<__bf16>(const _Float16*, const _Float16*, const _Float16*, __bf16*, int,
                                    int, int, float, hipStream_t);
template void dec_attention<_Float16>(const float*, int, int, const float*, float, float,
                                      _Float16*, _Float16*, const int*, const int*, const int*, int,
                                      int, _Float16*, int, int, float, hipStream_t, const int*,
                                      const int*, int, int, int, unsigned long long*);
template void dec_attention<__bf16>(const float*, int, int, const float*, float, float, _Float16*,
                                    _Float16*, const int*, const int*, const int*, int, int,
                                    __bf16*, int, int, float, hipStream_t, const int*, const int*, int, int,
                                    int, unsigned long long*);

}  // namespace mwx
