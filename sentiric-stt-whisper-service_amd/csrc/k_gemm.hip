// MFMA GEMMs for gfx950 with ggml-faithful fused epilogues.
//
// C[m][n] = sum_k A[m][k] * W[n][k]: both operands K-contiguous (W is the ggml
// [out][in] weight layout), f16 or bf16 inputs, f32 accumulation on
// v_mfma_f32_16x16x32_{f16,bf16}. Replaces ggml_mul_mat (+ the ggml_add /
// ggml_scale / ggml_gelu / ggml_cpy nodes that follow it in whisper.cpp's
// encoder, cross and decoder graphs — SURVEY.md §2.2 rows 2-11).
//
// Two kernels:
//  * gemm_big:    256x256x64 tiles, 8 waves (2x4, 128x64 per wave), operands
//                 DMA'd (global_load_lds) into double-buffered LDS with an XOR
//                 swizzle (16-B chunk ^= (row >> 1) & 7) so the ds_read_b128
//                 fragment reads are bank-conflict free; a 2-stage ring
//                 (or an 8-phase schedule, MWX_GEMM_8PH=1). Encoder / conv / cross-KV GEMMs
//                 (M = clips x 1500).
//  * gemm_skinny: decode GEMMs (M <= 64 rows): weight-streaming, fragments
//                 loaded straight to VGPRs (no LDS round trip), 4 waves split
//                 K (or N for wide outputs), LDS reduction, one 16-column
//                 strip per wave.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "kcommon.h"
#include "kernels.h"
#include "ln_core.h"

namespace mwx {

template <int EPI, typename T, bool OUT16>
__device__ __forceinline__ void epi_store(const EpiParams& P, int bz, int m, int n, float acc) {
  if constexpr (EPI == EPI_ENC_QKV) {
    const int d = P.d;
    const int part = n / d;
    const int nn = n - part * d;
    const int h = nn >> 6, e = nn & 63;
    const int b = m / P.L, t = m - b * P.L;
    const _Float16 hv = f16r(acc + P.bias[n]);
    if (part == 0)
      P.q[(((long)b * P.H + h) * P.L + t) * 64 + e] = hv;
    else if (part == 1)
      P.k[(((long)b * P.H + h) * P.L + t) * 64 + e] = hv;
    else
      P.v[(((long)b * P.H + h) * 64 + e) * P.ldv + t] = hv;
  } else if constexpr (EPI == EPI_GELU) {
    const float g = gelu_ggml(acc + P.bias[n]);
    const long idx = P.pack_out ? pack_index(m, n, P.ldc)
                                : (long)bz * P.c_bstride + (long)m * P.ldc + n;
    if constexpr (OUT16)
      ((_Float16*)P.c16)[idx] = (_Float16)g;
    else
      ((T*)P.c16)[idx] = to_t<T>(g);
  } else if constexpr (EPI == EPI_RES) {
    if (P.active && !P.active[m]) return;  // (decode: an inactive row's residual is left alone)
    const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + n;
    const float b = P.bias ? P.bias[n] : 0.0f;
    P.c32[idx] = (acc + b) + P.r32[idx];
  } else if constexpr (EPI == EPI_CONV2) {
    const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + n;
    P.c32[idx] = P.pe[(long)m * P.ldc + n] + gelu_ggml(acc + P.bias[n]);
  } else if constexpr (EPI == EPI_F32) {
    P.c32[(long)bz * P.c_bstride + (long)m * P.ldc + n] = acc;
  } else if constexpr (EPI == EPI_CROSS_KV) {
    const int d = P.d;
    const int layer = n / (2 * d);
    const int r = n - layer * 2 * d;
    const int kv = r >= d;
    const int nn = r - kv * d;
    const int h = nn >> 6, e = nn & 63;
    const int bl = m / P.L, t = m - bl * P.L;
    const long idx = ((((long)layer * P.ncap + P.slot[bl]) * P.H + h) * P.L + t) * 64 + e;
    if (!kv)
      P.k[idx] = f16r(acc * P.kscale);
    else
      P.v[idx] = f16r(acc + P.bias[n]);
  } else if constexpr (EPI == EPI_DEC_QKV) {
    if (!P.active[m]) return;
    const int d = P.d;
    const int part = n / d;
    const int nn = n - part * d;
    const int h = nn >> 6, e = nn & 63;
    if (part == 0) {
      P.q[(long)m * d + nn] = f16r((acc + P.bias[n]) * P.qscale);
    } else {
      const long idx = (((long)m * P.H + h) * P.L + P.pos[m]) * 64 + e;
      if (part == 1)
        P.k[idx] = f16r(acc * P.kscale);
      else
        P.v[idx] = f16r(acc + P.bias[n]);
    }
  } else if constexpr (EPI == EPI_STORE16) {
    ((_Float16*)P.c16)[(long)m * P.ldc + n] = f16r(acc + P.bias[n]);
  }
}

template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 ld8(const T* p) {
  return *reinterpret_cast<const typename Elt<T>::v8*>(p);
}

// MX-fp8 decode weights (MWX_COMPUTE_MXFP8, bf16 models): the fragment tiles
// hold e4m3 codes (1 byte per element, pack_index order) and one E8M0 scale
// per (column, 32-deep k-step): S[(strip * KT + kt) * 16 + column % 16]. A
// lane's 8 codes of a k-step share that scale; they are widened to bf16 in
// registers (v_cvt_scalef32_pk_bf16_fp8: code x 2^(scale - 127), exact) and
// the MFMA runs on bf16 as for 16-bit weights (weight-only fp8: half the
// weight bytes, activations unchanged).
__device__ __forceinline__ float e8m0_to_f32(uint32_t e) {
  return e ? __uint_as_float(e << 23) : __uint_as_float(0x00400000u);
}
template <typename T>
__device__ __forceinline__ typename Elt<T>::v8 dequant8(uint2 raw, float sc) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  t2 a, b, c, d;
  if constexpr (std::is_same<T, __bf16>::value) {
    a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw.x, sc, false);
    b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw.x, sc, true);
    c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw.y, sc, false);
    d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw.y, sc, true);
  } else {
    a = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.x, sc, false);
    b = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.x, sc, true);
    c = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.y, sc, false);
    d = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(raw.y, sc, true);
  }
  return typename Elt<T>::v8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// ---------------------------------------------------------------------------
// big tile GEMM (encoder, conv stem, cross K/V: M = clips x 1500 rows)
//
// 256x256 output tile per 512-thread workgroup (one per CU, 128 KB LDS), 8
// waves as 2 (M) x 4 (N), each wave 128x64 outputs = 8x4 MFMA 16x16 fragments.
// K advances in 64-deep tiles through a 2-stage LDS ring filled by LDS DMA
// (global_load_lds, 16 B per lane): while the MFMAs of tile k run, tile k+1
// lands in the other stage; one counted wait + raw barrier per tile. Measured
// on the large-v3 encoder shapes (scripts/probe/gemm_variants.hip): 0.92-1.07
// PFLOP/s vs 0.37-0.63 for a 128x128 register-staged tile.
// ---------------------------------------------------------------------------
constexpr int BM = 256, BN = 256, BK = 64;
#ifndef GEMM_PRIO
#define GEMM_PRIO 1
#endif
constexpr int GWM = 2, GWN = 4;                  // wave grid
constexpr int GFM = BM / GWM / 16, GFN = BN / GWN / 16;  // 8 x 4 fragments per wave
#ifndef GEMM_STAGES
// 16-bit operands: LDS ring of 2 x 64-deep tiles (default) or 4 x 32-deep
// tiles (three in flight); measured on the encoder shapes 817 vs 734 TF/s:
// the 32-deep tile's extra barrier and fragment-read restart per 32 k cost
// more than the deeper ring recovers
#define GEMM_STAGES 2
#endif

// MX = true: A and W are MX-fp8 (e4m3 bytes, one E8M0 scale per 32 k of a row:
// P.sa [M][K/32], P.sw [N][K/32]); a K tile is 128 deep (the same 128 B per
// row as a 64-deep 16-bit tile, so staging and swizzle are unchanged) and is
// one v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair. Operand layout of
// that instruction (pinned on the GPU, scripts/probe/mfma_scale_probe2.hip):
// lane l holds row l&15, k = 16*(l>>4) + [0,16) in bytes 0-15 and
// 64 + 16*(l>>4) + [0,16) in bytes 16-31 -- exactly the 16-B chunks (l>>4)
// and 4+(l>>4) of the row -- and its scale operand is that row's scale of
// k block l>>4.
// PH8 (16-bit operands): the main loop as an 8-phase schedule (two 64-deep K
// tiles per iteration, four phases per tile; MI355X guide §5 "256² 8-phase
// template", T3 + T4): the waves of wave-row 1 run one barrier behind those
// of wave-row 0, so on every SIMD one wave's 16-MFMA cluster overlaps the
// other wave's LDS fragment reads and LDS-DMA issue. The LDS image of a K tile
// is four half-tiles of 128 rows: HA0 / HA1 = the A rows of quadrant row 0 / 1
// of both wave rows, HB0 / HB1 = the W rows of quadrant column 0 / 1 of all
// four wave columns; each phase DMAs one half-tile (2 instructions per wave)
// and waits with a counted vmcnt that keeps four half-tiles in flight. A
// wave's quadrants are computed in the order (0,0), (0,1), (1,0), (1,1), each
// output fragment still accumulating its K in the same order as the 2-stage
// loop (tile by tile, 32-deep sub-steps 0, 1): bit-identical results.
template <typename T, int EPI, bool OUT16, bool MX = false, bool PH8 = false>
__global__ __launch_bounds__(512, 1) void gemm_big(const void* __restrict__ Av, long lda,
                                                   long a_bstride, const void* __restrict__ Wv,
                                                   long ldw, int M, int N, int K, EpiParams P) {
  using V8 = typename Elt<T>::v8;
  using TE = typename std::conditional<MX, uint8_t, T>::type;  // operand element
  constexpr int CE = 16 / sizeof(TE);                          // elements per 16-B chunk
  // ring: NSTG stages of (BM + BN) rows x RBY bytes (128 KB in total): 16-bit
  // operands 2 x 64-deep (or GEMM_STAGES = 4: 4 x 32-deep), MX-fp8 2 x 128-deep
  constexpr int NSTG = MX ? 2 : GEMM_STAGES;
  constexpr int RBY = MX ? 128 : (GEMM_STAGES == 4 ? 64 : 128);  // bytes per row per tile
  constexpr int CPR = RBY / 16;                                  // 16-B chunks per row
  constexpr int RPI = 64 / CPR;                                  // rows per 1-KB DMA instruction
  constexpr int BKE = CPR * CE;                                  // K-tile depth (elements)
  constexpr int GDA = BM / RPI / 8, GDB = BN / RPI / 8;          // DMA instructions per wave per tile
  // chunk swizzle: 16 consecutive rows read one chunk column conflict-free.
  // 128-B rows: a 256-B bank row holds rows 2m and 2m + 1, so the slot is
  // XORed with (row >> 1) & 7 -- rows 2m / 2m + 1 then take 16-B slots kc ^ m
  // in the two halves of the bank row, 16 distinct slots for 16 rows (with
  // (row & 7), rows r and r + 8 shared banks: 2-way conflicts on every read)
  auto swz = [](int row) { return CPR == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3); };
  span_start(P.span);
  const TE* A = reinterpret_cast<const TE*>(Av);
  const TE* W = reinterpret_cast<const TE*>(Wv);
  // one __shared__ array only (a second one can make hipcc drain the LDS DMA
  // before every ds_read): [stage][A rows 0..255 | W rows 0..255][128 B].
  // EPI_GELU: after the main loop, bytes [0, 64 KB) stage the outputs (8 waves
  // x 64 rows x 64 columns of 16 bits) and the GELU table follows at GT_OFF
  constexpr int RING_B = NSTG * (BM + BN) * BKE * (int)sizeof(TE);
  constexpr int GT_OFF = 65536;
  constexpr int LDS_B =
      EPI == EPI_GELU ? (RING_B > GT_OFF + 2 * GELU_TAB_N ? RING_B : GT_OFF + 2 * GELU_TAB_N) : RING_B;
  __shared__ __attribute__((aligned(16))) TE lds_raw[LDS_B / sizeof(TE)];
  TE(*lds)[(BM + BN) * BKE] = reinterpret_cast<TE(*)[(BM + BN) * BKE]>(lds_raw);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / GWN, wn = wid % GWN;
  const int nbn = (N + BN - 1) / BN;
  // XCD-aware tile order (bijective remap): workgroups are placed round-robin
  // over the 8 XCDs (id % 8), so consecutive tile ids -- the column tiles of
  // one row tile, sharing its A rows -- are given to workgroups of one XCD
  // and the A tile is fetched into that XCD's L2 once
  //
  // Grouped order (P.group_m = G > 0, the default): the logical tile ids of
  // that contiguous range walk G row tiles before moving to the next column
  // tile, so the ~32 workgroups an XCD runs at once cover G row tiles x 32/G
  // column tiles and share both operand tiles in its 4-MiB L2 (row-major:
  // 1-2 row tiles x every column tile, whose W slices miss L2 once per row
  // tile: the all-layer cross-K/V GEMM re-read its 210-MB W ~188 times).
  int wgid = blockIdx.x;
  if (P.xcd_remap) {
    const int nwg = gridDim.x, xcd = wgid % 8, q = nwg / 8, r = nwg % 8;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wgid / 8;
  }
  int mt = wgid / nbn, nt = wgid % nbn;
  if (P.group_m > 0) {
    const int nbm = (M + BM - 1) / BM;
    const int per = P.group_m * nbn, g = wgid / per, i = wgid - g * per;
    const int gm = min(P.group_m, nbm - g * P.group_m);
    mt = g * P.group_m + i % gm;
    nt = i / gm;
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int bz = blockIdx.y;
  A += (long)bz * a_bstride;
  // LDS DMA: one wave instruction fills 1 KB = 8 rows x 128 B of the tile
  // image linearly in lane order; the XOR swizzle (16-B chunk slot =
  // kc ^ swz(row), conflict-free fragment reads) is applied on the SOURCE
  // address. Rows past M / N are clamped (their outputs are discarded).
  const int lr = lane / CPR, ls = lane % CPR;
  const TE* asrc[GDA];
  const TE* wsrc[GDB];
#pragma unroll
  for (int i = 0; i < GDA; ++i) {
    const int r = (wid * GDA + i) * RPI + lr;
    asrc[i] = A + (long)min(m0 + r, M - 1) * lda + (ls ^ swz(r)) * CE;
  }
#pragma unroll
  for (int i = 0; i < GDB; ++i) {
    const int r = (wid * GDB + i) * RPI + lr;
    wsrc[i] = W + (long)min(n0 + r, N - 1) * ldw + (ls ^ swz(r)) * CE;
  }
  // MX scale rows of this lane's fragments (row = fragment row l&15)
  const int ksb = K / 32;
  const uint8_t* sap[GFM];
  const uint8_t* swp[GFN];
  if constexpr (MX) {
#pragma unroll
    for (int i = 0; i < GFM; ++i)
      sap[i] = P.sa + (long)bz * P.sa_bstride +
               (long)min(m0 + wm * (BM / GWM) + i * 16 + (lane & 15), M - 1) * ksb + (lane >> 4);
#pragma unroll
    for (int j = 0; j < GFN; ++j)
      swp[j] = P.sw + (long)min(n0 + wn * (BN / GWN) + j * 16 + (lane & 15), N - 1) * ksb +
               (lane >> 4);
  }
#define GLDS(kt, st)                                                                        \
  do {                                                                                      \
    const int ko = (kt) * BKE;                                                              \
    _Pragma("unroll") for (int i = 0; i < GDA; ++i) __builtin_amdgcn_global_load_lds(       \
        (const void __attribute__((address_space(1)))*)(asrc[i] + ko),                      \
        (void __attribute__((address_space(3)))*)(&lds[st][((wid * GDA + i) * RPI) * BKE]), 16, \
        0, 0);                                                                              \
    _Pragma("unroll") for (int i = 0; i < GDB; ++i) __builtin_amdgcn_global_load_lds(       \
        (const void __attribute__((address_space(1)))*)(wsrc[i] + ko),                      \
        (void __attribute__((address_space(3)))*)(&lds[st][(BM + (wid * GDB + i) * RPI) * BKE]), \
        16, 0, 0);                                                                          \
  } while (0)

  f32x4 acc[GFM][GFN];
#pragma unroll
  for (int i = 0; i < GFM; ++i)
#pragma unroll
    for (int j = 0; j < GFN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const int nk = K / BKE;
  if constexpr (PH8) {
    static_assert(!MX && CPR == 8 && NSTG == 2, "8-phase schedule: 16-bit operands, 64-deep tiles");
    constexpr int HT = 128 * 64;  // elements per half-tile (128 rows x 128 B)
    // DMA sources: instruction i (0, 1) of this wave fills half-tile rows
    // (2 wid + i) * 8 + lr; half-tile h: 0 = HA0, 1 = HA1, 2 = HB0, 3 = HB1
    const TE* hs[4][2];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = (wid * 2 + i) * 8 + lr, q = h & 1;
        if (h < 2) {
          const int gr = m0 + (r >> 6) * 128 + q * 64 + (r & 63);
          hs[h][i] = A + (long)min(gr, M - 1) * lda + (ls ^ swz(r)) * CE;
        } else {
          const int gr = n0 + (r >> 5) * 64 + q * 32 + (r & 31);
          hs[h][i] = W + (long)min(gr, N - 1) * ldw + (ls ^ swz(r)) * CE;
        }
      }
    // stage s of the sequence: tile s / 4, half-tile HA0, HB0, HB1, HA1 by s % 4
    // (K, the phase and the stage order are wave-uniform; H is compile-time)
#define STAGE8(H, tile)                                                                     \
    do {                                                                                    \
      const int t_ = (tile);                                                                \
      if (t_ < nk) {                                                                        \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) __builtin_amdgcn_global_load_lds(    \
            (const void __attribute__((address_space(1)))*)(hs[H][i] + t_ * BKE),           \
            (void __attribute__((address_space(3)))*)(&lds_raw[((t_ & 1) * 4 + (H)) * HT +  \
                                                               (wid * 2 + i) * 8 * BKE]),   \
            16, 0, 0);                                                                      \
      }                                                                                     \
    } while (0)
    // outstanding stages allowed after phase P's wait: stages <= P + 2 must
    // have landed (read from phase P + 1 on, after the barriers); issued so
    // far: min(P + 7, 4 nk)
    auto wait_stages = [&](int issued, int retire_upto) {
      const int out = min(max(issued - (retire_upto + 1), 0), 4);
      switch (out) {
        case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    };
    // prologue: tile 0 (all four) and tile 1's HA0 / HB0
    STAGE8(0, 0);
    STAGE8(2, 0);
    STAGE8(3, 0);
    STAGE8(1, 0);
    STAGE8(0, 1);
    STAGE8(2, 1);
    wait_stages(min(6, 4 * nk), 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // wave row 1 runs one barrier behind (a scalar branch: the condition is
    // provably wave-uniform)
    const bool lag = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;
    if (lag) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    V8 af[2][4], b0[2][2], b1[2][2];
    auto rd_a = [&](int h, int buf) {
      const TE* base = &lds_raw[(buf * 4 + h) * HT];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kc = s2 * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + (lane & 15);
          af[s2][i] = *reinterpret_cast<const V8*>(base + row * BKE + ((kc ^ swz(row)) << 3));
        }
      }
    };
    auto rd_b = [&](V8 (&bb)[2][2], int h, int buf) {
      const TE* base = &lds_raw[(buf * 4 + h) * HT];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kc = s2 * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wn * 32 + j * 16 + (lane & 15);
          bb[s2][j] = *reinterpret_cast<const V8*>(base + row * BKE + ((kc ^ swz(row)) << 3));
        }
      }
    };
    auto mfma_q = [&](int qm, int qn, V8 (&bb)[2][2]) {
      if (GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qm * 4 + i][qn * 2 + j] = Elt<T>::mfma(af[s2][i], bb[s2][j], acc[qm * 4 + i][qn * 2 + j]);
      if (GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
    };
    // one phase: fragment reads + one stage + counted wait | barrier |
    // lgkmcnt(0) + the quadrant's 16 MFMAs | barrier
#define PHASE8(PH, READS, SH, STILE, MF)                                  \
    do {                                                                   \
      READS;                                                               \
      STAGE8(SH, STILE);                                                   \
      wait_stages(min(phi + 7, 4 * nk), phi + 2);                          \
      __builtin_amdgcn_sched_barrier(0);                                   \
      __builtin_amdgcn_s_barrier();                                        \
      __builtin_amdgcn_sched_barrier(0);                                   \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                   \
      MF;                                                                  \
      __builtin_amdgcn_sched_barrier(0);                                   \
      __builtin_amdgcn_s_barrier();                                        \
      __builtin_amdgcn_sched_barrier(0);                                   \
      ++phi;                                                               \
    } while (0)
    int phi = 0;  // phase index (4 per K tile)
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      PHASE8(0, (rd_a(0, buf), rd_b(b0, 2, buf)), 3, kt + 1, mfma_q(0, 0, b0));
      PHASE8(1, rd_b(b1, 3, buf), 1, kt + 1, mfma_q(0, 1, b1));
      PHASE8(2, rd_a(1, buf), 0, kt + 2, mfma_q(1, 0, b0));
      PHASE8(3, (void)0, 2, kt + 2, mfma_q(1, 1, b1));
    }
#undef PHASE8
#undef STAGE8
    if (!lag) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
#pragma unroll
  for (int t = 0; t < NSTG - 1; ++t)
    if (t < nk) GLDS(t, t);
  // MX: each tile's scales are requested one tile ahead, right after that
  // tile's DMA, so the counted wait that lands the tile lands its scales too
  // (requested at the top of their own tile they exposed an L2 round trip at
  // every tile's wait)
  int sa_n[MX ? GFM : 1], sw_n[MX ? GFN : 1];
  if constexpr (MX) {
#pragma unroll
    for (int i = 0; i < GFM; ++i) sa_n[i] = sap[i][0];
#pragma unroll
    for (int j = 0; j < GFN; ++j) sw_n[j] = swp[j][0];
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NSTG;
    int sa_k[MX ? GFM : 1], sw_k[MX ? GFN : 1];
    if constexpr (MX) {
#pragma unroll
      for (int i = 0; i < GFM; ++i) sa_k[i] = sa_n[i];
#pragma unroll
      for (int j = 0; j < GFN; ++j) sw_k[j] = sw_n[j];
    }
    // tile kt has landed (this wave's DMA), then the barrier makes every
    // wave's part visible and orders all reads of the other stage (tile kt-1)
    // before it is refilled below
    // (tiles issued after kt may stay in flight: counted wait)
    {
      const int after = min(NSTG - 2, nk - 1 - kt);
      if constexpr (NSTG == 4) {
        if (after >= 2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (BM / 16 / 8 + BN / 16 / 8)) : "memory");
        else if (after == 1)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BM / 16 / 8 + BN / 16 / 8) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NSTG - 1 < nk) GLDS(kt + NSTG - 1, (kt + NSTG - 1) % NSTG);
    if constexpr (MX) {
      if (kt + 1 < nk) {
#pragma unroll
        for (int i = 0; i < GFM; ++i) sa_n[i] = sap[i][(kt + 1) * 4];
#pragma unroll
        for (int j = 0; j < GFN; ++j) sw_n[j] = swp[j][(kt + 1) * 4];
      }
      typedef int v8i __attribute__((ext_vector_type(8)));
      v8i af[GFM], bf[GFN];
      const int g = lane >> 4;
#pragma unroll
      for (int i = 0; i < GFM; ++i) {
        const int row = wm * (BM / GWM) + i * 16 + (lane & 15);
        const uint4 lo = *reinterpret_cast<const uint4*>(&lds[cur][row * BKE + ((g ^ swz(row)) << 4)]);
        const uint4 hi =
            *reinterpret_cast<const uint4*>(&lds[cur][row * BKE + (((4 + g) ^ swz(row)) << 4)]);
        af[i] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int j = 0; j < GFN; ++j) {
        const int row = BM + wn * (BN / GWN) + j * 16 + (lane & 15);
        const uint4 lo = *reinterpret_cast<const uint4*>(&lds[cur][row * BKE + ((g ^ swz(row)) << 4)]);
        const uint4 hi =
            *reinterpret_cast<const uint4*>(&lds[cur][row * BKE + (((4 + g) ^ swz(row)) << 4)]);
        bf[j] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int i = 0; i < GFM; ++i)
#pragma unroll
        for (int j = 0; j < GFN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              af[i], bf[j], acc[i][j], 0, 0, 0, sa_k[i], 0, sw_k[j]);
    } else {
      // both 32-deep sub-steps' fragments are read up front: the MFMAs of
      // sub-step 0 wait only for their own 12 reads (counted lgkmcnt) while
      // sub-step 1's are in flight
      constexpr int NSUB = CPR / 4;
      V8 af[NSUB][GFM], bf[NSUB][GFN];
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        const int kc = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < GFM; ++i) {
          const int row = wm * (BM / GWM) + i * 16 + (lane & 15);
          af[s][i] = *reinterpret_cast<const V8*>(&lds[cur][row * BKE + ((kc ^ swz(row)) << 3)]);
        }
#pragma unroll
        for (int j = 0; j < GFN; ++j) {
          const int row = BM + wn * (BN / GWN) + j * 16 + (lane & 15);
          bf[s][j] = *reinterpret_cast<const V8*>(&lds[cur][row * BKE + ((kc ^ swz(row)) << 3)]);
        }
      }
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < GFM; ++i)
#pragma unroll
          for (int j = 0; j < GFN; ++j) acc[i][j] = Elt<T>::mfma(af[s][i], bf[s][j], acc[i][j]);
        if (GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
      }
    }
    // this wave's reads of `cur` have returned before its next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  }  // (2-stage loop)
#undef GLDS
  const int wr0 = m0 + wm * (BM / GWM), wc0 = n0 + wn * (BN / GWN);
  constexpr bool STAGED16 = EPI == EPI_GELU || EPI == EPI_ENC_QKV || EPI == EPI_CROSS_KV;
  constexpr bool STAGED32 = EPI == EPI_RES || EPI == EPI_CONV2;
  if ((STAGED16 || STAGED32) && (N & 63) == 0 && !P.pack_out) {
    // Epilogue through LDS: the ring is idle now; each wave stages its 128x64
    // tile (16 KB) so every global store is a 16-B (8-B for V^T) vector.
    // Staging swizzles (bit-identical: layout only). A fragment store writes
    // rows 4g + r (lane group g = lane >> 4) of 16 columns, so without a
    // swizzle the four groups' rows (512 B apart) land on the same banks
    // (4-way), and the V^T image's 16 e-rows of one t (256 B apart) on one
    // bank (16-way; PMC r05: 0.39 of the QKV launch's LDS cycles conflicted).
    //   16-bit row-major [row][64]: 16-B chunk ^ sw16(row) = ((row >> 2) & 3) << 1
    //   f32 row-major [row][64]:    16-B chunk ^ sw32(row) = ((row >> 2) & 3) << 2
    //   V^T [e][128 t], 8-B (4-t) stores: 8-B chunk ^ swv(e) = (e & 15) << 1
    // so every store instruction covers distinct banks and the 16-B / 8-B
    // read-outs stay row-contiguous permutations (conflict-free).
    auto sw16 = [](int row) { return ((row >> 2) & 3) << 1; };
    auto sw32 = [](int row) { return ((row >> 2) & 3) << 2; };
    auto swv = [](int e) { return (e & 15) << 1; };
    __builtin_amdgcn_s_barrier();  // all waves are past their last ring read
    uint16_t* gtl = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(lds_raw) + GT_OFF);
    if constexpr (EPI == EPI_GELU) {
      if (P.gelu_tab) {  // (uniform) the table into LDS, 16 B per thread and step
        for (int i = tid; i < GELU_TAB_N / 8; i += 512)
          reinterpret_cast<uint4*>(gtl)[i] = reinterpret_cast<const uint4*>(P.gelu_tab)[i];
        __syncthreads();
      }
    }
    if (wc0 >= N) {                // (N % 64 == 0: a wave's 64 columns are all in or all out)
      span_end(P.span);
      return;
    }
    uint16_t* wl = reinterpret_cast<uint16_t*>(&lds[0][0]) + wid * 8192;
    float* wlf = reinterpret_cast<float*>(wl);
    if constexpr (EPI == EPI_GELU) {
      // two 64-row halves of the wave tile through 8 KB of LDS per wave
      uint16_t* wg = reinterpret_cast<uint16_t*>(&lds[0][0]) + wid * 4096;
      auto half = [&](int hh, auto tabc) {
        constexpr bool TB = decltype(tabc)::value;
#pragma unroll
        for (int i = hh * (GFM / 2); i < (hh + 1) * (GFM / 2); ++i)
#pragma unroll
          for (int j = 0; j < GFN; ++j) {
            const int lc = j * 16 + (lane & 15);
            const float bv = P.bias[wc0 + lc];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int lr = (i - hh * (GFM / 2)) * 16 + (lane >> 4) * 4 + r;
              const float a = acc[i][j][r] + bv;
              const float g = TB ? gelu_ggml_tab(a, gtl) : gelu_ggml(a);
              uint16_t bits;
              if constexpr (OUT16) {
                bits = __builtin_bit_cast(uint16_t, (_Float16)g);
              } else {
                bits = __builtin_bit_cast(uint16_t, to_t<T>(g));
              }
              wg[lr * 64 + (((lc >> 3) ^ sw16(lr)) << 3) + (lc & 7)] = bits;
            }
          }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 4
        for (int it = 0; it < 8; ++it) {
          const int row = it * 8 + (lane >> 3), ch = lane & 7;
          const int m = wr0 + hh * 64 + row;
          if (m >= M) continue;
          const uint4 v = *reinterpret_cast<const uint4*>(&wg[row * 64 + ((ch ^ sw16(row)) << 3)]);
          _Float16* dst = reinterpret_cast<_Float16*>(P.c16) + (long)bz * P.c_bstride +
                          (long)m * P.ldc + wc0 + ch * 8;
          *reinterpret_cast<uint4*>(dst) = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      };
      if (P.gelu_tab) {
        half(0, std::true_type{});
        half(1, std::true_type{});
      } else {
        half(0, std::false_type{});
        half(1, std::false_type{});
      }
    } else if constexpr (STAGED16) {
      // a wave's 64 columns are one head (d % 64 == 0): part / layer / head / k|v
      int part = 0, h = 0, layer = 0;
      if constexpr (EPI == EPI_ENC_QKV) {
        part = wc0 / P.d;
        h = (wc0 - part * P.d) >> 6;
      } else if constexpr (EPI == EPI_CROSS_KV) {
        layer = wc0 / (2 * P.d);
        const int rr = wc0 - layer * 2 * P.d;
        part = rr >= P.d;
        h = (rr - part * P.d) >> 6;
      }
      const bool transposed = EPI == EPI_ENC_QKV && part == 2;  // V^T [e][t]
#pragma unroll
      for (int i = 0; i < GFM; ++i)
#pragma unroll
        for (int j = 0; j < GFN; ++j) {
          const int lc = j * 16 + (lane & 15);
          const int n = wc0 + lc;
          uint16_t bits[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = acc[i][j][r];
            if constexpr (EPI == EPI_ENC_QKV) {
              const _Float16 hv = f16r(a + P.bias[n]);
              bits[r] = __builtin_bit_cast(uint16_t, hv);
            } else {  // cross K: f16(acc * kscale); V: f16(acc + b)
              const _Float16 hv = part ? f16r(a + P.bias[n]) : f16r(a * P.kscale);
              bits[r] = __builtin_bit_cast(uint16_t, hv);
            }
          }
          const int lr0 = i * 16 + (lane >> 4) * 4;
          if (transposed) {  // the lane's 4 consecutive t of column e = lc: one 8-B store
            *reinterpret_cast<uint2*>(&wl[lc * 128 + (((lr0 >> 2) ^ swv(lc)) << 2)]) =
                uint2{(uint32_t)bits[0] | ((uint32_t)bits[1] << 16),
                      (uint32_t)bits[2] | ((uint32_t)bits[3] << 16)};
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              wl[(lr0 + r) * 64 + (((lc >> 3) ^ sw16(lr0 + r)) << 3) + (lc & 7)] = bits[r];
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (!transposed) {
        // 128 rows x 128 B: 8 rows per wave instruction
#pragma unroll 4
        for (int it = 0; it < 16; ++it) {
          const int row = it * 8 + (lane >> 3), ch = lane & 7;
          const int m = wr0 + row;
          if (m >= M) continue;
          const uint4 v = *reinterpret_cast<const uint4*>(&wl[row * 64 + ((ch ^ sw16(row)) << 3)]);
          if constexpr (EPI == EPI_CROSS_KV) {
            if (P.ks8) {
              // MX-fp8 cross K/V cache: each (time, head) row of 64 f16
              // values is two MX blocks of 32 (4 lanes x 8 values each):
              // block amax over the 4 lanes, E8M0 exponent, e4m3 codes
              const int b = m / P.L, t = m - b * P.L;
              const long ridx = (((long)layer * P.ncap + P.slot[b]) * P.H + h) * P.L + t;
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              float f[8];
              float amax = 0.0f;
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const uint16_t hb = (uint16_t)(w4[e >> 1] >> (16 * (e & 1)));
                f[e] = (float)__builtin_bit_cast(_Float16, hb);
                amax = fmaxf(amax, fabsf(f[e]));
              }
              amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
              amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
              const int ex = mx_exp(amax);
              const float inv = ldexpf(1.0f, -ex);
              uint32_t lo = 0, hi = 0;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                lo |= (uint32_t)e4m3_rne(f[e] * inv) << (8 * e);
                hi |= (uint32_t)e4m3_rne(f[4 + e] * inv) << (8 * e);
              }
              uint8_t* dq = reinterpret_cast<uint8_t*>(part ? P.v : P.k) + ridx * 64 + ch * 8;
              *reinterpret_cast<uint2*>(dq) = uint2{lo, hi};
              if ((ch & 3) == 0) (part ? P.vs8 : P.ks8)[ridx * 2 + (ch >> 2)] = (uint8_t)(127 + ex);
              continue;
            }
          }
          _Float16* dst;
          {
            const int b = m / P.L, t = m - b * P.L;
            if constexpr (EPI == EPI_ENC_QKV) {
              dst = (part == 0 ? P.q : P.k) + (((long)b * P.H + h) * P.L + t) * 64 + ch * 8;
            } else {
              const long idx =
                  ((((long)layer * P.ncap + P.slot[b]) * P.H + h) * P.L + t) * 64 + ch * 8;
              dst = (part ? P.v : P.k) + idx;
            }
          }
          *reinterpret_cast<uint4*>(dst) = v;
        }
      } else {
        // V^T: 64 rows (e) x 128 t; 4-t groups (8 B) never straddle a clip
        // (L % 4 == 0, m0 % 4 == 0)
#pragma unroll 4
        for (int it = 0; it < 32; ++it) {
          const int e = it * 2 + (lane >> 5), tg = lane & 31;
          const int m = wr0 + tg * 4;
          if (m >= M) continue;
          const uint2 v = *reinterpret_cast<const uint2*>(&wl[e * 128 + ((tg ^ swv(e)) << 2)]);
          const int b = m / P.L, t = m - b * P.L;
          *reinterpret_cast<uint2*>(P.v + (((long)b * P.H + h) * 64 + e) * P.ldv + t) = v;
        }
      }
    } else {
      // f32 outputs (residual stream): two 64-row halves of the wave tile.
      // The half's residual (EPI_RES) / positional rows (EPI_CONV2) are
      // requested before its staging, so their latency runs under it
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x4 rin[16];
#pragma unroll
        for (int it = 0; it < 16; ++it) {
          const int row = it * 4 + (lane >> 4), ch = lane & 15;
          const int m = wr0 + hh * 64 + row;
          if (m < M) {
            if constexpr (EPI == EPI_RES)
              rin[it] = *reinterpret_cast<const f32x4*>(P.r32 + (long)bz * P.c_bstride +
                                                         (long)m * P.ldc + wc0 + ch * 4);
            else
              rin[it] = *reinterpret_cast<const f32x4*>(P.pe + (long)m * P.ldc + wc0 + ch * 4);
          }
        }
#pragma unroll
        for (int i = hh * (GFM / 2); i < (hh + 1) * (GFM / 2); ++i)
#pragma unroll
          for (int j = 0; j < GFN; ++j) {
            const int lc = j * 16 + (lane & 15);
            const float bv = P.bias ? P.bias[wc0 + lc] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int lr = (i - hh * (GFM / 2)) * 16 + (lane >> 4) * 4 + r;
              const float a = acc[i][j][r] + bv;
              wlf[lr * 64 + (((lc >> 2) ^ sw32(lr)) << 2) + (lc & 3)] = EPI == EPI_CONV2 ? gelu_ggml(a) : a;
            }
          }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int it = 0; it < 16; ++it) {
          const int row = it * 4 + (lane >> 4), ch = lane & 15;
          const int m = wr0 + hh * 64 + row;
          if (m >= M) continue;
          const f32x4 v = *reinterpret_cast<const f32x4*>(&wlf[row * 64 + ((ch ^ sw32(row)) << 2)]);
          const long idx = (long)bz * P.c_bstride + (long)m * P.ldc + wc0 + ch * 4;
          f32x4 o;
          if constexpr (EPI == EPI_RES)
            o = v + rin[it];  // (acc + bias) + residual
          else
            o = rin[it] + v;  // pe + gelu(acc + bias)
          *reinterpret_cast<f32x4*>(P.c32 + idx) = o;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    span_end(P.span);
    return;
  }
#pragma unroll
  for (int i = 0; i < GFM; ++i)
#pragma unroll
    for (int j = 0; j < GFN; ++j) {
      const int n = wc0 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wr0 + i * 16 + (lane >> 4) * 4 + r;
        if (m < M && n < N) epi_store<EPI, T, OUT16>(P, bz, m, n, acc[i][j][r]);
      }
    }
  span_end(P.span);
}

// the f16 GELU table (kernels.h GELU_TAB_*): gelu_ggml's expression for every
// f16 input of magnitude <= 10, by the same device code
__global__ void gelu_table_kernel(uint16_t* __restrict__ tab) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= GELU_TAB_N) return;
  uint16_t out = 0;
  if (i < 2 * GELU_TAB_HALF) {
    const int neg = i >= GELU_TAB_HALF;
    const uint16_t hb = (uint16_t)((i - neg * GELU_TAB_HALF) | (neg << 15));
    const float xh = (float)__builtin_bit_cast(_Float16, hb);
    out = __builtin_bit_cast(uint16_t, f16r(gelu_f32(xh)));
  }
  tab[i] = out;
}

void gelu_table_build(uint16_t* tab, hipStream_t st) {
  gelu_table_kernel<<<(GELU_TAB_N + 255) / 256, 256, 0, st>>>(tab);
}

// ---------------------------------------------------------------------------
// skinny (decode) GEMM: M <= 16*MT rows. One workgroup = one 16-column strip;
// its NW waves split K, each wave owns KCH consecutive 32-deep k-steps and
// issues all of its W and A fragment loads before the first MFMA (one memory
// round trip per launch), then the NW partial tiles are summed through LDS.
// ---------------------------------------------------------------------------
template <int EPI, typename T, bool OUT16>
__device__ __forceinline__ void skinny_store(const EpiParams& P, int m, int n, float v) {
  epi_store<EPI, T, OUT16>(P, 0, m, n, v);
}

// LNF (M = 1, MT = 1): the A operand is the folded LayerNorm of the row
// (LnFuse, ln_core.h), as gemm_splitk LNF.
template <typename T, int MT, int KCH, bool W8 = false, bool LNF = false>
__global__ __launch_bounds__(1024) void gemm_skinny(int epi, const T* __restrict__ Ap,
                                                    const void* __restrict__ Wv,
                                                    const uint8_t* __restrict__ Ws, int KT, int M,
                                                    int N, EpiParams P, LnFuse ln) {
  static_assert(!LNF || MT == 1, "the folded LayerNorm serves one row");
  using V8 = typename Elt<T>::v8;
  __shared__ f32x4 red[16][MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int bx = blockIdx.x, by = blockIdx.y;
  const int n0 = bx * 16;
  // row block of 16*MT rows (grid.y): per-row arithmetic does not depend on M
  // nor on the block size (each output is the same MFMA chain over k)
  const int m_base = by * 16 * MT;
  const int Mb = min(16 * MT, M - m_base);
  const int kt0 = wid * KCH;
  const long f0 = (long)bx * KT + kt0;  // first weight fragment of this wave
  V8 bfr[KCH];
  V8 afr[MT][KCH];
  uint2 wraw[W8 ? KCH : 1];
  uint32_t wsc[W8 ? KCH : 1];
  if constexpr (W8) {
    const uint8_t* wq = reinterpret_cast<const uint8_t*>(Wv) + f0 * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      wraw[c] = *reinterpret_cast<const uint2*>(wq + c * 512);
      wsc[c] = Ws[(f0 + c) * 16 + (lane & 15)];
    }
  } else {
    const T* wt = reinterpret_cast<const T*>(Wv) + f0 * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < KCH; ++c) bfr[c] = ld8(wt + c * 512);
  }
  if constexpr (LNF) {
    __shared__ double lnred[2][4];
    __shared__ __attribute__((aligned(16))) T srow[2048];
    ln_fold_prologue<T>(ln, KT * 32, bx == 0 && by == 0, srow, lnred);
#pragma unroll
    for (int c = 0; c < KCH; ++c) afr[0][c] = ln_fold_frag<T>(srow, kt0 + c, lane);
  } else {
    const T* at = Ap + ((long)(by * MT) * KT + kt0) * 512 + lane * 8;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int c = 0; c < KCH; ++c) afr[mt][c] = ld8(at + ((long)mt * KT + c) * 512);
  }
  if constexpr (W8) {
#pragma unroll
    for (int c = 0; c < KCH; ++c) bfr[c] = dequant8<T>(wraw[c], e8m0_to_f32(wsc[c]));
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < KCH; ++c) acc[mt] = Elt<T>::mfma(afr[mt][c], bfr[c], acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    for (int w = 1; w < NW; ++w) acc[mt] += red[w][mt][lane];
  const int n = n0 + (lane & 15);
  if (n >= N) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ml = mt * 16 + (lane >> 4) * 4 + r;
      if (ml >= Mb) continue;
      const int m = m_base + ml;
      const float v = acc[mt][r];
      switch (epi) {
        case EPI_GELU: skinny_store<EPI_GELU, T, false>(P, m, n, v); break;
        case EPI_RES: skinny_store<EPI_RES, T, false>(P, m, n, v); break;
        case EPI_F32: skinny_store<EPI_F32, T, false>(P, m, n, v); break;
        case EPI_DEC_QKV: skinny_store<EPI_DEC_QKV, T, false>(P, m, n, v); break;
        case EPI_STORE16: skinny_store<EPI_STORE16, T, false>(P, m, n, v); break;
        default: break;
      }
    }
}

// ---------------------------------------------------------------------------
// Decode GEMMs at M > 64 rows (beam / best-of decoders: 160 rows at beam 5):
// the A block of a workgroup (16*MT rows x its K range, fragment tiles) is
// DMA'd into LDS once and shared by the workgroup's 4 waves, each of which
// owns one 16-column strip over the whole K range. gemm_skinny / gemm_splitk
// give every 16-column strip its own workgroup, which re-reads the whole A
// block from L2: at 160 rows that is N / 16 reads of it (FFN1: ~130 MB of L2
// traffic per launch, 13 us with warm weights in the chain probe).
// Each output is formed exactly as there: NG k-groups of KCH k-steps, one
// MFMA chain per group (the k-steps of wave g of gemm_skinny / gemm_splitk),
// summed in wave order -- COMB 0: sequentially (gemm_skinny), COMB 1 (NG 4):
// (g0 + g1) + (g2 + g3) (gemm_splitk) -- so the results are bit-identical.
// 1-D grid: the nrb row-block workgroups of one (strip group, K slice) are
// dispatched within a window of 8 * nrb ids with equal id % 8 (one XCD under
// the round-robin placement), so they share the strips' weights in its L2.
// ---------------------------------------------------------------------------
template <typename T, int MT, int KCH, int NG, int COMB, bool W8>
__global__ __launch_bounds__(256) void gemm_dec_shared(int epi, const T* __restrict__ Ap,
                                                       const void* __restrict__ Wv,
                                                       const uint8_t* __restrict__ Ws, int KT,
                                                       int M, int N, int nsg, int nks, int nrb,
                                                       float* __restrict__ Pslab, EpiParams P) {
  static_assert(COMB == 0 || NG == 4, "split-K partials: four k-groups");
  using V8 = typename Elt<T>::v8;
  constexpr int KS = NG * KCH;  // k-steps of this workgroup's K range
  // the whole A block in LDS: 80 KB for the DS(10, 4) case (d = 1280,
  // 16-bit) fits gfx950's 160 KB of LDS per workgroup (not gfx942's 64 KB)
  static_assert(MT * KS * 512 * sizeof(T) <= 160 * 1024, "gemm_dec_shared: A block exceeds gfx950 LDS");
  __shared__ __attribute__((aligned(16))) T ash[MT * KS * 512];
  const int L = blockIdx.x, Wd = 8 * nrb;
  const int rb = (L % Wd) / 8, g = (L / Wd) * 8 + L % 8;
  if (g >= nsg * nks) return;  // (workgroup-uniform: before any barrier)
  const int ks = g / nsg, sg = g - ks * nsg;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kt0 = ks * KS;  // first k-step of the range
  const int strip = sg * 4 + wid;
  const bool live = strip * 16 < N;
  // (a wave past the last strip loads the last strip's weights: straight-line
  // loads keep the compiler's wait counts exact; it stores nothing)
  const long f0 = (long)min(strip, (N - 1) >> 4) * KT + kt0;  // this wave's first weight fragment
  // WB k-groups of weights in flight per wave, the first WB issued before the
  // A DMA (their latencies overlap). MX-fp8 weights: 4 (C5 one lane 985.6 ->
  // 994.8 against 2, same box, r05ad); 16-bit: 2 (4 measured 891.6 -> 887.0)
  // (all NG groups in flight measured slower: FFN1 at 160 rows 13.96 vs 11.47
  // µs, beam 5 878.9 vs 898.1, C5 983.6 vs 991.5; r05ah)
  constexpr int WB = NG < (W8 ? 4 : 2) ? NG : (W8 ? 4 : 2);
  V8 wb[WB][KCH];
  uint2 wraw[WB][W8 ? KCH : 1];
  uint32_t wsc[WB][W8 ? KCH : 1];
  auto load_w = [&](int buf, int grp) {
    if constexpr (W8) {
      const uint8_t* wq = reinterpret_cast<const uint8_t*>(Wv) + (f0 + grp * KCH) * 512 + lane * 8;
#pragma unroll
      for (int c = 0; c < KCH; ++c) {
        wraw[buf][c] = *reinterpret_cast<const uint2*>(wq + c * 512);
        wsc[buf][c] = Ws[(f0 + grp * KCH + c) * 16 + (lane & 15)];
      }
    } else {
      const T* wt = reinterpret_cast<const T*>(Wv) + (f0 + grp * KCH) * 512 + lane * 8;
#pragma unroll
      for (int c = 0; c < KCH; ++c) wb[buf][c] = ld8(wt + c * 512);
    }
  };
#pragma unroll
  for (int b = 0; b < WB; ++b) load_w(b, b);
  // A block -> LDS: fragment (mt, k) of row tile rb*MT + mt is 1 KB at
  // Ap + ((rb*MT + mt) * KT + kt0 + k) * 512; one DMA instruction per fragment
#pragma unroll
  for (int f = wid; f < MT * KS; f += 4) {
    const int mt = f / KS, k = f - mt * KS;
    const T* src = Ap + ((long)(rb * MT + mt) * KT + kt0 + k) * 512 + lane * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)&ash[f * 512], 16,
                                     0, 0);
  }
  // this wave's A fragments have landed (and its first weight groups: the
  // two streams' latencies overlap)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // (every wave has waited for its own DMA; then a raw barrier)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (!live) return;  // (no barrier below)
  f32x4 sum[MT], s23[MT];
#pragma unroll
  for (int grp = 0; grp < NG; ++grp) {
    const int buf = grp % WB;
    if constexpr (W8) {
#pragma unroll
      for (int c = 0; c < KCH; ++c) wb[buf][c] = dequant8<T>(wraw[buf][c], e8m0_to_f32(wsc[buf][c]));
    }
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      acc[mt] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < KCH; ++c) {
        const V8 a = *reinterpret_cast<const V8*>(&ash[((mt * KS) + grp * KCH + c) * 512 + lane * 8]);
        acc[mt] = Elt<T>::mfma(a, wb[buf][c], acc[mt]);
      }
    }
    if (grp + WB < NG) load_w(buf, grp + WB);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if constexpr (COMB == 0) {
        sum[mt] = grp == 0 ? acc[mt] : sum[mt] + acc[mt];
      } else {
        if (grp == 0 || grp == 2) {
          (grp == 0 ? sum[mt] : s23[mt]) = acc[mt];
        } else if (grp == 1) {
          sum[mt] = sum[mt] + acc[mt];
        } else {
          s23[mt] = s23[mt] + acc[mt];
        }
      }
    }
  }
  const int n = strip * 16 + (lane & 15);
  if (n >= N) return;
  float* Pk = COMB == 1 ? Pslab + (long)ks * M * N : nullptr;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 v = COMB == 1 ? sum[mt] + s23[mt] : sum[mt];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = (rb * MT + mt) * 16 + (lane >> 4) * 4 + r;
      if (m >= M) continue;
      if constexpr (COMB == 1) {
        Pk[(long)m * N + n] = v[r];
      } else {
        switch (epi) {
          case EPI_GELU: skinny_store<EPI_GELU, T, false>(P, m, n, v[r]); break;
          case EPI_RES: skinny_store<EPI_RES, T, false>(P, m, n, v[r]); break;
          case EPI_F32: skinny_store<EPI_F32, T, false>(P, m, n, v[r]); break;
          case EPI_DEC_QKV: skinny_store<EPI_DEC_QKV, T, false>(P, m, n, v[r]); break;
          case EPI_STORE16: skinny_store<EPI_STORE16, T, false>(P, m, n, v[r]); break;
          default: break;
        }
      }
    }
  }
}

// M > 64 (MWX_DEC_SHARED_MIN: the row threshold): the shared-A kernels
// (MWX_DEC_SHARED=0 or dec_shared_set(0): the per-strip grids, for the A/B and
// the bit-identity test). Row blocks of 32 (16- and 64-row blocks measured
// slower: beam 5 849.9 / 858.5 vs 891-894, C5 957.4 / 900.0 vs 982.2; 8 strips
// per workgroup instead of 4 neutral: 893.4 vs 892.1; r05y, r05z, r05aa)
static std::atomic<int>& dec_shared_mode() {
  static std::atomic<int> m{-1};
  return m;
}
static bool dec_shared() {
  int v = dec_shared_mode().load();
  if (v < 0) {
    v = (getenv("MWX_DEC_SHARED") && atoi(getenv("MWX_DEC_SHARED")) == 0) ? 0 : 1;
    dec_shared_mode().store(v);
  }
  return v != 0;
}
int dec_shared_set(int on) { return dec_shared_mode().exchange(on < 0 ? -1 : (on ? 1 : 0)); }
static bool dec_shared_rows(int M) {
  static const int mn = getenv("MWX_DEC_SHARED_MIN") ? atoi(getenv("MWX_DEC_SHARED_MIN")) : 65;
  return M >= mn && dec_shared();
}
template <typename T, int KCH, int NG, int COMB, bool W8>
static void dec_shared_launch(int epi, const T* Ap, const void* Wp, const uint8_t* Ws, int KT,
                              int M, int N, int nks, float* Pslab, const EpiParams& P,
                              hipStream_t st) {
  constexpr int MT = 2;
  const int nsg = ((N + 15) / 16 + 3) / 4, nrb = (M + 16 * MT - 1) / (16 * MT);
  const int groups = nsg * nks;
  const dim3 g((groups + 7) / 8 * 8 * nrb);
  gemm_dec_shared<T, MT, KCH, NG, COMB, W8><<<g, 256, 0, st>>>(epi, Ap, Wp, Ws, KT, M, N, nsg,
                                                               nks, nrb, Pslab, P);
}

// (waves, k-steps per wave) for a K: all 32-deep k-steps split evenly over at
// most 16 waves with at most 10 k-steps each. want_nw > 0: exactly that many
// waves (FFN1 runs 4, as the chained seam's skinny consumer does, k_chain.hip)
static bool skinny_split(int K, int& nw, int& kch, int want_nw = 0) {
  if (K % 32) return false;
  const int S = K / 32;
  static const int wmax = getenv("MWX_SKINNY_NW") ? atoi(getenv("MWX_SKINNY_NW")) : 16;
  const int wtop = want_nw > 0 ? want_nw : std::min(16, std::max(1, wmax));
  for (int w = wtop; w >= (want_nw > 0 ? want_nw : 1); --w) {
    if (S % w) continue;
    const int c = S / w;
    if (c == 1 || c == 2 || c == 3 || c == 4 || c == 6 || c == 8 || c == 10) {
      nw = w;
      kch = c;
      return true;
    }
  }
  return false;
}

template <typename T, int MT, bool W8>
static bool skinny_launch(int epi, const T* Ap, const void* Wp, const uint8_t* Ws, int M, int N,
                          int K, const EpiParams& P, hipStream_t st) {
  int nw = 0, kch = 0;
  if (!skinny_split(K, nw, kch, P.nw)) return false;
  if (dec_shared_rows(M)) {
    // (the k-group splits of the model widths: d 1280 / 1024 / 768 / 512 / 384)
#define DS(NWV, C)                                                                              \
  if (nw == NWV && kch == C) {                                                                  \
    dec_shared_launch<T, C, NWV, 0, W8>(epi, Ap, Wp, Ws, K / 32, M, N, 1, nullptr, P, st);      \
    return true;                                                                                \
  }
    DS(10, 4) DS(16, 2) DS(12, 2) DS(16, 1) DS(12, 1)
#undef DS
  }
  const int nrb = (M + 16 * MT - 1) / (16 * MT), nx = (N + 15) / 16;
  const dim3 g(nx, nrb), b(64 * nw);
  switch (kch) {
#define SK(C) \
  case C: gemm_skinny<T, MT, C, W8><<<g, b, 0, st>>>(epi, Ap, Wp, Ws, K / 32, M, N, P, LnFuse{}); return true;
    SK(1) SK(2) SK(3) SK(4) SK(6) SK(8) SK(10)
#undef SK
    default: return false;
  }
}

// ---------------------------------------------------------------------------
// split-K decode GEMM: P[ks][m][n] = sum_{k in slice ks} A[m][k] * W[n][k]
// (raw f32 partials, no epilogue). Grid (N/16, KS): far more workgroups than
// 16-column strips alone, each reading only its K slice of A and W, so every
// CU streams a small share of the weights. The KS partials are summed (in ks
// order) by the consumer kernel together with the epilogue ggml applies
// (bias, residual, scale, f16 rounding), so the reduction costs no launch.
// ---------------------------------------------------------------------------
// LNF (M = 1, MT = 1): the A operand is the LayerNorm of the row formed in the
// prologue (LnFuse, kernels.h), staged through LDS in natural order; the
// weight loads are issued first so they overlap the LayerNorm's reductions.
template <typename T, int MT, int KCH, bool W8 = false, bool LNF = false>
__global__ __launch_bounds__(256) void gemm_splitk(const T* __restrict__ Ap,
                                                   const void* __restrict__ Wv,
                                                   const uint8_t* __restrict__ Ws, int KT, int M,
                                                   int N, int kslice, float* __restrict__ P,
                                                   LnFuse ln) {
  using V8 = typename Elt<T>::v8;
  static_assert(!LNF || MT == 1, "the folded LayerNorm serves one row");
  __shared__ f32x4 red[4][MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int bx = blockIdx.x, ks = blockIdx.y, bz = blockIdx.z;
  const int n0 = bx * 16;
  const int m_base = bz * 16 * MT;  // row block (16*MT rows per grid.z slice)
  const int Mb = min(16 * MT, M - m_base);
  const int kt0 = (ks * kslice >> 5) + wid * KCH;
  const long f0 = (long)bx * KT + kt0;
  V8 bfr[KCH];
  V8 afr[MT][KCH];
  uint2 wraw[W8 ? KCH : 1];
  uint32_t wsc[W8 ? KCH : 1];
  if constexpr (W8) {
    const uint8_t* wq = reinterpret_cast<const uint8_t*>(Wv) + f0 * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      wraw[c] = *reinterpret_cast<const uint2*>(wq + c * 512);
      wsc[c] = Ws[(f0 + c) * 16 + (lane & 15)];
    }
  } else {
    const T* wt = reinterpret_cast<const T*>(Wv) + f0 * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < KCH; ++c) bfr[c] = ld8(wt + c * 512);
  }
  if constexpr (LNF) {
    __shared__ double lnred[2][4];
    __shared__ __attribute__((aligned(16))) T srow[2048];
    ln_fold_prologue<T>(ln, KT * 32, bx == 0 && ks == 0 && bz == 0, srow, lnred);
#pragma unroll
    for (int c = 0; c < KCH; ++c) afr[0][c] = ln_fold_frag<T>(srow, kt0 + c, lane);
  } else {
    const T* at = Ap + ((long)(bz * MT) * KT + kt0) * 512 + lane * 8;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int c = 0; c < KCH; ++c) afr[mt][c] = ld8(at + ((long)mt * KT + c) * 512);
  }
  if constexpr (W8) {
#pragma unroll
    for (int c = 0; c < KCH; ++c) bfr[c] = dequant8<T>(wraw[c], e8m0_to_f32(wsc[c]));
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < KCH; ++c) acc[mt] = Elt<T>::mfma(afr[mt][c], bfr[c], acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wid][mt][lane] = acc[mt];
  __syncthreads();
  if (wid != 0) return;
  const int n = n0 + (lane & 15);
  if (n >= N) return;
  float* Pk = P + (long)ks * M * N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 v = (red[0][mt][lane] + red[1][mt][lane]) + (red[2][mt][lane] + red[3][mt][lane]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 16 + (lane >> 4) * 4 + r;
      if (m < Mb) Pk[(long)(m_base + m) * N + n] = v[r];
    }
  }
}

int splitk_factor(int K) {
  if (K % 128) return 0;
  const int S = K / 32;  // 32-deep k-steps
  static const int ksmax = getenv("MWX_SPLITK_KSMAX") ? atoi(getenv("MWX_SPLITK_KSMAX")) : 8;
  for (int ks = std::min(8, std::max(1, ksmax)); ks >= 1; --ks)
    if (S % ks == 0 && (S / ks) % 4 == 0 && (S / ks) / 4 <= 5) return ks;
  return 0;
}

template <typename T>
int gemm_splitk_partials(const T* Ap, const DecW<T>& Wd, int M, int N, int K, float* P,
                         hipStream_t st) {
  const void* Wp = Wd.q ? (const void*)Wd.q : (const void*)Wd.w;
  const uint8_t* Ws = Wd.s;
  const bool w8 = Wd.q != nullptr;
  const int ks = splitk_factor(K);
  if (ks == 0) return 0;
  const int kslice = K / ks;
  const int kch = kslice / 128;
  int MT = (std::min(M, 64) + 15) / 16;
  // M > 64 (beam / best-of rows): row blocks of 32 rows (beam 5: 722 -> 742
  // audio-s/s, fewer A-fragment registers per wave); 16*MT rows with
  // MWX_SPLITK_MT = 2..4 (A/B; per-row arithmetic is the same in any block)
  static const int mt_big = getenv("MWX_SPLITK_MT") ? atoi(getenv("MWX_SPLITK_MT")) : 2;
  if (M > 64 && mt_big >= 2 && mt_big <= 4) MT = mt_big;
  static const bool mt1 = !(getenv("MWX_DEC_MT1") && atoi(getenv("MWX_DEC_MT1")) == 0);
  if (mt1 && M <= 64) MT = 1;  // 16-row blocks (greedy +3%; MWX_DEC_MT1=0 for A/B)
  const int nrb = (M + 16 * MT - 1) / (16 * MT), nx = (N + 15) / 16;
  if (dec_shared_rows(M)) {
#define DSK(C)                                                                                   \
  if (kch == C) {                                                                                \
    if (w8)                                                                                      \
      dec_shared_launch<T, C, 4, 1, true>(0, Ap, Wp, Ws, K / 32, M, N, ks, P, EpiParams{}, st);  \
    else                                                                                         \
      dec_shared_launch<T, C, 4, 1, false>(0, Ap, Wp, Ws, K / 32, M, N, ks, P, EpiParams{}, st); \
    return ks;                                                                                   \
  }
    DSK(1) DSK(2) DSK(3) DSK(4) DSK(5)
#undef DSK
  }
  const dim3 g(nx, ks, nrb);
#define SKL(MTV, C)                                                                         \
  if (MT == MTV && kch == C) {                                                              \
    if (w8)                                                                                 \
      gemm_splitk<T, MTV, C, true><<<g, 256, 0, st>>>(Ap, Wp, Ws, K / 32, M, N, kslice, P,   \
                                                      LnFuse{});                            \
    else                                                                                    \
      gemm_splitk<T, MTV, C, false><<<g, 256, 0, st>>>(Ap, Wp, Ws, K / 32, M, N, kslice, P,  \
                                                       LnFuse{});                           \
    return ks;                                                                              \
  }
#define SKM(MTV) SKL(MTV, 1) SKL(MTV, 2) SKL(MTV, 3) SKL(MTV, 4) SKL(MTV, 5)
  SKM(1) SKM(2) SKM(3) SKM(4)
#undef SKM
#undef SKL
  return 0;
}

template <typename T>
int gemm_splitk_ln(const LnFuse& ln, const DecW<T>& Wd, int N, int K, float* P, hipStream_t st) {
  if (K > 2048 || K % 8) return 0;
  const void* Wp = Wd.q ? (const void*)Wd.q : (const void*)Wd.w;
  const int ks = splitk_factor(K);
  if (ks == 0) return 0;
  const int kslice = K / ks;
  const int kch = kslice / 128;
  const dim3 g((N + 15) / 16, ks, 1);
#define SKL(C)                                                                                 \
  if (kch == C) {                                                                              \
    if (Wd.q)                                                                                  \
      gemm_splitk<T, 1, C, true, true><<<g, 256, 0, st>>>(nullptr, Wp, Wd.s, K / 32, 1, N,     \
                                                          kslice, P, ln);                      \
    else                                                                                       \
      gemm_splitk<T, 1, C, false, true><<<g, 256, 0, st>>>(nullptr, Wp, Wd.s, K / 32, 1, N,    \
                                                           kslice, P, ln);                     \
    return ks;                                                                                 \
  }
  SKL(1) SKL(2) SKL(3) SKL(4) SKL(5)
#undef SKL
  return 0;
}
template int gemm_splitk_ln<_Float16>(const LnFuse&, const DecW<_Float16>&, int, int, float*,
                                      hipStream_t);
template int gemm_splitk_ln<__bf16>(const LnFuse&, const DecW<__bf16>&, int, int, float*,
                                    hipStream_t);

template int gemm_splitk_partials<_Float16>(const _Float16*, const DecW<_Float16>&, int, int, int,
                                            float*, hipStream_t);
template int gemm_splitk_partials<__bf16>(const __bf16*, const DecW<__bf16>&, int, int, int, float*,
                                          hipStream_t);

template <typename T>
bool gemm_decode(int epi, const T* Ap, const DecW<T>& Wd, int M, int N, int K, const EpiParams& P,
                 hipStream_t st) {
  const void* Wp = Wd.q ? (const void*)Wd.q : (const void*)Wd.w;
  const uint8_t* Ws = Wd.s;
  int MT = (std::min(M, 64) + 15) / 16;
  // M > 64 (beam / best-of rows): row blocks of 32 rows (32 KB of LDS: 5 workgroups
  // per CU instead of 2; beam 5 703 -> 729 audio-s/s; A/B: MWX_SKINNY_MT = 2..4;
  // the A tiles read stay inside the 64-row padded buffers for MT = 2..4)
  static const int mt_big = getenv("MWX_SKINNY_MT") ? atoi(getenv("MWX_SKINNY_MT")) : 2;
  if (M > 64 && mt_big >= 2 && mt_big <= 4) MT = mt_big;
  static const bool mt1 = !(getenv("MWX_DEC_MT1") && atoi(getenv("MWX_DEC_MT1")) == 0);
  if (mt1 && M <= 64) MT = 1;  // 16-row blocks (greedy +3%; MWX_DEC_MT1=0 for A/B)
  if (P.mt >= 1 && P.mt <= 4) MT = P.mt;
#define SKM(MTV)                                                                          \
  if (MT == MTV)                                                                          \
    return Wd.q ? skinny_launch<T, MTV, true>(epi, Ap, Wp, Ws, M, N, K, P, st)            \
                : skinny_launch<T, MTV, false>(epi, Ap, Wp, Ws, M, N, K, P, st);
  SKM(1) SKM(2) SKM(3) SKM(4)
#undef SKM
  return false;
}
template <typename T>
bool gemm_decode_ln(int epi, const LnFuse& ln, const DecW<T>& Wd, int N, int K,
                    const EpiParams& P, hipStream_t st) {
  int nw = 0, kch = 0;
  if (K > 2048 || K % 8 || !skinny_split(K, nw, kch, P.nw) || nw < 4) return false;
  const void* Wp = Wd.q ? (const void*)Wd.q : (const void*)Wd.w;
  const dim3 g((N + 15) / 16, 1), b(64 * nw);
  switch (kch) {
#define SK(C)                                                                                     \
  case C:                                                                                         \
    if (Wd.q)                                                                                     \
      gemm_skinny<T, 1, C, true, true><<<g, b, 0, st>>>(epi, nullptr, Wp, Wd.s, K / 32, 1, N, P,  \
                                                         ln);                                     \
    else                                                                                          \
      gemm_skinny<T, 1, C, false, true><<<g, b, 0, st>>>(epi, nullptr, Wp, Wd.s, K / 32, 1, N, P, \
                                                          ln);                                    \
    return true;
    SK(1) SK(2) SK(3) SK(4) SK(6) SK(8) SK(10)
#undef SK
    default: return false;
  }
}
template bool gemm_decode_ln<_Float16>(int, const LnFuse&, const DecW<_Float16>&, int, int,
                                       const EpiParams&, hipStream_t);
template bool gemm_decode_ln<__bf16>(int, const LnFuse&, const DecW<__bf16>&, int, int,
                                     const EpiParams&, hipStream_t);

template bool gemm_decode<_Float16>(int, const _Float16*, const DecW<_Float16>&, int, int, int,
                                    const EpiParams&, hipStream_t);
template bool gemm_decode<__bf16>(int, const __bf16*, const DecW<__bf16>&, int, int, int,
                                  const EpiParams&, hipStream_t);

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
static bool xcd_remap_enabled() {
  static const bool on = getenv("MWX_NO_XCD_REMAP") == nullptr;
  return on;
}
// row tiles per group of the grouped tile order (MWX_GEMM_GROUP; 0 = row-major)
static int gemm_group_m() {
  static const int g = getenv("MWX_GEMM_GROUP") ? std::max(0, atoi(getenv("MWX_GEMM_GROUP"))) : 8;
  return g;
}

// the encoder GEMM's main-loop schedule: env MWX_GEMM_8PH read once, a test
// switches it with gemm_8ph_set (mwx_test_set_gemm_8ph)
static std::atomic<int>& gemm_8ph_mode() {
  static std::atomic<int> m{-1};
  return m;
}
static bool gemm_8ph() {
  int v = gemm_8ph_mode().load();
  if (v < 0) {
    v = (getenv("MWX_GEMM_8PH") && atoi(getenv("MWX_GEMM_8PH")) == 1) ? 1 : 0;
    gemm_8ph_mode().store(v);
  }
  return v != 0;
}
int gemm_8ph_set(int on) { return gemm_8ph_mode().exchange(on < 0 ? -1 : (on ? 1 : 0)); }

template <typename T, int EPI, bool OUT16>
static void gemm_dispatch(const T* A, long lda, long a_bstride, const T* W, long ldw, int M,
                          int N, int K, int batch, const EpiParams& P0, hipStream_t st) {
  if (K % BK) throw std::runtime_error("mwx: gemm K must be a multiple of 64");
  dim3 g(((N + BN - 1) / BN) * ((M + BM - 1) / BM), batch);
  EpiParams P = P0;
  // (row-major order measured: XCD remap -3..-5% on the encoder GEMMs, +5%
  // on the all-layer cross K/V GEMM whose 320 column tiles stream 210 MB of
  // weights per row tile; with the grouped order both take the remap)
  P.group_m = gemm_group_m();
  P.xcd_remap = xcd_remap_enabled() && (EPI != EPI_CROSS_KV || P.group_m > 0);
  // MWX_GEMM_8PH=1 (or gemm_8ph_set(1)): the 8-phase schedule (bit-identical;
  // measured no faster than the 2-stage ring on the large-v3 encoder shapes:
  // one lane 0.3633 vs 0.3647 of the dense peak, same box, r05f)
  if (gemm_8ph())
    gemm_big<T, EPI, OUT16, false, true><<<g, 512, 0, st>>>(A, lda, a_bstride, W, ldw, M, N, K, P);
  else
    gemm_big<T, EPI, OUT16><<<g, 512, 0, st>>>(A, lda, a_bstride, W, ldw, M, N, K, P);
}

template <typename T>
void gemm_mx(int epi, const uint8_t* A, long lda, long a_bstride, const uint8_t* W, long ldw,
             int M, int N, int K, int batch, const EpiParams& P0, hipStream_t st) {
  if (K % 128) throw std::runtime_error("mwx: MX-fp8 gemm K must be a multiple of 128");
  dim3 g(((N + BN - 1) / BN) * ((M + BM - 1) / BM), batch);
  EpiParams P = P0;
  P.group_m = gemm_group_m();
  P.xcd_remap = xcd_remap_enabled() && (epi != EPI_CROSS_KV || P.group_m > 0);
#define MXL(E) gemm_big<T, E, false, true><<<g, 512, 0, st>>>(A, lda, a_bstride, W, ldw, M, N, K, P)
  switch (epi) {
    case EPI_ENC_QKV: MXL(EPI_ENC_QKV); break;
    case EPI_GELU: MXL(EPI_GELU); break;
    case EPI_RES: MXL(EPI_RES); break;
    case EPI_CROSS_KV: MXL(EPI_CROSS_KV); break;
    case EPI_F32: MXL(EPI_F32); break;
    default: throw std::runtime_error("mwx: unsupported MX-fp8 epilogue");
  }
#undef MXL
}
template void gemm_mx<_Float16>(int, const uint8_t*, long, long, const uint8_t*, long, int, int,
                                int, int, const EpiParams&, hipStream_t);
template void gemm_mx<__bf16>(int, const uint8_t*, long, long, const uint8_t*, long, int, int,
                              int, int, const EpiParams&, hipStream_t);

template <typename T>
void gemm(int epi, bool out_f16, const T* A, long lda, long a_bstride, const T* W, long ldw,
          int M, int N, int K, int batch, const EpiParams& P, hipStream_t st) {
  switch (epi) {
    case EPI_ENC_QKV: gemm_dispatch<T, EPI_ENC_QKV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_GELU:
      if (out_f16)
        gemm_dispatch<T, EPI_GELU, true>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st);
      else
        gemm_dispatch<T, EPI_GELU, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st);
      break;
    case EPI_RES: gemm_dispatch<T, EPI_RES, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_CONV2: gemm_dispatch<T, EPI_CONV2, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_F32: gemm_dispatch<T, EPI_F32, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_CROSS_KV: gemm_dispatch<T, EPI_CROSS_KV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_DEC_QKV: gemm_dispatch<T, EPI_DEC_QKV, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    case EPI_STORE16: gemm_dispatch<T, EPI_STORE16, false>(A, lda, a_bstride, W, ldw, M, N, K, batch, P, st); break;
    default: break;
  }
}

template void gemm<_Float16>(int, bool, const _Float16*, long, long, const _Float16*, long, int,
                             int, int, int, const EpiParams&, hipStream_t);
template void gemm<__bf16>(int, bool, const __bf16*, long, long, const __bf16*, long, int, int,
                           int, int, const EpiParams&, hipStream_t);

}  // namespace mwx
