// Band-limited sinc resampler for non-16 kHz requests on gfx950.
//
// Replaces SttEngine::resample_audio (src/stt_engine.cpp:87-106): libsamplerate
// src_simple(SRC_SINC_FASTEST, one channel, end_of_input = 0), i.e. its sinc
// converter (src_sinc.c: sinc_mono_vari_process + calc_output_single). The
// converter's per-output bookkeeping — the input position advanced by
// 1 / ratio in double precision with its integer part moved into the buffer
// index (fmod_one / lrint) — is a serial recurrence and is replayed on the
// host (resample_plan in driver.inc); every output sample's filter sum
// (left wing, then right wing, coefficients linearly interpolated between the
// table points with 12-bit fixed-point indices, accumulated in double) is one
// thread here. libsamplerate is not in the image and its "fastest" coefficient
// table is not either: the table is reconstructed with the same geometry
// (128 points per zero crossing, 2464 entries, see resample_coeffs) — parity
// with libsamplerate is unpinned; the device matches the CPU restatement in
// oracle/resample_oracle.cpp bit for bit.
#include "kcommon.h"
#include "kernels.h"

namespace mwx {

// (coefficient differences in float, the rest in double: coeff_t is float in
// libsamplerate). One thread per output sample; pos[n] = {input index of the output's centre,
// start_filter_index (fixed point)}; the virtual input buffer is `half` zeros
// followed by the input (libsamplerate's prepare_data initial state)
__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ in, int half,
                                                      const float* __restrict__ coeffs,
                                                      int coeff_half_len, int increment, double scale,
                                                      const int2* __restrict__ pos, int n_out,
                                                      float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= n_out) return;
  const int2 p = pos[n];
  const int b_current = half + p.x;
  const int start = p.y;
  const int max_filter_index = coeff_half_len << RS_SHIFT;
  auto buf = [&](int j) -> float { return j < half ? 0.0f : in[j - half]; };
  // left wing
  int filter_index = start;
  int coeff_count = (max_filter_index - filter_index) / increment;
  filter_index = filter_index + coeff_count * increment;
  int data_index = b_current - coeff_count;
  if (data_index < 0) {  // (libsamplerate's underflow guard; unreachable with `half` zeros)
    const int steps = -data_index;
    filter_index -= increment * steps;
    data_index += steps;
  }
  double left = 0.0;
  while (filter_index >= 0) {
    const double fraction = (double)(filter_index & RS_FRAC_MASK) * RS_INV_FP_ONE;
    const int indx = filter_index >> RS_SHIFT;
    const double icoeff = (double)coeffs[indx] + fraction * (double)(coeffs[indx + 1] - coeffs[indx]);
    left += icoeff * (double)buf(data_index);
    filter_index -= increment;
    data_index = data_index + 1;
  }
  // right wing
  filter_index = increment - start;
  coeff_count = (max_filter_index - filter_index) / increment;
  filter_index = filter_index + coeff_count * increment;
  data_index = b_current + 1 + coeff_count;
  double right = 0.0;
  do {
    const double fraction = (double)(filter_index & RS_FRAC_MASK) * RS_INV_FP_ONE;
    const int indx = filter_index >> RS_SHIFT;
    const double icoeff = (double)coeffs[indx] + fraction * (double)(coeffs[indx + 1] - coeffs[indx]);
    right += icoeff * (double)buf(data_index);
    filter_index -= increment;
    data_index = data_index - 1;
  } while (filter_index > 0);
  out[n] = (float)(scale * (left + right));
}

void resample_launch(const float* in, int half, const float* coeffs, int coeff_half_len,
                     int increment, double scale, const int2* pos, int n_out, float* out,
                     hipStream_t st) {
  if (n_out <= 0) return;
  resample_kernel<<<(n_out + 255) / 256, 256, 0, st>>>(in, half, coeffs, coeff_half_len, increment,
                                                       scale, pos, n_out, out);
}

}  // namespace mwx
