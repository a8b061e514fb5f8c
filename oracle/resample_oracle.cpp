// CPU restatement of SttEngine::resample_audio (src/stt_engine.cpp:87-106) —
// TEST INFRASTRUCTURE ONLY (the checker for mwx_resample).
//
// The reference calls libsamplerate src_simple(&d, SRC_SINC_FASTEST, 1) with
// end_of_input = 0 and output_frames = (long)(n * ratio) + 100. libsamplerate
// is a third-party dependency (vcpkg.json:5-13, version not pinned in the
// reference) and is absent from the image, so this follows its published
// sinc converter (src_sinc.c, 0.2.x: sinc_mono_vari_process, prepare_data,
// calc_output_single): a buffer holding half_filter_chan_len zeros and then
// the input; per output sample the left and right filter wings summed in
// double with coefficients linearly interpolated at 12-bit fixed-point
// indices; the position advanced by 1 / ratio with fmod_one / lrint; the loop
// ends when no more than half_filter_chan_len samples remain (no
// end_of_input flush). Its "fastest" coefficient table (fastest_coeffs.h:
// increment 128, 2464 values) is not available either: the table below
// keeps that geometry with a reconstructed Kaiser-windowed sinc. Parity with
// libsamplerate itself is therefore unpinned.
#include <cmath>
#include <cstdint>
#include <vector>

namespace {

const int kIndexInc = 128;
const int kCoeffs = 2464;
const double kCutoff = 0.9;
const double kBeta = 9.0;
const int kShift = 12;

double i0(double x) {
  double sum = 1.0, term = 1.0;
  for (int k = 1; k < 64; ++k) {
    term *= (x / (2.0 * k)) * (x / (2.0 * k));
    sum += term;
    if (term < 1e-17 * sum) break;
  }
  return sum;
}

std::vector<float> table() {
  std::vector<double> h(kCoeffs);
  const double span = (double)kCoeffs / kIndexInc;
  for (int i = 0; i < kCoeffs; ++i) {
    const double x = (double)i / kIndexInc;
    const double t = x / span;
    const double arg = M_PI * kCutoff * x;
    const double sinc = i == 0 ? 1.0 : std::sin(arg) / arg;
    const double w = t >= 1.0 ? 0.0 : i0(kBeta * std::sqrt(1.0 - t * t)) / i0(kBeta);
    h[i] = kCutoff * sinc * w;
  }
  double dc = h[0];
  for (int k = kIndexInc; k < kCoeffs; k += kIndexInc) dc += 2.0 * h[k];
  std::vector<float> f(kCoeffs);
  for (int i = 0; i < kCoeffs; ++i) f[i] = (float)(h[i] / dc);
  return f;
}

typedef int32_t increment_t;
inline increment_t double_to_fp(double x) { return (increment_t)std::lrint(x * (double)(1 << kShift)); }
inline increment_t int_to_fp(int x) { return ((increment_t)x) << kShift; }
inline int fp_to_int(increment_t x) { return x >> kShift; }
inline double fp_to_double(increment_t x) {
  return (x & ((1 << kShift) - 1)) * (1.0 / (double)(1 << kShift));
}
inline double fmod_one(double x) {
  const double res = x - (double)std::lrint(x);
  return res < 0.0 ? res + 1.0 : res;
}

struct Filter {
  const float* coeffs;
  int coeff_half_len;
  std::vector<float> buffer;
  long b_current = 0, b_end = 0;
};

double calc_output_single(const Filter& f, increment_t increment, increment_t start_filter_index) {
  const increment_t max_filter_index = int_to_fp(f.coeff_half_len);
  increment_t filter_index = start_filter_index;
  int coeff_count = (max_filter_index - filter_index) / increment;
  filter_index = filter_index + coeff_count * increment;
  long data_index = f.b_current - coeff_count;
  if (data_index < 0) {
    const long steps = -data_index;
    filter_index -= increment * (increment_t)steps;
    data_index += steps;
  }
  double left = 0.0;
  while (filter_index >= 0) {
    const double fraction = fp_to_double(filter_index);
    const int indx = fp_to_int(filter_index);
    const double icoeff = f.coeffs[indx] + fraction * (f.coeffs[indx + 1] - f.coeffs[indx]);
    left += icoeff * f.buffer[data_index];
    filter_index -= increment;
    data_index = data_index + 1;
  }
  filter_index = increment - start_filter_index;
  coeff_count = (max_filter_index - filter_index) / increment;
  filter_index = filter_index + coeff_count * increment;
  data_index = f.b_current + 1 + coeff_count;
  double right = 0.0;
  do {
    const double fraction = fp_to_double(filter_index);
    const int indx = fp_to_int(filter_index);
    const double icoeff = f.coeffs[indx] + fraction * (f.coeffs[indx + 1] - f.coeffs[indx]);
    right += icoeff * f.buffer[data_index];
    filter_index -= increment;
    data_index = data_index - 1;
  } while (filter_index > 0);
  return left + right;
}

}  // namespace

extern "C" {

// Returns output_frames_gen (<= out_cap), 0 when src == dst or n == 0 (the
// reference then keeps its input), -1 on bad arguments or a ratio outside
// libsamplerate's [1/256, 256].
long orc_resample(const float* in, long n, int src_rate, int dst_rate, float* out, long out_cap) {
  if (n < 0 || src_rate <= 0 || dst_rate <= 0) return -1;
  if (src_rate == dst_rate || n == 0) return 0;
  const double ratio = (double)dst_rate / (double)src_rate;
  if (ratio < 1.0 / 256 || ratio > 256.0) return -1;
  static const std::vector<float> coeffs = table();
  Filter f;
  f.coeffs = coeffs.data();
  f.coeff_half_len = kCoeffs - 2;
  double count = (f.coeff_half_len + 2.0) / kIndexInc;
  if (ratio < 1.0) count /= ratio;
  const long half = std::lrint(count) + 1;
  // prepare_data, initial state: half zeros, then the input (all of it: the
  // ring buffer's refills move the same samples, indices are relative)
  f.buffer.assign(half, 0.0f);
  f.buffer.insert(f.buffer.end(), in, in + n);
  f.b_current = half;
  f.b_end = half + n;
  double input_index = 0.0;
  long out_gen = 0;
  while (out_gen < out_cap) {
    const long samples_in_hand = f.b_end - f.b_current;
    if (samples_in_hand <= half) break;
    const double float_increment = kIndexInc * (ratio < 1.0 ? ratio : 1.0);
    const increment_t increment = double_to_fp(float_increment);
    const increment_t start_filter_index = double_to_fp(input_index * float_increment);
    out[out_gen] = (float)((float_increment / kIndexInc) *
                           calc_output_single(f, increment, start_filter_index));
    out_gen++;
    input_index += 1.0 / ratio;
    const double rem = fmod_one(input_index);
    f.b_current = f.b_current + std::lrint(input_index - rem);
    input_index = rem;
  }
  return out_gen;
}

}  // extern "C"
