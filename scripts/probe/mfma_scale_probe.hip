// Probe: operand / scale layout of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A and B,
// E8M0 block scales) on gfx950, with exact small-integer data. Prints which
// hypothesis about the lane -> (row, k) map and the scale operand holds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// e4m3fn encode of small integers 0..8 and negatives (exact)
__host__ __device__ static uint8_t e4m3(float x) {
  if (x == 0.0f) return 0;
  uint8_t s = x < 0 ? 0x80 : 0;
  float a = fabsf(x);
  int e = (int)floorf(log2f(a));
  float m = a / exp2f((float)e) - 1.0f;  // [0,1)
  int mi = (int)lrintf(m * 8.0f);
  return s | (uint8_t)(((e + 7) & 0xF) << 3) | (uint8_t)(mi & 7);
}

// A[16][128], B[128][16] (K x N) given as fp8 bytes under hypothesis H:
// lane l holds A[l&15][32*(l>>4) + j] (j = 0..31) and B[32*(l>>4) + j][l&15].
__global__ void k(const uint8_t* A, const uint8_t* B, const int* sa, const int* sb, float* D,
                  int use_scale) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = (uint8_t*)&a;
  uint8_t* pb = (uint8_t*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4f c = {0, 0, 0, 0};
  // cbsz / blgp = 0: fp8 e4m3 for A and B; opsel 0; scales as given
  if (use_scale)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  else
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  std::vector<float> Af(16 * 128), Bf(128 * 16);
  std::vector<uint8_t> A(16 * 128), B(128 * 16);
  for (int i = 0; i < 16; ++i)
    for (int kk = 0; kk < 128; ++kk) {
      float v = (float)(((i * 7 + kk * 3) % 9) - 4);  // -4..4, asymmetric
      Af[i * 128 + kk] = v;
      A[i * 128 + kk] = e4m3(v);
    }
  for (int kk = 0; kk < 128; ++kk)
    for (int n = 0; n < 16; ++n) {
      float v = (float)(((kk * 5 + n * 11 + 1) % 7) - 3);
      Bf[kk * 16 + n] = v;
      B[kk * 16 + n] = e4m3(v);
    }
  // scales: E8M0 (bias 127). Hypothesis S: lane l's scale applies to A row l&15,
  // k-block l>>4 (and B col l&15, k-block l>>4). Use 2^(blk) for A, 2^(col%3) for B.
  std::vector<int> sa(64), sb(64);
  for (int l = 0; l < 64; ++l) {
    sa[l] = 127 + (l >> 4);
    sb[l] = 127 + ((l & 15) % 3);
  }
  uint8_t *dA, *dB;
  int *dsa, *dsb;
  float* dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dsa, 256);
  hipMalloc(&dsb, 256);
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
  for (int use = 0; use < 2; ++use) {
    k<<<1, 64>>>(dA, dB, dsa, dsb, dD, use);
    std::vector<float> D(256);
    hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
    double err0 = 0, errS = 0;
    for (int i = 0; i < 16; ++i)
      for (int n = 0; n < 16; ++n) {
        double r0 = 0, rs = 0;
        for (int kk = 0; kk < 128; ++kk) {
          const double p = (double)Af[i * 128 + kk] * Bf[kk * 16 + n];
          r0 += p;
          rs += p * std::pow(2.0, kk / 32) * std::pow(2.0, n % 3);
        }
        err0 = std::max(err0, std::fabs(D[i * 16 + n] - r0));
        errS = std::max(errS, std::fabs(D[i * 16 + n] - rs));
      }
    printf("use_scale=%d: max|D - plain| = %g, max|D - scaled(row-blk A, col B)| = %g, D[0]=%g D[17]=%g\n",
           use, err0, errS, D[0], D[17]);
  }
  return 0;
}
