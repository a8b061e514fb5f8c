// Probe 2: which (row|col, k-block) does each lane's E8M0 scale operand of
// v_mfma_scale_f32_16x16x128_f8f6f4 apply to? One lane's scale is set to 2.0
// (128), all others 1.0 (127); the rows / columns of D that change and the
// k-block whose partial product doubles identify the mapping.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static uint8_t e4m3(float x) {
  if (x == 0.0f) return 0;
  uint8_t s = x < 0 ? 0x80 : 0;
  float a = fabsf(x);
  int e = (int)floorf(log2f(a));
  float m = a / exp2f((float)e) - 1.0f;
  int mi = (int)lrintf(m * 8.0f);
  return s | (uint8_t)(((e + 7) & 0xF) << 3) | (uint8_t)(mi & 7);
}

__global__ void k(const uint8_t* A, const uint8_t* B, const int* sa, const int* sb, float* D) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = (uint8_t*)&a;
  uint8_t* pb = (uint8_t*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  std::vector<float> Af(16 * 128), Bf(128 * 16);
  std::vector<uint8_t> A(16 * 128), B(128 * 16);
  for (int i = 0; i < 16; ++i)
    for (int kk = 0; kk < 128; ++kk) {
      float v = (float)(((i * 7 + kk * 3) % 9) - 4);
      Af[i * 128 + kk] = v;
      A[i * 128 + kk] = e4m3(v);
    }
  for (int kk = 0; kk < 128; ++kk)
    for (int n = 0; n < 16; ++n) {
      float v = (float)(((kk * 5 + n * 11 + 1) % 7) - 3);
      Bf[kk * 16 + n] = v;
      B[kk * 16 + n] = e4m3(v);
    }
  // partial[i][n][blk]
  std::vector<double> part(16 * 16 * 4, 0.0);
  for (int i = 0; i < 16; ++i)
    for (int n = 0; n < 16; ++n)
      for (int kk = 0; kk < 128; ++kk)
        part[(i * 16 + n) * 4 + kk / 32] += (double)Af[i * 128 + kk] * Bf[kk * 16 + n];
  uint8_t *dA, *dB;
  int *dsa, *dsb;
  float* dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dsa, 256);
  hipMalloc(&dsb, 256);
  hipMalloc(&dD, 1024);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  for (int which = 0; which < 2; ++which) {
    for (int L = 0; L < 64; ++L) {
      std::vector<int> sa(64, 127), sb(64, 127);
      (which ? sb : sa)[L] = 128;
      hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
      k<<<1, 64>>>(dA, dB, dsa, dsb, dD);
      std::vector<float> D(256);
      hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
      printf("%s lane %2d:", which ? "B" : "A", L);
      // which subsets of the 16 8-element k-groups (as a 16-bit mask) explain
      // the change at every changed output, consistently
      int nchg = 0;
      std::vector<int> ok(1 << 16, 1);
      for (int i = 0; i < 16; ++i)
        for (int n = 0; n < 16; ++n) {
          double plain = 0, g8[16] = {0};
          for (int kk = 0; kk < 128; ++kk) {
            const double p = (double)Af[i * 128 + kk] * Bf[kk * 16 + n];
            plain += p;
            g8[kk / 8] += p;
          }
          const double dd = D[i * 16 + n] - plain;
          if (dd != 0.0) ++nchg;
          for (int m = 0; m < (1 << 16); ++m) {
            if (!ok[m]) continue;
            // mask applies to this output only if it is in the changed row/col set
            double s = 0;
            for (int g = 0; g < 16; ++g)
              if (m >> g & 1) s += g8[g];
            const bool in = which ? (n == (L & 15)) : (i == (L & 15));
            if (std::fabs((in ? s : 0.0) - dd) > 1e-6) ok[m] = 0;
          }
        }
      printf(" changed=%d masks:", nchg);
      int shown = 0;
      for (int m = 1; m < (1 << 16) && shown < 4; ++m)
        if (ok[m]) {
          printf(" %04x", m);
          ++shown;
        }
      printf("\n");
    }
  }
  return 0;
}
