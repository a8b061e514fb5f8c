// Probe: ds_read_b64_tr_b16 on gfx950 as the MX-fp8 cross-attention's P.V
// uses it: a wave's 32-key x 64-column f16 V tile in LDS, 16-column (32-B)
// blocks XOR-swizzled by (row >> 1) & 3; lane 16g + 4q + p addresses row
// 8g + 4h + q, columns 4p .. 4p+3 of logical block nt. Checks that lane
// 16g + i receives column 16 nt + i of rows 8g + 4h .. + 3 (elements 0..3).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef short v4s __attribute__((ext_vector_type(4)));

__global__ void k(uint16_t* out) {
  __shared__ __attribute__((aligned(16))) uint16_t img[32 * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 32 * 64; i += 64) {
    const int r = i / 64, c = i % 64;  // logical (row, col) -> physical slot
    const int blk = c >> 4, off = c & 15;
    img[r * 64 + ((blk ^ ((r >> 1) & 3)) << 4) + off] = (uint16_t)(r * 64 + c);
  }
  __syncthreads();
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  for (int nt = 0; nt < 4; ++nt)
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * g + 4 * h + q;
      const uint16_t* src = img + row * 64 + ((nt ^ ((row >> 1) & 3)) << 4) + 4 * p;
      v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(src));
      for (int e = 0; e < 4; ++e) out[((nt * 2 + h) * 64 + lane) * 4 + e] = (uint16_t)v[e];
    }
}

int main() {
  uint16_t* d;
  hipMalloc(&d, 8 * 64 * 4 * 2);
  k<<<1, 64>>>(d);
  uint16_t hbuf[8 * 64 * 4];
  hipMemcpy(hbuf, d, sizeof(hbuf), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int nt = 0; nt < 4; ++nt)
    for (int h = 0; h < 2; ++h)
      for (int lane = 0; lane < 64; ++lane) {
        const int g = lane >> 4, i = lane & 15;
        bool ok = true;
        for (int e = 0; e < 4; ++e)
          ok &= hbuf[((nt * 2 + h) * 64 + lane) * 4 + e] == (uint16_t)((8 * g + 4 * h + e) * 64 + 16 * nt + i);
        if (!ok) {
          if (bad < 24) {
            printf("nt %d h %d lane %2d got", nt, h, lane);
            for (int e = 0; e < 4; ++e) {
              const uint16_t v = hbuf[((nt * 2 + h) * 64 + lane) * 4 + e];
              printf(" (r%d c%d)", v / 64, v % 64);
            }
            printf(" want col %d rows %d..%d\n", 16 * nt + i, 8 * g + 4 * h, 8 * g + 4 * h + 3);
          }
          ++bad;
        }
      }
  printf("tr16 mapping: %s (%d mismatching lane reads of 512)\n", bad ? "WRONG" : "CONFIRMED", bad);
  hipFree(d);
  return 0;
}
