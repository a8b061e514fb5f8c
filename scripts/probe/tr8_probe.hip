// Probe: the lane <-> address / result mapping of ds_read_b64_tr_b8 on gfx950
// (used to gather 8 keys x 1 column of an fp8 V tile per lane for the MFMA
// B operand). A 32-row x 64-byte LDS image holds byte (row, col) = row*64+col
// (mod 256, with the row in the high bits of a second image); each lane
// supplies the GUESSED address: lane 16g + 2q + p -> row 8(g&1) + q, bytes
// 8p .. 8p+7 of the 16-byte column block c0 = 16*(g>>1). Prints, per lane,
// the 8 received bytes decoded as (row, col), and checks the expectation
// "lane 16g + i receives column c0 + i of rows 8(g&1) .. +7".
// Result on gfx950 (gpurun r04x): CONFIRMED, 0 mismatching lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void k(uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[32 * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 32 * 64; i += 64) {
    const int r = i / 64, c = i % 64;
    img[i] = (uint8_t)(r * 8 + (c & 7)) ^ (uint8_t)((c >> 3) << 5);  // unique per (r, c&7) and c>>3 bits
  }
  __syncthreads();
  const int g = lane >> 4, li = lane & 15, q = li >> 1, p = li & 1;
  const int row = 8 * (g & 1) + q, c0 = 16 * (g >> 1);
  const int addr = row * 64 + c0 + 8 * p;
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(img + addr));
  out[lane * 2] = (uint32_t)v[0];
  out[lane * 2 + 1] = (uint32_t)v[1];
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64 * 8);
  k<<<1, 64>>>(d);
  uint32_t h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // expected byte for (row, col)
  auto val = [](int r, int c) { return (uint8_t)((uint8_t)(r * 8 + (c & 7)) ^ (uint8_t)((c >> 3) << 5)); };
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int g = lane >> 4, i = lane & 15;
    const int r0 = 8 * (g & 1), c = 16 * (g >> 1) + i;
    uint8_t got[8];
    for (int b = 0; b < 8; ++b) got[b] = (uint8_t)(h[lane * 2 + b / 4] >> (8 * (b % 4)));
    bool ok = true;
    for (int b = 0; b < 8; ++b) ok &= got[b] == val(r0 + b, c);
    if (!ok) ++bad;
    if (lane < 20 || !ok)
      printf("lane %2d: %02x %02x %02x %02x %02x %02x %02x %02x  (expect col %d rows %d..%d: %02x %02x ..) %s\n",
             lane, got[0], got[1], got[2], got[3], got[4], got[5], got[6], got[7], c, r0, r0 + 7,
             val(r0, c), val(r0 + 1, c), ok ? "ok" : "MISMATCH");
  }
  printf("tr8 mapping guess: %s (%d mismatching lanes)\n", bad ? "WRONG" : "CONFIRMED", bad);
  hipFree(d);
  return 0;
}
