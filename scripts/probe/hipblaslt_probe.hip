// build: hipcc -O2 --offload-arch=gfx950 hipblaslt_probe.hip -lhipblaslt -o hipblaslt_probe
// Probe: what a library bf16 GEMM reaches on the encoder shapes (reference
// point for gemm_big; not used by the engine). C[M][N] = A[M][K] * W[N][K]^T.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <vector>
#define CK(x) do { auto e = (x); if (e) { printf("err %d at %d\n", (int)e, __LINE__); return 1; } } while (0)
int run(hipblasLtHandle_t h, int M, int N, int K) {
  void *A, *W, *C, *ws;
  size_t wss = 64 << 20;
  CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2)); CK(hipMalloc(&ws, wss));
  hipMemset(A, 0x3c, (size_t)M * K * 2); hipMemset(W, 0x3c, (size_t)N * K * 2);
  hipblasLtMatmulDesc_t op; CK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  // column-major view: C^T[N][M] = W[N][K] (as K x N col-major, transposed) * A^T
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta));
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb));
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K));
  CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, N, M, N));
  hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wss, sizeof wss));
  hipblasLtMatmulHeuristicResult_t res[8]; int nres = 0;
  CK(hipblasLtMatmulAlgoGetHeuristic(h, op, la, lb, lc, lc, pref, 8, res, &nres));
  float alpha = 1, beta = 0;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  double best = 0;
  for (int r = 0; r < nres; ++r) {
    for (int i = 0; i < 3; ++i) hipblasLtMatmul(h, op, &alpha, W, la, A, lb, &beta, C, lc, C, lc, &res[r].algo, ws, wss, 0);
    hipEventRecord(e0, 0);
    const int it = 10;
    for (int i = 0; i < it; ++i) hipblasLtMatmul(h, op, &alpha, W, la, A, lb, &beta, C, lc, C, lc, &res[r].algo, ws, wss, 0);
    hipEventRecord(e1, 0); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double tf = 2.0 * M * N * K / (ms / it * 1e-3) / 1e12;
    if (tf > best) best = tf;
    printf("M=%d N=%d K=%d algo %d: %.1f us  %.0f TF/s\n", M, N, K, r, ms / it * 1e3, tf);
  }
  printf("best %.0f TF/s\n", best);
  hipFree(A); hipFree(W); hipFree(C); hipFree(ws);
  return 0;
}
int main() {
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  run(h, 48000, 3840, 1280);
  run(h, 48000, 5120, 1280);
  run(h, 48000, 1280, 5120);
  run(h, 48000, 1280, 1280);
  return 0;
}
