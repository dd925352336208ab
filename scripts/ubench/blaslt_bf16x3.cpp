// Microbenchmark: the batch-32 encoder GEMM shapes (M = 32032 rows) as ONE hipBLASLt bf16 GEMM with f32 accumulate
// over K' = 3K (A' = [A_hi | A_lo | A_hi], W' = [W_hi | W_hi | W_lo] per row: the three bf16x3 products hi.hi + lo.hi +
// hi.lo), against the hand-written 256x256 bf16x3 tile's 212 us per launch (profiles/r05_encode_b32_planes_kernels.txt).
// Timing only (random bf16 data); graph-free, hipEvents around 20 back-to-back calls after 3 warm-ups.
// build: hipcc -O3 --offload-arch=gfx950 scripts/ubench/blaslt_bf16x3.cpp -lhipblaslt -o scripts/ubench/blaslt_bf16x3
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != 0) { printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); exit(1); } } while (0)

__global__ void fill_bf16(uint16_t* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (uint16_t)(0x3C00 + (h & 0x1FF) - 0x100);  // bf16 around +-1
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 32032;
  struct Shape { const char* name; int N, K; double ref_us; };
  std::vector<Shape> shapes = {{"qkv", 1536, 512, 212.0}, {"o", 512, 512, -1}, {"ffn1", 2048, 512, -1},
                               {"ffn2", 512, 2048, -1}, {"ctc", 60000, 512, 6674.0}};
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const uint64_t ws_bytes = 256ull << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  for (const auto& sh : shapes) {
    const int N = sh.N, Kp = 3 * sh.K;
    uint16_t *A, *W;
    float* D;
    CK(hipMalloc(&A, (size_t)M * Kp * 2));
    CK(hipMalloc(&W, (size_t)N * Kp * 2));
    CK(hipMalloc(&D, (size_t)M * N * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, s, A, (size_t)M * Kp, 1u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, s, W, (size_t)N * Kp, 2u);
    hipblasLtMatmulDesc_t md;
    CK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    // column-major: D (N x M, ld N) = W^T (W: Kp x N, ld Kp) * A (Kp x M, ld Kp)
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, Kp, N, Kp));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, Kp, M, Kp));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, N, M, N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws_bytes, sizeof(ws_bytes)));
    hipblasLtMatmulHeuristicResult_t res[16];
    int nres = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 16, res, &nres));
    const float alpha = 1.f, beta = 0.f;
    double best = 1e30;
    int best_i = -1;
    for (int i = 0; i < nres && i < 8; ++i) {
      bool ok = true;
      for (int w = 0; w < 3 && ok; ++w)
        ok = hipblasLtMatmul(h, md, &alpha, W, la, A, lb, &beta, D, lc, D, lc, &res[i].algo, ws, ws_bytes, s) == 0;
      if (!ok) continue;
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 20; ++r) hipblasLtMatmul(h, md, &alpha, W, la, A, lb, &beta, D, lc, D, lc, &res[i].algo, ws, ws_bytes, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / 20;
      if (us < best) { best = us; best_i = i; }
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
    }
    const double fl = 2.0 * M * (double)N * sh.K;  // f32-equivalent flops (one product per element pair)
    printf("%-5s M %d N %d K %d (K' %d): %d algos, best #%d %.1f us = %.0f TF/s f32-equivalent (%.0f TF/s bf16)%s",
           sh.name, M, N, sh.K, Kp, nres, best_i, best, fl / best * 1e-6, 3 * fl / best * 1e-6, "");
    if (sh.ref_us > 0) printf("; hand-written tile %.1f us", sh.ref_us);
    printf("\n");
    fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(md);
    CK(hipFree(A));
    CK(hipFree(W));
    CK(hipFree(D));
  }
  return 0;
}
