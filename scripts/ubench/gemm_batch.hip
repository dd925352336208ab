// Batched-decode q8_0 GEMMs (C3 shape, M = 32 tokens) one shape at a time: 28 launches over distinct weights,
// graph-replayed, us per launch for the split-K block kernel (kw 0), the K-in-block kernel (kw 2) and the engine's
// choice (kw 1). argv[1] = M (default 32). Also times the rmsnorm + q8_0 prep launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
#ifdef FA_GEMV_STAMPS
void gemv_stamps_read(unsigned long long* host, int n);
void gemm_stamps_read(unsigned long long* host, int n);
#endif
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
template <class T> T* dalloc(size_t n) { void* p; CK(hipMalloc(&p, n * sizeof(T))); return (T*)p; }
int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 32;
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int L = 28, E = 1024, F = 3072, QKV = 4096, V = 151936;
  float* tmp = dalloc<float>((size_t)V * E);
  auto q8 = [&](int64_t rows, int64_t cols, uint32_t key, int8_t** q, __half** d) {
    launch_synth_fill(tmp, rows * cols, key, 0.05f, 0.f, s);
    CK(hipMalloc(q, rows * cols)); CK(hipMalloc(d, rows * cols / 32 * 2));
    launch_quant_q8_0(tmp, rows * cols, *q, *d, s);
  };
  struct Shape { const char* name; int O, K, epi, n; std::vector<int8_t*> q, q2; std::vector<__half*> d, d2; };
  std::vector<Shape> shapes = {{"qkv", QKV, E, 0, L}, {"o", E, 2048, 1, L}, {"gate|up", F, E, 2, L}, {"down", E, F, 1, L},
                               {"lm_head", V, E, 3, 1}};
  uint32_t key = 100;
  for (auto& sh : shapes) {
    sh.q.resize(sh.n); sh.d.resize(sh.n); sh.q2.resize(sh.n); sh.d2.resize(sh.n);
    for (int i = 0; i < sh.n; ++i) {
      q8(sh.O, sh.K, key++, &sh.q[i], &sh.d[i]);
      if (sh.epi == 2) q8(sh.O, sh.K, key++, &sh.q2[i], &sh.d2[i]);
    }
  }
  CK(hipStreamSynchronize(s)); CK(hipFree(tmp));
  float* x = dalloc<float>((size_t)M * F); launch_synth_fill(x, (int64_t)M * F, 7, 1.f, 0.f, s);
  float* nw = dalloc<float>(F); launch_synth_fill(nw, F, 8, 0.1f, 1.f, s);
  int8_t* xq = dalloc<int8_t>((size_t)M * F); float* xd = dalloc<float>((size_t)M * F / 32);
  prep_q8(x, F, nullptr, 0.f, M, F, xq, xd, s);
  int8_t* q2 = dalloc<int8_t>((size_t)M * F); float* d2 = dalloc<float>((size_t)M * F / 32);
  float* out = dalloc<float>((size_t)M * V); float* res = dalloc<float>((size_t)M * F);
  CK(hipMemset(res, 0, (size_t)M * F * 4));
  float* pval = dalloc<float>((size_t)M * 8192); int* pidx = dalloc<int>((size_t)M * 8192);
  const int64_t kpart_n = (int64_t)4096 * 1024 * 8; float* kpart = dalloc<float>(kpart_n);
  const int64_t kcnt_n = 8192; int* kcnt = dalloc<int>(kcnt_n * CNT_LINE); CK(hipMemset(kcnt, 0, kcnt_n * CNT_LINE * 4));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timed = [&](auto&& body, int n) {
    hipGraph_t g; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)); body(); CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ex, s));
    CK(hipStreamSynchronize(s));
    const int R = 20;
    CK(hipEventRecord(a, s)); for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
    return ms * 1e3 / R / n;
  };
  printf("M = %d\n", M);
  printf("  %-8s prep (rmsnorm + q8_0, K 1024): %6.2f us\n", "",
         timed([&] { for (int i = 0; i < L; ++i) prep_q8(x, F, nw, 1e-6f, M, E, xq, xd, s); }, L));
  for (auto& sh : shapes) {
    for (int kw : {0, 2, 1}) {
      g_gemm_q8_kw = kw;
      g_lm_head_b = kw == 1;  // lm_head: kw 0 / 2 time the one-tile-per-block kernel, kw 1 the persistent loop
      const double us = timed([&] {
        for (int i = 0; i < sh.n; ++i) {
          GemvArgs ga{};
          ga.M = M; ga.eps = 1e-6f; ga.wq = sh.q[i]; ga.wd = sh.d[i]; ga.wq2 = sh.q2[i]; ga.wd2 = sh.d2[i]; ga.O = sh.O;
          ga.rpw = gemv_rows_per_wave(sh.O); ga.xq = xq; ga.xd = xd; ga.out = out; ga.ldo = sh.O;
          ga.res = sh.epi == 1 ? res : nullptr; ga.ldr = sh.O; ga.kpart = kpart; ga.kpart_n = kpart_n; ga.kcnt = kcnt;
          ga.kcnt_n = kcnt_n; ga.pval = pval; ga.pidx = pidx; ga.n_part = lm_head_parts(sh.O, M);
          if (sh.epi == 2) { ga.qout = q2; ga.dout = d2; }
          gemv_q8(ga, sh.K, sh.epi, s);
        }
      }, sh.n);
      const double wb = (double)sh.O * sh.K * (sh.epi == 2 ? 2 : 1) * 34 / 32;
      printf("  %-8s kw %d: %7.2f us per launch  (weights %.1f MB -> %.2f TB/s)\n", sh.name, kw, us, wb / 1e6,
             wb / (us * 1e-6) / 1e12);
    }
#ifdef FA_GEMV_STAMPS
    if (sh.epi != 3) {  // split-K kernel: one launch, stamps per block (wave 0)
      g_gemm_q8_kw = 0;
      for (int rep = 0; rep < 3; ++rep) {
        const int i = sh.n - 3 + rep;
        GemvArgs ga{};
        ga.M = M; ga.eps = 1e-6f; ga.wq = sh.q[i]; ga.wd = sh.d[i]; ga.wq2 = sh.q2[i]; ga.wd2 = sh.d2[i]; ga.O = sh.O;
        ga.rpw = gemv_rows_per_wave(sh.O); ga.xq = xq; ga.xd = xd; ga.out = out; ga.ldo = sh.O;
        ga.res = sh.epi == 1 ? res : nullptr; ga.ldr = sh.O; ga.kpart = kpart; ga.kpart_n = kpart_n; ga.kcnt = kcnt;
        ga.kcnt_n = kcnt_n;
        gemv_q8(ga, sh.K, sh.epi, s);
      }
      CK(hipStreamSynchronize(s));
      const int nb = (sh.O + 31) / 32 * gemm_k_splits(sh.O, M, sh.K, sh.epi);
      std::vector<unsigned long long> st((size_t)nb * 6);
      gemm_stamps_read(st.data(), nb);
      unsigned long long t0 = ~0ull;
      for (int bk = 0; bk < nb; ++bk) t0 = std::min(t0, st[bk * 6]);
      printf("    split-K kernel, %d blocks (%d splits):\n", nb, gemm_k_splits(sh.O, M, sh.K, sh.epi));
      const char* nm[] = {"start", "loads landed", "reduced", "published", "last arrival", "end"};
      for (int k = 0; k < 6; ++k) {
        std::vector<double> v;
        for (int bk = 0; bk < nb; ++bk) {
          const long long d = (long long)(st[bk * 6 + k] - t0);
          if (st[bk * 6 + k] && d >= 0) v.push_back(d * 0.01);
        }
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        printf("      %-14s n=%4zu min %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", nm[k], v.size(), v[0], v[v.size() / 2],
               v[v.size() * 9 / 10], v.back());
      }
    }
    if (sh.epi != 3) {  // one K-in-block launch (cold weights: the 3rd-last layer's copy), wave-0 stamps per block
      g_gemm_q8_kw = 2;
      for (int rep = 0; rep < 3; ++rep) {
        const int i = sh.n - 3 + rep;
        GemvArgs ga{};
        ga.M = M; ga.eps = 1e-6f; ga.wq = sh.q[i]; ga.wd = sh.d[i]; ga.wq2 = sh.q2[i]; ga.wd2 = sh.d2[i]; ga.O = sh.O;
        ga.rpw = gemv_rows_per_wave(sh.O); ga.xq = xq; ga.xd = xd; ga.out = out; ga.ldo = sh.O;
        ga.res = sh.epi == 1 ? res : nullptr; ga.ldr = sh.O;
        if (sh.epi == 2) { ga.qout = q2; ga.dout = d2; }
        gemv_q8(ga, sh.K, sh.epi, s);
      }
      CK(hipStreamSynchronize(s));
      const int nb = (sh.O + 31) / 32;
      std::vector<unsigned long long> st((size_t)nb * 4);
      gemv_stamps_read(st.data(), nb);
      unsigned long long t0 = ~0ull;
      for (int bk = 0; bk < nb; ++bk) t0 = std::min(t0, st[bk * 4]);
      const char* nm[] = {"start", "loads landed", "reduced", "end"};
      for (int k = 0; k < 4; ++k) {
        std::vector<double> v;
        for (int bk = 0; bk < nb; ++bk) v.push_back((long long)(st[bk * 4 + k] - t0) * 0.01);
        std::sort(v.begin(), v.end());
        printf("      %-14s min %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", nm[k], v[0], v[v.size() / 2],
               v[v.size() * 9 / 10], v.back());
      }
    }
#endif
  }
  return 0;
}
