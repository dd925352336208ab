// Timeline inside ONE decode GEMV launch (the last of a graph of 28 back-to-back launches over distinct weights):
// per-block s_memrealtime stamps [start, prologue done, rows done], relative to the first block's start.
// Build: llm.hip with -DFA_GEMV_STAMPS (scripts/ubench/build.sh). Usage: gemv_stamps [O K epi]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
void gemv_stamps_read(unsigned long long* host, int n);
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
static void stats(const char* name, std::vector<double> v) {
  std::sort(v.begin(), v.end());
  printf("  %-22s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", name, v[0], v[v.size() / 10],
         v[v.size() / 2], v[v.size() * 9 / 10], v.back());
}
int main(int argc, char** argv) {
  const int O = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 1024, epi = argc > 3 ? atoi(argv[3]) : 0;
  const int L = 28;
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* tmp; CK(hipMalloc(&tmp, (size_t)O * K * 4));
  std::vector<int8_t*> q(L); std::vector<__half*> d(L);
  for (int l = 0; l < L; ++l) {
    launch_synth_fill(tmp, (int64_t)O * K, 100 + l, 0.05f, 0.f, s);
    CK(hipMalloc(&q[l], (size_t)O * K)); CK(hipMalloc(&d[l], (size_t)O * K / 32 * 2));
    launch_quant_q8_0(tmp, (int64_t)O * K, q[l], d[l], s);
  }
  float *x, *nw, *y; CK(hipMalloc(&x, K * 4)); CK(hipMalloc(&nw, K * 4)); CK(hipMalloc(&y, O * 4));
  launch_synth_fill(x, K, 7, 1.f, 0.f, s); launch_synth_fill(nw, K, 8, 0.1f, 1.f, s);
  CK(hipStreamSynchronize(s));
  hipGraph_t g; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int l = 0; l < L; ++l) {
    GemvArgs a{}; a.M = 1; a.eps = 1e-6f; a.wq = q[l]; a.wd = d[l]; a.O = O; a.rpw = gemv_rows_per_wave(O);
    a.x = x; a.ldx = K; a.norm_w = epi == 1 ? nullptr : nw; a.out = y; a.ldo = O; a.res = y; a.ldr = O;
    if (epi == 2) { a.wq2 = q[(l + 1) % L]; a.wd2 = d[(l + 1) % L]; }  // SwiGLU: the up matrix
    if (epi == 3) { fprintf(stderr, "epi 3 (lm_head) needs argmax partial buffers: not supported here\n"); return 1; }
    gemv_q8(a, K, epi, s);
  }
  CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ex, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s)); for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const int nblk = (O + 4 * gemv_rows_per_wave(O) - 1) / (4 * gemv_rows_per_wave(O));
  std::vector<unsigned long long> st((size_t)nblk * 4);
  gemv_stamps_read(st.data(), nblk);
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < nblk; ++b) t0 = std::min(t0, st[b * 4]);
  printf("GEMV O=%d K=%d epi=%d: %d blocks, %.2f us per launch in the graph (%.2f MB of q8_0 weights)\n", O, K, epi, nblk,
         ms * 1e3 / (20 * L), (double)O * K * 34 / 32 / 1e6);
  const char* nm[3] = {"block start", "prologue done", "rows done"};
  for (int k = 0; k < 3; ++k) {
    std::vector<double> v;
    for (int b = 0; b < nblk; ++b) v.push_back((st[b * 4 + k] - t0) * 0.01);
    stats(nm[k], v);
  }
  return 0;
}
