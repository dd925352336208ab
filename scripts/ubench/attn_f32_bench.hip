// Encoder attention (attn_f32) timing: one 60 s clip (T = 1001, 4 heads x 128) and a batch of 32, per key-split
// count, graph-replayed (70 launches = the encoder's SANM blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
extern int g_attn_f32_force_splits;
extern int g_attn_wab;
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
int main(int argc, char** argv) {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  AttnF32Work wk; wk.part_n = ATTN_F32_PART_FLOATS; wk.cnt_n = ATTN_F32_COUNTERS;
  CK(hipMalloc(&wk.part, wk.part_n * 4)); CK(hipMalloc(&wk.cnt, wk.cnt_n * CNT_LINE * 4));
  CK(hipMemset(wk.cnt, 0, wk.cnt_n * CNT_LINE * 4));
  const int T = 1001, H = 4, Dh = 128, d = 512, L = 70;
  if (argc > 1 && std::string(argv[1]) == "wab") {  // k_attn_bf3 staging schedules, interleaved rounds, both graphs
    for (int B : {1, 32}) {
      float *qkv, *out;
      CK(hipMalloc(&qkv, (size_t)B * T * 3 * d * 4)); CK(hipMalloc(&out, (size_t)B * T * d * 4));
      launch_synth_fill(qkv, (int64_t)B * T * 3 * d, 5, 1.f, 0.f, s);
      std::vector<int> hl(B, T); int* lens; CK(hipMalloc(&lens, B * 4));
      CK(hipMemcpy(lens, hl.data(), B * 4, hipMemcpyHostToDevice));
      const double flops = 4.0 * B * T * (double)T * d;
      for (int r16 : {0, 1}) {
        std::vector<float> o0((size_t)B * T * d), o1(o0.size());
        for (int w = 0; w < 2; ++w) {
          g_attn_wab = w;
          CK(hipMemsetAsync(out, 0, o0.size() * 4, s));
          attn_f32(qkv, qkv + d, qkv + 2 * d, 3 * d, 3 * d, 3 * d, out, d, B, T, H, Dh, lens, wk, s, r16, 1);
          CK(hipStreamSynchronize(s));
          CK(hipMemcpy((w ? o1 : o0).data(), out, o0.size() * 4, hipMemcpyDeviceToHost));
        }
        size_t nd = 0;
        for (size_t i = 0; i < o0.size(); ++i) nd += o0[i] != o1[i];
        printf("%s batch %2d: schedule 1 vs 0: %zu outputs differ;", r16 ? "fp16  " : "bf16x3", B, nd);
        const int n = B > 1 ? 4 : L;
        for (int round = 0; round < 3; ++round)
          for (int w = 0; w < 2; ++w) {
            g_attn_wab = w;
            hipGraph_t g; hipGraphExec_t ex;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < n; ++i) attn_f32(qkv, qkv + d, qkv + 2 * d, 3 * d, 3 * d, 3 * d, out, d, B, T, H, Dh, lens, wk, s, r16, 1);
            CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
            hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
            CK(hipEventRecord(a, s)); for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1e3 / (3.0 * n);
            printf("  s%d %7.1f us %6.1f TF/s", w, us, flops / us / 1e6);
            CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
          }
        printf("\n");
      }
      CK(hipFree(qkv)); CK(hipFree(out)); CK(hipFree(lens));
    }
    return 0;
  }
  for (int B : {1, 32}) {
    float *qkv, *out;
    CK(hipMalloc(&qkv, (size_t)B * T * 3 * d * 4)); CK(hipMalloc(&out, (size_t)B * T * d * 4));
    launch_synth_fill(qkv, (int64_t)B * T * 3 * d, 5, 1.f, 0.f, s);
    std::vector<int> hl(B, T); int* lens; CK(hipMalloc(&lens, B * 4));
    CK(hipMemcpy(lens, hl.data(), B * 4, hipMemcpyHostToDevice));
    const double flops = 4.0 * B * T * (double)T * d;
   for (int bf3 : {0, 1}) {
    for (int ks : {0, 1, 2, 4, 8}) {
      if (B > 1 && ks > 1) continue;
      g_attn_f32_force_splits = ks;
      hipGraph_t g; hipGraphExec_t ex;
      const int n = B > 1 ? 4 : L;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < n; ++i) attn_f32(qkv, qkv + d, qkv + 2 * d, 3 * d, 3 * d, 3 * d, out, d, B, T, H, Dh, lens, wk, s, 0, bf3);
      CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
      hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
      CK(hipEventRecord(a, s)); for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / (3.0 * n);
      printf("%s batch %2d splits %d%s: %8.1f us per launch  %6.1f TF/s\n", bf3 ? "bf16x3" : "f32   ", B,
             ks ? ks : attn_f32_splits(B, T, H), ks ? "" : " (default)", us, flops / us / 1e6);
      CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
    }
   }
    CK(hipFree(qkv)); CK(hipFree(out)); CK(hipFree(lens));
  }
  return 0;
}
