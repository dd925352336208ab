// Per-kernel decode-step timings with production shapes (Qwen3-0.6B q8_0, batch 1, n_past ~330),
// each kernel replayed 200x back-to-back inside a hipGraph (includes the ~1.6 us kernel boundary).
// Build: hipcc -O3 --offload-arch=gfx950 -I include scripts/ubench/decode_kernels.hip fun-asr-gguf_amd/csrc/{llm,synth}.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <functional>
#include <string>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
template <class T> T* dalloc(size_t n) { void* p; CK(hipMalloc(&p, n * sizeof(T))); return (T*)p; }
static hipStream_t s;
static double time_graph(const char* name, std::function<void()> f, int reps = 200, double bytes = 0) {
  hipGraph_t g; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) f();
  CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s)); for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
  double us = ms * 1e3 / (5.0 * reps);
  if (bytes > 0) printf("%-34s %8.2f us   %7.1f GB/s\n", name, us, bytes / us / 1e3);
  else printf("%-34s %8.2f us\n", name, us);
  return us;
}
int main() {
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  AttnWork wk; wk.max_tokens = 1; wk.max_split_tokens = 1; wk.max_kv = 8;
  CK(hipMalloc(&wk.counters, 8 * CNT_LINE * 4)); CK(hipMemset(wk.counters, 0, 8 * CNT_LINE * 4));
  CK(hipMalloc(&wk.partials, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
  const int E = 1024, H = 16, KV = 8, D = 128, F = 3072, V = 151936, QKV = (H + 2 * KV) * D, NCTX = 2048;
  auto q8 = [&](int64_t rows, int64_t cols, uint32_t key, int8_t** q, __half** d) {
    float* tmp = dalloc<float>(rows * cols);
    launch_synth_fill(tmp, rows * cols, key, 0.05f, 0.f, s);
    *q = dalloc<int8_t>(rows * cols); *d = dalloc<__half>(rows * cols / 32);
    launch_quant_q8_0(tmp, rows * cols, *q, *d, s);
    CK(hipStreamSynchronize(s)); CK(hipFree(tmp));
  };
  int8_t *wqkv, *wo, *wg, *wu, *wd, *wemb; __half *dqkv, *dO, *dg, *du, *dd, *demb;
  q8(QKV, E, 1, &wqkv, &dqkv); q8(E, H * D, 2, &wo, &dO); q8(F, E, 3, &wg, &dg); q8(F, E, 4, &wu, &du);
  q8(E, F, 5, &wd, &dd); q8(V, E, 6, &wemb, &demb);
  float* x = dalloc<float>(E); launch_synth_fill(x, E, 7, 1.f, 0.f, s);
  float* nw = dalloc<float>(E); launch_synth_fill(nw, E, 8, 0.1f, 1.f, s);
  float* qkv = dalloc<float>(QKV); launch_synth_fill(qkv, QKV, 9, 1.f, 0.f, s);
  float* att = dalloc<float>(H * D); launch_synth_fill(att, H * D, 10, 1.f, 0.f, s);
  float* act = dalloc<float>(F); launch_synth_fill(act, F, 11, 1.f, 0.f, s);
  float* out = dalloc<float>(V);
  float* pval = dalloc<float>(8192); int* pidx = dalloc<int>(8192);
  __half* kc = dalloc<__half>((size_t)NCTX * KV * D); __half* vc = dalloc<__half>((size_t)NCTX * KV * D);
  CK(hipMemset(kc, 0, (size_t)NCTX * KV * D * 2)); CK(hipMemset(vc, 0, (size_t)NCTX * KV * D * 2));
  float* rc = dalloc<float>(NCTX * 64); float* rs = dalloc<float>(NCTX * 64);
  launch_synth_fill(rc, NCTX * 64, 12, 1.f, 0.f, s); launch_synth_fill(rs, NCTX * 64, 13, 1.f, 0.f, s);
  float* qn = dalloc<float>(D); launch_synth_fill(qn, D, 14, 0.1f, 1.f, s);
  int* seq = dalloc<int>(1); int* pos = dalloc<int>(1); CK(hipMemset(seq, 0, 4));
  int p0 = 330; CK(hipMemcpy(pos, &p0, 4, hipMemcpyHostToDevice));
  CK(hipStreamSynchronize(s));
  auto G = [&](const int8_t* q, const __half* d, int O, const float* xin, const float* nrm, float* o, const float* res) {
    GemvArgs a{}; a.M = 1; a.eps = 1e-6f; a.wq = q; a.wd = d; a.O = O; a.rpw = gemv_rows_per_wave(O);
    a.x = xin; a.ldx = 4096; a.norm_w = nrm; a.out = o; a.ldo = O; a.res = res; a.ldr = O; return a; };
  double tot = 0;
  { auto a = G(wqkv, dqkv, QKV, x, nw, qkv, nullptr); a.ldx = E;
    tot += time_graph("gemv qkv 4096x1024 (norm)", [&] { gemv_q8(a, E, 0, s); }, 200, QKV * E * 34.0 / 32); }
  { auto a = G(wo, dO, E, att, nullptr, out, out); a.ldx = H * D;
    tot += time_graph("gemv o 1024x2048 (+res)", [&] { gemv_q8(a, H * D, 1, s); }, 200, E * H * D * 34.0 / 32); }
  { auto a = G(wg, dg, F, x, nw, act, nullptr); a.ldx = E; a.wq2 = wu; a.wd2 = du;
    tot += time_graph("gemv gate|up 2x3072x1024 (swiglu)", [&] { gemv_q8(a, E, 2, s); }, 200, 2.0 * F * E * 34.0 / 32); }
  { auto a = G(wd, dd, E, act, nullptr, out, out); a.ldx = F;
    tot += time_graph("gemv down 1024x3072 (+res)", [&] { gemv_q8(a, F, 1, s); }, 200, E * F * 34.0 / 32); }
  tot += time_graph("attn_block decode n_past=330", [&] {
    attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc, vc, 1, H, KV, seq, pos, (int64_t)NCTX * KV * D, att, wk, s); });
  time_graph("attn_block prefill-mode n_past=330", [&] {
    attn_block(att, 0, qn, qn, 1e-6f, rc, rs, kc, vc, 1, H, KV, seq, pos, (int64_t)NCTX * KV * D, qkv, wk, s); });
  int p1 = 40; CK(hipMemcpy(pos, &p1, 4, hipMemcpyHostToDevice));
  time_graph("attn_block decode n_past=40", [&] {
    attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc, vc, 1, H, KV, seq, pos, (int64_t)NCTX * KV * D, att, wk, s); });
  p1 = 1000; CK(hipMemcpy(pos, &p1, 4, hipMemcpyHostToDevice));
  time_graph("attn_block decode n_past=1000", [&] {
    attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc, vc, 1, H, KV, seq, pos, (int64_t)NCTX * KV * D, att, wk, s); });
  p1 = 330; CK(hipMemcpy(pos, &p1, 4, hipMemcpyHostToDevice));
  printf("%-34s %8.2f us  (x28 = %.1f us/step)\n", "layer sum", tot, tot * 28);
  { auto a = G(wemb, demb, V, x, nw, out, nullptr); a.ldx = E; a.pval = pval; a.pidx = pidx;
    a.n_part = (V + 4 * a.rpw - 1) / (4 * a.rpw) * 4;
    time_graph("lm_head 151936x1024 (argmax)", [&] { gemv_q8(a, E, 3, s); }, 50, (double)V * E * 34.0 / 32); }
  // ---- continuous batch (M tokens, pre-quantised activations -> int8 MFMA GEMM) and prefill shapes
  for (int M : {32, 204}) {
    int8_t* xq = dalloc<int8_t>((size_t)M * F); float* xd = dalloc<float>((size_t)M * F / 32);
    float* xs = dalloc<float>((size_t)M * F); launch_synth_fill(xs, (int64_t)M * F, 21, 1.f, 0.f, s);
    float* ob = dalloc<float>((size_t)M * QKV);
    prep_q8(xs, F, nullptr, 0.f, M, F, xq, xd, s);
    CK(hipStreamSynchronize(s));
    char nm[96];
    snprintf(nm, sizeof nm, "M=%d prep_q8 K=1024 (norm)", M);
    time_graph(nm, [&] { prep_q8(xs, E, nw, 1e-6f, M, E, xq, xd, s); });
    int* kc_ = dalloc<int>(256); CK(hipMemset(kc_, 0, 1024));
    float* kp_ = dalloc<float>(256 * 8 * 2 * 1024);
    auto B = [&](const int8_t* q, const __half* d, int O) {
      GemvArgs a{}; a.M = M; a.eps = 1e-6f; a.wq = q; a.wd = d; a.O = O; a.xq = xq; a.xd = xd; a.out = ob; a.ldo = O;
      a.res = ob; a.ldr = O; a.kpart = kp_; a.kpart_n = 256 * 8 * 2 * 1024; a.kcnt = kc_; a.kcnt_n = 256; return a; };
    double t = 0;
    { auto a = B(wqkv, dqkv, QKV); snprintf(nm, sizeof nm, "M=%d gemm qkv 4096x1024", M);
      t += time_graph(nm, [&] { gemv_q8(a, E, 0, s); }, 200, QKV * E * 34.0 / 32); }
    { auto a = B(wo, dO, E); snprintf(nm, sizeof nm, "M=%d gemm o 1024x2048 (+res)", M);
      t += time_graph(nm, [&] { gemv_q8(a, H * D, 1, s); }, 200, E * H * D * 34.0 / 32); }
    { auto a = B(wg, dg, F); a.wq2 = wu; a.wd2 = du; snprintf(nm, sizeof nm, "M=%d gemm gate|up (swiglu)", M);
      t += time_graph(nm, [&] { gemv_q8(a, E, 2, s); }, 200, 2.0 * F * E * 34.0 / 32); }
    { auto a = B(wd, dd, E); snprintf(nm, sizeof nm, "M=%d gemm down 1024x3072 (+res)", M);
      t += time_graph(nm, [&] { gemv_q8(a, F, 1, s); }, 200, E * F * 34.0 / 32); }
    printf("%-34s %8.2f us\n", "  gemm sum", t);
    { float* lg = dalloc<float>((size_t)M * V); float* pv = dalloc<float>((size_t)M * 4800); int* pi = dalloc<int>((size_t)M * 4800);
      auto a = B(wemb, demb, V); a.out = lg; a.ldo = V; a.pval = pv; a.pidx = pi; a.n_part = lm_head_parts(V, M);
      snprintf(nm, sizeof nm, "M=%d lm_head (argmax)", M);
      time_graph(nm, [&] { gemv_q8(a, E, 3, s); }, 20, (double)V * E * 34.0 / 32);
      CK(hipFree(lg)); CK(hipFree(pv)); CK(hipFree(pi)); }
    CK(hipFree(xq)); CK(hipFree(xd)); CK(hipFree(xs)); CK(hipFree(ob));
  }
  {  // batch-32 decode attention: 32 sequences at n_past 330
    const int M = 32;
    AttnWork wb; wb.max_tokens = M; wb.max_split_tokens = M; wb.max_kv = 8;
    CK(hipMalloc(&wb.counters, M * 8 * 4)); CK(hipMemset(wb.counters, 0, M * 8 * 4));
    CK(hipMalloc(&wb.partials, (size_t)M * 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
    __half* kb = dalloc<__half>((size_t)M * NCTX * KV * D); __half* vb = dalloc<__half>((size_t)M * NCTX * KV * D);
    CK(hipMemset(kb, 0, (size_t)M * NCTX * KV * D * 2)); CK(hipMemset(vb, 0, (size_t)M * NCTX * KV * D * 2));
    float* qb = dalloc<float>((size_t)M * QKV); launch_synth_fill(qb, (int64_t)M * QKV, 22, 1.f, 0.f, s);
    float* ab = dalloc<float>((size_t)M * H * D);
    int hs[M], hp[M]; for (int i = 0; i < M; ++i) { hs[i] = i; hp[i] = 330; }
    int* ds = dalloc<int>(M); int* dp = dalloc<int>(M);
    CK(hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice)); CK(hipMemcpy(dp, hp, sizeof hp, hipMemcpyHostToDevice));
    time_graph("M=32 attn_block decode n_past=330", [&] {
      attn_block(qb, 1, qn, qn, 1e-6f, rc, rs, kb, vb, M, H, KV, ds, dp, (int64_t)NCTX * KV * D, ab, wb, s); });
  }
  return 0;
}
