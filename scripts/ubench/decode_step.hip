// Production replica of one batch-1 decode step (Qwen3-0.6B q8_0): 28 layers with DISTINCT weights
// (465 MB > 256 MB Infinity Cache, so weights stream from HBM like in the engine), n_past = 330.
// mode "graph": per-step time of the hipGraph'd step; mode "eager N": N eager steps (for rocprofv3 PMC).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
template <class T> T* dalloc(size_t n) { void* p; CK(hipMalloc(&p, n * sizeof(T))); return (T*)p; }
namespace fa { extern int g_lm_rpw; }
int main(int argc, char** argv) {
  if (const char* g = getenv("FUNASR_LM_RPW")) fa::g_lm_rpw = atoi(g);
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  AttnWork wk; wk.max_tokens = 1; wk.max_split_tokens = 1; wk.max_kv = 8;
  CK(hipMalloc(&wk.counters, 8 * CNT_LINE * 4)); CK(hipMemset(wk.counters, 0, 8 * CNT_LINE * 4));
  CK(hipMalloc(&wk.partials, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
  const int E = 1024, H = 16, KV = 8, D = 128, F = 3072, V = 151936, QKV = (H + 2 * KV) * D, NCTX = 2048, L = 28;
  float* tmp = dalloc<float>((size_t)V * E);
  // "arena": all q8_0 weights carved from ONE allocation (TLB experiment), else one hipMalloc per tensor
  const bool arena = argc > 1 && !strcmp(argv[1], "arena");
  // "mall": layers reuse 6 distinct weight sets (~100 MB < 256 MB Infinity Cache): the step reads MALL-resident
  // weights (what a run-ahead prefetcher could at best achieve)
  // "l2": every layer reuses ONE weight set (16.7 MB, 2.1 MB per XCD L2): the upper bound of an L2 prefetcher
  const int n_distinct = (argc > 1 && !strcmp(argv[1], "mall")) ? 6 : (argc > 1 && !strcmp(argv[1], "l2")) ? 1 : 28;
  char* arena_p = nullptr; size_t arena_off = 0;
  if (arena) CK(hipMalloc(&arena_p, (size_t)700 << 20));
  auto take = [&](size_t bytes) -> void* {
    if (!arena) { void* p; CK(hipMalloc(&p, bytes)); return p; }
    void* p = arena_p + arena_off; arena_off += (bytes + 4095) & ~(size_t)4095; return p; };
  auto q8 = [&](int64_t rows, int64_t cols, uint32_t key, int8_t** q, __half** d) {
    launch_synth_fill(tmp, rows * cols, key, 0.05f, 0.f, s);
    *q = (int8_t*)take(rows * cols); *d = (__half*)take(rows * cols / 32 * 2);
    launch_quant_q8_0(tmp, rows * cols, *q, *d, s);
  };
  struct LW { int8_t *qkv, *o, *g, *u, *d; __half *dqkv, *dO, *dg, *du, *dd; };
  std::vector<LW> lw(L);
  for (int l = 0; l < L; ++l) {
    q8(QKV, E, 100 + l, &lw[l].qkv, &lw[l].dqkv); q8(E, H * D, 200 + l, &lw[l].o, &lw[l].dO);
    q8(F, E, 300 + l, &lw[l].g, &lw[l].dg); q8(F, E, 400 + l, &lw[l].u, &lw[l].du); q8(E, F, 500 + l, &lw[l].d, &lw[l].dd);
  }
  int8_t* wemb; __half* demb; q8(V, E, 6, &wemb, &demb);
  CK(hipStreamSynchronize(s)); CK(hipFree(tmp));
  float* x = dalloc<float>(E); launch_synth_fill(x, E, 7, 1.f, 0.f, s);
  float* nw = dalloc<float>(E); launch_synth_fill(nw, E, 8, 0.1f, 1.f, s);
  float* qkv = dalloc<float>(QKV); float* att = dalloc<float>(H * D); float* act = dalloc<float>(F);
  float* logits = dalloc<float>(V); float* pval = dalloc<float>(8192); int* pidx = dalloc<int>(8192);
  __half* kc = dalloc<__half>((size_t)L * NCTX * KV * D); __half* vc = dalloc<__half>((size_t)L * NCTX * KV * D);
  CK(hipMemset(kc, 0, (size_t)L * NCTX * KV * D * 2)); CK(hipMemset(vc, 0, (size_t)L * NCTX * KV * D * 2));
  float* rc = dalloc<float>(NCTX * 64); float* rs = dalloc<float>(NCTX * 64);
  launch_synth_fill(rc, NCTX * 64, 12, 1.f, 0.f, s); launch_synth_fill(rs, NCTX * 64, 13, 1.f, 0.f, s);
  float* qn = dalloc<float>(D); launch_synth_fill(qn, D, 14, 0.1f, 1.f, s);
  int* seq = dalloc<int>(1); int* pos = dalloc<int>(1); CK(hipMemset(seq, 0, 4));
  int p0 = 330; CK(hipMemcpy(pos, &p0, 4, hipMemcpyHostToDevice));
  CK(hipStreamSynchronize(s));
  auto G = [&](const int8_t* q, const __half* d, int O, const float* xin, int ldx, const float* nrm, float* o, const float* res) {
    GemvArgs a{}; a.M = 1; a.eps = 1e-6f; a.wq = q; a.wd = d; a.O = O; a.rpw = gemv_rows_per_wave(O);
    a.x = xin; a.ldx = ldx; a.norm_w = nrm; a.out = o; a.ldo = O; a.res = res; a.ldr = O; return a; };
  int mask = 63;  // 1 qkv, 2 attn, 4 o, 8 gate/up, 16 down, 32 lm_head (ablation: time a subset of the chain)
  // "fused": the 3-launch batch-1 layer (A = qkv with the partial-sum prologue, B = attention + o slice, C = gate|up +
  // down slice); masks: 1 A, 2 B, 8 C, 32 lm_head
  // "fused2": the two-launch layer (AB = q|k|v GEMV + attention + o slice in one launch, C); mask 2 times AB
  const bool two = argc > 1 && !strcmp(argv[1], "fused2");
  const bool fused = two || (argc > 1 && !strcmp(argv[1], "fused"));
  FusedDecodeWork fw;
  fw.opart = dalloc<float>(8 * E); fw.dpart = dalloc<float>(8 * E); fw.act = dalloc<float>(2 * F); CK(hipMemset(fw.act, 0, 2 * F * 4)); fw.xmid = dalloc<float>(E);
  fw.cnt = dalloc<unsigned>(FUSED_CNT_LINES * CNT_LINE); fw.err = dalloc<int>(1);
  fw.gqkv = dalloc<unsigned long long>(4096); CK(hipMemset(fw.gqkv, 0, 4096 * 8));
  fw.gpart = dalloc<unsigned long long>(8 * ATTN_SPLITS * ATTN_PART_FLOATS);
  CK(hipMemset(fw.gpart, 0, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 8));
  CK(hipMemset(fw.cnt, 0, FUSED_CNT_LINES * CNT_LINE * 4)); CK(hipMemset(fw.err, 0, 4));
  CK(hipMemset(fw.opart, 0, 8 * E * 4)); CK(hipMemset(fw.dpart, 0, 8 * E * 4)); CK(hipMemset(fw.xmid, 0, E * 4));
  wk.max_tokens = 1;
  auto step_fused = [&]() {
    for (int l = 0; l < L; ++l) {
      auto& w = lw[l % n_distinct];
      auto a = G(w.qkv, w.dqkv, QKV, fw.xmid, E, nw, qkv, nullptr); a.psum = fw.dpart; a.xsum = x;
      if (two) {
        if (mask & 2) qkv_attn_o_fused(fw.xmid, fw.dpart, x, nw, w.qkv, w.dqkv, qkv, qn, qn, 1e-6f, rc, rs,
                                       kc + (size_t)l * NCTX * KV * D, vc + (size_t)l * NCTX * KV * D, H, KV, seq, pos,
                                       (int64_t)NCTX * KV * D, w.o, w.dO, E, wk, fw, s);
        if (mask & 8) ffn_fused(x, nw, 1e-6f, w.g, w.dg, w.u, w.du, w.d, w.dd, E, F, fw, s);
        continue;
      }
      if (mask & 1) gemv_q8(a, E, 0, s);
      if (mask & 2) attn_o_fused(qkv, qn, qn, 1e-6f, rc, rs, kc + (size_t)l * NCTX * KV * D, vc + (size_t)l * NCTX * KV * D,
                                 H, KV, seq, pos, (int64_t)NCTX * KV * D, w.o, w.dO, E, wk, fw, s);
      if (mask & 8) ffn_fused(x, nw, 1e-6f, w.g, w.dg, w.u, w.du, w.d, w.dd, E, F, fw, s);
    }
    auto h = G(wemb, demb, V, fw.xmid, E, nw, logits, nullptr); h.pval = pval; h.pidx = pidx; h.psum = fw.dpart;
    h.n_part = (V + 4 * h.rpw - 1) / (4 * h.rpw) * 4;
    if (mask & 32) gemv_q8(h, E, 3, s);
  };
  auto step = [&]() {
    if (fused) { step_fused(); return; }
    for (int l = 0; l < L; ++l) {
      auto& w = lw[l % n_distinct];
      if (mask & 1) gemv_q8(G(w.qkv, w.dqkv, QKV, x, E, nw, qkv, nullptr), E, 0, s);
      if (mask & 2) attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc + (size_t)l * NCTX * KV * D, vc + (size_t)l * NCTX * KV * D, 1, H, KV,
                 seq, pos, (int64_t)NCTX * KV * D, att, wk, s);
      if (mask & 4) gemv_q8(G(w.o, w.dO, E, att, H * D, nullptr, x, x), H * D, 1, s);
      auto gu = G(w.g, w.dg, F, x, E, nw, act, nullptr); gu.wq2 = w.u; gu.wd2 = w.du;
      if (mask & 8) gemv_q8(gu, E, 2, s);
      if (mask & 16) gemv_q8(G(w.d, w.dd, E, act, F, nullptr, x, x), F, 1, s);
    }
    auto h = G(wemb, demb, V, x, E, nw, logits, nullptr); h.pval = pval; h.pidx = pidx;
    h.n_part = (V + 4 * h.rpw - 1) / (4 * h.rpw) * 4;
    if (mask & 32) gemv_q8(h, E, 3, s);
  };
  const bool eager = argc > 1 && !strcmp(argv[1], "eager");
  printf("weights: %s, %d distinct layers\n", arena ? "one arena allocation" : "one hipMalloc per tensor", n_distinct);
  const int n = argc > 2 ? atoi(argv[2]) : 3;
  if (eager) { for (int i = 0; i < n; ++i) step(); CK(hipStreamSynchronize(s)); printf("eager %d steps done\n", n); return 0; }
  const double bytes = (double)L * (QKV * E + E * H * D + 2.0 * F * E + E * F) * 34 / 32 + (double)V * E * 34 / 32;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const char* names[] = {"full step", "qkv x28", "attn x28", "o x28", "gate/up x28", "down x28", "lm_head", "layers w/o attn",
                         "qkv+attn x28"};
  const int masks[] = {63, 1, 2, 4, 8, 16, 32, 29, 3};
  const char* fnames[] = {"full step", "A qkv+psum x28", "B attn+o x28", "", "C ffn+down x28", "", "lm_head", "A+C x28",
                          "A+B x28"};
  const int fmasks[] = {63, 1, 2, 0, 8, 0, 32, 9, 3};
  if (fused) { for (int t = 0; t < 9; ++t) { names[t] = fnames[t]; } }
  for (int t = 0; t < 9; ++t) {
    if (fused && fmasks[t] == 0) continue;
    if (fused) mask = fmasks[t];
    if (!fused) mask = masks[t];
    hipGraph_t g; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)); step(); CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ex, s));
    CK(hipStreamSynchronize(s));
    const int R = 50;
    CK(hipEventRecord(a, s)); for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (t == 0)
      printf("decode step (graph, 28 layers + lm_head, n_past 330): %.1f us  -> %.1f GB/s of q8_0 weights (%.1f MB)\n",
             ms * 1e3 / R, bytes / (ms * 1e-3 / R) / 1e9, bytes / 1e6);
    else
      printf("  %-18s %8.1f us  (%.2f us per launch)\n", names[t], ms * 1e3 / R,
             ms * 1e3 / R / (t == 6 ? 1 : (t == 7 ? (fused ? 2 : 4) * L : (t == 8 ? 2 * L : L))));
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
  }
  int err = 0; CK(hipMemcpy(&err, fw.err, 4, hipMemcpyDeviceToHost));
  if (err) printf("FUSED FAN-IN TIMEOUT\n");
  return 0;
}
