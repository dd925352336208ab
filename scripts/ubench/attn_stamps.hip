// s_memtime stamps along wave 0 of block 0 of k_attn_block (build with -DFA_ATTN_STAMPS)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
extern __device__ unsigned long long g_attn_stamps[16];
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
template <class T> T* dalloc(size_t n) { void* p; CK(hipMalloc(&p, n * sizeof(T))); return (T*)p; }
int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  AttnWork wk; wk.max_tokens = 1; wk.max_kv = 8;
  CK(hipMalloc(&wk.counters, 8 * CNT_LINE * 4)); CK(hipMemset(wk.counters, 0, 8 * CNT_LINE * 4));
  CK(hipMalloc(&wk.partials, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
  const int H = 16, KV = 8, D = 128, NCTX = 2048, QKV = 4096;
  float* qkv = dalloc<float>(QKV); launch_synth_fill(qkv, QKV, 9, 1.f, 0.f, s);
  float* att = dalloc<float>(H * D);
  __half* kc = dalloc<__half>((size_t)28 * NCTX * KV * D); __half* vc = dalloc<__half>((size_t)28 * NCTX * KV * D);
  float* rc = dalloc<float>(NCTX * 64); float* rs = dalloc<float>(NCTX * 64);
  launch_synth_fill(rc, NCTX * 64, 12, 1.f, 0.f, s); launch_synth_fill(rs, NCTX * 64, 13, 1.f, 0.f, s);
  float* qn = dalloc<float>(D); launch_synth_fill(qn, D, 14, 0.1f, 1.f, s);
  int* seq = dalloc<int>(1); int* pos = dalloc<int>(1); CK(hipMemset(seq, 0, 4));
  for (int p0 : {40, 330}) {
    CK(hipMemcpy(pos, &p0, 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 30; ++rep) {
      const int l = rep % 28;  // rotate layers: cold K/V like in the engine
      attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc + (size_t)l * NCTX * KV * D, vc + (size_t)l * NCTX * KV * D, 1, H, KV, seq,
                 pos, (int64_t)NCTX * KV * D, att, wk, s);
    }
    CK(hipStreamSynchronize(s));
    unsigned long long st[16];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_attn_stamps), sizeof(st)));
    printf("n_past=%d cycles from start:", p0);
    const char* nm[] = {"entry", "pos", "K issued", "q ready", "QK done", "softmax", "PV done", "pre-merge", "merge bar", "end"};
    for (int i = 1; i < 10; ++i) printf(" %s=%llu", nm[i], st[i] - st[0]);
    printf("\n");
  }
  return 0;
}
