// Per-block timeline of ONE decode attention launch (the last of 30 over rotating layers, cold K/V): s_memrealtime
// stamps of wave 0 (build llm.hip with -DFA_ATTN_STAMPS, scripts/ubench/build.sh), relative to the first block.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
void attn_stamps_read(unsigned long long* host, int n_blocks);
void attn_stamps_clear();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
template <class T> T* dalloc(size_t n) { void* p; CK(hipMalloc(&p, n * sizeof(T))); return (T*)p; }
static void stats(const char* name, std::vector<double> v) {
  v.erase(std::remove(v.begin(), v.end(), -1.0), v.end());
  if (v.empty()) return;
  std::sort(v.begin(), v.end());
  printf("  %-24s n=%3zu  min %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", name, v.size(), v[0], v[v.size() / 2],
         v[v.size() * 9 / 10], v.back());
}
int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  AttnWork wk; wk.max_tokens = 1; wk.max_kv = 8;
  CK(hipMalloc(&wk.counters, 8 * CNT_LINE * 4)); CK(hipMemset(wk.counters, 0, 8 * CNT_LINE * 4));
  CK(hipMalloc(&wk.partials, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
  const int H = 16, KV = 8, D = 128, NCTX = 2048, QKV = 4096;
  float* qkv = dalloc<float>(QKV); launch_synth_fill(qkv, QKV, 9, 1.f, 0.f, s);
  float* att = dalloc<float>(H * D);
  __half* kc = dalloc<__half>((size_t)28 * NCTX * KV * D); __half* vc = dalloc<__half>((size_t)28 * NCTX * KV * D);
  CK(hipMemset(kc, 0, (size_t)28 * NCTX * KV * D * 2)); CK(hipMemset(vc, 0, (size_t)28 * NCTX * KV * D * 2));
  float* rc = dalloc<float>(NCTX * 64); float* rs = dalloc<float>(NCTX * 64);
  launch_synth_fill(rc, NCTX * 64, 12, 1.f, 0.f, s); launch_synth_fill(rs, NCTX * 64, 13, 1.f, 0.f, s);
  float* qn = dalloc<float>(D); launch_synth_fill(qn, D, 14, 0.1f, 1.f, s);
  int* seq = dalloc<int>(1); int* pos = dalloc<int>(1); CK(hipMemset(seq, 0, 4));
  const int nblk = KV * ATTN_SPLITS;
  std::vector<unsigned long long> st((size_t)nblk * 12);
  for (int p0 : {40, 330, 700}) {
    CK(hipMemcpy(pos, &p0, 4, hipMemcpyHostToDevice));
    CK(hipStreamSynchronize(s));
    attn_stamps_clear();
    for (int rep = 0; rep < 30; ++rep) {
      const int l = rep % 28;  // rotate layers: cold K/V like in the engine
      attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc + (size_t)l * NCTX * KV * D, vc + (size_t)l * NCTX * KV * D, 1, H, KV, seq,
                 pos, (int64_t)NCTX * KV * D, att, wk, s);
    }
    CK(hipStreamSynchronize(s));
    attn_stamps_read(st.data(), nblk);
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nblk; ++b) if (st[b * 12]) t0 = std::min(t0, st[b * 12]);
    printf("decode attention, n_past %d:\n", p0);
    const int slot[] = {0, 1, 3, 7, 11, 9, 10};
    const char* nm[] = {"block start", "pos/splits known", "q normed/roped", "split merged", "partial stored",
                        "combine / direct start", "combined out"};
    for (int k = 0; k < 7; ++k) {
      std::vector<double> v;
      for (int b = 0; b < nblk; ++b) {  // stamps left by an earlier launch (before t0) are not this launch's
        const long long d = (long long)(st[b * 12 + slot[k]] - t0);
        v.push_back(st[b * 12 + slot[k]] && d >= 0 ? d * 0.01 : -1.0);
      }
      stats(nm[k], v);
    }
  }
  return 0;
}
