// Per-block timeline of ONE decode attention launch (the last of 30 over rotating layers, cold K/V): s_memrealtime
// stamps of wave 0 (build llm.hip with -DFA_ATTN_STAMPS, scripts/ubench/build.sh), relative to the first block.
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
int main(int argc, char** argv) {
  // argv[1] = M tokens (default 1: one sequence at n_past 40 / 330 / 700; M > 1: token m is sequence m at
  // n_past 200 + (97 m) % 261, the C3 batch shape)
  const int M = argc > 1 ? atoi(argv[1]) : 1;
  // argv[2] == "o": the fused batch-1 layer's B launch (k_attn_o: attention + fan-in + combine + o slice), M = 1
  const bool fused_o = argc > 2 && argv[2][0] == 'o';
  // argv[2] == "c": the fused layer's C launch (k_ffn_fused: x_mid + norm + gate|up + group fan-in + down slice)
  const bool fused_c = argc > 2 && argv[2][0] == 'c';
  // argv[2] == "a": the two-launch layer's AB launch (k_attn_o<true>: q|k|v GEMV + fan-in, then as "o"), M = 1
  const bool fused_a = argc > 2 && argv[2][0] == 'a';
  if (const char* e = getenv("FUNASR_ATTN_LEAN")) g_attn_lean = atoi(e);
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int H = 16, KV = 8, D = 128, NCTX = 1024, QKV = 4096;
  AttnWork wk; wk.max_tokens = M; wk.max_split_tokens = M; wk.max_kv = KV;
  CK(hipMalloc(&wk.counters, (size_t)M * KV * CNT_LINE * 4)); CK(hipMemset(wk.counters, 0, (size_t)M * KV * CNT_LINE * 4));
  CK(hipMalloc(&wk.partials, (size_t)M * KV * ATTN_SPLITS * ATTN_PART_FLOATS * 4));
  const int64_t seq_stride = (int64_t)NCTX * KV * D;
  const size_t layer = (size_t)M * seq_stride;
  float* qkv = dalloc<float>((size_t)M * QKV); launch_synth_fill(qkv, (int64_t)M * QKV, 9, 1.f, 0.f, s);
  float* att = dalloc<float>((size_t)M * H * D);
  __half* kc = dalloc<__half>(28 * layer); __half* vc = dalloc<__half>(28 * layer);
  CK(hipMemset(kc, 0, 28 * layer * 2)); CK(hipMemset(vc, 0, 28 * layer * 2));
  float* rc = dalloc<float>(NCTX * 64); float* rs = dalloc<float>(NCTX * 64);
  launch_synth_fill(rc, NCTX * 64, 12, 1.f, 0.f, s); launch_synth_fill(rs, NCTX * 64, 13, 1.f, 0.f, s);
  float* qn = dalloc<float>(D); launch_synth_fill(qn, D, 14, 0.1f, 1.f, s);
  int* seq = dalloc<int>(M); int* pos = dalloc<int>(M);
  std::vector<int> hseq(M);
  for (int m = 0; m < M; ++m) hseq[m] = m;
  CK(hipMemcpy(seq, hseq.data(), M * 4, hipMemcpyHostToDevice));
  int8_t* wg_q = dalloc<int8_t>((size_t)3072 * 1024);  // gate / up stand-in [3072][1024], down [1024][3072]
  int8_t* wd_q = dalloc<int8_t>((size_t)1024 * 3072);
  CK(hipMemset(wg_q, 1, (size_t)3072 * 1024)); CK(hipMemset(wd_q, 1, (size_t)1024 * 3072));
  int8_t* wo_q = dalloc<int8_t>((size_t)1024 * 2048);
  int8_t* wqkv_q = dalloc<int8_t>((size_t)4096 * 1024);  // q|k|v stand-in (scales: wo_d, 3072 x 96 >= 4096 x 32)
  CK(hipMemset(wqkv_q, 1, (size_t)4096 * 1024));
  __half* wo_d = dalloc<__half>((size_t)3072 * 96);  // scales for every stand-in matrix (zeros)
  CK(hipMemset(wo_q, 1, (size_t)1024 * 2048)); CK(hipMemset(wo_d, 0, (size_t)3072 * 96 * 2));
  FusedDecodeWork fw;
  fw.opart = dalloc<float>(8 * 1024); fw.dpart = dalloc<float>(8 * 1024); fw.act = dalloc<float>(2 * 3072); CK(hipMemset(fw.act, 0, 2 * 3072 * 4));
  fw.xmid = dalloc<float>(1024); fw.cnt = dalloc<unsigned>(FUSED_CNT_LINES * CNT_LINE); fw.err = dalloc<int>(1);
  fw.gqkv = dalloc<unsigned long long>(4096); CK(hipMemset(fw.gqkv, 0, 4096 * 8));
  fw.gpart = dalloc<unsigned long long>(8 * ATTN_SPLITS * ATTN_PART_FLOATS);
  CK(hipMemset(fw.gpart, 0, 8 * ATTN_SPLITS * ATTN_PART_FLOATS * 8));
  CK(hipMemset(fw.cnt, 0, FUSED_CNT_LINES * CNT_LINE * 4)); CK(hipMemset(fw.err, 0, 4));
  CK(hipMemset(fw.xmid, 0, 1024 * 4)); CK(hipMemset(fw.dpart, 0, 8 * 1024 * 4));
  const int nblk = fused_c ? 256 : M * KV * ATTN_SPLITS;
  if (nblk > 4096) { printf("M too large for the stamp buffer\n"); return 1; }
  std::vector<unsigned long long> st((size_t)nblk * 16);
  std::vector<int> cases = M == 1 ? std::vector<int>{40, 330, 700} : std::vector<int>{-1};
  for (int p0 : cases) {
    std::vector<int> hpos(M);
    for (int m = 0; m < M; ++m) hpos[m] = p0 >= 0 ? p0 : 200 + (m * 97) % 261;
    CK(hipMemcpy(pos, hpos.data(), M * 4, hipMemcpyHostToDevice));
    CK(hipStreamSynchronize(s));
    attn_stamps_clear();
    for (int rep = 0; rep < 30; ++rep) {
      const int l = rep % 28;  // rotate layers: cold K/V like in the engine
      if (fused_c)
        ffn_fused(qkv, qkv + 1024, 1e-6f, wg_q, wo_d, wg_q, wo_d, wd_q, wo_d, 1024, 3072, fw, s);
      else if (fused_a)
        qkv_attn_o_fused(fw.xmid, fw.dpart, att, qkv, wqkv_q, wo_d, qkv, qn, qn, 1e-6f, rc, rs, kc + l * layer,
                         vc + l * layer, H, KV, seq, pos, seq_stride, wo_q, wo_d, 1024, wk, fw, s);
      else if (fused_o)
        attn_o_fused(qkv, qn, qn, 1e-6f, rc, rs, kc + l * layer, vc + l * layer, H, KV, seq, pos, seq_stride, wo_q, wo_d,
                     1024, wk, fw, s);
      else
        attn_block(qkv, 1, qn, qn, 1e-6f, rc, rs, kc + l * layer, vc + l * layer, M, H, KV, seq, pos, seq_stride, att, wk, s);
    }
    CK(hipStreamSynchronize(s));
    attn_stamps_read(st.data(), nblk);
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nblk; ++b) if (st[b * 16]) t0 = std::min(t0, st[b * 16]);
    if (p0 >= 0) printf("decode attention, n_past %d:\n", p0);
    else printf("decode attention, batch %d, n_past 200-460:\n", M);
    const int slot_b[] = {0, 1, 3, 7, 11, 9, 10};
    const char* nm_b[] = {"block start", "pos/splits known", "q normed/roped", "split merged", "partial stored",
                          "combine / direct start", "combined out"};
    const int slot_o[] = {1, 3, 7, 9, 10, 11, -1};
    const char* nm_o[] = {"splits known", "q normed/roped", "split merged", "partial published", "fan-in passed",
                          "combined + quantised", ""};
    const int slot_a[] = {0, 12, 13, 14, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11};
    const char* nm_a[] = {"loads issued", "x normed + q8", "q|k|v rows stored", "q|k|v hand-off passed", "splits known",
                          "K/V issued", "q normed/roped", "scores", "softmax", "p.V", "split merged",
                          "partial published", "fan-in passed", "combined + quantised"};
    const int slot_c[] = {0, 1, 2, 3, 4, 5, -1};
    const char* nm_c[] = {"block start", "x normed + q8", "act published", "group fan-in passed", "act quantised",
                          "down slice stored", ""};
    const int* slot = fused_a ? slot_a : fused_c ? slot_c : fused_o ? slot_o : slot_b;
    const char* const* nm = fused_a ? nm_a : fused_c ? nm_c : fused_o ? nm_o : nm_b;
    for (int k = 0; k < (fused_a ? 14 : fused_c || fused_o ? 6 : 7); ++k) {
      std::vector<double> v;
      for (int b = 0; b < nblk; ++b) {  // stamps left by an earlier launch (before t0) are not this launch's
        const long long d = (long long)(st[b * 16 + slot[k]] - t0);
        v.push_back(st[b * 16 + slot[k]] && d >= 0 ? d * 0.01 : -1.0);
      }
      stats(nm[k], v);
    }
  }
  return 0;
}
