// libfunasr_hip: C-ABI engine for the Fun-ASR hot path on MI355X (see include/funasr_hip.h).
//
// Owns, per GPU: all weights (encoder f32, decoder q8_0 in engine layout), activation arenas sized
// for max_batch x max_samples, the fp16 KV cache [layer][seq][kv head][n_ctx][128], one HIP stream.
// Encoder math follows model_definition.py (SenseVoiceEncoderSmall / CorrectTransformerAdaptor /
// CTC head); decoder math follows llama.cpp's qwen3 graph with ggml q8_0 numerics (oracle/qwen3.py).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/funasr_hip.h"
#include "common.h"
#include "gguf.h"
#include "kernels.h"

namespace fa {

static thread_local std::string g_err;
static void (*g_log_cb)(int32_t, const char*, void*) = nullptr;
static void* g_log_ud = nullptr;

void set_error(const std::string& m) {
  g_err = m;
  log(2, m);
}
void log(int level, const std::string& m) {
  if (g_log_cb) g_log_cb(level, m.c_str(), g_log_ud);
}

static uint32_t fnv1a32(const std::string& s) {
  uint32_t h = 0x811C9DC5u;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x01000193u;
  }
  return h;
}
static uint32_t lowbias32_h(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// ------------------------------------------------------------------------------------------------
struct Slot {
  int kind = 0;  // 0 f32 encoder/norm tensor, 1 q8_0 decoder matrix rows
  float* f = nullptr;
  int8_t* q = nullptr;
  __half* d = nullptr;
  int64_t n = 0;      // elements
  int64_t rows = 0, cols = 0;
  float scale = 0.f, offset = 0.f;  // synthetic spec
  bool set = false;
};

struct EncBlockW {
  const float *ln1_w, *ln1_b, *ln2_w, *ln2_b, *qkv_w, *qkv_b, *out_w, *out_b, *fsmn_w, *w1, *b1, *w2, *b2;
  int d_in;
};
struct AdBlockW {
  const float *ln1_w, *ln1_b, *ln2_w, *ln2_b, *qkv_w, *qkv_b, *o_w, *o_b, *w1, *b1, *w2, *b2;
};
struct AdaptorW {
  const float *l1_w, *l1_b, *l2_w, *l2_b;
  std::vector<AdBlockW> blocks;
};
struct Q8Mat {
  int8_t* q = nullptr;
  __half* d = nullptr;
};
struct LlmLayerW {
  Q8Mat qkv, o, gate, up, down;
  float *attn_norm, *ffn_norm, *q_norm, *k_norm;
};

struct Engine {
  int device = 0;
  fa_encoder_config ec{};
  fa_llm_config lc{};
  int max_batch = 1;
  int64_t max_samples = 0;
  hipStream_t stream = nullptr;
  std::vector<void*> allocs;
  std::unordered_map<std::string, Slot> slots;
  std::vector<std::string> spec_order;

  // encoder weights
  std::vector<EncBlockW> enc_blocks;  // encoders0 + encoders + tp_encoders
  const float *after_w, *after_b, *tp_w, *tp_b;
  AdaptorW adaptor, ctc_dec;
  const float *ctc_w, *ctc_b;
  // frontend constants
  float *basis = nullptr, *fbank = nullptr, *pe = nullptr;
  // encoder arenas
  int tm_max = 0, tl_max = 0, R = 0;
  int64_t xp_stride_max = 0;
  float *d_pcm = nullptr, *xp = nullptr, *mean_part = nullptr, *power = nullptr, *mel = nullptr;
  float *xa = nullptr, *hbuf = nullptr, *qkv = nullptr, *att = nullptr, *mem = nullptr, *ffn = nullptr;
  float *enc = nullptr, *ad = nullptr, *cbuf = nullptr, *ctc_pval = nullptr;
  int *ctc_pidx = nullptr, *ctc_ids = nullptr;
  int64_t* d_nsamp = nullptr;
  int *d_tmel = nullptr, *d_tlfr = nullptr, *d_tgt = nullptr, *d_ctclen = nullptr;
  int *d_col_ids = nullptr, *d_col_frames = nullptr, *d_col_n = nullptr;
  int debug_flags = 0;
  int64_t pcm_uploaded = 0;
  float* tap_lfr = nullptr;
  // last encode geometry
  int last_batch = 0, last_tstride = 0;
  int64_t enc_gen = 0;         // +1 per encode / CTC-head call: the adaptor rows fa_llm_prefill_rows may read
  float* d_prow = nullptr;     // fa_llm_prefill_rows: the caller's host rows on the device (grown on demand)
  int64_t prow_cap = 0;
  int* d_rowsrc = nullptr;     // fa_llm_prefill_rows: row codes of one forward
  std::vector<int> h_tlfr, h_tgt, h_ctclen;

  // decoder
  std::vector<LlmLayerW> layers;
  Q8Mat tok_embd;
  float* out_norm = nullptr;
  float *rcos = nullptr, *rsin = nullptr;
  __half *kcache = nullptr, *vcache = nullptr;
  int64_t seq_stride = 0, layer_stride = 0;
  int m_max = 0, n_part = 0, n_part_cur = 0;  // partial stride allocated / written by the last lm_head
  int pf_max = 0;                               // row capacity of one forward (multi-sequence prefill batches)
  int4* d_ptiles = nullptr;                     // prefill query tiles {row0, n_rows, seq, 0} (attn_prefill)
  int n_ptiles = 0;                             // tiles of the forward being run (0: per-row attn_block)
  int attn_pf_min_m = 512;                      // query-tiled prefill attention from this many rows (env knob)
  int attn_pf_rl = 1;                           // ... in row-local forwards, at any size (FUNASR_ATTN_PF_RL; 0: never)
  float* lxg = nullptr;                         // gathered last rows of a prefill batch
  int* d_lastrow = nullptr;
  int chunk_cur = 1;                            // rows per partial of the last lm_head
  float *lx = nullptr, *lqkv = nullptr, *lq = nullptr, *latt = nullptr, *lact = nullptr, *logits = nullptr;
  int8_t *lxq = nullptr, *lxq2 = nullptr;
  float *lxd = nullptr, *lxd2 = nullptr;
  float* pval = nullptr;
  int* pidx = nullptr;
  int *d_tok_seq = nullptr, *d_tok_pos = nullptr, *d_step = nullptr, *d_tok_cur = nullptr, *d_tok_hist = nullptr,
      *d_ids = nullptr;
  int hist_max = 0;
  int* h_hist = nullptr;           // pinned host copy of the sampled-token history (fa_llm_generate_begin / _end)
  hipEvent_t ev_gen = nullptr;     // recorded after that copy
  bool gen_pending = false;        // a generate call is in flight
  std::vector<int> gen_seqs;       // its sequences (row order) and steps
  int gen_steps = 0;
  SampleParams* d_samp = nullptr;  // sampler chain parameters of the current call (read by the sampler launch)
  SampleParams h_samp{};
  std::vector<int> n_past, last_tok;
  std::vector<int> logits_row;  // per sequence: its row of `logits` in the most recent forward (-1: none)
  AttnWork attn_wk;
  FusedDecodeWork fdw;     // fused batch-1 decode layer (3 launches per layer)
  // decode batches up to this width take the two-launch layer (FUNASR_FUSED_MAX_M, <= FUSED_MAX_M). Measured per step
  // (scripts/prof_small_batch.py, full model, two tokens per fused-FFN block from M = 4): M 1-6 0.486 / 0.566 / 0.694 /
  // 0.698 / 0.933 / 0.915 ms vs 0.594 / 0.709 / 0.812 / 0.935 / 1.000 / 1.047 ms on the 5-launch layer; M 7 / 8 1.213 /
  // 1.261 vs 1.070 / 1.073 ms (the AB launch's token slabs, 128 blocks each, no longer fit the chip at once)
  int fused_max_m = 6;
  // decode steps per captured graph (FUNASR_GRAPH_STEPS): chunks replay graphs of this many steps, then single steps.
  // Measured (graph-replayed, full model): 1 / 8 / 32 steps per graph -> batch 1 0.489 / 0.499 / 0.525 ms per step,
  // batch 32 1.223 / 1.239 / 1.358 ms: one step per graph replay stays the default
  int graph_steps = 1;
  int graph_sync_every = 0;  // FUNASR_GRAPH_SYNC_EVERY (profiling aid, see enqueue_steps)
  // profiler experiment hook (FUNASR_STEP_MASK, default all): which launches a batch-1 fused decode step enqueues --
  // bit 0 the attention launches (AB), 1 the FFN launches (C), 2 the LM head, 3 the sampler. Steps with bits cleared
  // compute garbage; only for bisecting which graph node rocprofv3's kernel trace rejects (scripts/gpu_r5_graphprof.sh)
  int step_mask = 15;
  bool pf_row_local = false;  // the prefill forward being run is row-local (see llm_forward)
  int pf_rl_max = 1024;       // prompts longer than this prefill on the tiled forward, alone (FUNASR_PF_ROW_LOCAL_MAX)
  int fused_retries = 0;     // chunks re-run on the fused layer after a fan-in timeout (exact: the same arithmetic)
  int fused_recoveries = 0;  // chunks re-run on the 5-launch layer after the retry timed out too (not batch-exact)
  int fused_fail_streak = 0; // consecutive chunks that needed the 5-launch layer; at kFusedGiveUp the engine keeps it
  int use_fused = 1;       // batch-1 layer: 1 two-launch (q|k|v + attention + o, FFN), 2 three-launch (q|k|v GEMV,
                           // attention + o, FFN), 0 the 5-launch layer every batch width uses (FUNASR_FUSED_DECODE)
  bool use_nrm = true;     // FUNASR_DECODE_NRM=0: batched decode keeps the k_prep_q8 launches (A/B)
  float* d_ssp = nullptr;  // batched decode: per-token sum-of-squares partials [max_seqs][32] of the residual stream
  AttnF32Work enc_attn_wk;
  GemmF32Work enc_gemm_wk;
  unsigned* gd_cnt = nullptr;  // gemv_gu_down hand-off counters
  // batched decode: gate|up + down in one launch with a per-K-split hand-off (FUNASR_GU_DOWN; 0 = two launches, A/B)
  bool use_gu_down = false;  // measured: batch-32 step 1.216-1.218 vs 1.2085-1.209 ms (profiles/r05_exp_gu_down.txt)
  // batched decode at M = 32: attention + o projection + residual + NRM epilogue in one launch (llm.hip k_attn_ob;
  // FUNASR_ATTN_OB=1, A/B). Needs every one of its KV x 32 one-per-CU blocks resident (checked against the CU count).
  // Measured slower (profiles/r06_exp_attn_ob.txt: graph-replayed batch-32 step 1.228-1.231 vs 1.154-1.158 ms): the two
  // in-launch edges it adds (32-block head fan-in, cross-XCD head sum) cost more than the kernel boundary they replace
  bool use_attn_ob = false;
  // row-local prefill on producer-normalised rows (FUNASR_PREFILL_NRM=1, A/B): measured slower (profiles/
  // r06_exp_prefill_nrm.txt: one 204-row prompt 2.59-2.60 vs 2.41-2.43 ms, 512 rows 4.72 vs 4.16 ms): the normalising
  // epilogue and the rstd prologue cost the K-in-block GEMMs more than the two k_prep_q8 launches per layer they replace
  bool use_pnrm = false;
  fa::AttnObWork ob_wk;
  float* gk_part = nullptr;  // MFMA GEMM split-K workspace
  int* gk_cnt = nullptr;
  int64_t gk_part_n = 0, gk_cnt_n = 0;

  // result gather over RCCL (fa_comm_*): this engine's communicator and its device staging buffers
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_world = 0;
  int64_t* comm_sz = nullptr;  // [2 world]: the send slot + the gathered sizes (own allocation, reused across inits)
  int comm_sz_n = 0;
  uint8_t* comm_buf = nullptr;  // send (cap) + receive (world x cap)
  int64_t comm_cap = 0;
  // the communicator and its buffers (fa_comm_destroy; ~Engine for C-API users that never call it)
  void comm_teardown();

  // profiling
  bool prof = false;
  struct ProfCls {
    double ms = 0, bytes = 0, flops = 0;
    int64_t launches = 0;
  } pcls[7];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  struct Pending {
    int cls;
    hipEvent_t a, b;
    double bytes, flops;
  };
  std::vector<Pending> pending;
  size_t ev_next = 0;
  std::unordered_map<int, hipGraphExec_t> step_graphs;
  bool use_graphs = true;

  int fill_lo = -1, fill_hi = -2, fill_byte = 0;  // FUNASR_ALLOC_FILL (alloc)
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    FA_HIP(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
    allocs.push_back(p);
    // FUNASR_ALLOC_FILL=lo:hi:byte (test hook, read at engine creation): allocations lo..hi of this engine start filled
    // with that byte instead of whatever bytes earlier buffers left (0xFF: NaN patterns), so a read of a never-written
    // byte shows up in results (tests/test_gpu_parity.py::test_poisoned_allocations_decode_bit_identical)
    const int idx = (int)allocs.size() - 1;
    if (idx >= fill_lo && idx <= fill_hi) FA_HIP(hipMemset(p, fill_byte, std::max<size_t>(n, 1) * sizeof(T)));
    return (T*)p;
  }
  ~Engine() {
    try {
      comm_teardown();
    } catch (...) {
    }
    if (comm_sz) hipFree(comm_sz);
    if (hp_rowsrc) hipHostFree(hp_rowsrc);
    if (ev_rowsrc) hipEventDestroy(ev_rowsrc);
    if (d_prow) hipFree(d_prow);
    for (auto& l : enc_lanes)
      if (l.s) hipStreamSynchronize(l.s);
    if (stream) hipStreamSynchronize(stream);
    for (auto& l : enc_lanes) {
      if (l.done) hipEventDestroy(l.done);
      if (l.s) hipStreamDestroy(l.s);
    }
    if (ev_fork) hipEventDestroy(ev_fork);
    if (hp_meta) hipHostFree(hp_meta);
    for (hipEvent_t ev : ev_meta)
      if (ev) hipEventDestroy(ev);
    for (auto& g : step_graphs) hipGraphExecDestroy(g.second);
    for (auto& e : ev_pool) {
      hipEventDestroy(e.first);
      hipEventDestroy(e.second);
    }
    for (void* p : allocs) hipFree(p);
    if (h_hist) hipHostFree(h_hist);
    if (ev_gen) hipEventDestroy(ev_gen);
    if (stream) hipStreamDestroy(stream);
  }

  // ---- profiling helpers: bracket launches of class `cls` with events on the engine stream
  bool prof_sample = true;  // decode layers > 1 are not bracketed (keeps the eager host ahead of the GPU)
  bool prof_layer0 = false;  // layer 0's decoder launches go to class 5 (its weights arrive without prefetch)
  bool prof_prefill = false; // prefill forwards' layer launches go to class 6 (not the decode classes)
  int prof_pos = 0;         // position of the profiled eager batch-1 decode step
  void prof_begin(int cls, hipEvent_t* a) {
    if (!prof || !prof_sample) return;
    if (ev_next >= ev_pool.size()) {
      // timing-only events: no system-scope fence (cache writeback + invalidate) at each record, which would
      // otherwise be charged to the bracketed kernel
      hipEvent_t x, y;
      FA_HIP(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
      FA_HIP(hipEventCreateWithFlags(&y, hipEventDisableSystemFence));
      ev_pool.push_back({x, y});
    }
    *a = ev_pool[ev_next].first;
    FA_HIP(hipEventRecord(*a, stream));
    (void)cls;
  }
  void prof_end(int cls, double bytes, double flops) {
    if (!prof || !prof_sample) return;
    hipEvent_t a = ev_pool[ev_next].first, b = ev_pool[ev_next].second;
    FA_HIP(hipEventRecord(b, stream));
    if (cls == 0 || cls == 3) cls = prof_prefill ? 6 : prof_layer0 ? 5 : cls;
    pending.push_back({cls, a, b, bytes, flops});
    ev_next++;
  }
  void prof_collect() {
    if (pending.empty()) return;
    FA_HIP(hipStreamSynchronize(stream));
    for (auto& p : pending) {
      float ms = 0;
      FA_HIP(hipEventElapsedTime(&ms, p.a, p.b));
      pcls[p.cls].ms += ms;
      pcls[p.cls].bytes += p.bytes;
      pcls[p.cls].flops += p.flops;
      pcls[p.cls].launches++;
    }
    pending.clear();
    ev_next = 0;
  }

  // ---------------------------------------------------------------------------------------------
  void add_f32(const std::string& name, int64_t n, float scale, float offset, float* dst) {
    Slot s;
    s.kind = 0;
    s.f = dst;
    s.n = n;
    s.scale = scale;
    s.offset = offset;
    slots[name] = s;
    spec_order.push_back(name);
  }
  float* f32_tensor(const std::string& name, int64_t n, float scale, float offset) {
    float* p = alloc<float>(n);
    add_f32(name, n, scale, offset, p);
    return p;
  }
  void add_q8(const std::string& name, int64_t rows, int64_t cols, float scale, int8_t* q, __half* d) {
    Slot s;
    s.kind = 1;
    s.q = q;
    s.d = d;
    s.rows = rows;
    s.cols = cols;
    s.n = rows * cols;
    s.scale = scale;
    slots[name] = s;
    spec_order.push_back(name);
  }

  static float lin_scale(int n_in) { return (float)std::sqrt(3.0 / n_in); }

  void lin(const std::string& p, int n_in, int n_out, float* w, float* b) {
    add_f32(p + ".weight", (int64_t)n_in * n_out, lin_scale(n_in), 0.f, w);
    if (b) add_f32(p + ".bias", n_out, 0.02f, 0.f, b);
    gemm_w.push_back({w, (int64_t)n_in * n_out});
  }

  // ---- fp16 encoder mode (C5: the reference's float16 ONNX graphs, 02-Quantize-ONNX.py:13-27). Every GEMM weight
  // gets an fp16 copy in one arena, in registration order (the adaptor's q|k|v sub-matrices stay contiguous), built
  // on the first fp16 encode after weights change.
  struct WRegion {
    const float* w;
    int64_t n;
  };
  std::vector<WRegion> gemm_w;
  bool enc_fp16 = false, w16_stale = true;
  __half* w16_arena = nullptr;
  std::unordered_map<const float*, const __half*> w16;
  float *basis16 = nullptr, *fbank16 = nullptr;  // frontend initializers as fp16 values (held in f32)

  void prepare_fp16() {
    if (!w16_stale) return;
    int64_t total = 0;
    for (const WRegion& r : gemm_w) total += r.n;
    if (!w16_arena) w16_arena = alloc<__half>((size_t)total);
    int64_t off = 0;
    for (const WRegion& r : gemm_w) {
      launch_f2h_initializer(r.w, w16_arena + off, nullptr, r.n, stream);
      w16[r.w] = w16_arena + off;
      off += r.n;
    }
    if (!basis16) basis16 = alloc<float>((size_t)402 * 400);
    if (!fbank16) fbank16 = alloc<float>((size_t)80 * 204);
    launch_f2h_initializer(basis, nullptr, basis16, (int64_t)402 * 400, stream);
    launch_f2h_initializer(fbank, nullptr, fbank16, (int64_t)80 * 204, stream);
    w16_stale = false;
  }
  const __half* W16(const float* W) const {
    if (!enc_fp16) return nullptr;
    auto it = w16.find(W);
    FA_REQUIRE(it != w16.end(), "fp16 encoder: GEMM weight without an fp16 copy");
    return it->second;
  }
  int r16() const { return enc_fp16 ? 1 : 0; }

  // ---- f32 mode on the bf16x3 split GEMM (enc_gemm 1, default; 0 = exact-f32 MFMA): every GEMM weight split once into
  // bf16 hi / lo planes (hi plane then lo plane, registration order in each, so contiguous sub-matrices stay
  // contiguous), built on the first f32 encode after weights change.
  int enc_gemm = 1;
  bool wb_stale = true;
  uint16_t* wb_arena = nullptr;
  std::unordered_map<const float*, WSplit> wb;

  void prepare_bf3() {
    if (!wb_stale) return;
    int64_t total = 0;
    for (const WRegion& r : gemm_w) total += r.n;
    if (!wb_arena) wb_arena = alloc<uint16_t>((size_t)2 * total);
    int64_t off = 0;
    for (const WRegion& r : gemm_w) {
      WSplit s;
      s.hi = wb_arena + off;
      s.lo = wb_arena + total + off;
      launch_split_bf16(r.w, wb_arena + off, wb_arena + total + off, r.n, stream);
      wb[r.w] = s;
      off += r.n;
    }
    wb_stale = false;
  }
  WSplit WB(const float* W) const {
    if (enc_fp16 || !enc_gemm) return WSplit{};
    auto it = wb.find(W);
    FA_REQUIRE(it != wb.end(), "bf16x3 encoder: GEMM weight without a split copy");
    return it->second;
  }
  void weights_changed() { w16_stale = wb_stale = qn_stale = true; }

  // The f16-MFMA prefill attention (k_attn_prefill_h) holds q * D^-0.5 * 2^8 as f16 hi + lo. After the q RMSNorm
  // every |x_i| <= sqrt(D), so |q_i| <= max|q_norm| * sqrt(D), and RoPE rotates pairs (|q'| <= max|q_norm| * sqrt(D)
  // as well): the f16 image stays finite while max|q_norm| * 256 (D = 128, scale D^-0.5) is below 65504 with margin.
  // Above that (a q_norm weight > ~234) the prefill attention runs the exact-f32 MFMA kernel (k_attn_prefill), and
  // row-local forwards take the per-row path. Checked lazily after every weight change.
  bool qn_stale = true, qn_f16_safe = true;
  bool prefill_attn_f16() {
    if (!fa::g_attn_pf_f16) return false;
    if (qn_stale && !layers.empty()) {
      const int D = lc.head_dim;
      std::vector<float> h(D);
      float mx = 0.f;
      for (const LlmLayerW& w : layers) {
        // on the engine's stream: the weight uploads are async on it (a null-stream copy does not wait for a
        // non-blocking stream and could read the previous weights)
        FA_HIP(hipMemcpyAsync(h.data(), w.q_norm, D * 4, hipMemcpyDeviceToHost, stream));
        FA_HIP(hipStreamSynchronize(stream));
        for (float v : h) mx = std::max(mx, std::isfinite(v) ? std::fabs(v) : INFINITY);
      }
      const bool ok = mx * std::sqrt((float)D) * (1.0f / std::sqrt(128.0f)) * 256.0f < 60000.0f;  // kernel: D = 128
      if (!ok && qn_f16_safe)
        log(2, "prefill attention: max|q_norm| = " + std::to_string(mx) +
                   " would overflow the f16 query image; using the exact-f32 MFMA prefill attention");
      qn_f16_safe = ok;
      qn_stale = false;
    }
    return qn_f16_safe;
  }

  // ---- int8-dynamic CTC graph (Fun-ASR-Nano-CTC.int8.onnx, the reference README's default CTC model: 02-Quantize-ONNX.py
  // :38-46): every CTC-graph linear with an ORT dynamic-quant weight (fa_set_tensor_u8dq) runs DynamicQuantizeLinear +
  // MatMulInteger + f32 rescale (gemm_f32.hip) instead of the f32 GEMM, once all of them have one (and fa_set_ctc_int8
  // has not turned it off). Regions are the CTC graph's f32 GEMM weight regions (q|k|v concatenated as in f32).
  struct U8Region {
    int N = 0, K = 0;
    int8_t* q = nullptr;
    int *cs = nullptr, *bz = nullptr;
    float* ws = nullptr;
    std::vector<char> row_set;
    int n_set = 0;
  };
  std::vector<const float*> ctc_regions;          // registration order
  std::unordered_map<const float*, U8Region> u8w;  // f32 region base -> its int8 form
  int ctc_i8 = 1;
  fa::U8Work u8wk;                                 // activation workspace of the batch encode (lanes own theirs)
  void ctc_region(const float* w, int N, int K) {
    ctc_regions.push_back(w);
    U8Region& r = u8w[w];
    r.N = N;
    r.K = K;
    r.row_set.assign(N, 0);
  }
  // an f32 write to (or unset of) elements [p, p + n) of a CTC-graph weight makes the int8 form of the rows it touches
  // stale: those rows must be handed over again (fa_set_tensor_u8dq) before the int8 graph runs again
  void u8_invalidate(const float* p, int64_t n) {
    for (const float* w : ctc_regions) {
      U8Region& r = u8w.at(w);
      const int64_t lo = std::max<int64_t>(0, (p - w) / r.K), hi = std::min<int64_t>(r.N, (p + n - w + r.K - 1) / r.K);
      for (int64_t i = lo; i < hi; ++i)
        if (r.row_set[i]) {
          r.row_set[i] = 0;
          --r.n_set;
        }
    }
  }
  bool ctc_int8_active() const {
    if (!ctc_i8 || ctc_regions.empty()) return false;
    for (const float* w : ctc_regions)
      if (u8w.at(w).n_set < u8w.at(w).N) return false;
    return true;
  }
  U8W U8(const float* W) const {
    const U8Region& r = u8w.at(W);
    U8W o;
    o.q = r.q; o.cs = r.cs; o.bz = r.bz; o.ws = r.ws;
    return o;
  }
  fa::U8Work make_u8work(int rows, int clips) {
    int kmax = 0;
    for (const float* w : ctc_regions) kmax = std::max(kmax, u8w.at(w).K);
    fa::U8Work w;
    w.xq_n = (int64_t)rows * kmax;
    w.xq = alloc<int8_t>((size_t)w.xq_n);
    w.rs = alloc<int>(rows);
    w.part = alloc<float2>((size_t)clips * 64);
    w.qp = alloc<float2>(clips);
    w.max_clips = clips;
    return w;
  }
  // one int8 linear of the CTC graph: DynamicQuantizeLinear of x (per clip over its lens[b] rows), MatMulInteger, rescale
  void u8_lin(fa::U8Work& w, const float* x, int64_t ldx, const float* W, const float* b, float* C, int64_t ldc, int rows,
              int ts, const int* lens, int N, int K, int relu = 0, const float* add1 = nullptr, int64_t ld1 = 0) {
    hipEvent_t ev;
    prof_begin(1, &ev);
    fa::dq_quantize(x, ldx, K, lens, ts, rows / ts, w, stream);
    fa::gemm_u8_linear(w, U8(W), b, C, ldc, rows, N, K, ts, relu, add1, ld1, stream);
    prof_end(1, 0, 2.0 * rows * N * K);
  }
  // CorrectTransformerAdaptor of the CTC graph with its linears in int8-dynamic form (the attention and LayerNorms stay
  // f32, as in the quantized ONNX graph), then ctc_lo + row argmax -> ctc_ids
  void run_ctc_int8(const float* in, int rows, int ts, const int* lens) {
    const AdaptorW& a = ctc_dec;
    const int d = ec.d_model, f = ec.ctc_ffn, d4 = d / 4;
    if (!u8wk.xq) u8wk = make_u8work(R, max_batch);
    fa::U8Work& w = u8wk;
    u8_lin(w, in, d, a.l1_w, a.l1_b, ffn, f, rows, ts, lens, f, d, 1);
    u8_lin(w, ffn, f, a.l2_w, a.l2_b, cbuf, d, rows, ts, lens, d, f);
    for (const AdBlockW& b : a.blocks) {
      layernorm(cbuf, d, hbuf, d, b.ln1_w, b.ln1_b, rows, d, 1e-12f, nullptr, ts, stream, 0);
      u8_lin(w, hbuf, d, b.qkv_w, b.qkv_b, qkv, 3 * d, rows, ts, lens, 3 * d, d);
      {
        hipEvent_t ev;
        prof_begin(2, &ev);
        attn_f32(qkv, qkv + d, qkv + 2 * d, 3 * d, 3 * d, 3 * d, att, d, rows / ts, ts, ec.ctc_heads, d / ec.ctc_heads,
                 lens, enc_attn_wk, stream, 0, enc_gemm ? 1 : 0);
        prof_end(2, 0, 4.0 * rows * (double)ts * d);
      }
      u8_lin(w, att, d, b.o_w, b.o_b, cbuf, d, rows, ts, lens, d, d, 0, cbuf, d);
      layernorm(cbuf, d, hbuf, d, b.ln2_w, b.ln2_b, rows, d, 1e-12f, nullptr, ts, stream, 0);
      u8_lin(w, hbuf, d, b.w1, b.b1, ffn, d4, rows, ts, lens, d4, d, 1);
      u8_lin(w, ffn, d4, b.w2, b.b2, cbuf, d, rows, ts, lens, d, d4, 0, cbuf, d);
    }
    hipEvent_t ev;
    prof_begin(1, &ev);
    fa::dq_quantize(cbuf, d, d, lens, ts, rows / ts, w, stream);
    fa::gemm_u8_ctc_argmax(w, U8(ctc_w), ctc_b, rows, ec.ctc_vocab, d, ts, ctc_pval, ctc_pidx, ctc_ids, stream);
    prof_end(1, 0, 2.0 * rows * (double)ec.ctc_vocab * d);
  }
  int bf3_attn() const { return !enc_fp16 && enc_gemm ? 1 : 0; }  // encoder attention products in the same mode

  EncBlockW sanm_block(const std::string& p, int d_in) {
    const int d = ec.d_model, f = ec.d_ffn, k = ec.fsmn_k;
    EncBlockW w{};
    w.d_in = d_in;
    w.ln1_w = f32_tensor(p + ".norm1.weight", d_in, 0.1f, 1.0f);
    w.ln1_b = f32_tensor(p + ".norm1.bias", d_in, 0.02f, 0.f);
    w.ln2_w = f32_tensor(p + ".norm2.weight", d, 0.1f, 1.0f);
    w.ln2_b = f32_tensor(p + ".norm2.bias", d, 0.02f, 0.f);
    float* qw = alloc<float>((size_t)3 * d * d_in);
    float* qb = alloc<float>(3 * d);
    lin(p + ".self_attn.linear_q_k_v", d_in, 3 * d, qw, qb);
    w.qkv_w = qw;
    w.qkv_b = qb;
    float* ow = alloc<float>((size_t)d * d);
    float* ob = alloc<float>(d);
    lin(p + ".self_attn.linear_out", d, d, ow, ob);
    w.out_w = ow;
    w.out_b = ob;
    w.fsmn_w = f32_tensor(p + ".self_attn.fsmn_block.weight", (int64_t)d * k, (float)(std::sqrt(3.0 / k) * 0.5), 0.f);
    float* w1 = alloc<float>((size_t)f * d);
    float* b1 = alloc<float>(f);
    lin(p + ".feed_forward.w_1", d, f, w1, b1);
    float* w2 = alloc<float>((size_t)d * f);
    float* b2 = alloc<float>(d);
    lin(p + ".feed_forward.w_2", f, d, w2, b2);
    w.w1 = w1;
    w.b1 = b1;
    w.w2 = w2;
    w.b2 = b2;
    return w;
  }

  AdaptorW adaptor_w(const std::string& p, int d_enc, int d_out, int d_ffn, int n_blocks) {
    AdaptorW a;
    float* l1w = alloc<float>((size_t)d_ffn * d_enc);
    float* l1b = alloc<float>(d_ffn);
    lin(p + ".linear1", d_enc, d_ffn, l1w, l1b);
    float* l2w = alloc<float>((size_t)d_out * d_ffn);
    float* l2b = alloc<float>(d_out);
    lin(p + ".linear2", d_ffn, d_out, l2w, l2b);
    a.l1_w = l1w;
    a.l1_b = l1b;
    a.l2_w = l2w;
    a.l2_b = l2b;
    for (int b = 0; b < n_blocks; ++b) {
      std::string q = p + ".blocks." + std::to_string(b);
      AdBlockW w{};
      // linear_q/k/v are stored concatenated [3*d_out][d_out] so one GEMM produces q|k|v
      float* qkvw = alloc<float>((size_t)3 * d_out * d_out);
      float* qkvb = alloc<float>(3 * d_out);
      const char* nm[3] = {"linear_q", "linear_k", "linear_v"};
      for (int i = 0; i < 3; ++i)
        lin(q + ".self_attn." + nm[i], d_out, d_out, qkvw + (size_t)i * d_out * d_out, qkvb + i * d_out);
      w.qkv_w = qkvw;
      w.qkv_b = qkvb;
      float* ow = alloc<float>((size_t)d_out * d_out);
      float* ob = alloc<float>(d_out);
      lin(q + ".self_attn.linear_out", d_out, d_out, ow, ob);
      w.o_w = ow;
      w.o_b = ob;
      float* w1 = alloc<float>((size_t)(d_out / 4) * d_out);
      float* b1 = alloc<float>(d_out / 4);
      lin(q + ".feed_forward.w_1", d_out, d_out / 4, w1, b1);
      float* w2 = alloc<float>((size_t)d_out * (d_out / 4));
      float* b2 = alloc<float>(d_out);
      lin(q + ".feed_forward.w_2", d_out / 4, d_out, w2, b2);
      w.w1 = w1;
      w.b1 = b1;
      w.w2 = w2;
      w.b2 = b2;
      w.ln1_w = f32_tensor(q + ".norm1.weight", d_out, 0.1f, 1.0f);
      w.ln1_b = f32_tensor(q + ".norm1.bias", d_out, 0.02f, 0.f);
      w.ln2_w = f32_tensor(q + ".norm2.weight", d_out, 0.1f, 1.0f);
      w.ln2_b = f32_tensor(q + ".norm2.bias", d_out, 0.02f, 0.f);
      a.blocks.push_back(w);
    }
    return a;
  }

  void build_encoder() {
    const int d = ec.d_model;
    enc_blocks.push_back(sanm_block("audio_encoder.encoders0.0", ec.d_in));
    for (int i = 0; i < ec.n_blocks - 1; ++i) enc_blocks.push_back(sanm_block("audio_encoder.encoders." + std::to_string(i), d));
    for (int i = 0; i < ec.n_tp_blocks; ++i)
      enc_blocks.push_back(sanm_block("audio_encoder.tp_encoders." + std::to_string(i), d));
    after_w = f32_tensor("audio_encoder.after_norm.weight", d, 0.1f, 1.0f);
    after_b = f32_tensor("audio_encoder.after_norm.bias", d, 0.02f, 0.f);
    tp_w = f32_tensor("audio_encoder.tp_norm.weight", d, 0.1f, 1.0f);
    tp_b = f32_tensor("audio_encoder.tp_norm.bias", d, 0.02f, 0.f);
    adaptor = adaptor_w("audio_adaptor", d, ec.d_llm, ec.adaptor_ffn, ec.adaptor_blocks);
    ctc_dec = adaptor_w("ctc_decoder", d, d, ec.ctc_ffn, ec.ctc_blocks);
    float* cw = alloc<float>((size_t)ec.ctc_vocab * d);
    float* cb = alloc<float>(ec.ctc_vocab);
    lin("ctc_proj.ctc_lo", d, ec.ctc_vocab, cw, cb);
    ctc_w = cw;
    ctc_b = cb;
    ctc_region(ctc_dec.l1_w, ec.ctc_ffn, d);
    ctc_region(ctc_dec.l2_w, d, ec.ctc_ffn);
    for (const AdBlockW& b : ctc_dec.blocks) {
      ctc_region(b.qkv_w, 3 * d, d);
      ctc_region(b.o_w, d, d);
      ctc_region(b.w1, d / 4, d);
      ctc_region(b.w2, d, d / 4);
    }
    ctc_region(ctc_w, ec.ctc_vocab, d);
  }

  Q8Mat q8mat(int64_t rows, int64_t cols) {
    Q8Mat m;
    m.q = alloc<int8_t>((size_t)rows * cols);
    m.d = alloc<__half>((size_t)rows * cols / 32);
    return m;
  }

  void build_llm() {
    const int E = lc.n_embd, H = lc.n_head, KV = lc.n_head_kv, D = lc.head_dim, F = lc.n_ff;
    tok_embd = q8mat(lc.n_vocab, E);
    add_q8("token_embd.weight", lc.n_vocab, E, 0.05f, tok_embd.q, tok_embd.d);
    for (int l = 0; l < lc.n_layer; ++l) {
      std::string b = "blk." + std::to_string(l) + ".";
      LlmLayerW w{};
      w.attn_norm = f32_tensor(b + "attn_norm.weight", E, 0.1f, 1.0f);
      w.qkv = q8mat((int64_t)(H + 2 * KV) * D, E);
      add_q8(b + "attn_q.weight", (int64_t)H * D, E, lin_scale(E), w.qkv.q, w.qkv.d);
      add_q8(b + "attn_k.weight", (int64_t)KV * D, E, lin_scale(E), w.qkv.q + (size_t)H * D * E,
             w.qkv.d + (size_t)H * D * E / 32);
      add_q8(b + "attn_v.weight", (int64_t)KV * D, E, lin_scale(E), w.qkv.q + (size_t)(H + KV) * D * E,
             w.qkv.d + (size_t)(H + KV) * D * E / 32);
      w.q_norm = f32_tensor(b + "attn_q_norm.weight", D, 0.1f, 1.0f);
      w.k_norm = f32_tensor(b + "attn_k_norm.weight", D, 0.1f, 1.0f);
      w.o = q8mat(E, (int64_t)H * D);
      add_q8(b + "attn_output.weight", E, (int64_t)H * D, lin_scale(H * D), w.o.q, w.o.d);
      w.ffn_norm = f32_tensor(b + "ffn_norm.weight", E, 0.1f, 1.0f);
      w.gate = q8mat(F, E);
      add_q8(b + "ffn_gate.weight", F, E, lin_scale(E), w.gate.q, w.gate.d);
      w.up = q8mat(F, E);
      add_q8(b + "ffn_up.weight", F, E, lin_scale(E), w.up.q, w.up.d);
      w.down = q8mat(E, F);
      add_q8(b + "ffn_down.weight", E, F, lin_scale(F), w.down.q, w.down.d);
      layers.push_back(w);
    }
    out_norm = f32_tensor("output_norm.weight", E, 0.1f, 1.0f);
  }

  // ---------------------------------------------------------------------------------------------
  // host constants (STFT basis, mel fbank, PE, RoPE) — same float32 formulas as oracle/frontend.py
  static std::vector<float> linspace_f32(float start, float end, int steps) {
    std::vector<float> o(steps);
    float step = (end - start) / (float)(steps - 1);
    int half = steps / 2;
    for (int i = 0; i < steps; ++i) o[i] = i < half ? start + step * (float)i : end - step * (float)(steps - i - 1);
    return o;
  }

  void build_constants() {
    const double PI = 3.14159265358979323846;
    // STFT basis, rows interleaved (cos_f, -sin_f) [402][400]
    std::vector<float> basis_h(402 * 400), win(400);
    const float wstep = (float)(2.0 * PI / 400.0);
    for (int n = 0; n < 400; ++n) win[n] = (float)std::cos((double)((float)n * wstep)) * -0.46f + 0.54f;
    const float twopi = (float)(2.0 * PI);
    for (int f = 0; f < 201; ++f)
      for (int t = 0; t < 400; ++t) {
        float om = ((twopi * (float)f) * (float)t) / 400.0f;
        basis_h[(2 * f) * 400 + t] = (float)std::cos((double)om) * win[t];
        basis_h[(2 * f + 1) * 400 + t] = -(float)std::sin((double)om) * win[t];
      }
    basis = alloc<float>(basis_h.size());
    FA_HIP(hipMemcpy(basis, basis_h.data(), basis_h.size() * 4, hipMemcpyHostToDevice));
    // HTK mel filterbank [80][204] (torchaudio melscale_fbanks(201, 20, 8000, 80, 16000, None, 'htk'))
    std::vector<float> allf = linspace_f32(0.f, 8000.f, 201);
    double mmin = 2595.0 * std::log10(1.0 + 20.0 / 700.0), mmax = 2595.0 * std::log10(1.0 + 8000.0 / 700.0);
    std::vector<float> mp = linspace_f32((float)mmin, (float)mmax, 82), fp(82);
    for (int i = 0; i < 82; ++i) fp[i] = 700.0f * ((float)std::pow(10.0, (double)(mp[i] / 2595.0f)) - 1.0f);
    std::vector<float> fb(80 * 204, 0.f);
    for (int j = 0; j < 201; ++j)
      for (int i = 0; i < 80; ++i) {
        float fd0 = fp[i + 1] - fp[i], fd1 = fp[i + 2] - fp[i + 1];
        float down = (-1.0f * (fp[i] - allf[j])) / fd0;
        float up = (fp[i + 2] - allf[j]) / fd1;
        fb[i * 204 + j] = std::max(0.0f, std::min(down, up));
      }
    fbank = alloc<float>(fb.size());
    FA_HIP(hipMemcpy(fbank, fb.data(), fb.size() * 4, hipMemcpyHostToDevice));
    // sinusoidal PE [tl_max][d_in], positions 1..T (model_definition.py:13-28)
    const int depth = ec.d_in, half = depth / 2;
    std::vector<float> pe_h((size_t)tl_max * depth);
    float inc = (float)std::log(10000.0f) / (float)(depth / 2.0 - 1.0);
    std::vector<float> inv(half);
    for (int i = 0; i < half; ++i) inv[i] = (float)std::exp((double)((float)i * -inc));
    for (int t = 0; t < tl_max; ++t)
      for (int i = 0; i < half; ++i) {
        float st = (float)(t + 1) * inv[i];
        pe_h[(size_t)t * depth + i] = (float)std::sin((double)st);
        pe_h[(size_t)t * depth + half + i] = (float)std::cos((double)st);
      }
    pe = alloc<float>(pe_h.size());
    FA_HIP(hipMemcpy(pe, pe_h.data(), pe_h.size() * 4, hipMemcpyHostToDevice));
    // RoPE cos/sin [n_ctx][head_dim/2], ggml iterative f32 theta
    const int hd = lc.head_dim / 2;
    std::vector<float> c((size_t)lc.n_ctx * hd), sn((size_t)lc.n_ctx * hd);
    const float ts = std::pow(lc.rope_theta, -2.0f / (float)lc.head_dim);
    for (int p = 0; p < lc.n_ctx; ++p) {
      float th = (float)p;
      for (int i = 0; i < hd; ++i) {
        c[(size_t)p * hd + i] = (float)std::cos((double)th);
        sn[(size_t)p * hd + i] = (float)std::sin((double)th);
        th = th * ts;
      }
    }
    rcos = alloc<float>(c.size());
    rsin = alloc<float>(sn.size());
    FA_HIP(hipMemcpy(rcos, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    FA_HIP(hipMemcpy(rsin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
  }

  static int t_lfr_of(int64_t n) { return (int)(((n / 160 + 1) + 5) / 6); }

  void build_arenas() {
    const int64_t n_eff = std::max<int64_t>(max_samples, 16000);
    tm_max = (int)(n_eff / 160 + 1);
    tl_max = t_lfr_of(n_eff);
    R = max_batch * tl_max;
    xp_stride_max = ((int64_t)160 * (tm_max - 1) + 400 + 3) / 4 * 4;
    const int d = ec.d_model;
    d_pcm = alloc<float>((size_t)max_batch * n_eff);
    xp = alloc<float>((size_t)max_batch * xp_stride_max);
    mean_part = alloc<float>((size_t)max_batch * 64);
    power = alloc<float>((size_t)max_batch * tm_max * 204);
    enc_attn_wk.part_n = ATTN_F32_PART_FLOATS;
    enc_attn_wk.part = alloc<float>(enc_attn_wk.part_n);
    enc_attn_wk.cnt_n = ATTN_F32_COUNTERS;
    enc_attn_wk.cnt = alloc<int>(enc_attn_wk.cnt_n * CNT_LINE);
    FA_HIP(hipMemset(enc_attn_wk.cnt, 0, enc_attn_wk.cnt_n * CNT_LINE * sizeof(int)));
    enc_gemm_wk.cnt_n = 512;
    // f32 64x64 splits: tiles x splits <= 512 of 256 x 16 floats; bf16x3 128x128 splits (k_gemm_bf3_sk): tiles x
    // splits <= 256 of 16 x 1024 floats
    enc_gemm_wk.part_n = std::max<int64_t>((int64_t)512 * 256 * 16, (int64_t)256 * 16 * 1024);
    enc_gemm_wk.part = alloc<float>(enc_gemm_wk.part_n);
    enc_gemm_wk.cnt = alloc<int>(enc_gemm_wk.cnt_n * CNT_LINE);
    FA_HIP(hipMemset(enc_gemm_wk.cnt, 0, enc_gemm_wk.cnt_n * CNT_LINE * sizeof(int)));
    mel = alloc<float>((size_t)max_batch * tm_max * ec.n_mels);
    const int wmax = std::max({ec.d_in, ec.d_llm, d});
    xa = alloc<float>((size_t)R * wmax);
    hbuf = alloc<float>((size_t)R * wmax);
    qkv = alloc<float>((size_t)R * 3 * std::max(d, ec.d_llm));
    att = alloc<float>((size_t)R * std::max(d, ec.d_llm));
    mem = alloc<float>((size_t)R * d);
    ffn = alloc<float>((size_t)R * std::max({ec.d_ffn, ec.adaptor_ffn, ec.ctc_ffn}));
    enc = alloc<float>((size_t)R * d);
    ad = alloc<float>((size_t)R * ec.d_llm);
    cbuf = alloc<float>((size_t)R * d);
    const int nt = cdiv(ec.ctc_vocab, 64);
    ctc_pval = alloc<float>((size_t)R * nt);
    ctc_pidx = alloc<int>((size_t)R * nt);
    ctc_ids = alloc<int>(R);
    d_nsamp = alloc<int64_t>(max_batch);
    d_tmel = alloc<int>(max_batch);
    d_tlfr = alloc<int>(max_batch);
    d_tgt = alloc<int>(max_batch);
    d_ctclen = alloc<int>(max_batch);
    d_col_ids = alloc<int>(R);
    d_col_frames = alloc<int>(R);
    d_col_n = alloc<int>(max_batch);
    // decoder
    const int E = lc.n_embd, H = lc.n_head, KV = lc.n_head_kv, D = lc.head_dim;
    m_max = std::max(lc.n_ctx, lc.max_seqs);
    // rows of one forward: a single prefill (n_ctx), a decode step (max_seqs), or a multi-sequence prefill batch
    // (fa_llm_prefill_batch: up to 8192 rows, ~55 KB of activations per row)
    pf_max = lc.max_seqs > 1 ? std::max(m_max, std::min(lc.max_seqs * lc.n_ctx, 8192)) : m_max;
    seq_stride = (int64_t)lc.n_ctx * KV * D;
    layer_stride = seq_stride * lc.max_seqs;
    kcache = alloc<__half>((size_t)layer_stride * lc.n_layer);
    vcache = alloc<__half>((size_t)layer_stride * lc.n_layer);
    lx = alloc<float>((size_t)pf_max * E);
    lqkv = alloc<float>((size_t)pf_max * (H + 2 * KV) * D);
    lq = alloc<float>((size_t)pf_max * H * D);
    latt = alloc<float>((size_t)pf_max * H * D);
    lact = alloc<float>((size_t)pf_max * lc.n_ff);
    const int kmax = std::max({E, H * D, lc.n_ff});
    lxq = alloc<int8_t>((size_t)pf_max * kmax);
    lxd = alloc<float>((size_t)pf_max * kmax / 32);
    lxq2 = alloc<int8_t>((size_t)pf_max * kmax);  // q8_0 rows produced by epilogues (attention out, SwiGLU act)
    lxd2 = alloc<float>((size_t)pf_max * kmax / 32);
    lxg = alloc<float>((size_t)lc.max_seqs * E);   // prefill batch: the last row of each sequence (LM head input)
    d_lastrow = alloc<int>(lc.max_seqs);
    logits = alloc<float>((size_t)lc.max_seqs * lc.n_vocab);
    n_part = std::max(lm_head_parts(lc.n_vocab, 1, E), cdiv(lc.n_vocab, 32));  // the GEMV's partials or one per 32-row tile
    pval = alloc<float>((size_t)lc.max_seqs * n_part);
    pidx = alloc<int>((size_t)lc.max_seqs * n_part);
    d_ssp = alloc<float>((size_t)std::max(lc.max_seqs, pf_max) * 32);  // batched decode and row-local prefill rows

    d_tok_seq = alloc<int>(pf_max);
    d_tok_pos = alloc<int>(pf_max);
    d_ptiles = alloc<int4>(pf_max);
    d_step = alloc<int>(m_max);
    d_tok_cur = alloc<int>(lc.max_seqs);
    hist_max = 4096;
    d_tok_hist = alloc<int>((size_t)lc.max_seqs * hist_max);
    FA_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_hist), (size_t)lc.max_seqs * hist_max * 4, hipHostMallocDefault));
    FA_HIP(hipEventCreateWithFlags(&ev_gen, hipEventDisableTiming));
    d_ids = alloc<int>(m_max);
    d_rowsrc = alloc<int>(pf_max);
    d_samp = alloc<SampleParams>(1);
    attn_wk.max_tokens = pf_max;
    attn_wk.max_split_tokens = m_max;
    attn_wk.max_kv = KV;
    attn_wk.counters = alloc<int>((size_t)pf_max * KV * CNT_LINE);
    FA_HIP(hipMemset(attn_wk.counters, 0, (size_t)pf_max * KV * CNT_LINE * sizeof(int)));
    attn_wk.partials = alloc<float>((size_t)m_max * KV * ATTN_SPLITS * ATTN_PART_FLOATS);
    {  // fused-layer workspace: one slab per token of a batch of up to FUSED_MAX_M
      const size_t MF = FUSED_MAX_M, nq = (size_t)(lc.n_head + 2 * lc.n_head_kv) * lc.head_dim;
      fdw.opart = alloc<float>(MF * FUSED_PARTS * E);
      fdw.dpart = alloc<float>(MF * FUSED_PARTS * E);
      fdw.act = alloc<float>(MF * 2 * (size_t)lc.n_ff);
      FA_HIP(hipMemset(fdw.act, 0, MF * 2 * (size_t)lc.n_ff * sizeof(float)));
      fdw.xmid = alloc<float>(MF * E);
      fdw.cnt = alloc<unsigned>((size_t)FUSED_CNT_LINES * CNT_LINE);
      fdw.err = alloc<int>(1);
      fdw.gqkv = reinterpret_cast<unsigned long long*>(alloc<float>(MF * 2 * nq));
      FA_HIP(hipMemset(fdw.gqkv, 0, MF * nq * 8));
      const size_t ngp = MF * FUSED_PARTS * ATTN_SPLITS * ATTN_PART_FLOATS;
      fdw.gpart = reinterpret_cast<unsigned long long*>(alloc<float>(2 * ngp));
      FA_HIP(hipMemset(fdw.gpart, 0, ngp * 8));
      fdw.pzero = alloc<float>(MF * FUSED_PARTS * E);
      FA_HIP(hipMemset(fdw.pzero, 0, MF * FUSED_PARTS * E * sizeof(float)));
    }
    FA_HIP(hipMemset(fdw.cnt, 0, (size_t)FUSED_CNT_LINES * CNT_LINE * sizeof(unsigned)));
    FA_HIP(hipMemset(fdw.err, 0, sizeof(int)));
    // split-K GEMM workspace: splits are only used below 256 tiles (x <= 8 splits, x2 for gate|up)
    gk_cnt_n = 1024;                             // tiles of a split-K launch
    gk_part_n = (int64_t)1024 * 2 * 1024;        // tiles x splits x (1 or 2 matrices) x 32 x 32 partial floats
    gk_cnt = alloc<int>(gk_cnt_n * CNT_LINE);
    gd_cnt = alloc<unsigned>(64 * CNT_LINE);  // gate|up -> down hand-off counters (re-armed in-launch)
    FA_HIP(hipMemset(gd_cnt, 0, 64 * CNT_LINE * sizeof(unsigned)));
    FA_HIP(hipMemset(gk_cnt, 0, gk_cnt_n * CNT_LINE * sizeof(int)));
    gk_part = alloc<float>(gk_part_n);
    if (lc.max_seqs >= 32) {  // k_attn_ob (M = 32): q8_0 attention rows in lxq2 / lxd2, tile partials, counters
      ob_wk.aq = lxq2;
      ob_wk.ad = lxd2;
      ob_wk.opart = alloc<float>((size_t)32 * KV * 32 * 32);
      ob_wk.cnt_g = alloc<unsigned>((size_t)(KV + 32) * CNT_LINE);
      ob_wk.cnt_s = ob_wk.cnt_g + (size_t)KV * CNT_LINE;
      FA_HIP(hipMemset(ob_wk.cnt_g, 0, (size_t)(KV + 32) * CNT_LINE * sizeof(unsigned)));
      ob_wk.err = fdw.err;
      hipDeviceProp_t prop;
      FA_HIP(hipGetDeviceProperties(&prop, device));
      if (prop.multiProcessorCount < KV * 32) use_attn_ob = false;  // one 16-wave block per CU, all resident
    } else {
      use_attn_ob = false;
    }
    n_past.assign(lc.max_seqs, 0);
    last_tok.assign(lc.max_seqs, -1);
    logits_row.assign(lc.max_seqs, -1);
  }

  // ---------------------------------------------------------------------------------------------
  void synthetic(uint32_t seed) {
    float* tmp = nullptr;
    int64_t tmp_n = 0;
    for (const std::string& name : spec_order) {
      Slot& s = slots[name];
      const uint32_t key = lowbias32_h(fnv1a32(name) ^ (uint32_t)(seed * 0x9E3779B9u));
      if (s.kind == 0) {
        launch_synth_fill(s.f, s.n, key, s.scale, s.offset, stream);
      } else {
        if (tmp_n < s.n) {
          if (tmp) {
            FA_HIP(hipStreamSynchronize(stream));
            FA_HIP(hipFree(tmp));
          }
          FA_HIP(hipMalloc(&tmp, s.n * 4));
          tmp_n = s.n;
        }
        launch_synth_fill(tmp, s.n, key, s.scale, s.offset, stream);
        launch_quant_q8_0(tmp, s.n, s.q, s.d, stream);
      }
      s.set = true;
    }
    FA_HIP(hipStreamSynchronize(stream));
    if (tmp) FA_HIP(hipFree(tmp));
  }

  Slot& slot(const char* name) {
    auto it = slots.find(name);
    if (it == slots.end()) {
      set_error(std::string("unknown tensor ") + name);
      throw arg_failure();
    }
    return it->second;
  }

  // ---------------------------------------------------------------------------------------------
  // encoder forward (batch, device pcm)
  void enc_lin(const float* A, int64_t lda, const float* W, const float* b, float* C, int64_t ldc, int M, int N, int K,
               int relu = 0, const float* add1 = nullptr, int64_t ld1 = 0, const float* add2 = nullptr, int64_t ld2 = 0,
               APlanes ap = {}, APlanes cp = {}) {
    hipEvent_t ev;
    prof_begin(1, &ev);
    gemm_linear(A, lda, W, K, b, C, ldc, M, N, K, relu, add1, ld1, add2, ld2, stream, W16(W), &enc_gemm_wk, WB(W), ap,
                cp);
    prof_end(1, 0, 2.0 * M * N * K);
  }

  // bf16x3 encoder: the SANM blocks' GEMM inputs (LN1, attention, LN2 and ffn1 outputs, each read only by one bf16x3
  // GEMM) travel as bf16 hi / lo planes, written by their producers instead of f32 (FUNASR_ENC_PLANES=0: f32, A/B).
  // Same split as the GEMM staging applies to an f32 row: bit-identical products. The planes of a [rows][ld] tensor
  // live in the f32 buffer it replaces: hi at its start, lo rows * ld elements later (4 B per element either way).
  // Measured (profiles/r05_exp_enc_planes_ab.txt): one 60 s clip 11.3-11.5 -> 11.0-11.2 ms, but batch 32 103.7-104.3 ->
  // 105.8-106.2 ms (the 256x256 tile reads A as two half-line streams instead of one), so planes are used while no
  // GEMM of the call takes the 256x256 tile (below enc_planes_max_rows rows; FUNASR_ENC_PLANES=2: always)
  int enc_planes = 1;
  int enc_planes_max_rows = 6000;
  bool planes_on(int rows) const {
    return !enc_fp16 && enc_gemm && (enc_planes == 2 || (enc_planes == 1 && rows < enc_planes_max_rows));
  }
  static APlanes planes_in(float* buf, int rows, int ld) {
    uint16_t* hi = reinterpret_cast<uint16_t*>(buf);
    return APlanes{hi, hi + (size_t)rows * ld};
  }

  void sanm(const EncBlockW& w, int rows, int ts, const int* lens, bool first) {
    const int d = ec.d_model;
    const float* xin = first ? hbuf : xa;  // block0 input = PE'd LFR features (hbuf holds them)
    float* x = xa;
    // planes fit the f32 buffers they replace (att holds rows x max(d, d_llm) floats, ffn rows x >= d_ffn floats)
    const bool pl = planes_on(rows) && std::max(w.d_in, d) <= std::max(d, ec.d_llm) && WB(w.qkv_w).hi &&
                    WB(w.out_w).hi && WB(w.w1).hi && WB(w.w2).hi;
    const APlanes p_ln1 = pl ? planes_in(att, rows, w.d_in) : APlanes{}, p_att = pl ? planes_in(att, rows, d) : APlanes{};
    const APlanes p_ffn = pl ? planes_in(ffn, rows, ec.d_ffn) : APlanes{};
    // LN1
    layernorm(first ? xin : x, w.d_in, att, w.d_in, w.ln1_w, w.ln1_b, rows, w.d_in, 1e-5f, nullptr, ts, stream, r16(),
              p_ln1);
    enc_lin(att, w.d_in, w.qkv_w, w.qkv_b, qkv, 3 * d, rows, 3 * d, w.d_in, 0, nullptr, 0, nullptr, 0, p_ln1);
    fsmn(qkv + 2 * d, 3 * d, w.fsmn_w, mem, d, rows, d, ec.fsmn_k, lens, ts, stream, r16());
    {
      hipEvent_t ev;
      prof_begin(2, &ev);
      attn_f32(qkv, qkv + d, qkv + 2 * d, 3 * d, 3 * d, 3 * d, att, d, rows / ts, ts, ec.n_heads, d / ec.n_heads, lens,
               enc_attn_wk, stream, r16(), bf3_attn(), p_att);
      prof_end(2, 0, 4.0 * rows * (double)ts * d);
    }
    if (first) {
      enc_lin(att, d, w.out_w, w.out_b, x, d, rows, d, d, 0, nullptr, 0, mem, d, p_att);
      return;
    }
    enc_lin(att, d, w.out_w, w.out_b, x, d, rows, d, d, 0, x, d, mem, d, p_att);
    layernorm(x, d, hbuf, d, w.ln2_w, w.ln2_b, rows, d, 1e-5f, nullptr, ts, stream, r16(), p_att);
    enc_lin(hbuf, d, w.w1, w.b1, ffn, ec.d_ffn, rows, ec.d_ffn, d, 1, nullptr, 0, nullptr, 0, p_att, p_ffn);
    enc_lin(ffn, ec.d_ffn, w.w2, w.b2, x, d, rows, d, ec.d_ffn, 0, x, d, nullptr, 0, p_ffn);
  }

  // CorrectTransformerAdaptor: out [rows][d_out] in `out`; uses hbuf/qkv/att/ffn as scratch
  void run_adaptor(const AdaptorW& a, const float* in, int d_enc, int d_out, int d_ffn, int n_heads, float* out,
                   int rows, int ts, const int* lens) {
    enc_lin(in, d_enc, a.l1_w, a.l1_b, ffn, d_ffn, rows, d_ffn, d_enc, 1);
    enc_lin(ffn, d_ffn, a.l2_w, a.l2_b, out, d_out, rows, d_out, d_ffn);
    for (const AdBlockW& b : a.blocks) {
      layernorm(out, d_out, hbuf, d_out, b.ln1_w, b.ln1_b, rows, d_out, 1e-12f, nullptr, ts, stream, r16());
      enc_lin(hbuf, d_out, b.qkv_w, b.qkv_b, qkv, 3 * d_out, rows, 3 * d_out, d_out);
      {
        hipEvent_t ev;
        prof_begin(2, &ev);
        attn_f32(qkv, qkv + d_out, qkv + 2 * d_out, 3 * d_out, 3 * d_out, 3 * d_out, att, d_out, rows / ts, ts, n_heads,
                 d_out / n_heads, lens, enc_attn_wk, stream, r16(), bf3_attn());
        prof_end(2, 0, 4.0 * rows * (double)ts * d_out);
      }
      enc_lin(att, d_out, b.o_w, b.o_b, out, d_out, rows, d_out, d_out, 0, out, d_out);
      layernorm(out, d_out, hbuf, d_out, b.ln2_w, b.ln2_b, rows, d_out, 1e-12f, nullptr, ts, stream, r16());
      enc_lin(hbuf, d_out, b.w1, b.b1, ffn, d_out / 4, rows, d_out / 4, d_out, 1);
      enc_lin(ffn, d_out / 4, b.w2, b.b2, out, d_out, rows, d_out, d_out / 4, 0, out, d_out);
    }
  }

  // ---- independent-clip encodes (fa_set_encode_mode(1)): every clip runs the single-clip encode (its own row count,
  // tiles, key splits: the arithmetic of encoding it alone) in a lane of its own -- rows [b tl_max, +tl_max) of the
  // batch arenas, its own split-K / attention workspaces, its own HIP stream -- so up to kEncLanes one-clip encodes
  // (each too small to fill the chip) run concurrently. The fetch / collapse calls then read clip b at row b tl_max.
  static constexpr int kEncLanes = 8;
  struct EncBind {
    hipStream_t stream;
    AttnF32Work attn;
    GemmF32Work gemm;
    float *xp, *mean_part, *power, *mel, *xa, *hbuf, *qkv, *att, *mem, *ffn, *enc, *ad, *cbuf, *ctc_pval;
    int *ctc_pidx, *ctc_ids;
    int64_t* d_nsamp;
    int *d_tmel, *d_tlfr, *d_tgt, *d_ctclen;
    fa::U8Work u8;
  };
  struct EncLane {
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    AttnF32Work attn;
    GemmF32Work gemm;
    fa::U8Work u8;  // int8-dynamic CTC activations (allocated once the int8 graph is active)
  };
  std::vector<EncLane> enc_lanes;
  int encode_mode = 0;  // 0: padded batch; 1: independent clips in concurrent lanes
  int64_t* hp_meta = nullptr;  // pinned per-clip length records: region 0 = batch encode, 1 + lane = lane encode
  int meta_slot = 0;
  hipEvent_t ev_meta[kEncLanes + 1] = {};  // recorded after a region's copies; the host waits on it before rewriting
  // the pinned record of meta_slot, once the copies that last read it (an earlier call, still queued) have run
  int64_t* meta_region() {
    if (!hp_meta) {
      FA_HIP(hipHostMalloc(&hp_meta, (size_t)(kEncLanes + 1) * max_batch * 6 * sizeof(int64_t), hipHostMallocDefault));
    }
    hipEvent_t& ev = ev_meta[meta_slot];
    if (ev) FA_HIP(hipEventSynchronize(ev));
    else FA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return hp_meta + (size_t)meta_slot * max_batch * 6;
  }
  hipEvent_t ev_fork = nullptr;

  EncBind enc_bind() const {
    return EncBind{stream, enc_attn_wk, enc_gemm_wk, xp, mean_part, power, mel, xa, hbuf, qkv, att, mem, ffn, enc, ad, cbuf,
                   ctc_pval, ctc_pidx, ctc_ids, d_nsamp, d_tmel, d_tlfr, d_tgt, d_ctclen, u8wk};
  }
  void enc_rebind(const EncBind& b) {
    stream = b.stream; enc_attn_wk = b.attn; enc_gemm_wk = b.gemm; xp = b.xp; mean_part = b.mean_part; power = b.power;
    mel = b.mel; xa = b.xa; hbuf = b.hbuf; qkv = b.qkv; att = b.att; mem = b.mem; ffn = b.ffn; enc = b.enc; ad = b.ad;
    cbuf = b.cbuf; ctc_pval = b.ctc_pval; ctc_pidx = b.ctc_pidx; ctc_ids = b.ctc_ids; d_nsamp = b.d_nsamp;
    d_tmel = b.d_tmel; d_tlfr = b.d_tlfr; d_tgt = b.d_tgt; d_ctclen = b.d_ctclen; u8wk = b.u8;
  }
  EncLane& enc_lane(int i) {
    if ((int)enc_lanes.size() <= i) enc_lanes.resize(i + 1);
    EncLane& l = enc_lanes[i];
    if (!l.s) {
      FA_HIP(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking));
      FA_HIP(hipEventCreateWithFlags(&l.done, hipEventDisableTiming));
      // the arrival counters start at zero (zeroed once, re-armed by the combining blocks). The zeroing is enqueued on
      // the lane's own stream, ahead of its kernels: a plain hipMemset runs on the null stream, which a non-blocking
      // stream does not wait for, and reused device memory is not zero (a lane created mid-run then raced it)
      l.attn = enc_attn_wk;
      l.attn.part = alloc<float>(l.attn.part_n);
      l.attn.cnt = alloc<int>(l.attn.cnt_n * CNT_LINE);
      FA_HIP(hipMemsetAsync(l.attn.cnt, 0, l.attn.cnt_n * CNT_LINE * sizeof(int), l.s));
      l.gemm = enc_gemm_wk;
      l.gemm.part = alloc<float>(l.gemm.part_n);
      l.gemm.cnt = alloc<int>(l.gemm.cnt_n * CNT_LINE);
      FA_HIP(hipMemsetAsync(l.gemm.cnt, 0, l.gemm.cnt_n * CNT_LINE * sizeof(int), l.s));
    }
    return l;
  }

  void encode_independent(const float* pcm, const int64_t* n_samples, int batch, int64_t stride) {
    FA_REQUIRE(batch >= 1 && batch <= max_batch, "batch out of range");
    if (enc_fp16) prepare_fp16();
    else if (enc_gemm) prepare_bf3();
    if (!ev_fork) FA_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    FA_HIP(hipEventRecord(ev_fork, stream));
    const EncBind base = enc_bind();
    const int d = ec.d_model, wmax = std::max({ec.d_in, ec.d_llm, d}), nt = cdiv(ec.ctc_vocab, 64);
    const size_t T = tl_max;
    std::vector<int> tl(batch), tg(batch), cl(batch);
    try {
      for (int b = 0; b < batch; ++b) {
        EncLane& l = enc_lane(b % kEncLanes);
        // the lane's previous clip used the same workspaces and pinned length record: the host waits for it (the
        // record is rewritten at enqueue time)
        if (b >= kEncLanes) FA_HIP(hipEventSynchronize(l.done));
        FA_HIP(hipStreamWaitEvent(l.s, ev_fork, 0));
        if (ctc_int8_active() && !l.u8.xq) l.u8 = make_u8work(tl_max, 1);
        EncBind lb = base;
        lb.stream = l.s; lb.attn = l.attn; lb.gemm = l.gemm; lb.u8 = l.u8;
        lb.xp += b * xp_stride_max; lb.mean_part += b * 64; lb.power += b * (size_t)tm_max * 204;
        lb.mel += b * (size_t)tm_max * ec.n_mels; lb.xa += b * T * wmax; lb.hbuf += b * T * wmax;
        lb.qkv += b * T * 3 * std::max(d, ec.d_llm); lb.att += b * T * std::max(d, ec.d_llm); lb.mem += b * T * d;
        lb.ffn += b * T * std::max({ec.d_ffn, ec.adaptor_ffn, ec.ctc_ffn}); lb.enc += b * T * d; lb.ad += b * T * ec.d_llm;
        lb.cbuf += b * T * d; lb.ctc_pval += b * T * nt; lb.ctc_pidx += b * T * nt; lb.ctc_ids += b * T;
        lb.d_nsamp += b; lb.d_tmel += b; lb.d_tlfr += b; lb.d_tgt += b; lb.d_ctclen += b;
        enc_rebind(lb);
        meta_slot = 1 + b % kEncLanes;
        encode_device(pcm + (size_t)b * stride, n_samples + b, 1, stride);
        meta_slot = 0;
        FA_HIP(hipEventRecord(l.done, l.s));
        tl[b] = h_tlfr[0];
        tg[b] = h_tgt[0];
        cl[b] = h_ctclen[0];
        enc_rebind(base);
      }
    } catch (...) {
      enc_rebind(base);
      meta_slot = 0;
      throw;
    }
    for (int i = 0; i < std::min(batch, kEncLanes); ++i) FA_HIP(hipStreamWaitEvent(stream, enc_lanes[i].done, 0));
    h_tlfr = tl;
    h_tgt = tg;
    h_ctclen = cl;
    last_batch = batch;
    last_tstride = tl_max;  // clip b's rows start at b tl_max
    ++enc_gen;
  }

  void encode_device(const float* pcm, const int64_t* n_samples, int batch, int64_t stride) {
    FA_REQUIRE(batch >= 1 && batch <= max_batch, "batch out of range");
    std::vector<int> tmel(batch), ctcl(batch);
    h_tlfr.assign(batch, 0);
    h_tgt.assign(batch, 0);
    h_ctclen.assign(batch, 0);
    int tm_stride = 1, ts = 1;
    for (int b = 0; b < batch; ++b) {
      const int64_t n = n_samples[b];
      FA_REQUIRE(n >= 1 && n <= max_samples, "n_samples out of range");
      FA_REQUIRE(n <= stride, "n_samples > stride");
      tmel[b] = (int)(n / 160 + 1);
      h_tlfr[b] = (tmel[b] + 5) / 6;
      const int o1 = 1 + (h_tlfr[b] - 3 + 2) / 2;
      h_tgt[b] = (1 + (o1 - 3 + 2) / 2 - 1) / 2 + 1;
      // CPU-EP policy (nano_onnx.py:90-99): clips < 1 s are zero-padded to 1 s; the unmasked CTC head
      // then runs over the padded length (model_definition.py:336)
      h_ctclen[b] = t_lfr_of(std::max<int64_t>(n, 16000));
      tm_stride = std::max(tm_stride, tmel[b]);
      ts = std::max(ts, h_ctclen[b]);
    }
    const int64_t xps = ((int64_t)160 * (tm_stride - 1) + 400 + 3) / 4 * 4;
    const int rows = batch * ts;
    last_batch = batch;
    last_tstride = ts;
    ++enc_gen;
    // the per-clip lengths go up from pinned host memory owned by the engine (one region per encode lane), so no
    // copy depends on when the runtime reads a pageable source (the lane loop reuses the host vectors at once)
    int64_t* hm = meta_region();
    int32_t* hm32 = reinterpret_cast<int32_t*>(hm + max_batch);
    for (int b = 0; b < batch; ++b) {
      hm[b] = n_samples[b];
      hm32[b] = tmel[b];
      hm32[max_batch + b] = h_tlfr[b];
      hm32[2 * max_batch + b] = h_tgt[b];
      hm32[3 * max_batch + b] = h_ctclen[b];
    }
    FA_HIP(hipMemcpyAsync(d_nsamp, hm, batch * sizeof(int64_t), hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tmel, hm32, batch * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tlfr, hm32 + max_batch, batch * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tgt, hm32 + 2 * max_batch, batch * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_ctclen, hm32 + 3 * max_batch, batch * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipEventRecord(ev_meta[meta_slot], stream));
    // F1-F4
    if (enc_fp16) prepare_fp16();
    else if (enc_gemm) prepare_bf3();
    frontend_preemph(pcm, stride, d_nsamp, batch, mean_part, xp, xps, stream, r16());
    {
      hipEvent_t ev;
      prof_begin(1, &ev);
      gemm_stft_power(xp, xps, tm_stride, batch * tm_stride, enc_fp16 ? basis16 : basis, power, 204, stream, r16());
      prof_end(1, 0, 2.0 * batch * tm_stride * 402.0 * 400.0);
    }
    gemm_mel_log(power, 204, enc_fp16 ? fbank16 : fbank, 204, mel, batch * tm_stride, ec.n_mels, 201, stream, r16());
    frontend_lfr(mel, tm_stride, d_tmel, d_tlfr, pe, hbuf, batch, ts, ec.n_mels, ec.lfr_m, ec.lfr_n, stream, r16());
    if (debug_flags & 1) {
      if (!tap_lfr) tap_lfr = alloc<float>((size_t)tl_max * ec.d_in);
      // LFR features before the x*sqrt(512)+PE embed are not materialised; the tap holds the embedded rows
      FA_HIP(hipMemcpyAsync(tap_lfr, hbuf, (size_t)ts * ec.d_in * 4, hipMemcpyDeviceToDevice, stream));
    }
    // SenseVoiceEncoderSmall (embed is folded into frontend_lfr: x*sqrt(512) + PE)
    const int d = ec.d_model;
    for (size_t i = 0; i < enc_blocks.size(); ++i) {
      if ((int)i == ec.n_blocks) {
        layernorm(xa, d, xa, d, after_w, after_b, rows, d, 1e-5f, d_tlfr, ts, stream, r16());
      }
      sanm(enc_blocks[i], rows, ts, d_tlfr, i == 0);
    }
    if ((int)enc_blocks.size() == ec.n_blocks)
      layernorm(xa, d, xa, d, after_w, after_b, rows, d, 1e-5f, d_tlfr, ts, stream, r16());
    layernorm(xa, d, enc, d, tp_w, tp_b, rows, d, 1e-5f, d_tlfr, ts, stream, r16());
    // adaptor (key mask = valid frames) -> ad [rows][d_llm]
    run_adaptor(adaptor, enc, d, ec.d_llm, ec.adaptor_ffn, ec.adaptor_heads, ad, rows, ts, d_tlfr);
    // CTC head (reference: unmasked over the clip's own frames -> key length = ctc_len)
    if (ctc_int8_active()) {
      run_ctc_int8(enc, rows, ts, d_ctclen);
      return;
    }
    run_adaptor(ctc_dec, enc, d, d, ec.ctc_ffn, ec.ctc_heads, cbuf, rows, ts, d_ctclen);
    {
      hipEvent_t ev;
      prof_begin(1, &ev);
      gemm_ctc_argmax(cbuf, d, ctc_w, ctc_b, rows, ec.ctc_vocab, d, ctc_pval, ctc_pidx, ctc_ids, stream, W16(ctc_w),
                      WB(ctc_w));
      prof_end(1, 0, 2.0 * rows * (double)ec.ctc_vocab * d);
    }
  }

  // CTC head alone over a caller's encoder output (the CTC graph's own session, decoder.py:27: ctc_decoder with
  // mask=None, then ctc_lo and argmax, model_definition.py:335-337): T rows, every key unmasked. Uses the encode
  // buffers, so the previous encode's outputs are gone afterwards (fa_encode_fetch then fails).
  void ctc_head(const float* enc_host, int T, int32_t* ids_out) {
    FA_REQUIRE(T >= 1 && T <= tl_max, "fa_ctc_head: T out of range (1 .. the T_lfr of max_samples)");
    const int d = ec.d_model;
    last_batch = 0;
    ++enc_gen;
    if (enc_fp16) prepare_fp16();
    else if (enc_gemm) prepare_bf3();
    int32_t* hm32 = reinterpret_cast<int32_t*>(meta_region() + max_batch);
    hm32[3 * max_batch] = T;
    FA_HIP(hipMemcpyAsync(d_ctclen, hm32 + 3 * max_batch, 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipEventRecord(ev_meta[meta_slot], stream));
    FA_HIP(hipMemcpyAsync(enc, enc_host, (size_t)T * d * 4, hipMemcpyHostToDevice, stream));
    if (ctc_int8_active()) {
      run_ctc_int8(enc, T, T, d_ctclen);
    } else {
      run_adaptor(ctc_dec, enc, d, d, ec.ctc_ffn, ec.ctc_heads, cbuf, T, T, d_ctclen);
      gemm_ctc_argmax(cbuf, d, ctc_w, ctc_b, T, ec.ctc_vocab, d, ctc_pval, ctc_pidx, ctc_ids, stream, W16(ctc_w),
                      WB(ctc_w));
    }
    FA_HIP(hipMemcpyAsync(ids_out, ctc_ids, (size_t)T * 4, hipMemcpyDeviceToHost, stream));
    FA_HIP(hipStreamSynchronize(stream));
  }

  // ---------------------------------------------------------------------------------------------
  // prefill rows -> query tiles of <= 64 consecutive positions of one sequence (uploaded on the stream; host copy
  // kept in h_ptiles until the next call). Below attn_pf_min_m rows (or head dim != 128) the per-row path runs.
  std::vector<int4> h_ptiles;
  bool ptiles_f16 = true;  // the tiles run k_attn_prefill_h (prefill_attn_f16), else k_attn_prefill
  // rl (row-local forward): tiles at every row count (a threshold on the call's rows would give a prompt other
  // arithmetic alone than in a batch), on the f16-MFMA tile kernel only: a row's result there depends on its own keys
  // alone (fully masked key tiles add exact zeros, rescale by exactly 1), so the forward stays row-local
  void set_prefill_tiles(const int* sq, const int* ps, int rows, bool rl = false) {
    n_ptiles = 0;
    ptiles_f16 = prefill_attn_f16();
    if (rl ? (!ptiles_f16 || !attn_pf_rl) : rows < attn_pf_min_m) return;
    if (lc.head_dim != 128 || lc.n_head != 2 * lc.n_head_kv) return;
    h_ptiles.clear();
    for (int r = 0; r < rows; ++r) {
      const bool cont = r > 0 && h_ptiles.back().y < 64 && h_ptiles.back().z == sq[r] && ps[r - 1] + 1 == ps[r];
      if (cont) ++h_ptiles.back().y;
      else h_ptiles.push_back(make_int4(r, 1, sq[r], 0));
    }
    n_ptiles = (int)h_ptiles.size();
    FA_HIP(hipMemcpyAsync(d_ptiles, h_ptiles.data(), n_ptiles * sizeof(int4), hipMemcpyHostToDevice, stream));
  }

  // decoder forward over M token rows (embeddings already in lx, positions in d_tok_pos)
  // n_last > 0 (prefill batch): logits for rows d_lastrow[0 .. n_last) (each sequence's last prompt row)
  void llm_forward(int M, bool decode, int max_pos, int n_last = 0) {
    // decode: every row is a different sequence (continuous batch), logits for all rows;
    // prefill: rows are consecutive positions of one sequence, logits for the last row only.
    const int E = lc.n_embd, H = lc.n_head, KV = lc.n_head_kv, D = lc.head_dim, F = lc.n_ff;
    const int QKV = (H + 2 * KV) * D;
    // row-local prefill (pf_row_local): every row's arithmetic that of its own sequence's prefill (gemv_q8 row_local;
    // attention in f16 query tiles that never span two sequences (attn_pf_rl), or one key split per row; never the
    // fused-GEMV path, whose use would depend on the call's row count)
    const int rl = !decode && pf_row_local ? 1 : 0;
    const bool small = gemv_small(M) && !rl;
    // batched decode: the residual GEMMs (o, down) quantise their new rows times the next RMSNorm weight and leave
    // per-token sum-of-squares partials; q|k|v, gate|up and the LM head apply rstd to those rows' block scales
    // (no k_prep_q8 launches but layer 0's)
    const bool fused = decode && fused_layer_runs(M);
    const bool nrm = decode && !small && M <= 32 && E == 1024 && use_nrm && !fused;
    // row-local prefill: the same producer-normalised rows on the K-in-block GEMMs (k_gemm_q8_kw NRM): the o / down
    // residual epilogues quantise x * the next RMSNorm weight and leave sum-of-squares partials, q|k|v and gate|up apply
    // rstd to the block scales: no k_prep_q8 launch but layer 0's (FUNASR_PREFILL_NRM=0: the prep launches, A/B)
    const bool pnrm = rl && E == 1024 && use_pnrm && M <= pf_max;

    (void)max_pos;
    if (fused) {
      llm_forward_fused(M);
      if (M == 1) return;  // the batch-1 LM head completes the residual in its prologue
      psum_rows(fdw.xmid, fdw.dpart, M, E, lx, stream);
    }
    for (int l = 0; l < (fused ? 0 : lc.n_layer); ++l) {
      const LlmLayerW& w = layers[l];
      // sampled timing: layer 1's launches stand for layers 1 .. n_layer - 1 (identical shapes; from layer 1 on the
      // weights arrive L2-warm from the previous launches' prefetch slabs); layer 0, which also carries the first
      // slabs, is timed as its own class (5); prefill forwards go to class 6
      prof_sample = l <= (lc.n_layer > 2 ? 1 : 0);
      prof_layer0 = l == 0 && lc.n_layer > 2;
      prof_prefill = !decode;
      __half* kc = kcache + (size_t)l * layer_stride;
      __half* vc = vcache + (size_t)l * layer_stride;
      GemvArgs a{};
      a.M = M;
      a.eps = lc.rms_eps;
      a.row_local = rl;
      // q|k|v = W . rms_norm(x)*attn_norm
      a.wq = w.qkv.q; a.wd = w.qkv.d; a.O = QKV; a.rpw = gemv_rows_per_wave(QKV);
      a.out = lqkv; a.ldo = QKV;
      if (small) { a.x = lx; a.ldx = E; a.norm_w = w.attn_norm; }
      else if ((nrm || pnrm) && l > 0) { a.xq = lxq; a.xd = lxd; a.ssp = d_ssp; }  // rows from the previous down epilogue
      else { prep_q8(lx, E, w.attn_norm, lc.rms_eps, M, E, lxq, lxd, stream); a.xq = lxq; a.xd = lxd; }
      // batched decode: each split-K GEMM pulls the next one's weight rows into the reading XCDs' L2 (gemm_l2_prefetch)
      const bool gpf = nrm && fa::g_gemm_pf;
      auto set_pf = [&](GemvArgs& x, int bit, const Q8Mat& m, const Q8Mat* m2, int O, int K) {
        if (!gpf || !(fa::g_gemm_pf & bit)) return;
        x.pf_q = m.q; x.pf_d = m.d; x.pf_q2 = m2 ? m2->q : nullptr; x.pf_d2 = m2 ? m2->d : nullptr;
        x.pf_O = O; x.pf_K = K; x.pf_slabs = fa::g_gemm_pf_slabs; x.pf_delay = fa::g_gemm_pf_delay;
      };
      set_pf(a, 8, w.o, nullptr, E, H * D);
      gemv(a, E, 0);
      // M = 32 batched decode: attention, o projection, residual and the NRM epilogue in one launch (k_attn_ob)
      const bool ob = nrm && M == 32 && use_attn_ob && fused_shape_ok() && ob_wk.opart;
      if (ob) {
        hipEvent_t ev;
        prof_begin(3, &ev);
        attn_o_batched(lqkv, w.q_norm, w.k_norm, lc.rms_eps, rcos, rsin, kc, vc, M, H, KV, d_tok_seq, d_tok_pos,
                       seq_stride, w.o.q, w.o.d, E, ob_wk, lx, w.ffn_norm, lxq, lxd, d_ssp, stream);
        prof_end(3, 0, 0);
      }
      if (!ob) {
        hipEvent_t ev;
        prof_begin(3, &ev);
        if (!decode)
          qk_rope_store(lqkv, M, H, KV, lc.rms_eps, w.q_norm, w.k_norm, rcos, rsin, d_tok_seq, d_tok_pos, lq, kc, vc,
                        seq_stride, stream);
        // M > 4: the attention also leaves its rows as q8_0 blocks for the o GEMM (no prep launch)
        if (!decode && n_ptiles > 0)  // query tiles: each K/V tile serves 64 rows x 2 heads (set_prefill_tiles)
          attn_prefill(d_ptiles, n_ptiles, d_tok_pos, H, KV, seq_stride, kc, vc, lq, latt, small ? nullptr : lxq2,
                       small ? nullptr : lxd2, stream, ptiles_f16);
        else
          attn_block(decode ? lqkv : lq, decode ? 1 : 0, w.q_norm, w.k_norm, lc.rms_eps, rcos, rsin, kc, vc, M, H, KV,
                     d_tok_seq, d_tok_pos, seq_stride, latt, attn_wk, stream, small ? nullptr : lxq2,
                     small ? nullptr : lxd2, rl ? 1 : ATTN_SPLITS);
        prof_end(3, 0, 0);
      }
      // x += Wo . attn
      GemvArgs o{};
      o.M = M; o.eps = lc.rms_eps; o.wq = w.o.q; o.wd = w.o.d; o.O = E; o.rpw = gemv_rows_per_wave(E);
      o.row_local = rl;
      o.out = lx; o.ldo = E; o.res = lx; o.ldr = E;
      if (small) { o.x = latt; o.ldx = H * D; }
      else { o.xq = lxq2; o.xd = lxd2; }
      if (nrm || pnrm) { o.ssp_out = d_ssp; o.qout = lxq; o.dout = lxd; o.qn_w = w.ffn_norm; }
      set_pf(o, 1, w.gate, &w.up, F, E);
      if (!ob) gemv(o, H * D, 1);
      // act = silu(Wg . h) * (Wu . h), h = rms_norm(x)*ffn_norm
      GemvArgs g{};
      g.M = M; g.eps = lc.rms_eps; g.wq = w.gate.q; g.wd = w.gate.d; g.wq2 = w.up.q; g.wd2 = w.up.d; g.O = F;
      g.row_local = rl;
      g.rpw = gemv_rows_per_wave(F); g.out = lact; g.ldo = F;
      if (small) { g.x = lx; g.ldx = E; g.norm_w = w.ffn_norm; }
      else {
        if (nrm || pnrm) { g.xq = lxq; g.xd = lxd; g.ssp = d_ssp; }  // rows from the o epilogue
        else { prep_q8(lx, E, w.ffn_norm, lc.rms_eps, M, E, lxq, lxd, stream); g.xq = lxq; g.xd = lxd; }
        g.qout = lxq2; g.dout = lxd2;  // SwiGLU epilogue quantises act for the down GEMM (no prep launch)
      }
      set_pf(g, 2, w.down, nullptr, E, F);
      // x += Wdown . act
      GemvArgs dn{};
      dn.M = M; dn.eps = lc.rms_eps; dn.wq = w.down.q; dn.wd = w.down.d; dn.O = E; dn.rpw = gemv_rows_per_wave(E);
      dn.row_local = rl;
      dn.out = lx; dn.ldo = E; dn.res = lx; dn.ldr = E;
      if (small) { dn.x = lact; dn.ldx = F; }
      else { dn.xq = lxq2; dn.xd = lxd2; }
      if (nrm || (pnrm && l + 1 < lc.n_layer)) {  // (prefill: the LM head reads the last layer's f32 rows)
        dn.ssp_out = d_ssp; dn.qout = lxq; dn.dout = lxd;
        dn.qn_w = l + 1 < lc.n_layer ? layers[l + 1].attn_norm : out_norm;
      }
      if (l + 1 < lc.n_layer) set_pf(dn, 4, layers[l + 1].qkv, nullptr, QKV, E);
      if (!(nrm && decode && use_gu_down && gemv_gu_down(g, dn))) {
        gemv(g, E, 2);
        gemv(dn, F, 1);
      }
    }
    prof_sample = true;
    prof_layer0 = prof_prefill = false;
    // lm_head (tied token_embd) with fused argmax partials: all rows (decode), the last row (prefill) or each
    // sequence's last row (prefill batch)
    const int n_rows = decode ? M : n_last > 0 ? n_last : 1;
    const float* xrow = decode ? lx : lx + (size_t)(M - 1) * E;
    if (!decode && n_last > 0) {
      gather_rows(lx, d_lastrow, n_last, E, lxg, stream);
      xrow = lxg;
    }
    GemvArgs h{};
    h.M = n_rows; h.eps = lc.rms_eps; h.wq = tok_embd.q; h.wd = tok_embd.d; h.O = lc.n_vocab;
    h.rpw = gemv_rows_per_wave(lc.n_vocab);
    h.out = logits; h.ldo = lc.n_vocab;
    h.pval = pval; h.pidx = pidx; h.n_part = n_part_cur = lm_head_parts(lc.n_vocab, n_rows, E);
    chunk_cur = lm_head_chunk(lc.n_vocab, n_rows, E);
    if (gemv_small(n_rows)) { h.x = xrow; h.ldx = E; h.norm_w = out_norm; }
    else if (nrm) { h.xq = lxq; h.xd = lxd; h.ssp = d_ssp; }  // rows from the last down epilogue
    else { prep_q8(xrow, E, out_norm, lc.rms_eps, n_rows, E, lxq, lxd, stream); h.xq = lxq; h.xd = lxd; }
    gemv(h, E, 3);
  }

  // the two-launch layer gives every token of a batch of up to fused_max_m its own grid slab with the batch-1
  // arithmetic, and the LM head is the fused GEMV up to g_gemv_small_max tokens (the MFMA LM head above sums in
  // another f32 order); every other decode path is only known to be invariant at width 1
  int invariant_width() const {
    if (use_fused == 1 && fused_shape_ok()) return std::max(1, std::min(fused_max_m, fa::g_gemv_small_max));
    return 1;
  }

  // a decode step of M sequences runs on the fused layer (two- or three-launch); else on the 5-launch / batched layer
  bool fused_layer_runs(int M) const {
    return fused_shape_ok() && ((M == 1 && use_fused) || (M <= fused_max_m && use_fused == 1));
  }

  bool fused_shape_ok() const {
    return lc.n_embd == 1024 && lc.n_ff == 3072 && lc.n_head == 16 && lc.n_head_kv == 8 && lc.head_dim == 128;
  }

  // batch-1 decode step through the fused layer (llm.hip "Fused batch-1 decode layer"): per layer
  //   A  q|k|v GEMV, prologue x = x_mid + sum dpart (layer > 0; block 0 stores x to lx)
  //   B  attention + this split's slice of the o projection -> opart
  //   C  x_mid = lx + sum opart; gate|up + SwiGLU; group fan-in; slice of the down projection -> dpart
  // then the LM head with the same partial-sum prologue.
  // M > 1 (small decode batches, two-launch layer only): every launch has one grid slab per token; the layers end
  // with x_mid + partials per token, which llm_forward sums (psum_rows) for the regular LM head.
  void llm_forward_fused(int M = 1) {
    const int E = lc.n_embd, H = lc.n_head, KV = lc.n_head_kv, D = lc.head_dim, F = lc.n_ff;
    const int QKV = (H + 2 * KV) * D;
    for (int l = 0; l < lc.n_layer; ++l) {
      const LlmLayerW& w = layers[l];
      prof_sample = l <= (lc.n_layer > 2 ? 1 : 0);
      prof_layer0 = l == 0 && lc.n_layer > 2;  // as in llm_forward
      __half* kc = kcache + (size_t)l * layer_stride;
      __half* vc = vcache + (size_t)l * layer_stride;
      if (use_fused == 1) {
        // batch 1: extra blocks of the attention launch pull this layer's FFN weights and the next layer's attention
        // weights / K/V rows into the L2 of the XCDs that will read them (llm.hip l2_prefetch)
        fa::L2Prefetch pf;
        pf.gq = w.gate.q; pf.gd = w.gate.d; pf.uq = w.up.q; pf.ud = w.up.d; pf.dq = w.down.q; pf.dd = w.down.d;
        pf.F = F;
        if (l + 1 < lc.n_layer) {
          const LlmLayerW& wn = layers[l + 1];
          pf.qkv_q = wn.qkv.q; pf.qkv_d = wn.qkv.d; pf.o_q = wn.o.q; pf.o_d = wn.o.d;
          pf.kc = kcache + (size_t)(l + 1) * layer_stride;
          pf.vc = vcache + (size_t)(l + 1) * layer_stride;
        }
        // a q8_0 weight-streaming layer launch (class 0, like C): algorithmic bytes = q|k|v + Wo weights + the K/V
        // rows of positions [0, pos] of every kv head (fp16 K and V: 2 x KV x D x 2 B per position)
        hipEvent_t ev;
        prof_begin(0, &ev);
        if (step_mask & 1)
        qkv_attn_o_fused(l == 0 ? lx : fdw.xmid, l == 0 ? nullptr : fdw.dpart, lx, w.attn_norm, w.qkv.q, w.qkv.d, lqkv,
                         w.q_norm, w.k_norm, lc.rms_eps, rcos, rsin, kc, vc, H, KV, d_tok_seq, d_tok_pos, seq_stride,
                         w.o.q, w.o.d, E, attn_wk, fdw, stream, M, (debug_flags & 2) ? 1 : 0, &pf);
        prof_end(0, (double)(E * H * D + (size_t)QKV * E) * 34.0 / 32.0 + (M == 1 ? 4.0 * KV * D * (prof_pos + 1.0) : 0.0),
                 2.0 * M * (E * H * D + (double)QKV * E));
      } else {
        GemvArgs a{};
        a.M = 1;
        a.eps = lc.rms_eps;
        a.wq = w.qkv.q; a.wd = w.qkv.d; a.O = QKV; a.rpw = gemv_rows_per_wave(QKV);
        a.out = lqkv; a.ldo = QKV; a.ldx = E; a.norm_w = w.attn_norm;
        if (l == 0) a.x = lx;
        else { a.x = fdw.xmid; a.psum = fdw.dpart; a.xsum = lx; }
        gemv(a, E, 0);
      }
      if (use_fused != 1) {
        hipEvent_t ev;
        prof_begin(3, &ev);
        attn_o_fused(lqkv, w.q_norm, w.k_norm, lc.rms_eps, rcos, rsin, kc, vc, H, KV, d_tok_seq, d_tok_pos, seq_stride,
                     w.o.q, w.o.d, E, attn_wk, fdw, stream);
        prof_end(3, (double)E * H * D * 34.0 / 32.0, 0);
      }
      {
        hipEvent_t ev;
        prof_begin(0, &ev);
        if (step_mask & 2)
          ffn_fused(lx, w.ffn_norm, lc.rms_eps, w.gate.q, w.gate.d, w.up.q, w.up.d, w.down.q, w.down.d, E, F, fdw, stream,
                    M);
        prof_end(0, 3.0 * F * E * 34.0 / 32.0, 2.0 * 3.0 * M * F * E);
      }
    }
    prof_sample = true;
    prof_layer0 = false;
    if (M > 1) return;
    GemvArgs h{};
    h.M = 1; h.eps = lc.rms_eps; h.wq = tok_embd.q; h.wd = tok_embd.d; h.O = lc.n_vocab;
    h.rpw = gemv_rows_per_wave(lc.n_vocab);
    h.out = logits; h.ldo = lc.n_vocab;
    h.pval = pval; h.pidx = pidx; h.n_part = n_part_cur = lm_head_parts(lc.n_vocab, 1, E);
    chunk_cur = lm_head_chunk(lc.n_vocab, 1, E);
    h.x = fdw.xmid; h.ldx = E; h.norm_w = out_norm; h.psum = fdw.dpart;
    if (step_mask & 4) gemv(h, E, 3);
  }

  // a fused-decode fan-in timeout (a group not co-resident: another kernel held CUs) leaves the chunk's outputs
  // garbage; -> true (flag cleared) when one happened
  bool fused_error() {
    int err = 0;
    FA_HIP(hipMemcpy(&err, fdw.err, sizeof(int), hipMemcpyDeviceToHost));
    if (err) FA_HIP(hipMemsetAsync(fdw.err, 0, sizeof(int), stream));  // ordered before the next launches
    return err != 0;
  }

  // enqueue n_steps decode steps for seqs from the host state (n_past, last_tok): fa_llm_generate_begin's body, also
  // the re-run of a chunk whose fused layer timed out
  void enqueue_steps(const int32_t* seqs, int n_seqs, int n_steps) {
    std::vector<int> sq(n_seqs), ps(n_seqs), cur(n_seqs), zero(n_seqs, 0);
    for (int i = 0; i < n_seqs; ++i) {
      sq[i] = seqs[i];
      ps[i] = n_past[seqs[i]];
      cur[i] = last_tok[seqs[i]];
    }
    FA_HIP(hipMemcpyAsync(d_tok_seq, sq.data(), n_seqs * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tok_pos, ps.data(), n_seqs * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tok_cur, cur.data(), n_seqs * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_step, zero.data(), n_seqs * 4, hipMemcpyHostToDevice, stream));
    // input row of the first step (later steps get theirs from the sampler launch)
    fa::embed_rows(tok_embd.q, tok_embd.d, d_tok_cur, n_seqs, lc.n_embd, 0, lx, stream);
    // the sampler reads its parameters from device memory, so the captured step graph serves every setting.
    // Profiling runs eager (event nodes inside graphs do not time individual nodes on ROCm 7.2).
    if (use_graphs && !prof) {
      int st = 0;
      if (graph_steps > 1 && n_steps >= graph_steps) {
        const hipGraphExec_t exk = step_graph(n_seqs, graph_steps);
        for (; st + graph_steps <= n_steps; st += graph_steps) FA_HIP(hipGraphLaunch(exk, stream));
      }
      if (st < n_steps) {
        const hipGraphExec_t ex = step_graph(n_seqs);
        for (; st < n_steps; ++st) {
          FA_HIP(hipGraphLaunch(ex, stream));
          // profiling aid (FUNASR_GRAPH_SYNC_EVERY): bound the captured-graph packets in flight (under rocprofv3 with
          // HIP's graph packet capture on, more than a queue ring of them crashes the process: DESIGN.md section 4)
          if (graph_sync_every > 0 && (st + 1) % graph_sync_every == 0) FA_HIP(hipStreamSynchronize(stream));
        }
      }
    } else {
      for (int st = 0; st < n_steps; ++st) {
        prof_pos = ps[0] + st;  // the profiled fused layer's K/V bytes (batch 1)
        decode_step(n_seqs);
      }
    }
    // the sampled tokens land in pinned host memory; fa_llm_generate_end waits for them (the host may work meanwhile)
    FA_HIP(hipMemcpyAsync(h_hist, d_tok_hist, (size_t)n_seqs * hist_max * 4, hipMemcpyDeviceToHost, stream));
    FA_HIP(hipEventRecord(ev_gen, stream));
  }

  // the landed chunk ran on the fused layer and a fan-in timed out (a group was not co-resident: another kernel or
  // process held CUs). Decode the chunk again from the same host state (positions and input tokens were not advanced;
  // a re-run overwrites the chunk's K/V rows before any step reads them, and its draws are keyed on the same (seed,
  // seq, pos)): first on the fused layer again, which gives exactly the tokens an undisturbed chunk gives; only if that
  // times out too, on the 5-launch layer for this chunk (agreeing to the q8_0 noise floor), and the next chunk probes
  // the fused layer again. After kFusedGiveUp such chunks in a row the engine keeps the 5-launch layer.
  static constexpr int kFusedGiveUp = 3;
  void drop_step_graphs() {
    for (auto& g : step_graphs) FA_HIP(hipGraphExecDestroy(g.second));
    step_graphs.clear();  // captured steps bake the layer structure and the debug hook in
  }
  void rerun_chunk() {
    enqueue_steps(gen_seqs.data(), (int)gen_seqs.size(), gen_steps);
    FA_HIP(hipEventSynchronize(ev_gen));
  }
  void recover_fused_chunk() {
    if ((debug_flags & 2) && !(debug_flags & 4)) {  // test hook: bit 1 withholds one hand-off once, bit 2 every time
      debug_flags &= ~2;
      drop_step_graphs();
    }
    ++fused_retries;
    rerun_chunk();
    if (!fused_error()) {
      fused_fail_streak = 0;
      log(2, "fused decode: an in-launch fan-in timed out; the chunk's re-run on the fused layer completed");
      return;
    }
    ++fused_recoveries;
    const bool give_up = ++fused_fail_streak >= kFusedGiveUp;
    log(3, std::string("fused decode: the chunk's re-run timed out too; running it on the 5-launch layer") +
               (give_up ? " and keeping that layer for this engine" : " (the next chunk probes the fused layer again)"));
    const int fused_mode = use_fused;
    use_fused = 0;
    debug_flags &= ~6;
    drop_step_graphs();
    rerun_chunk();
    FA_REQUIRE(!fused_error(), "decode chunk re-run: error flag set on the 5-launch layer");
    drop_step_graphs();
    if (!give_up) use_fused = fused_mode;
  }

  // one prompt's prefill (fa_llm_prefill; also a long prompt of a row-local batch): row-local up to pf_rl_max rows (a
  // prompt's arithmetic is then the same alone and in a row-local batch); above, the tiled forward (query-tiled
  // attention, tiled GEMMs), which is faster there (scripts/prof_prefill_long.py: 2000 rows 19.8 vs 32.4 ms; 512 / 1024
  // rows 5.5 / 12.4 ms row-local vs 11.0 / 13.4 tiled; 1536 rows row-local 21.5 ms)
  // where a prefill's input rows come from: a host array [rows, n_embd] (fa_llm_prefill / _batch), or row codes
  // (fa_llm_prefill_rows: the caller's rows already in d_prow, or adaptor rows of the last encode)
  struct PromptSrc {
    const float* embd = nullptr;
    const int32_t* codes = nullptr;
  };
  // rows [off, off + n) of each part, back to back into lx
  void load_prompt_rows(const PromptSrc& src, const std::vector<std::pair<int64_t, int>>& parts) {
    const int E = lc.n_embd;
    if (src.embd) {
      int64_t r = 0;
      for (const auto& p : parts) {
        FA_HIP(hipMemcpyAsync(lx + r * E, src.embd + p.first * E, (size_t)p.second * E * 4, hipMemcpyHostToDevice,
                              stream));
        r += p.second;
      }
      return;
    }
    int64_t n = 0;
    for (const auto& p : parts) n += p.second;
    FA_REQUIRE(n <= pf_max, "prompt rows exceed the row capacity");
    // the codes go through an engine-owned pinned buffer: the copy may still be queued when this call returns, so
    // the source must outlive it (rewritten only after the event of its last copy)
    if (!hp_rowsrc) {
      FA_HIP(hipHostMalloc(reinterpret_cast<void**>(&hp_rowsrc), (size_t)std::max<int64_t>(pf_max, 1) * 4,
                           hipHostMallocDefault));
      FA_HIP(hipEventCreateWithFlags(&ev_rowsrc, hipEventDisableTiming));
    } else {
      FA_HIP(hipEventSynchronize(ev_rowsrc));
    }
    int64_t r = 0;
    for (const auto& p : parts) {
      std::memcpy(hp_rowsrc + r, src.codes + p.first, (size_t)p.second * 4);
      r += p.second;
    }
    FA_HIP(hipMemcpyAsync(d_rowsrc, hp_rowsrc, (size_t)n * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipEventRecord(ev_rowsrc, stream));
    fa::prompt_rows(d_prow, ad, last_tstride, d_rowsrc, (int)n, E, lx, stream);
  }
  int32_t* hp_rowsrc = nullptr;  // pinned staging of the prompt row codes (load_prompt_rows)
  hipEvent_t ev_rowsrc = nullptr;

  void prefill_one(int seq, const PromptSrc& src, int64_t off, int n_tokens, int32_t* tok_out, float* logits_out) {
    load_prompt_rows(src, {{off, n_tokens}});
    std::vector<int> sq(n_tokens, seq), ps(n_tokens);
    for (int i = 0; i < n_tokens; ++i) ps[i] = n_past[seq] + i;
    FA_HIP(hipMemcpyAsync(d_tok_seq, sq.data(), n_tokens * 4, hipMemcpyHostToDevice, stream));
    FA_HIP(hipMemcpyAsync(d_tok_pos, ps.data(), n_tokens * 4, hipMemcpyHostToDevice, stream));
    set_prefill_tiles(sq.data(), ps.data(), n_tokens, n_tokens <= pf_rl_max);
    pf_row_local = n_tokens <= pf_rl_max;
    try {
      llm_forward(n_tokens, false, n_past[seq] + n_tokens - 1);
    } catch (...) {
      pf_row_local = false;
      throw;
    }
    pf_row_local = false;
    n_ptiles = 0;
    // the first token's draw is keyed by the last prompt row's (seq, position)
    sample(1, d_tok_seq + (n_tokens - 1), d_tok_pos + (n_tokens - 1), nullptr, d_tok_cur, nullptr);
    int tok = 0;
    FA_HIP(hipMemcpyAsync(&tok, d_tok_cur, 4, hipMemcpyDeviceToHost, stream));
    if (logits_out) FA_HIP(hipMemcpyAsync(logits_out, logits, (size_t)lc.n_vocab * 4, hipMemcpyDeviceToHost, stream));
    FA_HIP(hipStreamSynchronize(stream));
    prof_collect();
    n_past[seq] += n_tokens;
    last_tok[seq] = tok;
    std::fill(logits_row.begin(), logits_row.end(), -1);
    logits_row[seq] = 0;
    if (tok_out) *tok_out = tok;
  }

  // one decode step for the n active sequences: embed last token -> forward -> sample -> advance
  void decode_step(int n) {
    // profiled (eager) steps: give the host a head start so the sampled event pairs time back-to-back kernels,
    // not host launch gaps
    if (prof) gpu_delay_us(1500, stream);
    llm_forward(n, true, 0);
    // sample, then the next step's input row + position advance in the same launch (the first step's row is
    // embedded by fa_llm_generate before the steps)
    EmbedNext en;
    en.qs = tok_embd.q; en.d = tok_embd.d; en.E = lc.n_embd; en.x = lx; en.tok_pos = d_tok_pos;
    if (step_mask & 8) sample(n, d_tok_seq, d_tok_pos, d_step, d_tok_cur, d_tok_hist, &en);
  }

  // hipGraph of one decode step (all per-step state, the sampler parameters included, lives in device memory;
  // grids are n_past-independent), one per batch width
  // k > 1: k consecutive steps in one graph (one replay instead of k: no inter-graph gap between the steps)
  hipGraphExec_t step_graph(int n, int k = 1) {
    const int key = n * 1024 + k;
    auto it = step_graphs.find(key);
    if (it != step_graphs.end()) return it->second;
    hipGraph_t g;
    hipGraphExec_t ex;
    FA_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < k; ++i) decode_step(n);
    FA_HIP(hipStreamEndCapture(stream, &g));
    FA_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    FA_HIP(hipGraphDestroy(g));
    return step_graphs[key] = ex;
  }

  // gate|up + down in one launch (batched decode, FUNASR_GU_DOWN); false: shape not covered
  bool gemv_gu_down(const GemvArgs& g0, const GemvArgs& d0) {
    GemvArgs g = g0;
    g.kpart = gk_part;
    g.kpart_n = gk_part_n;
    g.kcnt = gk_cnt;
    g.kcnt_n = gk_cnt_n;
    hipEvent_t ev;
    prof_begin(0, &ev);
    const bool ok = fa::gemm_q8_gu_down(g, d0, gd_cnt, fdw.err, stream);
    const double F = lc.n_ff, E = lc.n_embd;
    prof_end(0, ok ? 3.0 * F * E * 34.0 / 32.0 : 0.0, ok ? 2.0 * 3.0 * g.M * F * E : 0.0);
    return ok;
  }

  void gemv(const GemvArgs& a0, int K, int epi) {
    GemvArgs a = a0;
    a.kpart = gk_part;
    a.kpart_n = gk_part_n;
    a.kcnt = gk_cnt;
    a.kcnt_n = gk_cnt_n;
    hipEvent_t ev;
    const int cls = epi == 3 ? 4 : 0;  // LM head (fused argmax) is its own class: it is not layer-sampled
    prof_begin(cls, &ev);
    gemv_q8(a, K, epi, stream);
    const double wbytes = (double)a.O * K * (epi == 2 ? 2.0 : 1.0) * 34.0 / 32.0;
    prof_end(cls, wbytes, 2.0 * a.M * a.O * K * (epi == 2 ? 2.0 : 1.0));
  }

  // stage the call's sampler parameters in device memory (stream-ordered before the launches that read them;
  // h_samp stays untouched until the call's closing synchronise)
  void set_sampling(const fa_sampling* s) {
    h_samp = SampleParams{s ? s->temperature : 0.f, s ? s->top_p : 1.f, s ? s->top_k : 1, s ? s->seed : 0u};
    FA_REQUIRE(h_samp.temperature == h_samp.temperature && h_samp.top_p == h_samp.top_p, "sampling: NaN parameter");
    FA_HIP(hipMemcpyAsync(d_samp, &h_samp, sizeof(SampleParams), hipMemcpyHostToDevice, stream));
  }
  void sample(int M, const int* row_seq, const int* row_pos, int* step_ctr, int* tok_out, int* hist,
              const EmbedNext* en = nullptr) {
    sample_tokens(logits, lc.n_vocab, lc.n_vocab, pval, pidx, n_part_cur, chunk_cur, M, d_samp, row_seq, row_pos, step_ctr, tok_out,
                  hist, hist_max, en, stream);
  }
};

}  // namespace fa

using fa::Engine;

struct fa_engine {
  Engine* e;
};

#define FA_API_BEGIN try {
#define FA_API_END                 \
  }                                \
  catch (fa::hip_failure&) {       \
    return FA_ERR_HIP;             \
  }                                \
  catch (fa::arg_failure&) {       \
    return FA_ERR_ARG;             \
  }                                \
  catch (std::exception & ex) {    \
    fa::set_error(ex.what());      \
    return FA_ERR_STATE;           \
  }                                \
  return FA_OK;

extern "C" {

const char* fa_last_error(void) { return fa::g_err.c_str(); }

int fa_set_log_callback(void (*cb)(int32_t, const char*, void*), void* user) {
  fa::g_log_cb = cb;
  fa::g_log_ud = user;
  return FA_OK;
}

int fa_engine_create(int32_t device, const fa_encoder_config* enc, const fa_llm_config* llm, int32_t max_batch,
                     int64_t max_samples, fa_engine** out) {
  if (!enc || !llm || !out || max_batch < 1 || max_samples < 1) {
    fa::set_error("fa_engine_create: bad arguments");
    return FA_ERR_ARG;
  }
  Engine* e = new Engine();
  try {
    e->device = device;
    e->ec = *enc;
    e->lc = *llm;
    e->max_batch = max_batch;
    e->max_samples = max_samples;
    FA_REQUIRE(enc->d_model % 64 == 0 && enc->d_model / enc->n_heads <= 128, "d_model/heads");
    FA_REQUIRE(llm->head_dim == 128 && llm->n_head == 2 * llm->n_head_kv, "decoder head layout");
    FA_REQUIRE(llm->n_embd % 1024 == 0 && llm->n_ff % 1024 == 0, "decoder widths must be multiples of 1024");
    FA_HIP(hipSetDevice(device));
    if (const char* m = getenv("FUNASR_CU_MASK")) {  // experiment hook: comma-separated hex 32-bit CU mask words
      std::vector<uint32_t> words;
      for (const char* p = m; *p;) {
        char* end = nullptr;
        words.push_back((uint32_t)strtoul(p, &end, 16));
        if (!end || end == p) break;
        p = *end == ',' ? end + 1 : end;
      }
      FA_HIP(hipExtStreamCreateWithCUMask(&e->stream, (uint32_t)words.size(), words.data()));
    } else {
      FA_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    }
    if (const char* g = getenv("FUNASR_GRAPHS")) e->use_graphs = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_GEMM_KW")) fa::g_gemm_q8_kw = atoi(g) != 0;
    // A/B knobs of the decode GEMV: fused-GEMV batch limit (0..7; lm_head partials are sized for <= 7) and
    // tokens per fused-GEMV block (1 or 2: the instantiated and tested variants)
    {  // process-wide decode-path knob: re-read (or reset to the default 5) at every engine creation
      const char* g = getenv("FUNASR_GEMV_SMALL");
      fa::g_gemv_small_max = g ? std::min(7, std::max(0, atoi(g))) : 6;
    }
    if (const char* g = getenv("FUNASR_GEMV_MT")) fa::g_gemv_mt = atoi(g) >= 2 ? 2 : 1;
    if (const char* g = getenv("FUNASR_GEMM_F32_SPLIT")) fa::g_gemm_f32_split = atoi(g) != 0;
    {  // process-wide split-K shape knob: re-read (or reset) at every engine creation
      const char* g = getenv("FUNASR_SK_MIN_BLOCKS");
      fa::g_sk_min_blocks = g ? std::max(1, atoi(g)) : 128;
    }
    {
      const char* g = getenv("FUNASR_LM_HEAD_MT6");
      fa::g_lm_head_mt6 = g ? atoi(g) != 0 : 1;
    }
    {  // small-batch MFMA LM head (k_lm_head_s): re-read (or reset) at every engine creation
      const char* g = getenv("FUNASR_LM_HEAD_S");
      fa::g_lm_head_s = g ? std::min(2, std::max(0, atoi(g))) : 1;
      const char* g1 = getenv("FUNASR_LM_HEAD_S1");
      fa::g_lm_head_s1 = g1 ? std::min(2, std::max(0, atoi(g1))) : 0;
      const char* g2 = getenv("FUNASR_LM_GRID");
      fa::g_lm_grid = g2 ? std::max(0, atoi(g2)) : 0;
    }
    if (const char* g = getenv("FUNASR_STEP_MASK")) e->step_mask = atoi(g) & 15;
    if (const char* g = getenv("FUNASR_GRAPH_SYNC_EVERY")) e->graph_sync_every = std::max(0, atoi(g));
    if (const char* g = getenv("FUNASR_GRAPH_STEPS")) e->graph_steps = std::min(64, std::max(1, atoi(g)));
    if (const char* g = getenv("FUNASR_FUSED_DECODE")) e->use_fused = std::min(2, std::max(0, atoi(g)));
    if (const char* g = getenv("FUNASR_FUSED_MAX_M")) e->fused_max_m = std::min(fa::FUSED_MAX_M, std::max(1, atoi(g)));
    fa::g_ffn_pair_min_m = 2;
    fa::g_gemm_bf3_pf = 2;
    if (const char* g = getenv("FUNASR_BF3_PF")) fa::g_gemm_bf3_pf = atoi(g) >= 2 ? 2 : 1;
    // 256x256 bf16x3 tiles from 192 tiles per launch (batched encoder; bit-identical outputs): scripts/ubench/
    // gemm_f32_bench at M = 32032: 292-330 vs 243-276 TF/s f32-equivalent for the 128x128 tiles
    fa::g_gemm_bf3_256 = 192;
    if (const char* g = getenv("FUNASR_BF3_256")) fa::g_gemm_bf3_256 = std::max(0, atoi(g));
    if (const char* g = getenv("FUNASR_F16_GEMM")) fa::g_gemm_f16_b3 = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_BF3_MID")) fa::g_gemm_bf3_mid = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_BF3_KW4")) fa::g_gemm_bf3_kw4 = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_F16_DEEP")) fa::g_gemm_f16_deep = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_BF3_256_S")) fa::g_gemm_bf3_256_s = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_BF3_DMA")) fa::g_gemm_bf3_dma = atoi(g) != 0;
    {
      const char* g = getenv("FUNASR_ATTN_MERGE");  // encoder attention key splits merged by their own launch
      fa::g_attn_merge = g ? atoi(g) != 0 : 1;
      g = getenv("FUNASR_ATTN_MS");
      fa::g_attn_ms = g ? atoi(g) : 8;
      g = getenv("FUNASR_ATTN_KS");  // A/B: encoder attention key splits (0 = automatic, 1-8)
      fa::g_attn_f32_force_splits = g ? std::max(0, std::min(8, atoi(g))) : 0;
    }
    {  // the few-tile K splits: every creation takes the environment's setting or the default
      const char* g = getenv("FUNASR_BF3_SK");
      fa::g_gemm_bf3_sk = g ? atoi(g) != 0 : 1;
      g = getenv("FUNASR_F16_SK");
      fa::g_gemm_f16_sk = g ? atoi(g) != 0 : 1;
      g = getenv("FUNASR_BF3_SK_KMIN");
      fa::g_gemm_bf3_sk_kmin = g ? std::max(64, atoi(g)) : 2048;
      g = getenv("FUNASR_BF3_BIG");
      fa::g_gemm_bf3_big = g ? std::max(1, atoi(g)) : 1024;
      g = getenv("FUNASR_F16_PF32");
      fa::g_gemm_f16_pf32 = g ? atoi(g) != 0 : 1;
      g = getenv("FUNASR_BF3_PF_KB");
      fa::g_gemm_bf3_pf_kb = g ? (atoi(g) == 32 ? 32 : atoi(g) == 64 ? 64 : 0) : 0;
      g = getenv("FUNASR_EPI_GROUPED");
      fa::g_gemm_epi_grouped = g ? atoi(g) != 0 : 1;
      g = getenv("FUNASR_BF3_SK_KS");
      fa::g_gemm_bf3_sk_ks = g ? std::max(0, std::min(8, atoi(g))) : 0;
    }
    if (const char* g = getenv("FUNASR_BF3_PERSIST")) fa::g_gemm_bf3_persist = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_WAB")) fa::g_attn_wab = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_GEMM_T_WAB")) fa::g_gemm_t_wab = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_F32_WAB")) fa::g_gemm_f32_wab = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_LM_TR")) fa::g_lm_tr = atoi(g) != 0;
    {  // process-wide decode-path knobs: re-read (or reset) at every engine creation
      // o -> gate|up, gate|up -> down, down -> next q|k|v with 4 slabs after 0.5 us: graph-replayed step at batch
      // 8 / 16 / 24 / 32 1.145 / 1.163 / 1.228 / 1.241-1.246 -> 1.104 / 1.124 / 1.187 / 1.194 ms
      // (profiles/r04_exp_gemm_pf.txt; q|k|v -> o across the attention launch: slower)
      const char* gp = getenv("FUNASR_GEMM_PF");
      fa::g_gemm_pf = gp ? atoi(gp) & 15 : 7;
      const char* gs = getenv("FUNASR_GEMM_PF_SLABS");
      fa::g_gemm_pf_slabs = gs ? std::min(8, std::max(1, atoi(gs))) : 4;
      const char* gd = getenv("FUNASR_GEMM_PF_DELAY");
      fa::g_gemm_pf_delay = gd ? std::max(0, atoi(gd)) : 50;
      const char* g = getenv("FUNASR_L2PF");
      // 16 blocks per kv head (one block per CU with the 128 compute blocks), after 0.5 us: graph-replayed batch-1
      // step 0.4537-0.4549 vs 0.4740-0.4784 ms (scripts/gpu_r4_l2pf.sh; 8 / 12 / 20 / 24 blocks and 1.0-2.5 us slower)
      fa::g_l2pf_blocks = g ? std::min(64, std::max(0, atoi(g))) : 16;
      const char* d = getenv("FUNASR_L2PF_DELAY");
      fa::g_l2pf_delay = d ? std::max(0, atoi(d)) : 50;
      const char* mm = getenv("FUNASR_L2PF_MAX_M");  // set: one mask for every batch up to it (A/B); unset: the table
      fa::g_l2pf_max_m = mm ? std::max(1, atoi(mm)) : 0;
      const char* k = getenv("FUNASR_L2PF_MASK");
      fa::g_l2pf_mask = k ? atoi(k) & 7 : 7;
    }
    if (const char* g = getenv("FUNASR_PF_ROW_LOCAL_MAX")) e->pf_rl_max = std::max(1, atoi(g));
    if (const char* g = getenv("FUNASR_F16_ATTN")) fa::g_attn_f16_mfma = atoi(g) != 0;
    // batched decode attention: one 16-wave block per (token, kv head) once there are 256 of them (a CU each):
    // scripts/ubench/attn_batch at batch 32, 42.7 MB of K/V: 14.65 vs 15.7-15.9 us for the split blocks
    fa::g_attn_wide = 256;
    if (const char* g = getenv("FUNASR_ATTN_WIDE")) fa::g_attn_wide = std::max(0, atoi(g));
    if (const char* g = getenv("FUNASR_ATTN_LDSPF")) fa::g_attn_ldspf = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_PF_F16")) fa::g_attn_pf_f16 = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_XCD")) fa::g_attn_xcd = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_PF_RL")) e->attn_pf_rl = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_FSMN_VEC")) fa::g_fsmn_vec = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ENC_PLANES")) e->enc_planes = std::min(2, std::max(0, atoi(g)));
    if (const char* g = getenv("FUNASR_FFN_PAIR_MIN_M")) fa::g_ffn_pair_min_m = std::max(2, atoi(g));
    {  // process-wide knob: re-read (or reset) at every engine creation
      const char* g = getenv("FUNASR_FFN_WIDE");
      fa::g_ffn_wide = g ? atoi(g) != 0 : 0;
    }
    if (const char* g = getenv("FUNASR_DECODE_NRM")) e->use_nrm = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_GU_DOWN")) e->use_gu_down = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_OB")) e->use_attn_ob = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_PREFILL_NRM")) e->use_pnrm = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ALLOC_FILL")) sscanf(g, "%d:%d:%d", &e->fill_lo, &e->fill_hi, &e->fill_byte);
    {  // process-wide GEMM shape knob: re-read (or reset) at every engine creation
      const char* g = getenv("FUNASR_GEMM_T_MIN_M");
      fa::g_gemm_t_min_m = g ? std::max(1, atoi(g)) : 512;
    }
    if (const char* g = getenv("FUNASR_LM_HEAD_B")) fa::g_lm_head_b = atoi(g) != 0;
    if (const char* g = getenv("FUNASR_ATTN_PREFILL_MIN_M")) e->attn_pf_min_m = std::max(1, atoi(g));
    if (const char* g = getenv("FUNASR_ENC_GEMM")) e->enc_gemm = strcmp(g, "f32") == 0 ? 0 : 1;
    e->build_arenas();
    e->build_constants();
    e->build_encoder();
    e->build_llm();
    FA_HIP(hipDeviceSynchronize());
  } catch (...) {
    delete e;
    return FA_ERR_HIP;
  }
  *out = new fa_engine{e};
  return FA_OK;
}

int fa_engine_destroy(fa_engine* h) {
  if (!h) return FA_OK;
  delete h->e;
  delete h;
  return FA_OK;
}

int fa_weights_synthetic(fa_engine* h, uint32_t seed) {
  FA_API_BEGIN
  h->e->synthetic(seed);
  h->e->weights_changed();
  for (auto& kv : h->e->slots)
    if (kv.second.kind == 0) h->e->u8_invalidate(kv.second.f, kv.second.n);
  FA_API_END
}

int fa_set_tensor_f32(fa_engine* h, const char* name, const float* host, int64_t n) {
  FA_API_BEGIN
  Engine* e = h->e;
  fa::Slot& s = e->slot(name);
  FA_REQUIRE(n == s.n, std::string("size mismatch for ") + name);
  if (s.kind == 0) {
    FA_HIP(hipMemcpyAsync(s.f, host, n * 4, hipMemcpyHostToDevice, e->stream));
    e->weights_changed();
    e->u8_invalidate(s.f, s.n);
  } else {
    float* tmp = nullptr;
    FA_HIP(hipMalloc(&tmp, n * 4));
    FA_HIP(hipMemcpyAsync(tmp, host, n * 4, hipMemcpyHostToDevice, e->stream));
    fa::launch_quant_q8_0(tmp, n, s.q, s.d, e->stream);
    FA_HIP(hipStreamSynchronize(e->stream));
    FA_HIP(hipFree(tmp));
  }
  FA_HIP(hipStreamSynchronize(e->stream));
  s.set = true;
  FA_API_END
}

int fa_set_tensor_q8_0(fa_engine* h, const char* name, const uint8_t* blocks, int64_t n_bytes) {
  FA_API_BEGIN
  Engine* e = h->e;
  fa::Slot& s = e->slot(name);
  FA_REQUIRE(s.kind == 1, std::string("not a q8_0 tensor: ") + name);
  FA_REQUIRE(n_bytes == s.n / 32 * 34, std::string("q8_0 size mismatch for ") + name);
  uint8_t* tmp = nullptr;
  FA_HIP(hipMalloc(&tmp, n_bytes));
  FA_HIP(hipMemcpyAsync(tmp, blocks, n_bytes, hipMemcpyHostToDevice, e->stream));
  fa::launch_unpack_q8_0(tmp, s.n / 32, s.q, s.d, e->stream);
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_HIP(hipFree(tmp));
  s.set = true;
  FA_API_END
}

int fa_get_tensor_q8_0(fa_engine* h, const char* name, uint8_t* out, int64_t n_bytes) {
  FA_API_BEGIN
  Engine* e = h->e;
  fa::Slot& s = e->slot(name);
  FA_REQUIRE(s.kind == 1 && n_bytes == s.n / 32 * 34, "fa_get_tensor_q8_0: size/kind");
  uint8_t* tmp = nullptr;
  FA_HIP(hipMalloc(&tmp, n_bytes));
  fa::launch_pack_q8_0(s.q, s.d, s.n / 32, tmp, e->stream);
  FA_HIP(hipMemcpyAsync(out, tmp, n_bytes, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_HIP(hipFree(tmp));
  FA_API_END
}

int fa_get_tensor_f32(fa_engine* h, const char* name, float* out, int64_t n) {
  FA_API_BEGIN
  Engine* e = h->e;
  fa::Slot& s = e->slot(name);
  FA_REQUIRE(s.kind == 0 && n == s.n, "fa_get_tensor_f32: size/kind");
  FA_HIP(hipMemcpyAsync(out, s.f, n * 4, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_API_END
}

int fa_weights_mark_unset(fa_engine* h, const char* prefix) {
  FA_API_BEGIN
  const std::string p = prefix ? prefix : "";
  for (auto& kv : h->e->slots)
    if (kv.first.compare(0, p.size(), p) == 0) {
      kv.second.set = false;
      if (kv.second.kind == 0) h->e->u8_invalidate(kv.second.f, kv.second.n);
    }
  FA_API_END
}

int fa_tensor_names(fa_engine* h, const char* prefix, int32_t only_unset, char* buf, int64_t cap, int64_t* needed) {
  FA_API_BEGIN
  Engine* e = h->e;
  const std::string p = prefix ? prefix : "";
  std::string out;
  for (const std::string& name : e->spec_order) {
    if (name.compare(0, p.size(), p) != 0) continue;
    if (only_unset && e->slots[name].set) continue;
    if (!out.empty()) out += '\n';
    out += name;
  }
  if (needed) *needed = (int64_t)out.size() + 1;
  FA_REQUIRE(buf == nullptr || cap >= (int64_t)out.size() + 1, "fa_tensor_names: buffer too small");
  if (buf) memcpy(buf, out.c_str(), out.size() + 1);
  FA_API_END
}

int fa_load_gguf(fa_engine* h, const char* path) {
  FA_API_BEGIN
  Engine* e = h->e;
  fa::GGUFFile g;
  FA_REQUIRE(g.open(path), std::string("cannot read GGUF: ") + fa::gguf_error());
  for (const auto& t : g.tensors) {
    auto it = e->slots.find(t.name);
    if (it == e->slots.end()) {
      fa::log(3, "gguf: ignoring tensor " + t.name);
      continue;
    }
    fa::Slot& s = it->second;
    FA_REQUIRE(t.n_elements == s.n, "gguf: element count mismatch for " + t.name);
    const uint8_t* data = g.data(t);
    if (t.type == fa::GGML_Q8_0) {
      FA_REQUIRE(fa_set_tensor_q8_0(h, t.name.c_str(), data, t.n_bytes) == FA_OK, "gguf q8_0 upload");
    } else if (t.type == fa::GGML_F32) {
      FA_REQUIRE(fa_set_tensor_f32(h, t.name.c_str(), (const float*)data, t.n_elements) == FA_OK, "gguf f32 upload");
    } else if (t.type == fa::GGML_F16) {
      std::vector<float> tmp(t.n_elements);
      const uint16_t* hp = (const uint16_t*)data;
      for (int64_t i = 0; i < t.n_elements; ++i) tmp[i] = fa::half_to_float_host(hp[i]);
      FA_REQUIRE(fa_set_tensor_f32(h, t.name.c_str(), tmp.data(), t.n_elements) == FA_OK, "gguf f16 upload");
    } else {
      FA_REQUIRE(false, "gguf: unsupported tensor type for " + t.name);
    }
  }
  FA_API_END
}

int fa_encode_device(fa_engine* h, const float* d_pcm, const int64_t* n_samples, int32_t batch, int64_t stride) {
  FA_API_BEGIN
  Engine* e = h->e;
  if (!d_pcm) {
    FA_REQUIRE((int64_t)batch * stride <= e->pcm_uploaded, "fa_encode_device(NULL): upload the PCM first");
    d_pcm = e->d_pcm;
  }
  if (e->encode_mode == 1 && batch > 1) e->encode_independent(d_pcm, n_samples, batch, stride);
  else e->encode_device(d_pcm, n_samples, batch, stride);
  FA_API_END
}

int fa_pcm_upload(fa_engine* h, const float* pcm, int64_t n_floats) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(pcm && n_floats >= 1 && n_floats <= (int64_t)e->max_batch * std::max<int64_t>(e->max_samples, 16000),
             "fa_pcm_upload: size");
  FA_HIP(hipMemcpyAsync(e->d_pcm, pcm, n_floats * 4, hipMemcpyHostToDevice, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  e->pcm_uploaded = n_floats;
  FA_API_END
}

int fa_encode_fetch(fa_engine* h, float* audio_embd_out, int64_t tgt_stride, int32_t* ctc_ids_out, int64_t ids_stride,
                    int32_t* t_lfr_out, int32_t* target_len_out, float* enc_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  const int B = e->last_batch, ts = e->last_tstride, d = e->ec.d_model, L = e->ec.d_llm;
  FA_REQUIRE(B > 0, "no encode to fetch");
  for (int b = 0; b < B; ++b) {
    if (audio_embd_out) {
      FA_REQUIRE(tgt_stride >= e->h_tgt[b], "tgt_stride too small");
      FA_HIP(hipMemcpyAsync(audio_embd_out + (size_t)b * tgt_stride * L, e->ad + (size_t)b * ts * L,
                            (size_t)e->h_tgt[b] * L * 4, hipMemcpyDeviceToHost, e->stream));
    }
    if (ctc_ids_out) {
      FA_REQUIRE(ids_stride >= e->h_ctclen[b], "ids_stride too small");
      FA_HIP(hipMemcpyAsync(ctc_ids_out + (size_t)b * ids_stride, e->ctc_ids + (size_t)b * ts,
                            (size_t)e->h_ctclen[b] * 4, hipMemcpyDeviceToHost, e->stream));
    }
    if (enc_out) {
      FA_REQUIRE(ids_stride >= e->h_ctclen[b], "ids_stride too small");
      FA_HIP(hipMemcpyAsync(enc_out + (size_t)b * ids_stride * d, e->enc + (size_t)b * ts * d,
                            (size_t)e->h_ctclen[b] * d * 4, hipMemcpyDeviceToHost, e->stream));
    }
    if (t_lfr_out) t_lfr_out[b] = e->h_ctclen[b];
    if (target_len_out) target_len_out[b] = e->h_tgt[b];
  }
  FA_HIP(hipStreamSynchronize(e->stream));
  e->prof_collect();
  FA_API_END
}

int fa_encode(fa_engine* h, const float* pcm, const int64_t* n_samples, int32_t batch, int64_t stride,
              float* audio_embd_out, int64_t tgt_stride, int32_t* ctc_ids_out, int64_t ids_stride, int32_t* t_lfr_out,
              int32_t* target_len_out, float* enc_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(pcm && n_samples && batch >= 1 && batch <= e->max_batch && stride >= 1, "fa_encode args");
  FA_REQUIRE(stride <= std::max<int64_t>(e->max_samples, 16000), "stride > max_samples");
  FA_HIP(hipMemcpyAsync(e->d_pcm, pcm, (size_t)batch * stride * 4, hipMemcpyHostToDevice, e->stream));
  e->pcm_uploaded = (int64_t)batch * stride;
  if (e->encode_mode == 1 && batch > 1) e->encode_independent(e->d_pcm, n_samples, batch, stride);
  else e->encode_device(e->d_pcm, n_samples, batch, stride);
  int r = fa_encode_fetch(h, audio_embd_out, tgt_stride, ctc_ids_out, ids_stride, t_lfr_out, target_len_out, enc_out);
  if (r != FA_OK) return r;
  FA_API_END
}

int fa_ctc_head(fa_engine* h, const float* enc, int32_t T, int32_t* ids_out) {
  FA_API_BEGIN
  FA_REQUIRE(enc && ids_out, "fa_ctc_head args");
  h->e->ctc_head(enc, T, ids_out);
  FA_API_END
}

int fa_ctc_collapse(fa_engine* h, int32_t blank_id, int32_t* ids_out, int32_t* frames_out, int64_t out_stride,
                    int32_t* n_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  const int B = e->last_batch, ts = e->last_tstride;
  FA_REQUIRE(B > 0, "no encode");
  fa::ctc_collapse(e->ctc_ids, ts, e->d_ctclen, B, blank_id, e->d_col_ids, e->d_col_frames, ts, e->d_col_n, e->stream);
  std::vector<int> n(B);
  FA_HIP(hipMemcpyAsync(n.data(), e->d_col_n, B * 4, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  for (int b = 0; b < B; ++b) {
    FA_REQUIRE(out_stride >= n[b], "collapse out_stride too small");
    if (n[b]) {
      FA_HIP(hipMemcpyAsync(ids_out + (size_t)b * out_stride, e->d_col_ids + (size_t)b * ts, n[b] * 4,
                            hipMemcpyDeviceToHost, e->stream));
      FA_HIP(hipMemcpyAsync(frames_out + (size_t)b * out_stride, e->d_col_frames + (size_t)b * ts, n[b] * 4,
                            hipMemcpyDeviceToHost, e->stream));
    }
    n_out[b] = n[b];
  }
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_API_END
}

int fa_set_encode_mode(fa_engine* h, int32_t mode) {
  FA_API_BEGIN
  FA_REQUIRE(mode == 0 || mode == 1, "encode mode must be 0 (padded batch) or 1 (independent clips)");
  h->e->encode_mode = mode;
  FA_API_END
}

int fa_set_tensor_u8dq(fa_engine* h, const char* name, const uint8_t* q, const float* scale, const uint8_t* zero_point,
                       int64_t rows, int64_t cols) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(q && scale && zero_point && rows > 0 && cols > 0, "fa_set_tensor_u8dq args");
  fa::Slot& s = e->slot(name);
  FA_REQUIRE(s.kind == 0 && rows * cols == s.n, std::string("fa_set_tensor_u8dq: not an f32 matrix of that size: ") + name);
  const float* base = nullptr;
  for (const float* w : e->ctc_regions) {
    const Engine::U8Region& r = e->u8w.at(w);
    if (s.f >= w && s.f < w + (int64_t)r.N * r.K) base = w;
  }
  FA_REQUIRE(base, std::string("fa_set_tensor_u8dq: not a CTC-graph linear weight: ") + name);
  Engine::U8Region& r = e->u8w.at(base);
  FA_REQUIRE(cols == r.K && (s.f - base) % r.K == 0, std::string("fa_set_tensor_u8dq: shape mismatch for ") + name);
  const int64_t row0 = (s.f - base) / r.K;
  if (!r.q) {
    r.q = e->alloc<int8_t>((size_t)r.N * r.K);
    r.cs = e->alloc<int>(r.N);
    r.bz = e->alloc<int>(r.N);
    r.ws = e->alloc<float>(r.N);
  }
  uint8_t* tq = nullptr;
  float* ts = nullptr;
  uint8_t* tz = nullptr;
  FA_HIP(hipMalloc(&tq, rows * cols));
  FA_HIP(hipMalloc(&ts, rows * 4));
  FA_HIP(hipMalloc(&tz, rows));
  FA_HIP(hipMemcpyAsync(tq, q, rows * cols, hipMemcpyHostToDevice, e->stream));
  FA_HIP(hipMemcpyAsync(ts, scale, rows * 4, hipMemcpyHostToDevice, e->stream));
  FA_HIP(hipMemcpyAsync(tz, zero_point, rows, hipMemcpyHostToDevice, e->stream));
  fa::u8_weight_prep(tq, ts, tz, (int)rows, (int)cols, r.q + row0 * r.K, r.cs + row0, r.bz + row0, r.ws + row0, e->stream);
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_HIP(hipFree(tq));
  FA_HIP(hipFree(ts));
  FA_HIP(hipFree(tz));
  for (int64_t i = row0; i < row0 + rows; ++i)
    if (!r.row_set[i]) {
      r.row_set[i] = 1;
      ++r.n_set;
    }
  FA_API_END
}

int fa_set_ctc_int8(fa_engine* h, int32_t on) {
  FA_API_BEGIN
  h->e->ctc_i8 = on != 0;
  FA_API_END
}

int fa_ctc_int8_active(fa_engine* h, int32_t* out) {
  FA_API_BEGIN
  FA_REQUIRE(out, "fa_ctc_int8_active: out");
  *out = h->e->ctc_int8_active() ? 1 : 0;
  FA_API_END
}

int fa_set_encoder_fp16(fa_engine* h, int32_t on) {
  FA_API_BEGIN
  h->e->enc_fp16 = on != 0;
  FA_API_END
}

int fa_set_encoder_gemm(fa_engine* h, int32_t mode) {
  FA_API_BEGIN
  FA_REQUIRE(mode == 0 || mode == 1, "encoder GEMM mode must be 0 (exact f32) or 1 (bf16x3)");
  h->e->enc_gemm = mode;
  FA_API_END
}

int fa_set_decode_fused(fa_engine* h, int32_t on) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(on >= 0 && on <= 2, "fa_set_decode_fused: 0 (5-launch), 1 (two-launch), 2 (three-launch)");
  if (e->use_fused != on) {
    FA_HIP(hipStreamSynchronize(e->stream));
    for (auto& g : e->step_graphs) FA_HIP(hipGraphExecDestroy(g.second));
    e->step_graphs.clear();  // captured steps bake the layer structure in
  }
  e->use_fused = on;
  FA_API_END
}

int fa_set_debug(fa_engine* h, int32_t flags) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  if ((e->debug_flags ^ flags) & 2) {  // the fused-layer hook is a launch argument: captured steps must be re-made
    for (auto& g : e->step_graphs) FA_HIP(hipGraphExecDestroy(g.second));
    e->step_graphs.clear();
  }
  e->debug_flags = flags;
  FA_API_END
}

int fa_encode_tap(fa_engine* h, int32_t which, float* out, int64_t n) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(which == 0 && (e->debug_flags & 1) && e->tap_lfr, "tap 0 needs fa_set_debug(e, 1) before fa_encode");
  const int64_t have = (int64_t)e->last_tstride * e->ec.d_in;
  FA_REQUIRE(n <= have, "tap size");
  FA_HIP(hipMemcpy(out, e->tap_lfr, n * 4, hipMemcpyDeviceToHost));
  FA_API_END
}

int fa_embd_rows(fa_engine* h, const int32_t* ids, int32_t n, int32_t fp16_round, float* out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(n >= 1 && n <= e->m_max, "fa_embd_rows: n");
  for (int i = 0; i < n; ++i) FA_REQUIRE(ids[i] >= 0 && ids[i] < e->lc.n_vocab, "token id out of range");
  FA_HIP(hipMemcpyAsync(e->d_ids, ids, n * 4, hipMemcpyHostToDevice, e->stream));
  fa::embed_rows(e->tok_embd.q, e->tok_embd.d, e->d_ids, n, e->lc.n_embd, fp16_round, e->lx, e->stream);
  FA_HIP(hipMemcpyAsync(out, e->lx, (size_t)n * e->lc.n_embd * 4, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_API_END
}

int fa_llm_reset(fa_engine* h, int32_t seq) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  FA_REQUIRE(seq >= 0 && seq < e->lc.max_seqs, "seq out of range");
  e->n_past[seq] = 0;
  e->last_tok[seq] = -1;
  e->logits_row[seq] = -1;
  FA_API_END
}

int fa_llm_prefill(fa_engine* h, int32_t seq, const float* embd, int32_t n_tokens, const fa_sampling* s,
                   int32_t* tok_out, float* logits_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  FA_REQUIRE(seq >= 0 && seq < e->lc.max_seqs, "seq out of range");
  FA_REQUIRE(n_tokens >= 1 && e->n_past[seq] + n_tokens <= e->lc.n_ctx, "prefill exceeds n_ctx");
  e->set_sampling(s);
  Engine::PromptSrc src;
  src.embd = embd;
  e->prefill_one(seq, src, 0, n_tokens, tok_out, logits_out);
  FA_API_END
}

static void check_prefill_batch(Engine* e, const int32_t* seqs, int32_t n_seqs, const int32_t* n_tokens) {
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  FA_REQUIRE(n_seqs >= 1 && n_seqs <= e->lc.max_seqs, "prefill batch: n_seqs out of range");
  std::vector<char> seen(e->lc.max_seqs, 0);
  for (int i = 0; i < n_seqs; ++i) {
    const int q = seqs[i];
    FA_REQUIRE(q >= 0 && q < e->lc.max_seqs && !seen[q], "prefill batch: sequence ids must be distinct and in range");
    seen[q] = 1;
    FA_REQUIRE(n_tokens[i] >= 1 && n_tokens[i] <= e->pf_max && e->n_past[q] + n_tokens[i] <= e->lc.n_ctx,
               "prefill batch: prompt exceeds n_ctx or the row capacity");
  }
}

static void prefill_batch(Engine* e, const int32_t* seqs, int32_t n_seqs, const Engine::PromptSrc& src,
                          const int32_t* n_tokens, int32_t* tok_out) {
  std::vector<int64_t> off(n_seqs + 1, 0);
  for (int i = 0; i < n_seqs; ++i) off[i + 1] = off[i] + n_tokens[i];
  // within the invariant width the batch is row-local: every prompt gets exactly its fa_llm_prefill arithmetic (the
  // reference prefills every segment alone). A prompt above pf_rl_max rows gets the tiled forward when alone, so it is
  // prefilled alone here too.
  const bool rl = n_seqs <= e->invariant_width();
  std::vector<int> rest;
  for (int i = 0; i < n_seqs; ++i) {
    if (rl && n_tokens[i] > e->pf_rl_max) e->prefill_one(seqs[i], src, off[i], n_tokens[i], tok_out ? tok_out + i : nullptr, nullptr);
    else rest.push_back(i);
  }
  e->pf_row_local = rl;
  // sequences in order, as many per forward as the row capacity holds; one weight pass per forward
  for (size_t i0 = 0; i0 < rest.size();) {
    size_t i1 = i0;
    int rows = 0;
    while (i1 < rest.size() && rows + n_tokens[rest[i1]] <= e->pf_max) rows += n_tokens[rest[i1++]];
    const int n = (int)(i1 - i0);
    std::vector<int> sq(rows), ps(rows), last(n), lseq(n), lpos(n);
    std::vector<std::pair<int64_t, int>> parts;
    for (size_t k = i0, r = 0; k < i1; ++k) {
      const int i = rest[k];
      parts.emplace_back(off[i], n_tokens[i]);
      for (int t = 0; t < n_tokens[i]; ++t, ++r) {
        sq[r] = seqs[i];
        ps[r] = e->n_past[seqs[i]] + t;
      }
      last[k - i0] = (int)r - 1;
      lseq[k - i0] = seqs[i];
      lpos[k - i0] = ps[r - 1];
    }
    e->load_prompt_rows(src, parts);
    FA_HIP(hipMemcpyAsync(e->d_tok_seq, sq.data(), rows * 4, hipMemcpyHostToDevice, e->stream));
    FA_HIP(hipMemcpyAsync(e->d_tok_pos, ps.data(), rows * 4, hipMemcpyHostToDevice, e->stream));
    FA_HIP(hipMemcpyAsync(e->d_lastrow, last.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    e->set_prefill_tiles(sq.data(), ps.data(), rows, e->pf_row_local);
    try {
      e->llm_forward(rows, false, 0, n);
    } catch (...) {
      e->pf_row_local = false;
      throw;
    }
    e->n_ptiles = 0;
    // each first token's draw is keyed by its sequence's last prompt row (seq, position), as fa_llm_prefill's
    FA_HIP(hipMemcpyAsync(e->d_ids, lseq.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    FA_HIP(hipMemcpyAsync(e->d_step, lpos.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    e->sample(n, e->d_ids, e->d_step, nullptr, e->d_tok_cur, nullptr);
    std::vector<int> tok(n);
    FA_HIP(hipMemcpyAsync(tok.data(), e->d_tok_cur, n * 4, hipMemcpyDeviceToHost, e->stream));
    FA_HIP(hipStreamSynchronize(e->stream));
    e->prof_collect();
    std::fill(e->logits_row.begin(), e->logits_row.end(), -1);
    for (size_t k = i0; k < i1; ++k) {
      const int i = rest[k];
      e->n_past[seqs[i]] += n_tokens[i];
      e->last_tok[seqs[i]] = tok[k - i0];
      e->logits_row[seqs[i]] = (int)(k - i0);
      if (tok_out) tok_out[i] = tok[k - i0];
    }
    i0 = i1;
  }
  e->pf_row_local = false;
}

int fa_llm_prefill_batch(fa_engine* h, const int32_t* seqs, int32_t n_seqs, const float* embd, const int32_t* n_tokens,
                         const fa_sampling* s, int32_t* tok_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  check_prefill_batch(e, seqs, n_seqs, n_tokens);
  e->set_sampling(s);
  Engine::PromptSrc src;
  src.embd = embd;
  prefill_batch(e, seqs, n_seqs, src, n_tokens, tok_out);
  FA_API_END
}

int fa_encode_generation(fa_engine* h, int64_t* gen_out) {
  FA_API_BEGIN
  FA_REQUIRE(gen_out, "fa_encode_generation args");
  *gen_out = h->e->last_batch > 0 ? h->e->enc_gen : -1;
  FA_API_END
}

int fa_llm_prefill_rows(fa_engine* h, const int32_t* seqs, int32_t n_seqs, const float* host_rows, int32_t n_host_rows,
                        const int32_t* row_src, const int32_t* n_tokens, int64_t enc_gen, const fa_sampling* s,
                        int32_t* tok_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(row_src && n_tokens && n_host_rows >= 0 && (host_rows || n_host_rows == 0), "fa_llm_prefill_rows args");
  check_prefill_batch(e, seqs, n_seqs, n_tokens);
  const int E = e->lc.n_embd;
  int64_t total = 0;
  for (int i = 0; i < n_seqs; ++i) total += n_tokens[i];
  for (int64_t r = 0; r < total; ++r) {
    const int32_t c = row_src[r];
    if (c >= 0) {
      FA_REQUIRE(c < n_host_rows, "fa_llm_prefill_rows: host row index out of range");
    } else {
      const int v = -1 - c, b = v >> 16, t = v & 0xffff;
      FA_REQUIRE(e->last_batch > 0 && enc_gen == e->enc_gen,
                 "fa_llm_prefill_rows: the adaptor rows of that encode are gone (another encode or CTC-head call ran)");
      FA_REQUIRE(e->ec.d_llm == E, "fa_llm_prefill_rows: adaptor width != n_embd");
      FA_REQUIRE(b < e->last_batch && t < e->h_tgt[b], "fa_llm_prefill_rows: audio row out of range");
    }
  }
  if (n_host_rows > e->prow_cap) {
    if (e->d_prow) FA_HIP(hipFree(e->d_prow));
    e->d_prow = nullptr;
    e->prow_cap = 0;
    FA_HIP(hipMalloc(&e->d_prow, (size_t)n_host_rows * E * 4));
    e->prow_cap = n_host_rows;
  }
  if (n_host_rows > 0)
    FA_HIP(hipMemcpyAsync(e->d_prow, host_rows, (size_t)n_host_rows * E * 4, hipMemcpyHostToDevice, e->stream));
  e->set_sampling(s);
  Engine::PromptSrc src;
  src.codes = row_src;
  if (n_seqs == 1) e->prefill_one(seqs[0], src, 0, n_tokens[0], tok_out, nullptr);  // fa_llm_prefill's path
  else prefill_batch(e, seqs, n_seqs, src, n_tokens, tok_out);
  FA_API_END
}

int fa_llm_generate_begin(fa_engine* h, const int32_t* seqs, int32_t n_seqs, int32_t n_steps, const fa_sampling* s) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is already in flight (fa_llm_generate_end first)");
  FA_REQUIRE(n_seqs >= 1 && n_seqs <= e->lc.max_seqs && n_steps >= 1 && n_steps <= e->hist_max, "generate args");
  std::vector<char> seen(e->lc.max_seqs, 0);
  for (int i = 0; i < n_seqs; ++i) {
    const int q = seqs[i];
    FA_REQUIRE(q >= 0 && q < e->lc.max_seqs, "seq out of range");
    FA_REQUIRE(!seen[q], "duplicate sequence id in one generate call");  // rows would share a KV slot / position
    seen[q] = 1;
    FA_REQUIRE(e->last_tok[q] >= 0, "sequence has no sampled token (prefill first)");
    FA_REQUIRE(e->n_past[q] + n_steps <= e->lc.n_ctx, "generate exceeds n_ctx");
  }
  e->set_sampling(s);
  e->enqueue_steps(seqs, n_seqs, n_steps);
  e->gen_seqs.assign(seqs, seqs + n_seqs);
  e->gen_steps = n_steps;
  e->gen_pending = true;
  FA_API_END
}

int fa_llm_generate_end(fa_engine* h, int32_t* tokens_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(e->gen_pending, "no generate call in flight");
  e->gen_pending = false;
  FA_HIP(hipEventSynchronize(e->ev_gen));
  const int n_seqs = (int)e->gen_seqs.size(), n_steps = e->gen_steps;
  e->prof_collect();
  // the recovery follows the layer the chunk actually ran on (a batch of 7-8 with FUNASR_GU_DOWN=1 is above the fused
  // width: its error flag can only come from the gate|up -> down hand-off)
  if (e->fused_layer_runs(n_seqs)) {
    if (e->fused_error()) e->recover_fused_chunk();
    else e->fused_fail_streak = 0;  // a clean fused chunk ends a run of fallbacks ("three in a row", funasr_hip.h)
  } else if ((e->use_gu_down || (e->use_attn_ob && n_seqs == 32)) && e->fused_error()) {
    // a batched-decode in-launch hand-off timed out (the gate|up -> down one, or the attention + o launch's head fan-in:
    // not expected, every block is resident): the separate launches from now on
    fa::log(3, "batched decode: an in-launch hand-off timed out; re-running the chunk on separate launches");
    e->use_gu_down = false;
    e->use_attn_ob = false;
    ++e->fused_recoveries;  // counted with the chunks re-run on another layer form (fa_llm_decode_recoveries)
    e->drop_step_graphs();
    e->rerun_chunk();
    FA_REQUIRE(!e->fused_error(), "decode chunk re-run: error flag set on the separate launches");
  }
  std::fill(e->logits_row.begin(), e->logits_row.end(), -1);
  for (int i = 0; i < n_seqs; ++i) {
    const int q = e->gen_seqs[i];
    const int* hrow = e->h_hist + (size_t)i * e->hist_max;
    if (tokens_out)
      for (int st = 0; st < n_steps; ++st) tokens_out[(size_t)i * n_steps + st] = hrow[st];
    e->n_past[q] += n_steps;
    e->last_tok[q] = hrow[n_steps - 1];
    e->logits_row[q] = i;
  }
  FA_API_END
}

int fa_llm_generate(fa_engine* h, const int32_t* seqs, int32_t n_seqs, int32_t n_steps, const fa_sampling* s,
                    int32_t* tokens_out) {
  const int rc = fa_llm_generate_begin(h, seqs, n_seqs, n_steps, s);
  if (rc != FA_OK) return rc;
  return fa_llm_generate_end(h, tokens_out);
}

int fa_llm_invariant_width(fa_engine* h, int32_t* out) {
  FA_API_BEGIN
  *out = h->e->invariant_width();
  FA_API_END
}

int fa_llm_decode_recoveries(fa_engine* h, int32_t* retries, int32_t* fallbacks) {
  FA_API_BEGIN
  FA_REQUIRE(retries && fallbacks, "fa_llm_decode_recoveries: outputs");
  *retries = h->e->fused_retries;
  *fallbacks = h->e->fused_recoveries;
  FA_API_END
}

int fa_llm_set_token(fa_engine* h, int32_t seq, int32_t token) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  FA_REQUIRE(seq >= 0 && seq < e->lc.max_seqs, "seq out of range");
  FA_REQUIRE(e->n_past[seq] > 0, "fa_llm_set_token: prefill the sequence first");
  FA_REQUIRE(token >= 0 && token < e->lc.n_vocab, "fa_llm_set_token: token out of range");
  e->last_tok[seq] = token;
  FA_API_END
}

int fa_llm_logits(fa_engine* h, int32_t seq, float* out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(!e->gen_pending, "a generate call is in flight (fa_llm_generate_end first)");
  FA_REQUIRE(seq >= 0 && seq < e->lc.max_seqs, "seq out of range");
  const int row = e->logits_row[seq];
  FA_REQUIRE(row >= 0, "fa_llm_logits: the most recent forward did not include this sequence");
  FA_HIP(hipMemcpy(out, e->logits + (size_t)row * e->lc.n_vocab, (size_t)e->lc.n_vocab * 4, hipMemcpyDeviceToHost));
  FA_API_END
}

int fa_llm_n_past(fa_engine* h, int32_t seq, int32_t* out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(seq >= 0 && seq < e->lc.max_seqs, "seq");
  *out = e->n_past[seq];
  FA_API_END
}

int fa_profile_enable(fa_engine* h, int32_t on) {
  FA_API_BEGIN
  Engine* e = h->e;
  e->prof_collect();
  e->prof = on != 0;
  for (auto& c : e->pcls) c = Engine::ProfCls{};
  FA_API_END
}

int fa_profile_read(fa_engine* h, int32_t cls, double* ms, int64_t* launches, double* bytes, double* flops) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(cls >= 0 && cls < 7, "class");
  e->prof_collect();
  if (ms) *ms = e->pcls[cls].ms;
  if (launches) *launches = e->pcls[cls].launches;
  if (bytes) *bytes = e->pcls[cls].bytes;
  if (flops) *flops = e->pcls[cls].flops;
  FA_API_END
}

int fa_synchronize(fa_engine* h) {
  FA_API_BEGIN
  FA_HIP(hipStreamSynchronize(h->e->stream));
  FA_API_END
}

// ---- result gather over RCCL: the only exchange of the sharded long-audio / clip-batch path. librccl is
// resolved at first use (dlopen: no load-time dependency; a process that already holds RCCL, e.g. torch's, shares it)
namespace {
struct RcclApi {
  bool ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};
RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
    api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
    api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
    api.ok = api.get_unique_id && api.comm_init_rank && api.all_gather && api.comm_destroy && api.error_string;
  });
  return api;
}
}  // namespace
#define FA_NCCL(expr)                                                                                    \
  do {                                                                                                   \
    const ncclResult_t _r = (expr);                                                                      \
    FA_REQUIRE(_r == ncclSuccess, std::string("RCCL: ") + rccl().error_string(_r) + " (" #expr ")"); \
  } while (0)

int fa_comm_unique_id(uint8_t* id_out) {
  FA_API_BEGIN
  FA_REQUIRE(id_out, "fa_comm_unique_id: id_out");
  FA_REQUIRE(rccl().ok, "fa_comm_unique_id: librccl.so.1 not loadable");
  ncclUniqueId id;
  FA_NCCL(rccl().get_unique_id(&id));
  std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  FA_API_END
}

int fa_comm_init(fa_engine* h, int32_t rank, int32_t world, const uint8_t* id) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(id && world >= 1 && rank >= 0 && rank < world, "fa_comm_init args");
  FA_REQUIRE(!e->comm, "fa_comm_init: this engine already has a communicator");
  FA_REQUIRE(rccl().ok, "fa_comm_init: librccl.so.1 not loadable");
  FA_HIP(hipSetDevice(e->device));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  if (e->comm_sz_n < 2 * world) {
    if (e->comm_sz) FA_HIP(hipFree(e->comm_sz));
    e->comm_sz = nullptr;
    e->comm_sz_n = 0;
    FA_HIP(hipMalloc(&e->comm_sz, (size_t)2 * world * sizeof(int64_t)));
    e->comm_sz_n = 2 * world;
  }
  FA_NCCL(rccl().comm_init_rank(&e->comm, world, uid, rank));
  e->comm_rank = rank;
  e->comm_world = world;
  FA_API_END
}

int fa_comm_allgather_sizes(fa_engine* h, int64_t n, int64_t* sizes_out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(e->comm && sizes_out && n >= 0, "fa_comm_allgather_sizes: no communicator / args");
  FA_HIP(hipSetDevice(e->device));
  FA_HIP(hipMemcpyAsync(e->comm_sz + e->comm_world, &n, 8, hipMemcpyHostToDevice, e->stream));
  FA_NCCL(rccl().all_gather(e->comm_sz + e->comm_world, e->comm_sz, 1, ncclInt64, e->comm, e->stream));
  FA_HIP(hipMemcpyAsync(sizes_out, e->comm_sz, (size_t)e->comm_world * 8, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_API_END
}

int fa_comm_allgather_bytes(fa_engine* h, const uint8_t* data, int64_t n, int64_t slot, uint8_t* out) {
  FA_API_BEGIN
  Engine* e = h->e;
  FA_REQUIRE(e->comm && out && n >= 0 && slot >= n && slot >= 1 && (n == 0 || data),
             "fa_comm_allgather_bytes: no communicator / args (every rank passes the same slot >= its n)");
  FA_HIP(hipSetDevice(e->device));
  if (slot > e->comm_cap) {
    if (e->comm_buf) FA_HIP(hipFree(e->comm_buf));
    e->comm_buf = nullptr;
    FA_HIP(hipMalloc(&e->comm_buf, (size_t)slot * (e->comm_world + 1)));
    e->comm_cap = slot;
  }
  uint8_t* send = e->comm_buf + (size_t)e->comm_world * slot;
  FA_HIP(hipMemsetAsync(send, 0, slot, e->stream));
  if (n) FA_HIP(hipMemcpyAsync(send, data, n, hipMemcpyHostToDevice, e->stream));
  FA_NCCL(rccl().all_gather(send, e->comm_buf, (size_t)slot, ncclUint8, e->comm, e->stream));
  FA_HIP(hipMemcpyAsync(out, e->comm_buf, (size_t)slot * e->comm_world, hipMemcpyDeviceToHost, e->stream));
  FA_HIP(hipStreamSynchronize(e->stream));
  FA_API_END
}

void fa::Engine::comm_teardown() {
  if (comm) {
    FA_HIP(hipStreamSynchronize(stream));
    const ncclComm_t c = comm;
    comm = nullptr;
    FA_NCCL(rccl().comm_destroy(c));
  }
  comm_rank = 0;
  comm_world = 0;
  if (comm_buf) FA_HIP(hipFree(comm_buf));
  comm_buf = nullptr;
  comm_cap = 0;
}

int fa_comm_destroy(fa_engine* h) {
  FA_API_BEGIN
  h->e->comm_teardown();
  FA_API_END
}

}  // extern "C"
