// Host-callable launchers of the HIP kernels (all enqueue on stream `s`, no synchronisation).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace fa {

// Arrival counters of the in-launch split combines (decode attention, encoder attention, split-K GEMM) sit one per
// 128-B line: device-scope adds to one line serialise (~12 ns each; MI355X_MICROARCH.md row fanin). Measured on
// the decode attention launch: 7.0 -> 6.5 us.
constexpr int CNT_LINE = 32;  // ints

// synth.hip
void launch_synth_fill(float* out, int64_t n, uint32_t key, float scale, float offset, hipStream_t s);
void launch_quant_q8_0(const float* x, int64_t n, int8_t* qs, __half* d, hipStream_t s);
void launch_unpack_q8_0(const uint8_t* blocks, int64_t n_blocks, int8_t* qs, __half* d, hipStream_t s);
void launch_pack_q8_0(const int8_t* qs, const __half* d, int64_t n_blocks, uint8_t* blocks, hipStream_t s);
void launch_h2f(const __half* a, float* b, int64_t n, hipStream_t s);
// float16-ONNX initializer conversion (clamp to [1e-7, 65504] magnitude, RN): f16 copy b and/or its f32 value b32
void launch_f2h_initializer(const float* a, __half* b, float* b32, int64_t n, hipStream_t s);

// gemm_f32.hip
// K-split workspace of the f32 GEMM (few-tile shapes, e.g. a single clip's N = 512 projections): partial
// accumulators of up to cnt_n tiles x GEMM_F32_KS_MAX splits x 256 threads x 16 floats, one arrival counter per
// tile (zeroed once; re-armed by the summing block)
#define GEMM_F32_KS_MAX 4
struct GemmF32Work {
  float* part = nullptr;
  int64_t part_n = 0;
  int* cnt = nullptr;  // [cnt_n][CNT_LINE]
  int64_t cnt_n = 0;
};
extern int g_gemm_f32_split;  // 1 (default): K splits where the tiles leave the chip idle; 0: none
extern int g_attn_merge;     // encoder attention key splits merged by their own launch (k_attn_merge; default 1)
extern int g_attn_ms;                 // query slices per tile of k_attn_merge (8)
extern int g_attn_f32_force_splits;  // encoder attention key splits (0: automatic; FUNASR_ATTN_KS)
extern int g_attn_f16_mfma;  // 1 (default): fp16-graph attention on f16 MFMAs; 0: exact f32 + fp16 rounding
extern int g_gemm_f16_b3;  // 1 (default): fp16-graph GEMMs on the bf16x3 kernel family with one f16 plane; 0: k_gemm_f16
extern int g_lm_tr;  // LM head of 2-8 tokens: transposed row x token reduction (default 1)
extern int g_gemm_f32_wab;  // exact-f32 GEMM tiles: 1 = write-after-barrier staging
extern int g_gemm_t_wab;  // k_gemm_q8_t: 1 = write-after-barrier staging
extern int g_attn_wab;  // k_attn_bf3: 1 = write-after-barrier K/V staging
extern int g_gemm_bf3_256_s;  // 256x256 tile: 1 = write-after-barrier staging
extern int g_gemm_bf3_persist;  // 256x256 tiles as persistent blocks, one per CU (A/B, default 0)
extern int g_gemm_bf3_dma;    // planes-A 256x256 tiles staged by LDS-DMA (k_gemm_bf3_256d; default 0: measured slower)
extern int g_gemm_bf3_sk;     // bf16x3 few-tile K >= 2048 linear GEMMs: 128x128 tiles, K split over blocks (default 1)
extern int g_gemm_f16_sk;     // fp16 graph: the same split on the register-staged 128x128 tile (default 1)
extern int g_gemm_epi_grouped;  // one-clip encoder GEMMs on the four-row grouped epilogue (default 1)
extern int g_gemm_bf3_big;  // launches of at least this many 128x128 tiles take them (1024)
extern int g_gemm_f16_pf32;   // fp16 batched 128-deep launches on the 32-deep prefetch tile (default 1)
extern int g_gemm_bf3_pf_kb;  // k depth of the 64x64 two-step-prefetch tile (0: 32 for batched launches, 64 for one clip)
extern int g_gemm_bf3_sk_kmin;  // smallest K of a split few-tile launch (2048: one clip's ffn2)
extern int g_gemm_bf3_sk_ks;  // force the K split of k_gemm_bf3_sk launches (0 = automatic)
extern int g_gemm_f16_deep;  // fp16 one-clip GEMMs on 128-deep stages (default 1)
extern int g_gemm_bf3_kw4;  // 1: four K groups per block for few-tile K >= 2048 shapes (FUNASR_BF3_KW4)
extern int g_gemm_bf3_mid;  // 1: 128x64 tiles for one clip's 256-1024-tile GEMM shapes (A/B, default 0)
// bf16x3 split of an f32 weight (raw bf16 bits): hi = bf16_rn(w), lo = bf16_rn(w - hi), planes laid out as w
struct WSplit {
  const uint16_t* hi = nullptr;
  const uint16_t* lo = nullptr;
};
void launch_split_bf16(const float* w, uint16_t* hi, uint16_t* lo, int64_t n, hipStream_t s);
// the same split of an f32 ACTIVATION, written by its producer (layernorm, encoder attention, ffn1 epilogue) in place of
// the f32 tensor when only a bf16x3 GEMM reads it: element (row, col) at hi / lo + row * ld + col, ld = the f32 tensor's
// row stride (raw bf16 bits)
struct APlanes {
  uint16_t* hi = nullptr;
  uint16_t* lo = nullptr;
};
// W16 != nullptr: fp16 mode (C5) on the f16 MFMA kernel with the fp16 weight copy W16, every op output rounded to fp16;
// else wb.hi != nullptr: f32 mode on the bf16x3 split kernel; else the exact-f32 MFMA kernel
void gemm_linear(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, float* C, int64_t ldc,
                 int M, int N, int K, int relu, const float* add1, int64_t ld1, const float* add2, int64_t ld2,
                 hipStream_t s, const __half* W16 = nullptr, const GemmF32Work* wk = nullptr, WSplit wb = {},
                 APlanes ap = {}, APlanes cp = {});  // ap.hi: A read from planes (lda); cp.hi: C written as planes (ldc)
void gemm_stft_power(const float* xp, int64_t xp_stride, int t_stride, int M, const float* basis, float* power,
                     int64_t ldp, hipStream_t s, int r16 = 0);
void gemm_mel_log(const float* power, int64_t ldp, const float* fbank, int64_t ldf, float* mel, int M, int n_mels,
                  int n_freq, hipStream_t s, int r16 = 0);
void gemm_ctc_argmax(const float* A, int64_t lda, const float* W, const float* bias, int M, int N, int K, float* pval,
                     int* pidx, int* out, hipStream_t s, const __half* W16 = nullptr, WSplit wb = {});

// int8-dynamic CTC graph (gemm_f32.hip): ORT quantize_dynamic weights (per output channel uint8) held as int8 w' = wq - 128
// with per-row sums cs, bz = 128 - zero point and the f32 scale; activations DynamicQuantizeLinear'd per clip into U8Work
struct U8W {
  const int8_t* q = nullptr;  // [N][K]
  const int* cs = nullptr;
  const int* bz = nullptr;
  const float* ws = nullptr;
};
struct U8Work {
  int8_t* xq = nullptr;    // [rows][K]
  int64_t xq_n = 0;
  int* rs = nullptr;       // [rows]
  float2* part = nullptr;  // [max_clips][64] min / max partials
  float2* qp = nullptr;    // [max_clips] {x scale, 128 - x zero point}
  int max_clips = 0;
};
void u8_weight_prep(const uint8_t* q, const float* scale, const uint8_t* zp, int N, int K, int8_t* wq, int* cs, int* bz,
                    float* ws, hipStream_t s);
void dq_quantize(const float* x, int64_t ldx, int K, const int* lens, int ts, int B, U8Work& w, hipStream_t s);
void gemm_u8_linear(const U8Work& w, const U8W& wt, const float* bias, float* C, int64_t ldc, int M, int N, int K,
                    int ts, int relu, const float* add1, int64_t ld1, hipStream_t s);
void gemm_u8_ctc_argmax(const U8Work& w, const U8W& wt, const float* bias, int M, int N, int K, int ts, float* pval,
                        int* pidx, int* out, hipStream_t s);

// attn_f32.hip
// Key-split workspace of the encoder attention (used only while (query tile, head, clip) blocks leave the
// chip idle): splits x tiles <= 512, so 512 partials of 128 x (128 + 2) floats and 512 arrival counters
// (zeroed once; re-armed by the merging block) always suffice.
struct AttnF32Work {
  float* part = nullptr;
  int64_t part_n = 0;
  int* cnt = nullptr;
  int64_t cnt_n = 0;
};
constexpr int64_t ATTN_F32_PART_FLOATS = (int64_t)512 * (128 * 128 + 2 * 128);
constexpr int64_t ATTN_F32_COUNTERS = 512;
int attn_f32_splits(int batch, int t_stride, int n_heads);
void attn_f32(const float* Q, const float* K, const float* V, int64_t ldq, int64_t ldk, int64_t ldv, float* O,
              int64_t ldo, int batch, int t_stride, int n_heads, int head_dim, const int* lens,
              const AttnF32Work& wk, hipStream_t s, int r16 = 0, int bf3 = 0,  // bf3: bf16x3 split MFMA products
              APlanes op = {});  // op.hi (bf3 only): O written as bf16 planes (ldo) instead of f32

// enc_misc.hip
void frontend_preemph(const float* pcm, int64_t stride, const int64_t* d_n_samples, int batch, float* partial,
                      float* xp, int64_t xp_stride, hipStream_t s, int r16 = 0);
void frontend_lfr(const float* mel, int mel_stride, const int* t_mel_valid, const int* t_lfr_valid, const float* pe,
                  float* x, int batch, int t_stride, int n_mels, int lfr_m, int lfr_n, hipStream_t s, int r16 = 0);
void layernorm(const float* x, int64_t ldx, float* y, int64_t ldy, const float* w, const float* b, int rows, int D,
               float eps, const int* lens, int t_stride, hipStream_t s, int r16 = 0,
               APlanes yp = {});  // yp.hi: y written as bf16 planes (ldy) instead of f32
void fsmn(const float* v, int64_t ldv, const float* w, float* out, int64_t ldo, int rows, int C, int ksize,
          const int* lens, int t_stride, hipStream_t s, int r16 = 0);
void ctc_collapse(const int* ids, int64_t ids_stride, const int* lens, int batch, int blank, int* out_ids,
                  int* out_frames, int64_t out_stride, int* n_out, hipStream_t s);

// llm.hip
struct GemvArgs {
  const int8_t* wq; const __half* wd;      // [O][K], [O][K/32]
  const int8_t* wq2; const __half* wd2;    // up matrix for SwiGLU
  const float* x; int64_t ldx; const float* norm_w; float eps;  // FUSED input
  const int8_t* xq; const float* xd;       // pre-quantised input
  float* out; int64_t ldo;                 // [M][O]
  const float* res; int64_t ldr;
  float* pval; int* pidx; int n_part;      // argmax partials [M][n_part]
  int M, O, rpw;
  float* kpart; int64_t kpart_n;           // MFMA GEMM split-K workspace (floats) + arrival counters
  int* kcnt; int64_t kcnt_n;               //   (counters zeroed once; re-armed by the combining block)
  int8_t* qout; float* dout;               // MFMA GEMM SwiGLU epilogue: also the q8_0 rows of out (next GEMM's input)
  const float* psum; float* xsum;          // fused decode (M = 1): x += psum[0..7][K] before the norm; block 0 -> xsum
  // batched decode (8 <= M <= 32, no k_prep_q8 launches): a residual GEMM (epi 1, O = 1024) with ssp_out also
  // quantises its new rows times qn_w (the next RMSNorm's weight) per 32-block into qout / dout (unscaled f32 block
  // scales) and writes per-token sum-of-squares partials ssp_out [M][32]; a GEMM with ssp != nullptr reads such rows
  // (xq / xd) and applies rstd = 1/sqrtf(sum ssp / K + eps) to the block scales
  const float* ssp; float* ssp_out; const float* qn_w;
  // prefill whose token rows must each get the arithmetic of their own sequence's prefill, whatever else the call
  // holds (fa_llm_prefill, and fa_llm_prefill_batch within the invariant width): every GEMM on the K-in-block MFMA
  // kernel, whose per-row result does not depend on the token count (no split-K, no 128-token tiles)
  int row_local;
  // batched decode, split-K form only: extra grid slabs (pf_slabs) that pull the NEXT GEMM's weight rows ([pf_O][pf_K]
  // q8_0, two matrices for SwiGLU) into the L2 of the XCD whose blocks will read them (gemm_l2_prefetch); nullptr: off
  const int8_t* pf_q; const __half* pf_d; const int8_t* pf_q2; const __half* pf_d2;
  int pf_O, pf_K, pf_slabs, pf_delay;
};
extern int g_gemm_pf;        // batched-decode GEMM L2 prefetch: bit 1 o -> gate|up, 2 gate|up -> down, 4 down -> next q|k|v,
                             // 8 q|k|v -> o (0 = off)
extern int g_gemm_pf_slabs;  // prefetch slabs per GEMM launch
extern int g_gemm_pf_delay;  // their start delay, ticks of the 100 MHz clock
void prep_q8(const float* x, int64_t ldx, const float* w, float eps, int M, int K, int8_t* xq, float* xd, hipStream_t s);
void gemv_q8(const GemvArgs& a, int K, int epi, hipStream_t s);
int gemv_rows_per_wave(int O);
// argmax partials per token written by the lm_head launch for M tokens (GEMV for gemv_small(M), MFMA GEMM above)
int lm_head_parts(int O, int M, int K = 1024);
int gemm_k_splits(int O, int M, int K, int epi);  // K splits of the split-K GEMM form for this shape
// batched decode (M <= 32, producer-normalised inputs): gate|up + SwiGLU and the down projection in one launch with a
// group-local hand-off per down K split; cnt = 64 zeroed counter lines (re-armed in-launch), err = timeout flag.
// false: shape not covered (the caller runs the two launches)
bool gemm_q8_gu_down(const GemvArgs& g, const GemvArgs& d, unsigned* cnt, int* err, hipStream_t s);
extern int g_attn_lean;    // -1 auto, 0/1 force the 128-VGPR attention variant (A/B)
extern int g_attn_blocks;  // attention key-split target (blocks per launch), 1024 by default
extern int g_attn_wide;    // decode launches with >= this many (token, kv head) pairs: 16-wave blocks, no splits
extern int g_attn_xcd;  // encoder attention (k_attn_bf3): the query tiles of one (head, clip) on one XCD
extern int g_attn_pf_f16;  // query-tiled prefill attention on f16 MFMAs (q split hi + lo; 0: exact-f32 MFMAs)
extern int g_attn_ldspf;   // ... with the next pass's K/V pulled into LDS by LDS-DMA during the current pass
extern int g_lm_head_mt6;    // LM head of 3-6 token batches in one block row (default 1)
extern int g_sk_min_blocks;  // split-K shape choice: fewest blocks before fewer splits are preferred (default 256)
extern int g_fsmn_vec;       // 1 (default): 16-B-lane FSMN kernel for batched encodes; 0: 4-B lanes (A/B)
extern int g_gemv_small_max;  // fused-GEMV decode path for M <= this (default 5); MFMA GEMM above
extern int g_gemv_mt;         // tokens per fused-GEMV block from M = 3 on (default 2)
bool gemv_small(int M);
extern int g_gemm_q8_kw;  // 1 (default): K-in-block int8 MFMA GEMM where instantiated; 0: split-K block kernel
extern int g_lm_head_s;     // LM head of 2-8 tokens (fused decode path) on k_lm_head_s (bit-identical to batch 1): 0 off, 1/2 = PF
extern int g_lm_grid;       // blocks of the persistent LM-head launches (0: all resident)
extern int g_lm_head_s1;    // ... and of one token (0: the GEMV)
extern int g_lm_head_b;     // 1: batched LM head on the persistent tile loop (k_lm_head_b); 0: split-K block kernel
extern int g_gemm_t_min_m;  // token count from which the 128x128-tile int8 GEMM runs (prefill batches; default 512)
void qk_rope_store(const float* qkv, int M, int H, int KV, float eps, const float* qn, const float* kn, const float* rcos,
                   const float* rsin, const int* tok_seq, const int* tok_pos, float* qout, __half* kc, __half* vc,
                   int64_t seq_stride, hipStream_t s);
// Split-key attention workspace: per (token, kv head) an arrival counter (zeroed once; the combining block
// re-arms it) and ATTN_SPLITS partials of ATTN_PART_FLOATS floats (o[2][128], then m0, l0, m1, l1).
#define ATTN_SPLITS 16
#define ATTN_PART_FLOATS 260

struct AttnWork {
  int* counters = nullptr;    // [max_tokens][max_kv][CNT_LINE]
  float* partials = nullptr;  // [max_split_tokens][max_kv][ATTN_SPLITS][ATTN_PART_FLOATS]
  int max_tokens = 0, max_kv = 0;
  int max_split_tokens = 0;   // launches with more rows than this run unsplit (large prefill batches always do)
};
// Prefill over query tiles (multi-sequence batches): tiles[i] = {row0, n_rows <= 64, seq, 0}, rows of one sequence at
// consecutive positions; q from qk_rope_store (head dim 128); out / qout / dout as attn_block's
// f16: the f16-MFMA kernel (k_attn_prefill_h; the caller checks the q range, Engine::prefill_attn_f16), else exact f32
void attn_prefill(const int4* tiles, int n_tiles, const int* tok_pos, int H, int KV, int64_t seq_stride, const __half* kc,
                  const __half* vc, const float* q, float* out, int8_t* qout, float* dout, hipStream_t s, bool f16);
// qout/dout (optional): the output rows also as q8_0 blocks (the o GEMM's pre-quantised input, no prep launch)
void attn_block(const float* qsrc, int decode_mode, const float* qn, const float* kn, float eps, const float* rcos,
                const float* rsin, __half* kc, __half* vc, int M, int H, int KV, const int* tok_seq, const int* tok_pos,
                int64_t seq_stride, float* out, const AttnWork& wk, hipStream_t s, int8_t* qout = nullptr,
                float* dout = nullptr, int max_splits = 16);
// Fused batch-1 decode layer (M = 1; llm.hip): attention + split o projection, and gate|up + SwiGLU + split down
// projection, each with an in-launch group fan-in (see the kernels). FUSED_PARTS = partial vectors summed by the next
// launch's prologue (8 kv heads for o, 8 groups of 384 act rows for down).
constexpr int FUSED_PARTS = 8;
constexpr int FUSED_MAX_M = 8;  // decode batch widths the two-launch layer takes (one grid slab per token)
constexpr int FUSED_CNT_LINES = 3 * FUSED_MAX_M * FUSED_PARTS;
struct FusedDecodeWork {
  float* opart = nullptr;   // [FUSED_MAX_M][FUSED_PARTS][E]
  float* dpart = nullptr;   // [FUSED_MAX_M][FUSED_PARTS][E]
  float* act = nullptr;     // [FUSED_MAX_M][2 F] act hand-off (F 8-byte granules per token; zeroed once)
  float* xmid = nullptr;    // [FUSED_MAX_M][E] residual stream after the attention block
  unsigned* cnt = nullptr;  // [FUSED_CNT_LINES][CNT_LINE] ticket counters (zeroed once, never re-armed): o fan-in,
                            // down-group fan-in, q|k|v fan-in (two-launch layer), FUSED_PARTS lines each
  int* err = nullptr;       // set to 1 by a timed-out fan-in wait
  float* pzero = nullptr;   // [FUSED_MAX_M][FUSED_PARTS][E] zeros: layer 0's partials in the two-launch layer
  unsigned long long* gqkv = nullptr;  // [FUSED_MAX_M][(H + 2 KV) D] q|k|v granules of the two-launch layer (zeroed once)
  unsigned long long* gpart = nullptr; // [FUSED_MAX_M][FUSED_PARTS][ATTN_SPLITS][ATTN_PART_FLOATS] attention split
                                       // partials of the two-launch layer as granules (zeroed once)
};
// L2 prefetch of the batch-1 two-launch layer (llm.hip l2_prefetch): the bytes the blocks of the NEXT launches read,
// pulled into the L2 of the XCD those blocks run on by extra blocks of the attention launch (its chain leaves HBM idle).
// ffn_*: this layer's FFN launch; qkv_* / o_* / kc / vc: the next layer's attention launch (nullptr: none).
struct L2Prefetch {
  const int8_t *gq = nullptr, *uq = nullptr, *dq = nullptr;
  const __half *gd = nullptr, *ud = nullptr, *dd = nullptr;
  const int8_t *qkv_q = nullptr, *o_q = nullptr;
  const __half *qkv_d = nullptr, *o_d = nullptr;
  const __half *kc = nullptr, *vc = nullptr;
  int F = 0;
};
extern int g_l2pf_blocks;  // L2 prefetch blocks per kv head in the two-launch attention launch (0 = off, <= 16)
extern int g_l2pf_max_m;   // > 0 (A/B): ... with g_l2pf_mask for decode batches up to this width (0: per-batch table)
extern int g_l2pf_delay;   // their start delay, ticks of the 100 MHz clock
extern int g_l2pf_mask;    // A/B: which byte sets they pull (1 FFN weights, 2 next attention weights, 4 next K/V)
void attn_o_fused(const float* qkv, const float* qn, const float* kn, float eps, const float* rcos, const float* rsin,
                  __half* kc, __half* vc, int H, int KV, const int* tok_seq, const int* tok_pos, int64_t seq_stride,
                  const int8_t* wo_q, const __half* wo_d, int E, const AttnWork& wk, const FusedDecodeWork& fw,
                  hipStream_t s);
// Two-launch layer: the q|k|v GEMV (prologue x = x + sum psum, block (0, 0) stores it to xsum) in the attention
// launch (k_attn_o<true>); psum = nullptr for layer 0.
void qkv_attn_o_fused(const float* x, const float* psum, float* xsum, const float* norm_w, const int8_t* wqkv_q,
                      const __half* wqkv_d, float* qkv, const float* qn, const float* kn, float eps, const float* rcos,
                      const float* rsin, __half* kc, __half* vc, int H, int KV, const int* tok_seq, const int* tok_pos,
                      int64_t seq_stride, const int8_t* wo_q, const __half* wo_d, int E, const AttnWork& wk,
                      const FusedDecodeWork& fw, hipStream_t s, int M = 1, int dbg_drop = 0,
                      const L2Prefetch* pf = nullptr);
// M tokens (rows of x / xsum, slabs of the workspace); M = 1: the batch-1 layer
void ffn_fused(const float* x, const float* norm_w, float eps, const int8_t* gq, const __half* gd, const int8_t* uq,
               const __half* ud, const int8_t* dq, const __half* dd, int E, int F, const FusedDecodeWork& fw,
               hipStream_t s, int M = 1);
// Batched decode at M = 32 (llm.hip k_attn_ob): attention + o projection + residual + the o GEMM's normalising
// epilogue in one launch. Workspace: aq / ad the q8_0 attention rows ([32][H D] int8, [32][H D / 32] f32), opart
// [32][KV][32][32] floats, cnt_g [KV] / cnt_s [32] counter lines (zeroed once), err the timeout flag.
struct AttnObWork {
  int8_t* aq = nullptr;
  float* ad = nullptr;
  float* opart = nullptr;
  unsigned* cnt_g = nullptr;
  unsigned* cnt_s = nullptr;
  int* err = nullptr;
};
void attn_o_batched(const float* qkv, const float* qn, const float* kn, float eps, const float* rcos, const float* rsin,
                    __half* kc, __half* vc, int M, int H, int KV, const int* tok_seq, const int* tok_pos,
                    int64_t seq_stride, const int8_t* wo_q, const __half* wo_d, int E, const AttnObWork& w, float* x,
                    const float* qn_w, int8_t* qout, float* dout, float* ssp_out, hipStream_t s);
extern int g_gemm_bf3_pf;     // few-tile bf16x3 GEMMs: global loads 1 or 2 k-steps ahead (default 2)
extern int g_gemm_bf3_256;    // bf16x3 GEMMs: 256x256 tiles when a launch has at least this many (0 = off)
extern int g_ffn_wide;  // small decode batches of 3-6: the fused FFN as one slab, all tokens per block (A/B)
extern int g_ffn_pair_min_m;  // small decode batches from this width: two tokens per fused-FFN block (default 2)
// out[m] = xmid[m] + sum_p dpart[m][p] for m < M (a small batch's residual rows after its last fused layer)
void psum_rows(const float* xmid, const float* dpart, int M, int E, float* out, hipStream_t s);
// dst[i] = src[rows[i]] (n rows of E floats; row stride E both sides)
void gather_rows(const float* src, const int* rows, int n, int E, float* dst, hipStream_t s);
void prompt_rows(const float* host, const float* audio, int64_t ts, const int* codes, int n, int E, float* dst,
                 hipStream_t s);
void embed_rows(const int8_t* qs, const __half* d, const int* ids, int n, int E, int fp16_round, float* out,
                hipStream_t s);
// Decode-step tail fused into the sampler: embedding row of the sampled token -> x (the next step's input), and
// tok_pos / step_ctr advanced by one (x == nullptr: sample only, e.g. after prefill)
struct EmbedNext {
  const int8_t* qs = nullptr;
  const __half* d = nullptr;
  int E = 0;
  float* x = nullptr;
  int* tok_pos = nullptr;
};
// Sampler chain parameters (fa_sampling) in device memory: one captured decode-step graph serves every setting.
struct SampleParams {
  float temperature, top_p;
  int top_k;
  uint32_t seed;
};
// row_seq / row_pos [M]: sequence id and position of each row's token (the draw's counter: (seed, seq, pos));
// partial t of a row covers logits [chunk t, chunk (t + 1)) (the lm_head launch's rows per partial)
void sample_tokens(const float* logits, int64_t ldl, int V, const float* pval, const int* pidx, int n_part, int chunk,
                   int M, const SampleParams* d_params, const int* row_seq, const int* row_pos, int* step_ctr,
                   int* tok_out, int* tok_hist, int hist_stride, const EmbedNext* en, hipStream_t s);
int lm_head_chunk(int O, int M, int K = 1024);  // rows per argmax partial of the lm_head launch for M tokens
void advance_positions(int* tok_pos, int* step_ctr, int M, hipStream_t s);
void gpu_delay_us(int us, hipStream_t s);

}  // namespace fa
