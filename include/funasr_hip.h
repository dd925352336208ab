/*
 * funasr_hip.h — C-ABI of the MI355X-native Fun-ASR hot-path engine (libfunasr_hip.so).
 *
 * Replaces the two native runtimes the reference drives from Python on its per-segment hot path
 * (SURVEY.md §8(b)):
 *   - onnxruntime sessions for the encoder+adaptor graph and the CTC graph
 *       /root/reference/fun_asr_gguf/nano_onnx.py:78-133 (encode_audio -> run_with_ort_values)
 *       /root/reference/fun_asr_gguf/core/decoder.py:27 (ctc_sess.run -> indices int32)
 *   - llama.cpp b7798 bound by ctypes (llama.py:150-349): llama_model_load_from_file,
 *     llama_init_from_model, llama_batch_init/set_embd, llama_decode, llama_memory_clear,
 *     llama_sampler_* , llama_get_logits (llama.py:462-659)
 *
 * Conventions: plain pointers + sizes, no torch types. Host buffers are owned by the caller and
 * read-only during a call; every device allocation is owned by the engine. Every fa_* returns 0 on
 * success and a negative code on failure; fa_last_error() returns a thread-local message.
 * Calls on one engine are serialised by the caller (the reference engine is not re-entrant either:
 * one KV cache, decoder.py:71). One engine per GPU.
 */
#ifndef FUNASR_HIP_H
#define FUNASR_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_OK 0
#define FA_ERR_ARG -1
#define FA_ERR_HIP -2
#define FA_ERR_STATE -3
#define FA_ERR_IO -4
#define FA_ERR_NOTFOUND -5

typedef struct fa_engine fa_engine;

/* Encoder/adaptor/CTC dimensions (model_definition.py:191-229). */
typedef struct fa_encoder_config {
  int32_t n_mels, lfr_m, lfr_n, d_in, d_model, n_heads, d_ffn, n_blocks, n_tp_blocks, fsmn_k;
  int32_t d_llm, adaptor_ffn, adaptor_blocks, adaptor_heads;
  int32_t ctc_blocks, ctc_heads, ctc_ffn, ctc_vocab;
} fa_encoder_config;

/* Qwen3 decoder dimensions (GGUF qwen3 arch). n_ctx matches LlamaContext(n_ctx=2048),
 * model_manager.py:63-69; max_seqs is the continuous-batch width (1 in the reference). */
typedef struct fa_llm_config {
  int32_t n_layer, n_embd, n_head, n_head_kv, head_dim, n_ff, n_vocab, n_ctx, max_seqs;
  float rope_theta, rms_eps;
} fa_llm_config;

/* Sampler chain of LlamaSampler (llama.py:577-605): temperature <= 0 (or top_k == 1) -> greedy;
 * else top_k (<= 0: all) -> top_p (min_keep 1; >= 1: no-op) -> temp -> dist. The draw of a token is keyed
 * by (seed, sequence id, position), so every step and every call draws afresh. */
typedef struct fa_sampling {
  float temperature, top_p;
  int32_t top_k;
  uint32_t seed;
} fa_sampling;

/* ---- lifecycle (replaces load_onnx_models nano_onnx.py:21-76, LlamaModel/LlamaContext llama.py:352-488) */
int fa_engine_create(int32_t device, const fa_encoder_config* enc, const fa_llm_config* llm,
                     int32_t max_batch, int64_t max_samples, fa_engine** out);
int fa_engine_destroy(fa_engine* e);
const char* fa_last_error(void);
/* llama_log_set-style callback (llama.py:692-732): level 2 error, 3 warn, 4 info, 5 debug. */
int fa_set_log_callback(void (*cb)(int32_t level, const char* msg, void* user), void* user);

/* ---- weights */
/* Deterministic synthetic weights generated on device (spec: oracle/synth.py; real weights absent). */
int fa_weights_synthetic(fa_engine* e, uint32_t seed);
/* Upload one tensor by reference state_dict / GGUF name. Decoder 2-D tensors given as f32 are
 * quantised to q8_0 on device with the ggml reference quantiser (gguf/quants.py:378-393). */
int fa_set_tensor_f32(fa_engine* e, const char* name, const float* host, int64_t n);
int fa_set_tensor_q8_0(fa_engine* e, const char* name, const uint8_t* blocks, int64_t n_bytes);
/* One CTC-graph linear in ONNX Runtime dynamic-quant form, as Fun-ASR-Nano-CTC.int8.onnx holds it (02-Quantize-ONNX.py
 * :38-46: quantize_dynamic over MatMul, per_channel, QUInt8 weights): q [rows = out][cols = in] uint8 (the ONNX
 * `<w>_quantized` [in][out] initializer transposed), scale[out] (`<w>_scale`), zero_point[out] (`<w>_zero_point`). `name`
 * is the f32 weight's state_dict name (ctc_decoder.* / ctc_proj.ctc_lo.weight). Once every CTC-graph linear has its
 * int8 form, the CTC head runs the quantized graph's arithmetic (DynamicQuantizeLinear of each MatMul input per clip,
 * MatMulInteger, f32 rescale; attention and LayerNorm f32) instead of the f32 graph — replaces the CTC InferenceSession
 * over the int8 model (decoder.py:27, nano_onnx.py:21-46). */
int fa_set_tensor_u8dq(fa_engine* e, const char* name, const uint8_t* q, const float* scale, const uint8_t* zero_point,
                       int64_t rows, int64_t cols);
/* 1 (default): the int8-dynamic CTC graph once all its weights are set; 0: the f32 (or fp16) CTC graph. */
int fa_set_ctc_int8(fa_engine* e, int32_t on);
/* *out = 1 when the next CTC head runs the int8-dynamic graph. */
int fa_ctc_int8_active(fa_engine* e, int32_t* out);
/* Decoder weights from a GGUF v3 file (q8_0 / f32 / f16 tensors) — replaces llama_model_load_from_file. */
int fa_load_gguf(fa_engine* e, const char* path);
/* Copy a decoder tensor back as ggml q8_0 blocks (test hook). */
int fa_get_tensor_q8_0(fa_engine* e, const char* name, uint8_t* out, int64_t n_bytes);
/* Copy an f32 tensor (encoder / norm weights) back (test hook). */
int fa_get_tensor_f32(fa_engine* e, const char* name, float* out, int64_t n);
/* Load-completeness bookkeeping (the reference's init fails when a model file cannot fill its graph:
 * ORT/llama.cpp raise, model_manager.py:98-100 -> asr_engine.py:135). Every upload (fa_set_tensor_*,
 * fa_load_gguf) marks its tensor as loaded; fa_weights_mark_unset clears that mark for every tensor whose
 * name starts with `prefix` ("" = all); fa_tensor_names lists the tensors under `prefix` in registration
 * order ('\n'-separated, NUL-terminated into buf of cap bytes; *needed = bytes required including the NUL),
 * only the ones not loaded since the last mark when only_unset != 0. */
int fa_weights_mark_unset(fa_engine* e, const char* prefix);
int fa_tensor_names(fa_engine* e, const char* prefix, int32_t only_unset, char* buf, int64_t cap, int64_t* needed);

/* ---- encoder operator (replaces encoder_sess.run_with_ort_values + ctc_sess.run)
 * pcm: batch clips, clip b at pcm + b*stride with n_samples[b] valid samples (16 kHz f32).
 * Outputs (host, may be NULL to skip):
 *   audio_embd_out [batch, tgt_stride, d_llm]   adaptor rows < target_len[b] (nano_onnx.py:129-131)
 *   ctc_ids_out    [batch, ids_stride]          argmax ids for frames < t_lfr[b] (model_definition.py:337)
 *   enc_out        [batch, ids_stride, d_model] encoder output (test hook)
 * t_lfr_out/target_len_out [batch]. A padded batch reproduces the unpadded per-clip result. */
int fa_encode(fa_engine* e, const float* pcm, const int64_t* n_samples, int32_t batch, int64_t stride,
              float* audio_embd_out, int64_t tgt_stride, int32_t* ctc_ids_out, int64_t ids_stride,
              int32_t* t_lfr_out, int32_t* target_len_out, float* enc_out);
/* Same, but pcm is a DEVICE pointer (NULL = the engine's buffer filled by fa_pcm_upload) (inputs already resident in HBM) and the ids/lengths are left on
 * device; fa_encode_fetch copies them out. Used by the benchmark and the batch scheduler. */
int fa_encode_device(fa_engine* e, const float* d_pcm, const int64_t* n_samples, int32_t batch, int64_t stride);
/* Upload PCM into the engine's own HBM buffer (same layout as fa_encode); a following
 * fa_encode_device(e, NULL, ...) encodes from it. Lets callers keep inputs resident across calls. */
int fa_pcm_upload(fa_engine* e, const float* pcm, int64_t n_floats);
int fa_encode_fetch(fa_engine* e, float* audio_embd_out, int64_t tgt_stride, int32_t* ctc_ids_out,
                    int64_t ids_stride, int32_t* t_lfr_out, int32_t* target_len_out, float* enc_out);
/* The CTC graph alone (ctc_sess.run({"enc_output": ...}), decoder.py:27): ctc_decoder with no mask, ctc_lo and
 * argmax (model_definition.py:335-337) over T caller-given encoder rows enc [T, d_model] f32 (fp16 graph: fp16
 * values) -> ids_out [T]. Reuses the encode buffers: the outputs of the previous fa_encode cannot be fetched after. */
int fa_ctc_head(fa_engine* e, const float* enc, int32_t T, int32_t* ids_out);
/* Greedy CTC collapse on device (nano_ctc.py:65-104): for clip b, compacted (id, first_frame) pairs
 * with blanks (= blank_id) and repeats removed; n_out[b] = count. */
int fa_ctc_collapse(fa_engine* e, int32_t blank_id, int32_t* ids_out, int32_t* frames_out, int64_t out_stride,
                    int32_t* n_out);
/* Encode mode: 0 (default) = one padded batch; 1 = independent clips: every clip of a multi-clip call runs the
 * single-clip encode (exactly the arithmetic of encoding it alone) in a lane of its own -- its own rows of the batch
 * arenas, its own workspaces and HIP stream -- so up to 8 one-clip encodes run concurrently. Used where a batch must
 * give each clip its one-at-a-time result (the reference encodes every segment alone, orchestrator.py:139-171). */
int fa_set_encode_mode(fa_engine* e, int32_t mode);
/* Debug hooks (tests): flags bit 0 keeps clip 0's embedded LFR features (x*sqrt(512)+PE, [T, d_in]) of
 * the next fa_encode; fa_encode_tap(e, 0, out, n) copies them out. Bit 1 makes one block of the fused decode layer
 * withhold its q|k|v hand-off, forcing the in-launch fan-in timeout (10 ms per wait): fa_llm_generate_end then
 * re-runs the chunk on the 5-launch layer, which the engine keeps from then on (the bit clears itself). */
/* Encoder precision: 0 = fp32 graph (Fun-ASR-Nano-Encoder-Adaptor.fp32.onnx / CTC.fp32.onnx), 1 = the float16
 * graphs of 02-Quantize-ONNX.py:13-27 (fp16 weights and op outputs, LayerNorm in fp32, fp16 input audio;
 * replaces the dtype switch of nano_onnx.py:84,101). The fp16 weight copies are built on the next encode. */
int fa_set_encoder_fp16(fa_engine* e, int32_t on);
/* fp32-graph GEMM arithmetic: 1 (default) = bf16x3 split operands on the bf16 matrix cores (x w ~= xh wh + xh wl +
 * xl wh, f32 accumulate; ~2^-16 relative error per product, held to the fp32 goldens' tolerances by the tests);
 * 0 = exact-f32 MFMA (v_mfma_f32_32x32x2_f32). Env FUNASR_ENC_GEMM=f32 selects 0 at engine creation. The split
 * weight copies are built on the next encode. No effect in fp16 mode. */
int fa_set_encoder_gemm(fa_engine* e, int32_t mode);
/* Decode layer structure: 1 (default) = 2 launches per layer (q|k|v GEMV + attention + a split o projection with
 * in-launch group hand-offs; gate|up + a split down projection) for batch 1 and for decode batches up to
 * FUNASR_FUSED_MAX_M (default 6) sequences; 2 = 3 launches at batch 1 (the q|k|v GEMV as its own launch;
 * bit-identical to 1); 0 = the 5-launch layer (what wider batches always use). Same numerics contract (ggml q8_0),
 * different f32 summation order of the o / down projections between 0 and 1/2. */
int fa_set_decode_fused(fa_engine* e, int32_t on);
/* Test hooks: bit 0 taps the LFR rows of the next encode (fa_encode_tap); bit 1 makes one block of the fused attention
 * launch withhold its q|k|v hand-off in the next decode chunk (a forced fan-in timeout, cleared by the recovery); bit 2
 * with bit 1 keeps withholding it (the fused re-run times out too). */
int fa_set_debug(fa_engine* e, int32_t flags);
int fa_encode_tap(fa_engine* e, int32_t which, float* out, int64_t n);

/* ---- decoder operator (replaces llama_decode / llama_sampler_sample / llama_memory_clear) */
/* Embedding rows from token_embd (q8_0). fp16_round=1 reproduces the numpy f16 product of
 * get_token_embeddings_gguf (llama.py:782-784) used for prompt rows; 0 = ggml get_rows (f32). */
int fa_embd_rows(fa_engine* e, const int32_t* ids, int32_t n, int32_t fp16_round, float* out);
/* llama_memory_clear for one sequence slot. */
int fa_llm_reset(fa_engine* e, int32_t seq);
/* Prefill a sequence with n_tokens input embeddings [n_tokens, n_embd] f32 (LlamaBatch.set_embd with
 * token=NULL, logits on the last row only; llama.py:536-558, decoder.py:70-80), then sample the first
 * token with `s`. logits_out (nullable) receives the last-row logits [n_vocab]. */
int fa_llm_prefill(fa_engine* e, int32_t seq, const float* embd, int32_t n_tokens, const fa_sampling* s,
                   int32_t* tok_out, float* logits_out);
/* fa_llm_prefill for n_seqs sequences (distinct ids) at once: embd holds their prompts back to back
 * [sum n_tokens, n_embd], n_tokens[i] rows for seqs[i]. As many sequences as fit the row capacity share one
 * forward (one pass over the weights instead of one per sequence; each row attends its own sequence's keys), then
 * every sequence samples its first token keyed on its own (seq, last position): tok_out [n_seqs]. Replaces the
 * per-sequence llama_decode of a prompt batch (decoder.py:70-80 run per stream). */
int fa_llm_prefill_batch(fa_engine* e, const int32_t* seqs, int32_t n_seqs, const float* embd, const int32_t* n_tokens,
                         const fa_sampling* s, int32_t* tok_out);
/* fa_llm_prefill / fa_llm_prefill_batch with the prompt rows assembled on the device instead of uploaded: the
 * reference concatenates [prefix rows | audio_embd | suffix rows] on the host (core/decoder.py:199) and hands the
 * result to llama_decode (decoder.py:73-77); here the audio rows stay where the last encode left them. row_src holds
 * one code per prompt row (sum n_tokens, prompts back to back): code >= 0 = row `code` of host_rows [n_host_rows,
 * n_embd] (the caller's prefix / suffix rows, uploaded once per call); code < 0 = adaptor output row t of clip b of
 * the last encode, code = -1 - (b << 16 | t) (t < target_len[b]). enc_gen = fa_encode_generation() right after that
 * encode: the call fails (FA_ERR_ARG) if another encode or CTC-head call has run since. The rows equal the host
 * concatenation bit for bit, so the results are fa_llm_prefill's (n_seqs == 1) / fa_llm_prefill_batch's. */
int fa_llm_prefill_rows(fa_engine* e, const int32_t* seqs, int32_t n_seqs, const float* host_rows, int32_t n_host_rows,
                        const int32_t* row_src, const int32_t* n_tokens, int64_t enc_gen, const fa_sampling* s,
                        int32_t* tok_out);
/* Generation of the last encode's outputs (-1 if none are held, e.g. after fa_ctc_head). */
int fa_encode_generation(fa_engine* e, int64_t* gen_out);
/* Run n_steps decode steps for n_seqs sequences (distinct ids) in one continuous batch: each step feeds
 * every sequence's last sampled token at its next position and samples the next one on device
 * (decoder.py:91-98). tokens_out [n_seqs, n_steps]. No host round trip inside the call. */
int fa_llm_generate(fa_engine* e, const int32_t* seqs, int32_t n_seqs, int32_t n_steps, const fa_sampling* s,
                    int32_t* tokens_out);
/* fa_llm_generate in two halves: _begin validates, enqueues the n_steps graph replays and the copy of the sampled
 * tokens into pinned host memory, and returns at once; _end waits for that copy and does the host bookkeeping
 * (positions, last tokens, logits rows), writing the tokens as fa_llm_generate does (tokens_out may be NULL). One call
 * in flight per engine; the other fa_llm_* calls refuse while it is. The host can work on the previous chunk's tokens
 * in between (the llama_decode loop of decoder.py:91-98 has no such overlap: its sampling is on the host). */
int fa_llm_generate_begin(fa_engine* e, const int32_t* seqs, int32_t n_seqs, int32_t n_steps, const fa_sampling* s);
int fa_llm_generate_end(fa_engine* e, int32_t* tokens_out);
/* (fa_llm_generate_end: when the chunk ran on the fused small-batch layer and one of its in-launch fan-ins timed out --
 * a group of blocks not co-resident because another kernel held CUs -- the chunk is decoded again on the 5-launch layer
 * from the same positions and input tokens, and the engine keeps that layer; the tokens returned are the re-run's.) */
/* Logits [n_vocab] of sequence `seq` from the most recent forward (fa_llm_prefill, or the last step of
 * fa_llm_generate) when that forward included it; FA_ERR_ARG otherwise (test hook; llama_get_logits_ith). */
int fa_llm_logits(fa_engine* e, int32_t seq, float* out);
/* Largest decode batch width whose per-token arithmetic is bit-identical to decoding that sequence alone (the
 * reference decodes every segment alone, core/decoder.py:70-123): sequences decoded together in batches up to this
 * width, each prefilled alone, produce exactly their single-sequence tokens. Wider batches agree to the q8_0 noise
 * floor. */
int fa_llm_invariant_width(fa_engine* e, int32_t* out);
/* Fused-layer timeout recoveries of this engine (llm.hip k_attn_o / k_ffn_fused bound every in-launch wait): *retries =
 * decode chunks re-run on the fused layer after a fan-in timed out (same arithmetic: results unchanged); *fallbacks =
 * chunks whose re-run timed out too and ran on the 5-launch layer (agreeing with single-sequence decoding to the q8_0
 * noise floor, not bit for bit). Three fallbacks in a row keep the 5-launch layer (fa_llm_invariant_width drops to 1);
 * otherwise the next chunk runs the fused layer again. No reference counterpart (llama.cpp has no in-launch waits). */
int fa_llm_decode_recoveries(fa_engine* e, int32_t* retries, int32_t* fallbacks);
/* Make `token` the input of the sequence's next generate step in place of the token it sampled last: the
 * caller-chosen token of the reference loop's llama_decode(batch{token, pos}) (decoder.py:91-98, llama.py:490-498),
 * used for teacher-forced parity runs. */
int fa_llm_set_token(fa_engine* e, int32_t seq, int32_t token);
/* Current length (n_past) of a sequence slot. */
int fa_llm_n_past(fa_engine* e, int32_t seq, int32_t* out);

/* ---- tokenizer / detokenizer from GGUF metadata (replaces llama_model_get_vocab + llama_tokenize +
 * llama_token_to_piece, llama.py:738-748; used by PromptBuilder.build_prompt prompt_utils.py:44-52 and the
 * streamed output ASRStreamDecoder.push llama.py:671-683). Byte-level BPE with the Qwen2 pre-tokenizer
 * (tokenizer.ggml.pre "qwen2"); control / user-defined tokens are matched in the text when parse_special != 0.
 * Pure host code (no device). */
typedef struct fa_vocab fa_vocab;
int fa_vocab_load_gguf(const char* path, fa_vocab** out);
int fa_vocab_free(fa_vocab* v);
int fa_vocab_info(const fa_vocab* v, int32_t* n_tokens, int32_t* eos_id);
/* text: UTF-8 bytes (add_special = false). *n_out = number of tokens; FA_ERR_ARG when cap is too small. */
int fa_tokenize(const fa_vocab* v, const char* text, int32_t n_bytes, int32_t parse_special, int32_t* out,
                int32_t cap, int32_t* n_out);
/* raw bytes of one token (special = true: control tokens render as their text). */
int fa_token_piece(const fa_vocab* v, int32_t id, char* buf, int32_t cap, int32_t* n_out);
/* One GGUF tensor (q8_0 / f16 / f32) dequantised to f32 [n]; fp16_product = 1 reproduces the numpy-f16
 * product of get_token_embeddings_gguf (llama.py:778-784), 0 = ggml dequantize_row_q8_0. */
int fa_gguf_read_tensor(const char* path, const char* name, int32_t fp16_product, float* out, int64_t n);

/* ---- host-side char alignment (replaces nano_ctc.align_timestamps, nano_ctc.py:118-232)
 * ctc_keys/llm_keys: per-char integer keys (equal iff the chars' .lower() strings are equal);
 * ctc_starts: per-CTC-char start seconds (token start + i*0.08). starts_out[n_llm] receives each LLM
 * char's start; aligned_out[n_llm] (nullable) the matched CTC char index or -1. Bit-identical to the
 * reference (same tie order, same float64 evaluation order). Pure host code, no device needed. */
int fa_align_timestamps(const int32_t* ctc_keys, const double* ctc_starts, int32_t n_ctc, const int32_t* llm_keys,
                        int32_t n_llm, double* starts_out, int32_t* aligned_out);

/* ---- hotword retrieval (host): the FastRAG coarse distance of rag_fast.py:35-77 (numba in the reference):
 * min over end positions of the edit distance between sub_codes [n] and a substring of main_codes [m] (free
 * start). *dist_out = n when either is empty. */
int fa_fuzzy_substring_distance(const int32_t* main_codes, int32_t m, const int32_t* sub_codes, int32_t n,
                                float* dist_out);

/* ---- timing hooks for bench.py roofline (HIP events on the engine's stream) */
/* Enable per-kernel-class event timing; fa_profile_read returns accumulated ms and launch counts for
 * class ids: 0 q8 GEMV/GEMM of the decoder layers, 1 f32 GEMM (encoder), 2 encoder attention,
 * 3 decoder attention, 4 LM head, 5 layer 0's decoder launches (classes 0 and 3 of layer 0), 6 prefill forwards'
 * layer launches (sampled layers only). Classes 0 and 3
 * are sampled on layer 1 only (identical shapes in every layer; from layer 1 on the weights arrive L2-warm from
 * the previous launches' prefetch slabs, layer 0's do not): the device time of all layers is class 5 +
 * (n_layer - 1) x (classes 0 + 3). */
int fa_profile_enable(fa_engine* e, int32_t on);
int fa_profile_read(fa_engine* e, int32_t cls, double* ms, int64_t* launches, double* bytes, double* flops);
int fa_synchronize(fa_engine* e);

/* ---- result gather over RCCL (the reference decodes segments sequentially, orchestrator.py:139-171,
 * so this is the only exchange of the sharded path): one communicator per engine. Rank 0 creates a 128-byte id, the
 * caller hands it to every rank by any side channel, each rank joins with fa_comm_init. The gather is two all-gathers
 * (every rank calls both, in order): the record sizes, then the records zero-padded to one slot >= the largest. */
int fa_comm_unique_id(uint8_t* id_out /* 128 bytes */);
int fa_comm_init(fa_engine* e, int32_t rank, int32_t world, const uint8_t* id);
int fa_comm_allgather_sizes(fa_engine* e, int64_t n, int64_t* sizes_out /* [world] */);
int fa_comm_allgather_bytes(fa_engine* e, const uint8_t* data, int64_t n, int64_t slot, uint8_t* out /* [world * slot] */);
int fa_comm_destroy(fa_engine* e);

#ifdef __cplusplus
}
#endif
#endif
