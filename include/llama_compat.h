/* llama.cpp-compatible C ABI over the MI355X engine (lib/llama_compat/libllama.so).
 *
 * The reference drives its decoder through ctypes bindings of llama.cpp b7798 (fun_asr_gguf/llama.py:150-349),
 * loading libggml.so, libggml-base.so and libllama.so from fun_asr_gguf/bin (llama.py:170-188). This library
 * exports the subset of that API the reference binds, with the b7798 struct layouts the bindings declare
 * (llama.py:27-104), so the reference's own llama.py / core/decoder.py run unmodified on the HIP engine when these
 * three files and libfunasr_hip.so (libllama.so's dependency, found through rpath $ORIGIN) stand in its bin/ directory
 * (INTEGRATION.md §5). Every call goes through the public fa_* ABI of
 * include/funasr_hip.h:
 *   llama_model_load_from_file  GGUF metadata + tokenizer (fa_vocab_load_gguf); weights load at context creation
 *   llama_init_from_model       fa_engine_create (n_ctx, n_seq_max from the context params) + fa_load_gguf, failing
 *                               when the file leaves any decoder tensor unset
 *   llama_decode                embedding batches -> fa_llm_prefill; one-token batches -> fa_llm_set_token +
 *                               fa_llm_generate (one step); logits of the batch's last row -> fa_llm_logits
 *   llama_memory_clear          fa_llm_reset of every sequence slot
 *   llama_tokenize / llama_token_to_piece / llama_vocab_*   fa_tokenize / fa_token_piece / fa_vocab_info
 *   llama_sampler_*             the top_k -> top_p -> temp -> dist / greedy chain of LlamaSampler (llama.py:577-605)
 *                               on the host over llama_get_logits (as llama.cpp samples on the host)
 * Limits (each refused with a logged error and a non-zero return, never silently): one output row per decode (the
 * batch's last row; the reference flags only that one, llama.py:556, 569), a batch holds one sequence at positions
 * continuing its current length, token batches of more than one row are embedded and prefilled. Greedy selection is
 * bit-identical to llama.cpp's; the dist sampler draws from std::mt19937(seed) (the reference seeds it randomly per
 * call, decoder.py:89, so its stream is not a parity target). */
#ifndef LLAMA_COMPAT_H
#define LLAMA_COMPAT_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t llama_token;
typedef int32_t llama_pos;
typedef int32_t llama_seq_id;

typedef struct llama_model llama_model;
typedef struct llama_context llama_context;
typedef struct llama_vocab llama_vocab;
typedef struct llama_sampler llama_sampler;
typedef struct llama_context llama_memory; /* llama_get_memory hands out the context itself */

/* llama.py:27-46 */
typedef struct llama_model_params {
  void* devices;
  const void* tensor_buft_overrides;
  int32_t n_gpu_layers;
  int32_t split_mode;
  int32_t main_gpu; /* HIP device of the engine */
  const float* tensor_split;
  bool (*progress_callback)(float progress, void* user_data);
  void* progress_callback_user_data;
  const void* kv_overrides;
  bool vocab_only, use_mmap, use_direct_io, use_mlock, check_tensors, use_extra_bufts, no_host, no_alloc;
} llama_model_params;

/* llama.py:48-82 */
typedef struct llama_context_params {
  uint32_t n_ctx, n_batch, n_ubatch, n_seq_max;
  int32_t n_threads, n_threads_batch;
  int32_t rope_scaling_type, pooling_type, attention_type, flash_attn_type;
  float rope_freq_base, rope_freq_scale, yarn_ext_factor, yarn_attn_factor, yarn_beta_fast, yarn_beta_slow;
  uint32_t yarn_orig_ctx;
  float defrag_thold;
  void* cb_eval;
  void* cb_eval_user_data;
  int32_t type_k, type_v;
  void* abort_callback;
  void* abort_callback_data;
  bool embeddings, offload_kqv, no_perf, op_offload, swa_full, kv_unified;
  void* samplers;
  size_t n_samplers;
} llama_context_params;

/* llama.py:84-93 */
typedef struct llama_sampler_chain_params {
  bool no_perf;
} llama_sampler_chain_params;
typedef struct llama_logit_bias {
  llama_token token;
  float bias;
} llama_logit_bias;

/* llama.py:95-104 */
typedef struct llama_batch {
  int32_t n_tokens;
  llama_token* token;
  float* embd;
  llama_pos* pos;
  int32_t* n_seq_id;
  llama_seq_id** seq_id;
  int8_t* logits;
} llama_batch;

typedef void (*ggml_log_callback)(int level, const char* text, void* user_data);

/* lifecycle (llama.py:192-246) */
void llama_log_set(ggml_log_callback cb, void* user_data);
void llama_backend_init(void);
void llama_backend_free(void);
llama_model_params llama_model_default_params(void);
llama_model* llama_model_load_from_file(const char* path, llama_model_params params);
void llama_model_free(llama_model* model);
const llama_vocab* llama_model_get_vocab(const llama_model* model);
int32_t llama_model_n_embd(const llama_model* model);
llama_context_params llama_context_default_params(void);
llama_context* llama_init_from_model(llama_model* model, llama_context_params params);
void llama_free(llama_context* ctx);

/* batches and decode (llama.py:249-269) */
llama_batch llama_batch_init(int32_t n_tokens, int32_t embd, int32_t n_seq_max);
void llama_batch_free(llama_batch batch);
int32_t llama_decode(llama_context* ctx, llama_batch batch);
float* llama_get_logits(llama_context* ctx);
float* llama_get_logits_ith(llama_context* ctx, int32_t i);
float* llama_get_embeddings(llama_context* ctx);

/* vocabulary (llama.py:272-291) */
int32_t llama_tokenize(const llama_vocab* vocab, const char* text, int32_t text_len, llama_token* tokens,
                       int32_t n_tokens_max, bool add_special, bool parse_special);
int32_t llama_vocab_n_tokens(const llama_vocab* vocab);
llama_token llama_vocab_eos(const llama_vocab* vocab);
int32_t llama_token_to_piece(const llama_vocab* vocab, llama_token token, char* buf, int32_t length, int32_t lstrip,
                             bool special);

/* KV cache (llama.py:294-300) */
llama_memory* llama_get_memory(const llama_context* ctx);
void llama_memory_clear(llama_memory* mem, bool data);

/* sampler chain (llama.py:303-346) */
llama_sampler_chain_params llama_sampler_chain_default_params(void);
llama_sampler* llama_sampler_chain_init(llama_sampler_chain_params params);
void llama_sampler_chain_add(llama_sampler* chain, llama_sampler* smpl);
llama_sampler* llama_sampler_init_greedy(void);
llama_sampler* llama_sampler_init_dist(uint32_t seed);
llama_sampler* llama_sampler_init_temp(float t);
llama_sampler* llama_sampler_init_top_k(int32_t k);
llama_sampler* llama_sampler_init_top_p(float p, size_t min_keep);
llama_sampler* llama_sampler_init_logit_bias(int32_t n_vocab, int32_t n_logit_bias, const llama_logit_bias* logit_bias);
llama_token llama_sampler_sample(llama_sampler* smpl, llama_context* ctx, int32_t idx);
void llama_sampler_free(llama_sampler* smpl);

/* test hooks (not llama.cpp API): the sampler chain over a caller's logits row; the struct sizes this library was
 * built with (model params, context params, batch) and their field offsets, for the layout check against the
 * reference's ctypes declarations (tests/golden/llama_abi.json) */
llama_token fa_llama_sampler_apply(llama_sampler* smpl, const float* logits, int32_t n_vocab);
void fa_llama_struct_sizes(size_t* out3);
int64_t fa_llama_field_offset(const char* strct, const char* field); /* offsetof, -1 for an unknown name */

#ifdef __cplusplus
}
#endif
#endif
