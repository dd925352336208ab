// llama.cpp b7798-compatible C ABI over the engine (include/llama_compat.h): the subset the reference binds in
// fun_asr_gguf/llama.py:150-349, so its LlamaModel / LlamaContext / LlamaBatch / LlamaSampler classes and the
// decode loop of core/decoder.py:55-123 run on MI355X without modification. Host code only: every device operation
// is a public fa_* call (include/funasr_hip.h).
#include "llama_compat.h"

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "funasr_hip.h"
#include "gguf.h"

namespace {

ggml_log_callback g_log_cb = nullptr;
void* g_log_user = nullptr;

void logf(int level, const std::string& m) {  // ggml levels: 2 error, 3 warn, 4 info, 5 debug
  const std::string line = m + "\n";
  if (g_log_cb) g_log_cb(level, line.c_str(), g_log_user);
  else if (level <= 3) fprintf(stderr, "llama_compat: %s", line.c_str());
}

bool fa_ok(int rc, const char* what) {
  if (rc == FA_OK) return true;
  logf(2, std::string(what) + ": " + fa_last_error());
  return false;
}

// Encoder dimensions of the engine a llama context owns: the decoder-only use never runs it, so the smallest
// configuration the engine accepts (oracle/synth.py ENC_TINY widths) with d_llm tied to the model's n_embd.
fa_encoder_config tiny_encoder(int32_t n_embd) {
  fa_encoder_config c{};
  c.n_mels = 80; c.lfr_m = 7; c.lfr_n = 6; c.d_in = 560; c.d_model = 512; c.n_heads = 4; c.d_ffn = 2048;
  c.n_blocks = 3; c.n_tp_blocks = 2; c.fsmn_k = 11;
  c.d_llm = n_embd; c.adaptor_ffn = 2048; c.adaptor_blocks = 1; c.adaptor_heads = 8;
  c.ctc_blocks = 1; c.ctc_heads = 8; c.ctc_ffn = 2048; c.ctc_vocab = 3001;
  return c;
}

const char* const kLlmGroups[] = {"token_embd.", "blk.", "output_norm."};  // core/model_manager.py LLM_GROUPS

}  // namespace

struct llama_vocab {
  fa_vocab* v = nullptr;
  int32_t n_tokens = 0, eos = -1;
  std::vector<int32_t> type;  // tokenizer.ggml.token_type (3 = control): hidden by token_to_piece(special = false)
};

struct llama_model {
  std::string path;
  int32_t device = 0;
  fa_llm_config cfg{};
  llama_vocab vocab;
};

struct llama_context {
  llama_model* model = nullptr;
  fa_engine* e = nullptr;
  int32_t n_seq_max = 1;
  std::vector<float> logits;  // the last decode's output row [n_vocab]
  bool has_logits = false;
};

struct llama_sampler {
  enum Kind { CHAIN, GREEDY, DIST, TEMP, TOP_K, TOP_P, LOGIT_BIAS } kind = CHAIN;
  std::vector<llama_sampler*> chain;
  float f = 0.f;
  int32_t k = 0;
  size_t min_keep = 1;
  std::mt19937 rng;
  std::vector<llama_logit_bias> bias;
};

namespace {

struct Cand {
  int32_t id;
  float logit, p;
};

// softmax over the candidates (sorted by logit, descending), as llama_sampler_softmax_impl
void softmax_sorted(std::vector<Cand>& c) {
  std::stable_sort(c.begin(), c.end(), [](const Cand& a, const Cand& b) { return a.logit > b.logit; });
  const float mx = c.empty() ? 0.f : c[0].logit;
  double sum = 0.0;
  for (auto& x : c) {
    x.p = std::exp(x.logit - mx);
    sum += x.p;
  }
  for (auto& x : c) x.p = (float)(x.p / sum);
}

// One stage of the chain; returns the selected token for the selecting stages (greedy, dist), else -1.
int32_t apply(llama_sampler* s, std::vector<Cand>& c) {
  switch (s->kind) {
    case llama_sampler::GREEDY: {  // first maximum, as llama_sampler_greedy_apply
      size_t best = 0;
      for (size_t i = 1; i < c.size(); ++i)
        if (c[i].logit > c[best].logit) best = i;
      return c.empty() ? -1 : c[best].id;
    }
    case llama_sampler::LOGIT_BIAS:
      for (const auto& b : s->bias)
        for (auto& x : c)
          if (x.id == b.token) x.logit += b.bias;
      return -1;
    case llama_sampler::TOP_K:
      if (s->k > 0 && (size_t)s->k < c.size()) {
        std::stable_sort(c.begin(), c.end(), [](const Cand& a, const Cand& b) { return a.logit > b.logit; });
        c.resize(s->k);
      }
      return -1;
    case llama_sampler::TOP_P: {
      if (s->f >= 1.0f) return -1;
      softmax_sorted(c);
      float cum = 0.f;
      size_t last = c.size();
      for (size_t i = 0; i < c.size(); ++i) {
        cum += c[i].p;
        if (cum >= s->f && i + 1 >= s->min_keep) {
          last = i + 1;
          break;
        }
      }
      c.resize(last);
      return -1;
    }
    case llama_sampler::TEMP:
      if (s->f <= 0.f) {  // temperature 0 keeps the maximum only
        size_t best = 0;
        for (size_t i = 1; i < c.size(); ++i)
          if (c[i].logit > c[best].logit) best = i;
        for (size_t i = 0; i < c.size(); ++i)
          if (i != best) c[i].logit = -INFINITY;
      } else {
        for (auto& x : c) x.logit /= s->f;
      }
      return -1;
    case llama_sampler::DIST: {
      softmax_sorted(c);
      std::uniform_real_distribution<double> u(0.0, 1.0);
      const double r = u(s->rng);
      double cum = 0.0;
      for (const auto& x : c) {
        cum += x.p;
        if (r < cum) return x.id;
      }
      return c.empty() ? -1 : c.back().id;
    }
    case llama_sampler::CHAIN: {
      int32_t sel = -1;
      for (auto* st : s->chain) {
        sel = apply(st, c);
        if (sel >= 0) break;
      }
      if (sel < 0 && !c.empty()) {  // a chain without a selecting stage: its most likely candidate
        size_t best = 0;
        for (size_t i = 1; i < c.size(); ++i)
          if (c[i].logit > c[best].logit) best = i;
        sel = c[best].id;
      }
      return sel;
    }
  }
  return -1;
}

llama_token sample_row(llama_sampler* s, const float* logits, int32_t n) {
  std::vector<Cand> c(n);
  for (int32_t i = 0; i < n; ++i) c[i] = Cand{i, logits[i], 0.f};
  return apply(s, c);
}

// GGUF metadata -> decoder dimensions (llama.cpp reads the same keys under the architecture prefix)
bool read_config(const fa::GGUFFile& g, fa_llm_config& c) {
  auto it = g.kv.find("general.architecture");
  const std::string arch = it != g.kv.end() ? it->second.s : "qwen3";
  auto num = [&](const std::string& k, double def, bool required) -> double {
    auto f = g.kv.find(arch + "." + k);
    if (f == g.kv.end()) {
      if (required) logf(2, "model file lacks " + arch + "." + k);
      return required ? NAN : def;
    }
    return f->second.type == 6 || f->second.type == 12 ? f->second.f : (double)f->second.i;
  };
  const double nl = num("block_count", 0, true), ne = num("embedding_length", 0, true),
               nh = num("attention.head_count", 0, true);
  if (std::isnan(nl) || std::isnan(ne) || std::isnan(nh)) return false;
  c.n_layer = (int32_t)nl;
  c.n_embd = (int32_t)ne;
  c.n_head = (int32_t)nh;
  c.n_head_kv = (int32_t)num("attention.head_count_kv", nh, false);
  c.head_dim = (int32_t)num("attention.key_length", ne / nh, false);
  c.rope_theta = (float)num("rope.freq_base", 10000.0, false);
  c.rms_eps = (float)num("attention.layer_norm_rms_epsilon", 1e-6, false);
  c.n_ff = 0;
  c.n_vocab = 0;
  for (const auto& t : g.tensors) {  // ggml dims: ne[0] = the inner (input) dimension
    if (t.name == "blk.0.ffn_gate.weight" && t.dims.size() == 2) c.n_ff = (int32_t)t.dims[1];
    if (t.name == "token_embd.weight" && t.dims.size() == 2) c.n_vocab = (int32_t)t.dims[1];
  }
  const double ff = num("feed_forward_length", c.n_ff, false);
  if (c.n_ff == 0) c.n_ff = (int32_t)ff;
  if (c.n_ff <= 0 || c.n_vocab <= 0) {
    logf(2, "model file lacks blk.0.ffn_gate.weight / token_embd.weight");
    return false;
  }
  return true;
}

bool check_loaded(fa_engine* e, const std::string& path) {
  for (const char* g : kLlmGroups) {
    int64_t need = 0;
    fa_tensor_names(e, g, 1, nullptr, 0, &need);
    std::string buf((size_t)std::max<int64_t>(need, 1), '\0');
    if (!fa_ok(fa_tensor_names(e, g, 1, &buf[0], (int64_t)buf.size(), &need), "fa_tensor_names")) return false;
    buf.resize(std::strlen(buf.c_str()));
    if (!buf.empty()) {
      logf(2, "model file " + path + " leaves decoder tensors unset:\n" + buf);
      return false;
    }
  }
  return true;
}

}  // namespace

extern "C" {

void llama_log_set(ggml_log_callback cb, void* user_data) {
  g_log_cb = cb;
  g_log_user = user_data;
  fa_set_log_callback(reinterpret_cast<void (*)(int32_t, const char*, void*)>(cb), user_data);
}

void llama_backend_init(void) {}
void llama_backend_free(void) {}

llama_model_params llama_model_default_params(void) {
  llama_model_params p{};
  p.n_gpu_layers = 999;
  p.split_mode = 1;
  p.main_gpu = 0;
  p.use_mmap = true;
  p.use_extra_bufts = true;
  return p;
}

llama_model* llama_model_load_from_file(const char* path, llama_model_params params) {
  if (!path) return nullptr;
  fa::GGUFFile g;
  if (!g.open(path)) {
    logf(2, std::string("llama_model_load_from_file: cannot read ") + path + ": " + fa::gguf_error());
    return nullptr;
  }
  auto* m = new llama_model();
  m->path = path;
  m->device = params.main_gpu;
  if (!read_config(g, m->cfg) || !fa_ok(fa_vocab_load_gguf(path, &m->vocab.v), "fa_vocab_load_gguf") ||
      !fa_ok(fa_vocab_info(m->vocab.v, &m->vocab.n_tokens, &m->vocab.eos), "fa_vocab_info")) {
    llama_model_free(m);
    return nullptr;
  }
  auto tt = g.kv.find("tokenizer.ggml.token_type");
  if (tt != g.kv.end()) m->vocab.type.assign(tt->second.arr_i.begin(), tt->second.arr_i.end());
  logf(4, "llama_model_load_from_file: " + std::string(path) + ": " + std::to_string(m->cfg.n_layer) + " layers, n_embd " +
              std::to_string(m->cfg.n_embd) + ", vocab " + std::to_string(m->cfg.n_vocab) + " (MI355X engine)");
  return m;
}

void llama_model_free(llama_model* model) {
  if (!model) return;
  if (model->vocab.v) fa_vocab_free(model->vocab.v);
  delete model;
}

const llama_vocab* llama_model_get_vocab(const llama_model* model) { return model ? &model->vocab : nullptr; }
int32_t llama_model_n_embd(const llama_model* model) { return model ? model->cfg.n_embd : 0; }

llama_context_params llama_context_default_params(void) {
  llama_context_params p{};
  p.n_ctx = 512;
  p.n_batch = 2048;
  p.n_ubatch = 512;
  p.n_seq_max = 1;
  p.n_threads = 4;
  p.n_threads_batch = 4;
  p.rope_scaling_type = -1;
  p.pooling_type = -1;
  p.attention_type = -1;
  p.flash_attn_type = -1;
  p.rope_freq_scale = 0.f;
  p.yarn_ext_factor = -1.f;
  p.yarn_attn_factor = 1.f;
  p.yarn_beta_fast = 32.f;
  p.yarn_beta_slow = 1.f;
  p.defrag_thold = -1.f;
  p.type_k = 1;  // GGML_TYPE_F16: the engine's KV cache is fp16
  p.type_v = 1;
  p.offload_kqv = true;
  p.no_perf = true;
  p.op_offload = true;
  p.kv_unified = false;
  return p;
}

llama_context* llama_init_from_model(llama_model* model, llama_context_params params) {
  if (!model) return nullptr;
  if (params.embeddings) {
    logf(2, "llama_init_from_model: embeddings output is not supported (the ASR path reads logits only)");
    return nullptr;
  }
  fa_llm_config lc = model->cfg;
  lc.n_ctx = params.n_ctx > 0 ? (int32_t)params.n_ctx : 2048;
  lc.max_seqs = std::max<int32_t>(1, (int32_t)params.n_seq_max);
  const fa_encoder_config ec = tiny_encoder(lc.n_embd);
  auto* c = new llama_context();
  c->model = model;
  c->n_seq_max = lc.max_seqs;
  c->logits.assign(lc.n_vocab, 0.f);
  // every decoder tensor must come from the file (core/model_manager.py: fail loudly, never a synthetic fallback)
  if (!fa_ok(fa_engine_create(model->device, &ec, &lc, 1, 16000, &c->e), "fa_engine_create") ||
      !fa_ok(fa_weights_mark_unset(c->e, ""), "fa_weights_mark_unset") ||
      !fa_ok(fa_load_gguf(c->e, model->path.c_str()), "fa_load_gguf") || !check_loaded(c->e, model->path)) {
    llama_free(c);
    return nullptr;
  }
  return c;
}

void llama_free(llama_context* ctx) {
  if (!ctx) return;
  if (ctx->e) fa_engine_destroy(ctx->e);
  delete ctx;
}

llama_batch llama_batch_init(int32_t n_tokens, int32_t embd, int32_t n_seq_max) {
  // the allocation scheme of llama.cpp's llama_batch_init (the reference writes into these arrays directly,
  // llama.py:536-570): token or embd rows, pos, n_seq_id, seq_id[n_tokens + 1] (NULL-terminated), logits
  llama_batch b{};
  if (n_tokens <= 0) return b;
  if (embd > 0) b.embd = (float*)calloc((size_t)n_tokens * embd, sizeof(float));
  else b.token = (llama_token*)calloc((size_t)n_tokens, sizeof(llama_token));
  b.pos = (llama_pos*)calloc((size_t)n_tokens, sizeof(llama_pos));
  b.n_seq_id = (int32_t*)calloc((size_t)n_tokens, sizeof(int32_t));
  b.seq_id = (llama_seq_id**)calloc((size_t)n_tokens + 1, sizeof(llama_seq_id*));
  for (int32_t i = 0; i < n_tokens; ++i) b.seq_id[i] = (llama_seq_id*)calloc((size_t)std::max(1, n_seq_max), sizeof(llama_seq_id));
  b.logits = (int8_t*)calloc((size_t)n_tokens, sizeof(int8_t));
  return b;
}

void llama_batch_free(llama_batch batch) {
  free(batch.token);
  free(batch.embd);
  free(batch.pos);
  free(batch.n_seq_id);
  if (batch.seq_id)
    for (int32_t i = 0; batch.seq_id[i]; ++i) free(batch.seq_id[i]);
  free(batch.seq_id);
  free(batch.logits);
}

int32_t llama_decode(llama_context* ctx, llama_batch b) {
  if (!ctx || b.n_tokens <= 0 || (!b.token && !b.embd) || !b.pos) {
    logf(2, "llama_decode: empty batch");
    return -1;
  }
  const int32_t n = b.n_tokens;
  const int32_t seq = b.seq_id && b.seq_id[0] ? b.seq_id[0][0] : 0;
  if (seq < 0 || seq >= ctx->n_seq_max) {
    logf(2, "llama_decode: seq_id out of range");
    return -1;
  }
  int32_t n_past = 0;
  if (!fa_ok(fa_llm_n_past(ctx->e, seq, &n_past), "fa_llm_n_past")) return -1;
  bool want = false;
  for (int32_t i = 0; i < n; ++i) {
    const int32_t s = b.seq_id && b.seq_id[i] ? b.seq_id[i][0] : 0;
    if (s != seq || (b.n_seq_id && b.n_seq_id[i] > 1) || b.pos[i] != n_past + i) {
      logf(2, "llama_decode: a batch must hold one sequence at positions continuing its length (" +
                  std::to_string(n_past) + ")");
      return -1;
    }
    if (b.logits && b.logits[i]) {
      if (i != n - 1) {
        logf(2, "llama_decode: only the batch's last row can output logits");
        return -1;
      }
      want = true;
    }
  }
  if (!b.logits) want = true;  // llama.cpp: a NULL logits array outputs the last row
  ctx->has_logits = false;
  const fa_sampling greedy{0.f, 1.f, 1, 0};
  int32_t tok = 0;
  if (b.embd || n > 1 || n_past == 0) {
    // embedding rows (the reference's audio injection, decoder.py:70-80), or token rows embedded as ggml get_rows
    const int32_t E = ctx->model->cfg.n_embd;
    std::vector<float> rows;
    const float* embd = b.embd;
    if (!embd) {
      rows.resize((size_t)n * E);
      if (!fa_ok(fa_embd_rows(ctx->e, b.token, n, 0, rows.data()), "fa_embd_rows")) return -1;
      embd = rows.data();
    }
    if (!fa_ok(fa_llm_prefill(ctx->e, seq, embd, n, &greedy, &tok, want ? ctx->logits.data() : nullptr),
               "fa_llm_prefill"))
      return -1;
  } else {
    // one token at the next position (decode_token, llama.py:493-498): the engine's decode step with this token as
    // its input
    int32_t out = 0;
    if (!fa_ok(fa_llm_set_token(ctx->e, seq, b.token[0]), "fa_llm_set_token") ||
        !fa_ok(fa_llm_generate(ctx->e, &seq, 1, 1, &greedy, &out), "fa_llm_generate"))
      return -1;
    if (want && !fa_ok(fa_llm_logits(ctx->e, seq, ctx->logits.data()), "fa_llm_logits")) return -1;
  }
  ctx->has_logits = want;
  return 0;
}

float* llama_get_logits(llama_context* ctx) { return ctx && ctx->has_logits ? ctx->logits.data() : nullptr; }

float* llama_get_logits_ith(llama_context* ctx, int32_t i) {
  return ctx && ctx->has_logits && (i == 0 || i == -1) ? ctx->logits.data() : nullptr;
}

float* llama_get_embeddings(llama_context*) { return nullptr; }

int32_t llama_tokenize(const llama_vocab* vocab, const char* text, int32_t text_len, llama_token* tokens,
                       int32_t n_tokens_max, bool /*add_special: qwen2 adds no BOS*/, bool parse_special) {
  if (!vocab || !vocab->v) return INT32_MIN;
  int32_t n = 0;
  const int rc = fa_tokenize(vocab->v, text, text_len, parse_special ? 1 : 0, tokens, n_tokens_max, &n);
  if (rc != FA_OK) return n > n_tokens_max ? -n : INT32_MIN;  // llama.cpp: -(tokens needed) when they do not fit
  return n;
}

int32_t llama_vocab_n_tokens(const llama_vocab* vocab) { return vocab ? vocab->n_tokens : 0; }
llama_token llama_vocab_eos(const llama_vocab* vocab) { return vocab ? vocab->eos : -1; }

int32_t llama_token_to_piece(const llama_vocab* vocab, llama_token token, char* buf, int32_t length, int32_t lstrip,
                             bool special) {
  if (!vocab || !vocab->v || token < 0 || token >= vocab->n_tokens) return 0;
  if (!special && token < (int32_t)vocab->type.size() && vocab->type[token] == 3) return 0;  // control token
  int32_t n = 0;
  fa_token_piece(vocab->v, token, nullptr, 0, &n);
  std::string p((size_t)n, '\0');
  if (n > 0 && !fa_ok(fa_token_piece(vocab->v, token, &p[0], n, &n), "fa_token_piece")) return 0;
  size_t skip = 0;
  while (lstrip > 0 && skip < p.size() && p[skip] == ' ') {
    ++skip;
    --lstrip;
  }
  const int32_t m = (int32_t)(p.size() - skip);
  if (m > length) return -m;
  if (m > 0) std::memcpy(buf, p.data() + skip, (size_t)m);
  return m;
}

llama_memory* llama_get_memory(const llama_context* ctx) { return const_cast<llama_context*>(ctx); }

void llama_memory_clear(llama_memory* mem, bool /*data*/) {
  if (!mem) return;
  for (int32_t s = 0; s < mem->n_seq_max; ++s) fa_ok(fa_llm_reset(mem->e, s), "fa_llm_reset");
  mem->has_logits = false;
}

llama_sampler_chain_params llama_sampler_chain_default_params(void) { return llama_sampler_chain_params{true}; }

llama_sampler* llama_sampler_chain_init(llama_sampler_chain_params) { return new llama_sampler(); }

void llama_sampler_chain_add(llama_sampler* chain, llama_sampler* smpl) {
  if (chain && smpl && chain->kind == llama_sampler::CHAIN) chain->chain.push_back(smpl);
}

llama_sampler* llama_sampler_init_greedy(void) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::GREEDY;
  return s;
}

llama_sampler* llama_sampler_init_dist(uint32_t seed) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::DIST;
  s->rng.seed(seed);
  return s;
}

llama_sampler* llama_sampler_init_temp(float t) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::TEMP;
  s->f = t;
  return s;
}

llama_sampler* llama_sampler_init_top_k(int32_t k) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::TOP_K;
  s->k = k;
  return s;
}

llama_sampler* llama_sampler_init_top_p(float p, size_t min_keep) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::TOP_P;
  s->f = p;
  s->min_keep = std::max<size_t>(1, min_keep);
  return s;
}

llama_sampler* llama_sampler_init_logit_bias(int32_t, int32_t n_logit_bias, const llama_logit_bias* logit_bias) {
  auto* s = new llama_sampler();
  s->kind = llama_sampler::LOGIT_BIAS;
  if (logit_bias && n_logit_bias > 0) s->bias.assign(logit_bias, logit_bias + n_logit_bias);
  return s;
}

llama_token llama_sampler_sample(llama_sampler* smpl, llama_context* ctx, int32_t idx) {
  if (!smpl || !ctx || !ctx->has_logits || (idx != -1 && idx != 0)) {
    logf(2, "llama_sampler_sample: no logits for that output row");
    return -1;
  }
  return sample_row(smpl, ctx->logits.data(), (int32_t)ctx->logits.size());
}

void llama_sampler_free(llama_sampler* smpl) {
  if (!smpl) return;
  for (auto* s : smpl->chain) llama_sampler_free(s);
  delete smpl;
}

llama_token fa_llama_sampler_apply(llama_sampler* smpl, const float* logits, int32_t n_vocab) {
  return smpl && logits && n_vocab > 0 ? sample_row(smpl, logits, n_vocab) : -1;
}

void fa_llama_struct_sizes(size_t* out3) {
  out3[0] = sizeof(llama_model_params);
  out3[1] = sizeof(llama_context_params);
  out3[2] = sizeof(llama_batch);
}

int64_t fa_llama_field_offset(const char* strct, const char* field) {
#define F(S, M) {#S, #M, (int64_t)offsetof(S, M)}
  static const struct {
    const char *s, *f;
    int64_t off;
  } table[] = {
      F(llama_model_params, devices), F(llama_model_params, tensor_buft_overrides), F(llama_model_params, n_gpu_layers),
      F(llama_model_params, split_mode), F(llama_model_params, main_gpu), F(llama_model_params, tensor_split),
      F(llama_model_params, progress_callback), F(llama_model_params, progress_callback_user_data),
      F(llama_model_params, kv_overrides), F(llama_model_params, vocab_only), F(llama_model_params, use_mmap),
      F(llama_model_params, use_direct_io), F(llama_model_params, use_mlock), F(llama_model_params, check_tensors),
      F(llama_model_params, use_extra_bufts), F(llama_model_params, no_host), F(llama_model_params, no_alloc),
      F(llama_context_params, n_ctx), F(llama_context_params, n_batch), F(llama_context_params, n_ubatch),
      F(llama_context_params, n_seq_max), F(llama_context_params, n_threads), F(llama_context_params, n_threads_batch),
      F(llama_context_params, rope_scaling_type), F(llama_context_params, pooling_type),
      F(llama_context_params, attention_type), F(llama_context_params, flash_attn_type),
      F(llama_context_params, rope_freq_base), F(llama_context_params, rope_freq_scale),
      F(llama_context_params, yarn_ext_factor), F(llama_context_params, yarn_attn_factor),
      F(llama_context_params, yarn_beta_fast), F(llama_context_params, yarn_beta_slow),
      F(llama_context_params, yarn_orig_ctx), F(llama_context_params, defrag_thold), F(llama_context_params, cb_eval),
      F(llama_context_params, cb_eval_user_data), F(llama_context_params, type_k), F(llama_context_params, type_v),
      F(llama_context_params, abort_callback), F(llama_context_params, abort_callback_data),
      F(llama_context_params, embeddings), F(llama_context_params, offload_kqv), F(llama_context_params, no_perf),
      F(llama_context_params, op_offload), F(llama_context_params, swa_full), F(llama_context_params, kv_unified),
      F(llama_context_params, samplers), F(llama_context_params, n_samplers), F(llama_sampler_chain_params, no_perf),
      F(llama_logit_bias, token), F(llama_logit_bias, bias), F(llama_batch, n_tokens), F(llama_batch, token),
      F(llama_batch, embd), F(llama_batch, pos), F(llama_batch, n_seq_id), F(llama_batch, seq_id),
      F(llama_batch, logits),
  };
#undef F
  for (const auto& t : table)
    if (!std::strcmp(t.s, strct) && !std::strcmp(t.f, field)) return t.off;
  return -1;
}

}  // extern "C"
