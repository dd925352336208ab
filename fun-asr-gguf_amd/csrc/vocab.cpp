// Native byte-level BPE tokenizer and detokenizer from GGUF metadata: replaces llama_tokenize(add_special=false,
// parse_special=true) and llama_token_to_piece(special=true) that the reference binds for its prompts and its
// streamed output (/root/reference/fun_asr_gguf/llama.py:738-748, prompt_utils.py:44-52, llama.py:671-683).
//
// GGUF keys (convert_hf_to_gguf.py:1283-1291, _set_vocab_gpt2; Qwen3 = tokenizer.ggml.pre "qwen2"):
//   tokenizer.ggml.tokens (byte-level unicode strings), tokenizer.ggml.token_type (1 normal, 3 control,
//   4 user defined), tokenizer.ggml.merges ("a b", rank = index), tokenizer.ggml.eos_token_id.
// Tokenisation: the text is partitioned at control / user-defined token strings (longest first), each other
// fragment is split by the Qwen2 pre-tokenizer regex
//   (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
// (matched by hand, alternatives in order, as a backtracking regex engine would), the pieces' UTF-8 bytes are
// mapped to the GPT-2 byte alphabet and merged by lowest merge rank, leftmost first.
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/funasr_hip.h"
#include "common.h"
#include "gguf.h"
#include "unicode_tables.h"

namespace fa {

namespace {

bool in_ranges(const CpRange* r, int n, uint32_t cp) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) / 2;
    if (cp < r[mid].lo) hi = mid - 1;
    else if (cp > r[mid].hi) lo = mid + 1;
    else return true;
  }
  return false;
}
bool is_letter(uint32_t c) { return in_ranges(kLetterRanges, kLetterRanges_N, c); }
bool is_number(uint32_t c) { return in_ranges(kNumberRanges, kNumberRanges_N, c); }
bool is_space(uint32_t c) {  // Unicode White_Space
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool is_crlf(uint32_t c) { return c == '\r' || c == '\n'; }

// UTF-8 -> code points (+ byte offset of each); invalid bytes become U+FFFD of one byte
void decode_utf8(const std::string& s, std::vector<uint32_t>& cps, std::vector<size_t>& off) {
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp = 0xFFFD;
    size_t n = 1;
    if (c < 0x80) {
      cp = c;
    } else if ((c >> 5) == 6 && i + 1 < s.size()) {
      cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F);
      n = 2;
    } else if ((c >> 4) == 14 && i + 2 < s.size()) {
      cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
      n = 3;
    } else if ((c >> 3) == 30 && i + 3 < s.size()) {
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      n = 4;
    }
    cps.push_back(cp);
    off.push_back(i);
    i += n;
  }
  off.push_back(s.size());
}

std::string encode_utf8(uint32_t cp) {
  std::string o;
  if (cp < 0x80) {
    o += (char)cp;
  } else if (cp < 0x800) {
    o += (char)(0xC0 | (cp >> 6));
    o += (char)(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    o += (char)(0xE0 | (cp >> 12));
    o += (char)(0x80 | ((cp >> 6) & 0x3F));
    o += (char)(0x80 | (cp & 0x3F));
  } else {
    o += (char)(0xF0 | (cp >> 18));
    o += (char)(0x80 | ((cp >> 12) & 0x3F));
    o += (char)(0x80 | ((cp >> 6) & 0x3F));
    o += (char)(0x80 | (cp & 0x3F));
  }
  return o;
}

// Qwen2 pre-tokenizer: [start, end) code-point spans of the pieces
void qwen2_split(const std::vector<uint32_t>& c, std::vector<std::pair<int, int>>& out) {
  const int n = (int)c.size();
  int i = 0;
  auto lower = [](uint32_t x) { return (x >= 'A' && x <= 'Z') ? x + 32 : x; };
  while (i < n) {
    int e = -1;
    // 1. (?i:'s|'t|'re|'ve|'m|'ll|'d)
    if (c[i] == '\'' && i + 1 < n) {
      const uint32_t a = lower(c[i + 1]);
      const uint32_t b = i + 2 < n ? lower(c[i + 2]) : 0;
      if (a == 's' || a == 't' || a == 'm' || a == 'd') e = i + 2;
      else if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) e = i + 3;
    }
    // 2. [^\r\n\p{L}\p{N}]?\p{L}+
    if (e < 0) {
      int j = i;
      if (!is_crlf(c[j]) && !is_letter(c[j]) && !is_number(c[j]) && j + 1 < n && is_letter(c[j + 1])) ++j;
      if (is_letter(c[j])) {
        while (j < n && is_letter(c[j])) ++j;
        e = j;
      }
    }
    // 3. \p{N}
    if (e < 0 && is_number(c[i])) e = i + 1;
    // 4. ' ?[^\s\p{L}\p{N}]+[\r\n]*'
    if (e < 0) {
      int j = i;
      if (c[j] == ' ' && j + 1 < n && !is_space(c[j + 1]) && !is_letter(c[j + 1]) && !is_number(c[j + 1])) ++j;
      if (!is_space(c[j]) && !is_letter(c[j]) && !is_number(c[j])) {
        while (j < n && !is_space(c[j]) && !is_letter(c[j]) && !is_number(c[j])) ++j;
        while (j < n && is_crlf(c[j])) ++j;
        e = j;
      }
    }
    if (e < 0 && is_space(c[i])) {
      int r = i;
      while (r < n && is_space(c[r])) ++r;  // whitespace run [i, r)
      // 5. \s*[\r\n]+ : ends after the run's last CR/LF
      int last_nl = -1;
      for (int j = i; j < r; ++j)
        if (is_crlf(c[j])) last_nl = j;
      if (last_nl >= 0) e = last_nl + 1;
      // 6. \s+(?!\S) : the whole run at the end of text, else the run minus its last char (if that leaves any)
      else if (r == n) e = r;
      else if (r - i >= 2) e = r - 1;
      // 7. \s+
      else e = r;
    }
    if (e < 0) e = i + 1;  // no alternative matched (not reachable for valid input)
    out.push_back({i, e});
    i = e;
  }
}

}  // namespace

struct Vocab {
  std::vector<std::string> tokens;
  std::vector<int> types;
  std::unordered_map<std::string, int> tok2id;
  std::unordered_map<std::string, int> ranks;  // "a b" -> rank
  std::vector<int> specials;                   // control / user-defined ids, longest text first
  int eos = -1;
  std::string b2u[256];                        // byte -> UTF-8 of its GPT-2 byte-alphabet code point
  std::unordered_map<uint32_t, int> u2b;
  mutable std::unordered_map<std::string, std::vector<int>> cache;

  void init_bytes() {
    std::vector<int> bs;
    for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
    for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
    for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
    std::vector<bool> have(256, false);
    for (int b : bs) have[b] = true;
    int extra = 0;
    for (int b = 0; b < 256; ++b) {
      const uint32_t cp = have[b] ? (uint32_t)b : (uint32_t)(256 + extra++);
      b2u[b] = encode_utf8(cp);
      u2b[cp] = b;
    }
  }

  std::vector<int> bpe(const std::string& word) const {  // word in the byte alphabet (UTF-8)
    auto it = cache.find(word);
    if (it != cache.end()) return it->second;
    std::vector<uint32_t> cps;
    std::vector<size_t> off;
    decode_utf8(word, cps, off);
    std::vector<std::string> parts;
    for (size_t k = 0; k + 1 < off.size(); ++k) parts.push_back(word.substr(off[k], off[k + 1] - off[k]));
    while (parts.size() > 1) {
      int best = -1;
      size_t bi = 0;
      for (size_t k = 0; k + 1 < parts.size(); ++k) {
        auto r = ranks.find(parts[k] + " " + parts[k + 1]);
        if (r != ranks.end() && (best < 0 || r->second < best)) {
          best = r->second;
          bi = k;
        }
      }
      if (best < 0) break;
      parts[bi] += parts[bi + 1];
      parts.erase(parts.begin() + bi + 1);
    }
    std::vector<int> ids;
    for (const std::string& p : parts) {
      auto t = tok2id.find(p);
      if (t != tok2id.end()) {
        ids.push_back(t->second);
      } else {  // merge result missing from the vocab: its single symbols
        std::vector<uint32_t> pc;
        std::vector<size_t> po;
        decode_utf8(p, pc, po);
        for (size_t k = 0; k + 1 < po.size(); ++k) {
          auto s = tok2id.find(p.substr(po[k], po[k + 1] - po[k]));
          if (s != tok2id.end()) ids.push_back(s->second);
        }
      }
    }
    cache[word] = ids;
    return ids;
  }

  void encode_plain(const std::string& text, std::vector<int>& out) const {
    std::vector<uint32_t> cps;
    std::vector<size_t> off;
    decode_utf8(text, cps, off);
    std::vector<std::pair<int, int>> pieces;
    qwen2_split(cps, pieces);
    for (const auto& pc : pieces) {
      std::string w;
      for (size_t b = off[pc.first]; b < off[pc.second]; ++b) w += b2u[(unsigned char)text[b]];
      const std::vector<int> ids = bpe(w);
      out.insert(out.end(), ids.begin(), ids.end());
    }
  }

  void tokenize(const std::string& text, bool parse_special, std::vector<int>& out) const {
    if (!parse_special || specials.empty()) {
      encode_plain(text, out);
      return;
    }
    size_t i = 0, frag = 0;
    while (i < text.size()) {
      int hit = -1;
      for (int id : specials) {
        const std::string& s = tokens[id];
        if (!s.empty() && text.compare(i, s.size(), s) == 0) {
          hit = id;
          break;
        }
      }
      if (hit < 0) {
        ++i;
        continue;
      }
      if (i > frag) encode_plain(text.substr(frag, i - frag), out);
      out.push_back(hit);
      i += tokens[hit].size();
      frag = i;
    }
    if (frag < text.size()) encode_plain(text.substr(frag), out);
  }

  std::string piece(int id) const {
    if (id < 0 || id >= (int)tokens.size()) return "";
    const std::string& t = tokens[id];
    if (types[id] == 3 || types[id] == 4) return t;
    std::vector<uint32_t> cps;
    std::vector<size_t> off;
    decode_utf8(t, cps, off);
    std::string o;
    for (uint32_t cp : cps) {
      auto it = u2b.find(cp);
      if (it != u2b.end()) o += (char)it->second;
    }
    return o;
  }
};

}  // namespace fa

struct fa_vocab {
  fa::Vocab v;
};

#define FA_VAPI_BEGIN try {
#define FA_VAPI_END                 \
  }                                 \
  catch (fa::arg_failure&) {        \
    return FA_ERR_ARG;              \
  }                                 \
  catch (std::exception & ex) {     \
    fa::set_error(ex.what());       \
    return FA_ERR_STATE;            \
  }                                 \
  return FA_OK;

extern "C" {

int fa_vocab_load_gguf(const char* path, fa_vocab** out) {
  FA_VAPI_BEGIN
  FA_REQUIRE(path && out, "fa_vocab_load_gguf: args");
  fa::GGUFFile g;
  if (!g.open(path)) {
    fa::set_error(std::string("cannot read GGUF: ") + fa::gguf_error());
    return FA_ERR_IO;
  }
  auto tk = g.kv.find("tokenizer.ggml.tokens");
  FA_REQUIRE(tk != g.kv.end() && !tk->second.arr_s.empty(), "GGUF has no tokenizer.ggml.tokens");
  fa_vocab* h = new fa_vocab();
  fa::Vocab& v = h->v;
  v.tokens = tk->second.arr_s;
  v.types.assign(v.tokens.size(), 1);
  auto ty = g.kv.find("tokenizer.ggml.token_type");
  if (ty != g.kv.end() && ty->second.arr_i.size() == v.tokens.size())
    for (size_t i = 0; i < v.tokens.size(); ++i) v.types[i] = (int)ty->second.arr_i[i];
  auto mg = g.kv.find("tokenizer.ggml.merges");
  if (mg != g.kv.end())
    for (size_t i = 0; i < mg->second.arr_s.size(); ++i) v.ranks.emplace(mg->second.arr_s[i], (int)i);
  auto eo = g.kv.find("tokenizer.ggml.eos_token_id");
  v.eos = eo != g.kv.end() ? (int)eo->second.i : -1;
  for (size_t i = 0; i < v.tokens.size(); ++i) {
    v.tok2id.emplace(v.tokens[i], (int)i);
    if (v.types[i] == 3 || v.types[i] == 4) v.specials.push_back((int)i);
  }
  std::stable_sort(v.specials.begin(), v.specials.end(),
                   [&](int a, int b) { return v.tokens[a].size() > v.tokens[b].size(); });
  v.init_bytes();
  *out = h;
  FA_VAPI_END
}

int fa_vocab_free(fa_vocab* v) {
  delete v;
  return FA_OK;
}

int fa_vocab_info(const fa_vocab* v, int32_t* n_tokens, int32_t* eos) {
  FA_VAPI_BEGIN
  FA_REQUIRE(v, "fa_vocab_info: null vocab");
  if (n_tokens) *n_tokens = (int32_t)v->v.tokens.size();
  if (eos) *eos = v->v.eos;
  FA_VAPI_END
}

int fa_tokenize(const fa_vocab* v, const char* text, int32_t n_bytes, int32_t parse_special, int32_t* out, int32_t cap,
                int32_t* n_out) {
  FA_VAPI_BEGIN
  FA_REQUIRE(v && (text || n_bytes == 0) && n_bytes >= 0 && n_out, "fa_tokenize: args");
  std::vector<int> ids;
  v->v.tokenize(std::string(text ? text : "", (size_t)n_bytes), parse_special != 0, ids);
  *n_out = (int32_t)ids.size();
  FA_REQUIRE((int32_t)ids.size() <= cap && (out || ids.empty()), "fa_tokenize: output capacity (see *n_out)");
  std::copy(ids.begin(), ids.end(), out);
  FA_VAPI_END
}

int fa_token_piece(const fa_vocab* v, int32_t id, char* buf, int32_t cap, int32_t* n_out) {
  FA_VAPI_BEGIN
  FA_REQUIRE(v && n_out, "fa_token_piece: args");
  const std::string p = v->v.piece(id);
  *n_out = (int32_t)p.size();
  FA_REQUIRE((int32_t)p.size() <= cap && (buf || p.empty()), "fa_token_piece: buffer capacity (see *n_out)");
  std::memcpy(buf, p.data(), p.size());
  FA_VAPI_END
}

// Dequantised GGUF tensor (q8_0 / f16 / f32) -> f32. fp16_product = 1 reproduces get_token_embeddings_gguf's numpy
// f16 product (llama.py:778-784): fp16(f16(d) * q); 0 = ggml dequantize_row_q8_0 (f32(d) * q).
int fa_gguf_read_tensor(const char* path, const char* name, int32_t fp16_product, float* out, int64_t n) {
  FA_VAPI_BEGIN
  FA_REQUIRE(path && name && out, "fa_gguf_read_tensor: args");
  fa::GGUFFile g;
  if (!g.open(path)) {
    fa::set_error(std::string("cannot read GGUF: ") + fa::gguf_error());
    return FA_ERR_IO;
  }
  const fa::GGUFTensor* t = nullptr;
  for (const auto& x : g.tensors)
    if (x.name == name) t = &x;
  if (!t) {
    fa::set_error(std::string("GGUF has no tensor ") + name);
    return FA_ERR_NOTFOUND;
  }
  FA_REQUIRE(n == t->n_elements, "fa_gguf_read_tensor: element count");
  const uint8_t* p = g.data(*t);
  if (t->type == fa::GGML_F32) {
    std::memcpy(out, p, (size_t)n * 4);
  } else if (t->type == fa::GGML_F16) {
    for (int64_t i = 0; i < n; ++i) {
      uint16_t h;
      std::memcpy(&h, p + 2 * i, 2);
      out[i] = fa::half_to_float_host(h);
    }
  } else if (t->type == fa::GGML_Q8_0) {
    for (int64_t b = 0; b < n / 32; ++b) {
      uint16_t dh;
      std::memcpy(&dh, p + 34 * b, 2);
      const float d = fa::half_to_float_host(dh);
      const int8_t* q = (const int8_t*)(p + 34 * b + 2);
      for (int j = 0; j < 32; ++j) {
        const float v = d * (float)q[j];
        out[32 * b + j] = fp16_product ? fa::half_to_float_host(fa::float_to_half_host(v)) : v;
      }
    }
  } else {
    FA_REQUIRE(false, std::string("fa_gguf_read_tensor: unsupported tensor type for ") + name);
  }
  FA_VAPI_END
}

}  // extern "C"
