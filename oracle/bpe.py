"""Byte-level BPE tokenizer restatement (pure Python) — TEST INFRASTRUCTURE ONLY.

Restates what llama.cpp b7798 does for the reference's llama_tokenize(add_special=False, parse_special=True) and
llama_token_to_piece(special=True) (/root/reference/fun_asr_gguf/llama.py:738-748) on a GGUF vocabulary with
tokenizer.ggml.pre = "qwen2" (convert_hf_to_gguf.py:1283-1291): control / user-defined tokens are split out of the
text first (longest first), every other fragment is cut by the Qwen2 pre-tokenizer regex, its UTF-8 bytes are
mapped to the GPT-2 byte alphabet and merged by lowest merge rank (leftmost on ties). llama.cpp itself is absent
(SURVEY §8(c)); this restatement and the product's native tokenizer (csrc/vocab.cpp) are both pinned against
HuggingFace `tokenizers` (third party, the tokenizer Qwen ships) in tests/test_tokenizer.py.
"""
import regex

from fun_asr_gguf.vocab import read_gguf_metadata

QWEN2_PRETOKENIZE = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                     r"|\s*[\r\n]+|\s+(?!\S)|\s+")
TOKEN_TYPE_NORMAL, TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED = 1, 3, 4


def bytes_to_unicode():
    """GPT-2 byte <-> printable-unicode table used by byte-level BPE vocabularies."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class BPEVocab:
    def __init__(self, path=None, kv=None):
        kv = kv if kv is not None else read_gguf_metadata(path)
        self.tokens = kv["tokenizer.ggml.tokens"]
        self.types = kv.get("tokenizer.ggml.token_type", [TOKEN_TYPE_NORMAL] * len(self.tokens))
        self.ranks = {tuple(m.split(" ", 1)): i for i, m in enumerate(kv.get("tokenizer.ggml.merges", []))}
        self.tok2id = {t: i for i, t in enumerate(self.tokens)}
        self.eos = int(kv.get("tokenizer.ggml.eos_token_id", -1))
        self.b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in self.b2u.items()}
        self.special = sorted((t for t, ty in zip(self.tokens, self.types)
                               if ty in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED)), key=len, reverse=True)
        self._pat = regex.compile(QWEN2_PRETOKENIZE)

    def _bpe(self, word):
        parts = list(word)
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        ids = []
        for p in parts:
            if p in self.tok2id:
                ids.append(self.tok2id[p])
            else:
                ids.extend(self.tok2id[c] for c in p if c in self.tok2id)
        return ids

    def _encode_plain(self, text):
        out = []
        for w in self._pat.findall(text):
            out.extend(self._bpe("".join(self.b2u[b] for b in w.encode("utf-8"))))
        return out

    def tokenize(self, text, parse_special=True):
        if not parse_special or not self.special:
            return self._encode_plain(text)
        out, i, frag = [], 0, 0
        while i < len(text):
            hit = next((s for s in self.special if text.startswith(s, i)), None)
            if hit is None:
                i += 1
                continue
            if i > frag:
                out.extend(self._encode_plain(text[frag:i]))
            out.append(self.tok2id[hit])
            i += len(hit)
            frag = i
        if frag < len(text):
            out.extend(self._encode_plain(text[frag:]))
        return out

    def token_to_bytes(self, tid):
        if tid < 0 or tid >= len(self.tokens):
            return b""
        t = self.tokens[tid]
        if self.types[tid] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED):
            return t.encode("utf-8")
        return bytes(self.u2b[c] for c in t if c in self.u2b)
