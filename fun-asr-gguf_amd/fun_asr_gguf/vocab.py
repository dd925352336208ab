"""Decoder vocabularies: the llama_tokenize / llama_token_to_piece surface the reference binds
(llama.py:738-748 text_to_tokens(add_special=False, parse_special=True), token_to_bytes(special=True);
ASRStreamDecoder incremental UTF-8 decode llama.py:661-690).

GGUFVocab   byte-level BPE read from GGUF metadata (tokenizer.ggml.tokens/merges/token_type, the
            layout convert_hf_to_gguf.py writes for Qwen, :1283-1291) with the Qwen2 pre-tokenizer split.
SyntheticVocab  deterministic stand-in used with synthetic weights (no tokenizer ships in the reference):
            one token per character, Qwen special-token strings mapped to the top ids.
"""
import struct

try:
    import regex as _re
except ImportError:  # pragma: no cover
    _re = None

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


def read_gguf_metadata(path):
    """Metadata KV of a GGUF v2/v3 file (tensor data is read by the native loader)."""
    def rd(f, fmt):
        return struct.unpack("<" + fmt, f.read(struct.calcsize("<" + fmt)))[0]

    def rs(f):
        return f.read(rd(f, "Q")).decode("utf-8", errors="replace")

    scal = {0: "B", 1: "b", 2: "H", 3: "h", 4: "I", 5: "i", 6: "f", 7: "?", 10: "Q", 11: "q", 12: "d"}

    def rv(f, t):
        if t == 8:
            return rs(f)
        if t == 9:
            at, n = rd(f, "I"), rd(f, "Q")
            return [rv(f, at) for _ in range(n)]
        return rd(f, scal[t])

    kv = {}
    with open(path, "rb") as f:
        if f.read(4) != b"GGUF":
            raise ValueError("not a GGUF file")
        rd(f, "I")
        rd(f, "Q")
        n_kv = rd(f, "Q")
        for _ in range(n_kv):
            k = rs(f)
            kv[k] = rv(f, rd(f, "I"))
    return kv


class GGUFVocab:
    def __init__(self, path=None, kv=None):
        kv = kv if kv is not None else read_gguf_metadata(path)
        self.tokens = kv["tokenizer.ggml.tokens"]
        self.types = kv.get("tokenizer.ggml.token_type", [TOKEN_TYPE_NORMAL] * len(self.tokens))
        merges = kv.get("tokenizer.ggml.merges", [])
        self.ranks = {tuple(m.split(" ", 1)): i for i, m in enumerate(merges)}
        self.tok2id = {t: i for i, t in enumerate(self.tokens)}
        self.eos = int(kv.get("tokenizer.ggml.eos_token_id", -1))
        self.n_vocab = len(self.tokens)
        self.b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in self.b2u.items()}
        self.special = sorted((t for t, ty in zip(self.tokens, self.types)
                               if ty in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED)), key=len, reverse=True)
        self._pat = _re.compile(QWEN2_PRETOKENIZE) if _re is not None else None
        self._cache = {}

    def _bpe(self, word):
        if word in self._cache:
            return self._cache[word]
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
            else:  # unknown merge result: fall back to single byte symbols
                ids.extend(self.tok2id[c] for c in p if c in self.tok2id)
        self._cache[word] = ids
        return ids

    def _encode_plain(self, text):
        if self._pat is None:
            raise RuntimeError("the 'regex' module is required for BPE pre-tokenisation")
        out = []
        for w in self._pat.findall(text):
            out.extend(self._bpe("".join(self.b2u[b] for b in w.encode("utf-8"))))
        return out

    def tokenize(self, text, parse_special=True):
        if not parse_special or not self.special:
            return self._encode_plain(text)
        out, i = [], 0
        while i < len(text):
            hit = None
            for s in self.special:
                if text.startswith(s, i):
                    hit = s
                    break
            if hit is not None:
                out.append(self.tok2id[hit])
                i += len(hit)
                continue
            j = i + 1
            while j < len(text) and not any(text.startswith(s, j) for s in self.special):
                j += 1
            out.extend(self._encode_plain(text[i:j]))
            i = j
        return out

    def token_to_bytes(self, tid):
        if tid < 0 or tid >= self.n_vocab:
            return b""
        t = self.tokens[tid]
        if self.types[tid] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED):
            return t.encode("utf-8")
        return bytes(self.u2b[c] for c in t if c in self.u2b)


class SyntheticVocab:
    """Character-level stand-in vocabulary for synthetic-weight runs."""
    SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]

    def __init__(self, n_vocab):
        self.n_vocab = n_vocab
        self.special_ids = {s: n_vocab - 3 + i for i, s in enumerate(self.SPECIALS)}
        self.eos = self.special_ids["<|endoftext|>"]
        self.span = n_vocab - 3

    def tokenize(self, text, parse_special=True):
        out, i = [], 0
        while i < len(text):
            hit = next((s for s in self.SPECIALS if parse_special and text.startswith(s, i)), None)
            if hit:
                out.append(self.special_ids[hit])
                i += len(hit)
            else:
                out.append((ord(text[i]) * 2654435761) % self.span)
                i += 1
        return out

    def token_to_bytes(self, tid):
        for s, i in self.special_ids.items():
            if tid == i:
                return s.encode()
        return chr(0x4E00 + tid % 20000).encode("utf-8")


class CTCSyntheticTokens(dict):
    """id -> text for the synthetic CTC head (blank = max id, as tokens.txt's last line `<blk>`)."""

    def __init__(self, n):
        super().__init__({i: chr(0x4E00 + (i * 7) % 20000) for i in range(n - 1)})
        self[n - 1] = "<blk>"
