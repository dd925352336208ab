"""Decoder vocabularies: the llama_tokenize / llama_token_to_piece surface the reference binds
(llama.py:738-748 text_to_tokens(add_special=False, parse_special=True), token_to_bytes(special=True);
ASRStreamDecoder incremental UTF-8 decode llama.py:661-690).

GGUFVocab   byte-level BPE from GGUF metadata (tokenizer.ggml.tokens/merges/token_type, the layout
            convert_hf_to_gguf.py writes for Qwen, :1283-1291) with the Qwen2 pre-tokenizer split, run by the
            native tokenizer (csrc/vocab.cpp).
SyntheticVocab  deterministic stand-in used with synthetic weights (no tokenizer ships in the reference):
            one token per character, Qwen special-token strings mapped to the top ids.
"""
import struct


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
    """The GGUF's tokenizer, run natively (fa_tokenize / fa_token_piece in libfunasr_hip.so): the llama_tokenize /
    llama_token_to_piece surface of the reference. The pure-Python restatement is oracle/bpe.py (test only)."""

    def __init__(self, path):
        from ._native import Vocab
        self._v = Vocab(path)
        self.n_vocab = self._v.n_vocab
        self.eos = self._v.eos

    def tokenize(self, text, parse_special=True):
        return self._v.tokenize(text, parse_special)

    def token_to_bytes(self, tid):
        return self._v.token_to_bytes(tid)


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
