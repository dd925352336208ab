"""Tokenizer parity (A10 / §8(f) row 3): the product's native GGUF tokenizer (fa_tokenize / fa_token_piece,
csrc/vocab.cpp) and the Python restatement (oracle/bpe.py) against HuggingFace `tokenizers` on a synthetic
Qwen2-style byte-level BPE written to GGUF by the reference's vendored GGUFWriter
(tests/golden/make_tokenizer_golden.py). llama.cpp's own llama_tokenize (llama.py:738-743) is absent here, so
`tokenizers` — the library Qwen's tokenizer.json runs on — is the anchor. Exact ids / bytes; no GPU needed.
"""
import json
import os

import pytest

from conftest import GOLDEN

GGUF = os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf")
G = json.load(open(os.path.join(GOLDEN, "tokenizer_golden.json")))


@pytest.fixture(scope="module")
def native():
    from fun_asr_gguf.vocab import GGUFVocab
    return GGUFVocab(GGUF)


@pytest.fixture(scope="module")
def pyref():
    from oracle.bpe import BPEVocab
    return BPEVocab(GGUF)


@pytest.mark.parametrize("i", range(len(G["cases"])))
def test_tokenize_matches_hf_tokenizers(native, pyref, i):
    c = G["cases"][i]
    assert native.tokenize(c["text"]) == c["ids"], repr(c["text"])
    assert pyref.tokenize(c["text"]) == c["ids"], repr(c["text"])


def test_token_pieces_and_roundtrip(native, pyref):
    assert native.n_vocab == G["n_vocab"] and native.eos == G["eos"]
    for tid, b in G["pieces"].items():
        assert native.token_to_bytes(int(tid)) == bytes(b)
        assert pyref.token_to_bytes(int(tid)) == bytes(b)
    for c in G["cases"]:  # detokenisation = concatenated pieces (special tokens render as their text)
        assert b"".join(native.token_to_bytes(t) for t in c["ids"]).decode("utf-8") == c["text"]
    assert native.token_to_bytes(-1) == b"" and native.token_to_bytes(10 ** 6) == b""


def test_parse_special_off_tokenizes_marker_text(native, pyref):
    t = "<|im_end|>"
    assert native.tokenize(t, parse_special=False) == pyref.tokenize(t, parse_special=False)
    assert G["specials"]["<|im_end|>"] not in native.tokenize(t, parse_special=False)
    assert native.tokenize(t) == [G["specials"]["<|im_end|>"]]


def test_gguf_tensor_reader_vs_reference_embedding_golden():
    """fa_gguf_read_tensor on the tiny GGUF the reference's GGUFWriter wrote (tests/golden/q8_0.npz tiny_gguf) against
    the reference's own get_token_embeddings_gguf output (numpy f16 product, llama.py:778-784)."""
    import tempfile

    import numpy as np

    from fun_asr_gguf._native import gguf_read_tensor
    z = np.load(os.path.join(GOLDEN, "q8_0.npz"))
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "tiny.gguf")
        z["tiny_gguf"].tofile(p)
        got = gguf_read_tensor(p, "token_embd.weight", z["emb_table"].size, fp16_product=True)
        assert (got.reshape(z["emb_table"].shape) == z["emb_table"]).all()
        f32 = gguf_read_tensor(p, "token_embd.weight", z["emb_table"].size, fp16_product=False)
        assert np.abs(f32.reshape(z["emb_table"].shape) - z["emb_table"]).max() <= 2e-3 * np.abs(z["emb_table"]).max()
