"""CPU checks of the llama.cpp-compatible library set (include/llama_compat.h, lib/llama_compat/): the reference binds
llama.cpp b7798 through ctypes (fun_asr_gguf/llama.py:150-349), so a drop-in must export every symbol it binds with the
struct layouts it declares (llama.py:27-104), both pinned by tests/golden/llama_abi.json (make_llama_abi_golden.py,
generated from the reference's own module). Model loading, the tokenizer and the sampler chain run without a GPU; the
decode path is tests/test_gpu_llama_compat.py. When /root/reference is present, the reference's own llama.py drives
the library in a subprocess (LlamaModel, text_to_tokens, token_to_bytes)."""
import ctypes
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

COMPAT = os.path.join(ROOT, "fun-asr-gguf_amd", "lib", "llama_compat")
ABI = json.load(open(os.path.join(GOLDEN, "llama_abi.json")))
TOK = json.load(open(os.path.join(GOLDEN, "tokenizer_golden.json")))
REF = "/root/reference/fun_asr_gguf"


def load_libs():
    for name in ("libggml-base.so", "libggml.so"):
        ctypes.CDLL(os.path.join(COMPAT, name))
    lib = ctypes.CDLL(os.path.join(COMPAT, "libllama.so"))
    lib.llama_model_load_from_file.restype = ctypes.c_void_p
    lib.llama_model_get_vocab.restype = ctypes.c_void_p
    lib.llama_model_get_vocab.argtypes = [ctypes.c_void_p]
    lib.llama_model_n_embd.argtypes = [ctypes.c_void_p]
    lib.llama_model_free.argtypes = [ctypes.c_void_p]
    lib.llama_vocab_n_tokens.argtypes = [ctypes.c_void_p]
    lib.llama_vocab_eos.argtypes = [ctypes.c_void_p]
    lib.llama_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                   ctypes.c_int32, ctypes.c_bool, ctypes.c_bool]
    lib.llama_token_to_piece.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_bool]
    for f in ("llama_sampler_chain_init", "llama_sampler_init_greedy", "llama_sampler_init_dist",
              "llama_sampler_init_temp", "llama_sampler_init_top_k", "llama_sampler_init_top_p",
              "llama_sampler_init_logit_bias"):
        getattr(lib, f).restype = ctypes.c_void_p
    lib.llama_sampler_init_dist.argtypes = [ctypes.c_uint32]
    lib.llama_sampler_init_temp.argtypes = [ctypes.c_float]
    lib.llama_sampler_init_top_k.argtypes = [ctypes.c_int32]
    lib.llama_sampler_init_top_p.argtypes = [ctypes.c_float, ctypes.c_size_t]
    lib.llama_sampler_init_logit_bias.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    lib.llama_sampler_chain_init.argtypes = [ctypes.c_bool]
    lib.llama_sampler_chain_add.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.llama_sampler_free.argtypes = [ctypes.c_void_p]
    lib.fa_llama_sampler_apply.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    lib.fa_llama_field_offset.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.fa_llama_field_offset.restype = ctypes.c_int64
    return lib


def abi_struct(name):
    """A ctypes Structure with the byte layout the reference declares for `name` (field widths from the golden). The
    structs travel by value and are larger than 16 bytes, so they are passed in memory: only the layout matters."""
    by = {1: ctypes.c_uint8, 4: ctypes.c_uint32, 8: ctypes.c_uint64}
    st = ABI["structs"][name]
    cls = type(name, (ctypes.Structure,), {"_fields_": [(f, by[sz]) for f, _, sz in st["fields"]]})
    assert ctypes.sizeof(cls) == st["size"] and all(getattr(cls, f).offset == o for f, o, _ in st["fields"])
    return cls


def tiny_model_gguf(path, n_embd=64, n_ff=128):
    """Tokenizer metadata of tests/golden/tokenizer_qwen2_synth.gguf plus the qwen3 dimension keys and the two tensors
    whose shapes llama_model_load_from_file reads (weights are only uploaded at context creation)."""
    from fun_asr_gguf.vocab import read_gguf_metadata
    from gguf_io import GGML_F32, write_gguf
    kv = {k: v for k, v in read_gguf_metadata(os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf")).items()
          if k.startswith("tokenizer.")}
    kv.update({"qwen3.block_count": 2, "qwen3.embedding_length": n_embd, "qwen3.attention.head_count": 4,
               "qwen3.attention.head_count_kv": 2})
    n_vocab = len(kv["tokenizer.ggml.tokens"])
    write_gguf(str(path), kv, [("token_embd.weight", np.zeros((n_vocab, n_embd), np.float32), GGML_F32),
                               ("blk.0.ffn_gate.weight", np.zeros((n_ff, n_embd), np.float32), GGML_F32)])
    return n_vocab


def test_exports_every_symbol_the_reference_binds():
    load_libs()
    for lib, names in ABI["symbols"].items():
        h = ctypes.CDLL(os.path.join(COMPAT, lib))
        missing = [n for n in names if not hasattr(h, n)]
        assert not missing, (lib, missing)
    hdr = open(os.path.join(ROOT, "include", "llama_compat.h")).read()
    declared = set(re.findall(r"\b((?:llama|fa_llama)_[a-z0-9_]+)\s*\(", hdr))
    h = ctypes.CDLL(os.path.join(COMPAT, "libllama.so"))
    assert not [n for n in declared if not hasattr(h, n)]
    assert set(ABI["symbols"]["libllama.so"]) <= declared


def test_struct_layouts_match_the_reference_ctypes_declarations():
    lib = load_libs()
    sizes = (ctypes.c_size_t * 3)()
    lib.fa_llama_struct_sizes(sizes)
    assert list(sizes) == [ABI["structs"][n]["size"] for n in ("llama_model_params", "llama_context_params",
                                                               "llama_batch")]
    for sname, st in ABI["structs"].items():
        for field, off, _ in st["fields"]:
            assert lib.fa_llama_field_offset(sname.encode(), field.encode()) == off, (sname, field)


def test_model_metadata_tokenizer_and_pieces(tmp_path):
    lib = load_libs()
    p = tmp_path / "m.gguf"
    n_vocab = tiny_model_gguf(p)
    mp = abi_struct("llama_model_params")
    lib.llama_model_default_params.restype = mp
    lib.llama_model_load_from_file.argtypes = [ctypes.c_char_p, mp]
    m = lib.llama_model_load_from_file(str(p).encode(), lib.llama_model_default_params())
    assert m
    try:
        v = lib.llama_model_get_vocab(m)
        assert lib.llama_model_n_embd(m) == 64
        assert lib.llama_vocab_n_tokens(v) == n_vocab == TOK["n_vocab"]
        assert lib.llama_vocab_eos(v) == TOK["eos"]
        for case in TOK["cases"]:
            b = case["text"].encode("utf-8")
            buf = (ctypes.c_int32 * (len(b) + 32))()
            n = lib.llama_tokenize(v, b, len(b), buf, len(buf), False, True)
            assert list(buf[:n]) == case["ids"], case["text"]
            if n > 1:  # too small a buffer: minus the tokens needed (llama.cpp contract)
                assert lib.llama_tokenize(v, b, len(b), buf, 1, False, True) == -n
            out = b""
            for t in case["ids"]:
                pb = ctypes.create_string_buffer(256)
                k = lib.llama_token_to_piece(v, t, pb, 256, 0, True)
                out += pb.raw[:k]
            assert out == b, case["text"]
        pb = ctypes.create_string_buffer(1)
        ids = TOK["cases"][1]["ids"]
        long_tok = max(ids, key=lambda t: len(TOK["pieces"][str(t)]) if "pieces" in TOK and str(t) in TOK["pieces"] else 0)
        k = lib.llama_token_to_piece(v, long_tok, pb, 0, 0, True)
        assert k <= 0
    finally:
        lib.llama_model_free(m)


def test_tokenizer_edge_cases(tmp_path):
    """llama.cpp's contracts at the edges: empty text -> 0 tokens; control tokens render only with special = true
    (tokenizer.ggml.token_type 3), lstrip drops leading spaces, out-of-range ids give 0 bytes."""
    lib = load_libs()
    p = tmp_path / "m.gguf"
    tiny_model_gguf(p)
    mp = abi_struct("llama_model_params")
    lib.llama_model_default_params.restype = mp
    lib.llama_model_load_from_file.argtypes = [ctypes.c_char_p, mp]
    m = lib.llama_model_load_from_file(str(p).encode(), lib.llama_model_default_params())
    try:
        v = lib.llama_model_get_vocab(m)
        buf = (ctypes.c_int32 * 8)()
        assert lib.llama_tokenize(v, b"", 0, buf, 8, False, True) == 0
        pb = ctypes.create_string_buffer(64)
        im_start = TOK["specials"]["<|im_start|>"]
        k = lib.llama_token_to_piece(v, im_start, pb, 64, 0, True)
        assert pb.raw[:k] == b"<|im_start|>"
        assert lib.llama_token_to_piece(v, im_start, pb, 64, 0, False) == 0
        sp = [c["ids"] for c in TOK["cases"] if c["text"].startswith(" ")]
        if sp:  # a piece with a leading space loses it under lstrip
            t = sp[0][0]
            k = lib.llama_token_to_piece(v, t, pb, 64, 0, True)
            full = pb.raw[:k]
            if full.startswith(b" "):
                k = lib.llama_token_to_piece(v, t, pb, 64, 1, True)
                assert pb.raw[:k] == full[1:]
        assert lib.llama_token_to_piece(v, 10 ** 6, pb, 64, 0, True) == 0
    finally:
        lib.llama_model_free(m)


def test_missing_model_file_returns_null(tmp_path):
    lib = load_libs()
    mp = abi_struct("llama_model_params")
    lib.llama_model_default_params.restype = mp
    lib.llama_model_load_from_file.argtypes = [ctypes.c_char_p, mp]
    assert not lib.llama_model_load_from_file(str(tmp_path / "absent.gguf").encode(), lib.llama_model_default_params())


def _chain(lib, *stages):
    c = lib.llama_sampler_chain_init(True)
    for s in stages:
        lib.llama_sampler_chain_add(c, s)
    return c


def test_sampler_chain():
    lib = load_libs()
    rng = np.random.default_rng(0)
    logits = (rng.standard_normal(151936) * 3).astype(np.float32)
    ptr = logits.ctypes.data
    greedy = _chain(lib, lib.llama_sampler_init_greedy())
    assert lib.fa_llama_sampler_apply(greedy, ptr, logits.size) == int(np.argmax(logits))
    tied = np.zeros(10, np.float32)
    tied[[3, 7]] = 1.0
    assert lib.fa_llama_sampler_apply(greedy, tied.ctypes.data, 10) == 3  # first maximum
    lib.llama_sampler_free(greedy)
    # LlamaSampler(temperature > 0): top_k -> top_p -> temp -> dist (llama.py:599-603)
    top = set(np.argsort(-logits)[:50].tolist())
    draws = []
    for seed in range(200):
        c = _chain(lib, lib.llama_sampler_init_top_k(50), lib.llama_sampler_init_top_p(1.0, 1),
                   lib.llama_sampler_init_temp(0.4), lib.llama_sampler_init_dist(seed))
        draws.append(lib.fa_llama_sampler_apply(c, ptr, logits.size))
        lib.llama_sampler_free(c)
    assert set(draws) <= top and len(set(draws)) > 1
    # top_k 1 and temperature 0 are greedy; top_p keeps the smallest prefix reaching p
    for stages in ((lib.llama_sampler_init_top_k(1), lib.llama_sampler_init_dist(1)),
                   (lib.llama_sampler_init_temp(0.0), lib.llama_sampler_init_dist(2))):
        c = _chain(lib, *stages)
        assert lib.fa_llama_sampler_apply(c, ptr, logits.size) == int(np.argmax(logits))
        lib.llama_sampler_free(c)
    peaked = np.full(100, -10.0, np.float32)
    peaked[42] = 10.0
    c = _chain(lib, lib.llama_sampler_init_top_p(0.5, 1), lib.llama_sampler_init_dist(3))
    assert lib.fa_llama_sampler_apply(c, peaked.ctypes.data, 100) == 42
    lib.llama_sampler_free(c)
    # logit bias (the reference's optional first stage, llama.py:588-597)
    bias = np.zeros(2, dtype=[("token", np.int32), ("bias", np.float32)])
    bias[0] = (5, 1e4)
    c = _chain(lib, lib.llama_sampler_init_logit_bias(logits.size, 1, bias.ctypes.data), lib.llama_sampler_init_greedy())
    assert lib.fa_llama_sampler_apply(c, ptr, logits.size) == 5
    lib.llama_sampler_free(c)


def test_batch_init_free_and_context_without_gpu(tmp_path):
    lib = load_libs()

    class Batch(ctypes.Structure):
        _fields_ = [("n_tokens", ctypes.c_int32), ("token", ctypes.POINTER(ctypes.c_int32)),
                    ("embd", ctypes.POINTER(ctypes.c_float)), ("pos", ctypes.POINTER(ctypes.c_int32)),
                    ("n_seq_id", ctypes.POINTER(ctypes.c_int32)),
                    ("seq_id", ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))), ("logits", ctypes.POINTER(ctypes.c_int8))]
    lib.llama_batch_init.restype = Batch
    lib.llama_batch_free.argtypes = [Batch]
    for n, e in ((204, 1024), (1, 0)):
        b = lib.llama_batch_init(n, e, 1)
        assert bool(b.embd) == (e > 0) and bool(b.token) == (e == 0)
        for i in range(n):
            b.pos[i] = i
            b.seq_id[i][0] = 0
        assert not b.seq_id[n]  # NULL-terminated, as llama.cpp's
        lib.llama_batch_free(b)
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: the context path is tests/test_gpu_llama_compat.py")
    except Exception:
        pass
    p = tmp_path / "m.gguf"
    tiny_model_gguf(p)
    mp, cp = abi_struct("llama_model_params"), abi_struct("llama_context_params")
    lib.llama_model_default_params.restype = mp
    lib.llama_model_load_from_file.argtypes = [ctypes.c_char_p, mp]
    lib.llama_context_default_params.restype = cp
    lib.llama_init_from_model.restype = ctypes.c_void_p
    lib.llama_init_from_model.argtypes = [ctypes.c_void_p, cp]
    m = lib.llama_model_load_from_file(str(p).encode(), lib.llama_model_default_params())
    assert not lib.llama_init_from_model(m, lib.llama_context_default_params())  # no device: NULL, logged
    lib.llama_model_free(m)


_REF_SCRIPT = r'''
import importlib.util, logging, os, sys, types
ref, fake_dir, model, cases = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
import json
pkg = types.ModuleType("fun_asr_gguf_ref"); pkg.__path__ = [ref]; pkg.logger = logging.getLogger("ref")
sys.modules["fun_asr_gguf_ref"] = pkg
sys.path.append(ref)  # the reference's vendored gguf-py
spec = importlib.util.spec_from_file_location("fun_asr_gguf_ref.llama", os.path.join(ref, "llama.py"))
m = importlib.util.module_from_spec(spec)
m.__file__ = os.path.join(fake_dir, "llama.py")  # its bin/ = our library set
sys.modules[spec.name] = m
spec.loader.exec_module(m)
lm = m.LlamaModel(model)
out = {"n_embd": lm.n_embd, "eos": lm.eos_token, "ids": [], "text": []}
for c in json.load(open(cases))["cases"]:
    ids = m.text_to_tokens(lm.vocab, c["text"])
    out["ids"].append(ids)
    out["text"].append(lm.detokenize(ids))
print("RESULT " + json.dumps(out))
'''


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is only present in the build container")
def test_reference_llama_py_drives_the_library(tmp_path):
    """The reference's unmodified llama.py (init_llama_lib binds all 34 symbols, LlamaModel loads through
    llama_model_load_from_file, text_to_tokens / token_to_bytes) against lib/llama_compat/ standing in its bin/."""
    fake = tmp_path / "fun_asr_gguf"
    (fake / "bin").mkdir(parents=True)
    for name in ("libllama.so", "libggml.so", "libggml-base.so"):
        os.symlink(os.path.join(COMPAT, name), fake / "bin" / name)
    os.symlink(os.path.join(COMPAT, "..", "libfunasr_hip.so"), fake / "bin" / "libfunasr_hip.so")  # libllama's DT_NEEDED
    p = tmp_path / "m.gguf"
    tiny_model_gguf(p)
    r = subprocess.run([sys.executable, "-c", _REF_SCRIPT, REF, str(fake), str(p),
                        os.path.join(GOLDEN, "tokenizer_golden.json")], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert r.returncode == 0 and line, r.stderr[-3000:]
    out = json.loads(line[0][7:])
    assert out["n_embd"] == 64 and out["eos"] == TOK["eos"]
    assert out["ids"] == [c["ids"] for c in TOK["cases"]]
    assert out["text"] == [c["text"] for c in TOK["cases"]]
