"""The llama.cpp-compatible library (include/llama_compat.h) on the GPU: the call sequence of the reference's
LLMDecoder.decode (core/decoder.py:55-123 through llama.py's classes: memory clear, an embedding batch with logits on its
last row, then sample -> one-token batch at the next position, greedy) driven through ctypes declarations of the b7798
ABI, against the engine's own prefill + generate on the same GGUF. The reference module itself cannot travel to the
GPU box; tests/test_llama_compat.py runs it against the library in the build container."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from gguf_io import GGML_F32, GGML_Q8_0, write_gguf
from oracle import synth

pytestmark = pytest.mark.gpu

COMPAT = os.path.join(ROOT, "fun-asr-gguf_amd", "lib", "llama_compat")
LLM_V = dict(synth.LLM_TINY, n_vocab=711)


class ModelParams(ctypes.Structure):
    _fields_ = [("devices", ctypes.c_void_p), ("tensor_buft_overrides", ctypes.c_void_p), ("n_gpu_layers", ctypes.c_int32),
                ("split_mode", ctypes.c_int32), ("main_gpu", ctypes.c_int32), ("tensor_split", ctypes.c_void_p),
                ("progress_callback", ctypes.c_void_p), ("progress_callback_user_data", ctypes.c_void_p),
                ("kv_overrides", ctypes.c_void_p)] + [(n, ctypes.c_bool) for n in (
                    "vocab_only", "use_mmap", "use_direct_io", "use_mlock", "check_tensors", "use_extra_bufts", "no_host",
                    "no_alloc")]


class ContextParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("n_ctx", "n_batch", "n_ubatch", "n_seq_max")] + \
               [(n, ctypes.c_int32) for n in ("n_threads", "n_threads_batch", "rope_scaling_type", "pooling_type",
                                              "attention_type", "flash_attn_type")] + \
               [(n, ctypes.c_float) for n in ("rope_freq_base", "rope_freq_scale", "yarn_ext_factor", "yarn_attn_factor",
                                              "yarn_beta_fast", "yarn_beta_slow")] + \
               [("yarn_orig_ctx", ctypes.c_uint32), ("defrag_thold", ctypes.c_float), ("cb_eval", ctypes.c_void_p),
                ("cb_eval_user_data", ctypes.c_void_p), ("type_k", ctypes.c_int32), ("type_v", ctypes.c_int32),
                ("abort_callback", ctypes.c_void_p), ("abort_callback_data", ctypes.c_void_p)] + \
               [(n, ctypes.c_bool) for n in ("embeddings", "offload_kqv", "no_perf", "op_offload", "swa_full",
                                             "kv_unified")] + [("samplers", ctypes.c_void_p), ("n_samplers", ctypes.c_size_t)]


class Batch(ctypes.Structure):
    _fields_ = [("n_tokens", ctypes.c_int32), ("token", ctypes.POINTER(ctypes.c_int32)),
                ("embd", ctypes.POINTER(ctypes.c_float)), ("pos", ctypes.POINTER(ctypes.c_int32)),
                ("n_seq_id", ctypes.POINTER(ctypes.c_int32)), ("seq_id", ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))),
                ("logits", ctypes.POINTER(ctypes.c_int8))]


def bind():
    for name in ("libggml-base.so", "libggml.so"):
        ctypes.CDLL(os.path.join(COMPAT, name))
    L = ctypes.CDLL(os.path.join(COMPAT, "libllama.so"))
    sig = {
        "llama_model_default_params": ([], ModelParams), "llama_context_default_params": ([], ContextParams),
        "llama_model_load_from_file": ([ctypes.c_char_p, ModelParams], ctypes.c_void_p),
        "llama_init_from_model": ([ctypes.c_void_p, ContextParams], ctypes.c_void_p),
        "llama_model_get_vocab": ([ctypes.c_void_p], ctypes.c_void_p), "llama_vocab_eos": ([ctypes.c_void_p], ctypes.c_int32),
        "llama_free": ([ctypes.c_void_p], None), "llama_model_free": ([ctypes.c_void_p], None),
        "llama_batch_init": ([ctypes.c_int32, ctypes.c_int32, ctypes.c_int32], Batch), "llama_batch_free": ([Batch], None),
        "llama_decode": ([ctypes.c_void_p, Batch], ctypes.c_int32),
        "llama_get_logits": ([ctypes.c_void_p], ctypes.POINTER(ctypes.c_float)),
        "llama_get_memory": ([ctypes.c_void_p], ctypes.c_void_p), "llama_memory_clear": ([ctypes.c_void_p, ctypes.c_bool], None),
        "llama_sampler_chain_init": ([ctypes.c_bool], ctypes.c_void_p),
        "llama_sampler_chain_add": ([ctypes.c_void_p, ctypes.c_void_p], None),
        "llama_sampler_init_greedy": ([], ctypes.c_void_p),
        "llama_sampler_sample": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32], ctypes.c_int32),
        "llama_sampler_free": ([ctypes.c_void_p], None),
    }
    for n, (a, r) in sig.items():
        f = getattr(L, n)
        f.argtypes, f.restype = a, r
    return L


def model_gguf(path, drop=None):
    from fun_asr_gguf.vocab import read_gguf_metadata
    kv = {k: v for k, v in read_gguf_metadata(os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf")).items()
          if k.startswith("tokenizer.")}
    kv.update({"qwen3.block_count": LLM_V["n_layer"], "qwen3.embedding_length": LLM_V["n_embd"],
               "qwen3.feed_forward_length": LLM_V["n_ff"], "qwen3.attention.head_count": LLM_V["n_head"],
               "qwen3.attention.head_count_kv": LLM_V["n_head_kv"], "qwen3.attention.key_length": LLM_V["head_dim"],
               "qwen3.rope.freq_base": float(LLM_V["rope_theta"]),
               "qwen3.attention.layer_norm_rms_epsilon": float(LLM_V["rms_eps"])})
    W = synth.make_weights(synth.llm_tensors(LLM_V), seed=0)
    write_gguf(str(path), kv, [(n, w, GGML_Q8_0 if w.ndim == 2 else GGML_F32) for n, w in W.items() if n != drop])


@pytest.fixture(scope="module")
def gguf(tmp_path_factory):
    p = tmp_path_factory.mktemp("llama_compat") / "decoder.q8_0.gguf"
    model_gguf(p)
    return str(p)


def reference_decode_loop(L, ctx, embd, n_predict):
    """LLMDecoder.decode (core/decoder.py:70-114) at temperature 0: clear, embedding batch, sample, one-token batches."""
    L.llama_memory_clear(L.llama_get_memory(ctx), True)
    n, E = embd.shape
    b = L.llama_batch_init(n, E, 1)
    ctypes.memmove(b.embd, embd.ctypes.data, embd.nbytes)
    b.n_tokens = n
    for i in range(n):
        b.pos[i], b.n_seq_id[i], b.logits[i] = i, 1, 1 if i == n - 1 else 0
        b.seq_id[i][0] = 0
    tok_ptr = b.token
    b.token = ctypes.cast(None, ctypes.POINTER(ctypes.c_int32))
    assert L.llama_decode(ctx, b) == 0
    first_logits = np.ctypeslib.as_array(L.llama_get_logits(ctx), shape=(LLM_V["n_vocab"],)).copy()
    b.token = tok_ptr
    L.llama_batch_free(b)
    bt = L.llama_batch_init(1, 0, 1)
    smpl = L.llama_sampler_chain_init(True)
    L.llama_sampler_chain_add(smpl, L.llama_sampler_init_greedy())
    toks, pos = [], n
    for _ in range(n_predict):
        t = L.llama_sampler_sample(smpl, ctx, -1)
        toks.append(t)
        bt.n_tokens = 1
        bt.token[0], bt.pos[0], bt.n_seq_id[0], bt.logits[0] = t, pos, 1, 1
        bt.seq_id[0][0] = 0
        assert L.llama_decode(ctx, bt) == 0
        pos += 1
    last_logits = np.ctypeslib.as_array(L.llama_get_logits(ctx), shape=(LLM_V["n_vocab"],)).copy()
    L.llama_sampler_free(smpl)
    L.llama_batch_free(bt)
    return toks, first_logits, last_logits


def test_reference_decode_loop_equals_engine(gguf):
    from fun_asr_gguf import _native
    L = bind()
    mp = L.llama_model_default_params()
    model = L.llama_model_load_from_file(gguf.encode(), mp)
    assert model
    cp = L.llama_context_default_params()
    cp.n_ctx, cp.n_batch, cp.n_ubatch, cp.n_seq_max, cp.flash_attn_type, cp.offload_kqv = 256, 256, 256, 1, 1, True
    ctx = L.llama_init_from_model(model, cp)
    assert ctx
    e = _native.Engine(synth.ENC_TINY, dict(LLM_V, n_ctx=256, max_seqs=1), max_batch=1, max_samples=16000)
    try:
        e.load_gguf(gguf)
        rng = np.random.default_rng(3)
        embd = (rng.standard_normal((37, LLM_V["n_embd"])) * 0.05).astype(np.float32)
        toks, lg0, lg_last = reference_decode_loop(L, ctx, embd, 16)
        e.llm_reset(0)
        t0, elg = e.llm_prefill(0, embd, want_logits=True)
        rest = e.llm_generate([0], 15)[0].tolist()
        assert (lg0 == elg).all()  # the prefill forward is the engine's
        assert toks == [t0] + rest  # host greedy over the copied logits == the engine's device greedy, step for step
        el15 = e.llm_logits(0)
        e.llm_generate([0], 1)
        el = e.llm_logits(0)
        assert (lg_last == el).all(), (
            f"max |diff| {np.abs(lg_last - el).max():.3g}, vs the engine's previous step {np.abs(lg_last - el15).max():.3g}"
            f", engine recoveries {e.llm_decode_recoveries()}, n_past {e.llm_n_past(0)}")
        # a cleared context decodes the same prompt to the same tokens
        assert reference_decode_loop(L, ctx, embd, 16)[0] == toks
        eos = L.llama_vocab_eos(L.llama_model_get_vocab(model))
        assert eos == json.load(open(os.path.join(GOLDEN, "tokenizer_golden.json")))["eos"]
    finally:
        e.close()
        L.llama_free(ctx)
        L.llama_model_free(model)


def test_context_fails_when_the_file_lacks_a_decoder_tensor(tmp_path):
    L = bind()
    p = tmp_path / "partial.gguf"
    model_gguf(p, drop="blk.1.ffn_down.weight")
    model = L.llama_model_load_from_file(str(p).encode(), L.llama_model_default_params())
    assert model
    cp = L.llama_context_default_params()
    cp.n_ctx = 128
    assert not L.llama_init_from_model(model, cp)  # core/model_manager.py: fail loudly, no synthetic fallback
    L.llama_model_free(model)
