"""The reference's per-segment path through both reference-ABI drop-ins at once, on the GPU: the onnxruntime-API sessions
(encoder-adaptor + CTC, nano_onnx.load_onnx_models / encode_audio, decoder.py:27) and the llama.cpp-ABI library
(PromptBuilder's tokenisation, LLMDecoder.decode's embedding batch + greedy loop with its stop rule, ASRStreamDecoder's
incremental UTF-8 detokenisation; decoder.py:55-123, llama.py:661-690), restated as call sequences (the reference
modules cannot travel to the GPU box), against the public API (`create_asr_engine(...).transcribe`) on the same model
files: the same text."""
import codecs
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import synth
from test_gpu_llama_compat import LLM_V, bind, model_gguf
from test_gpu_ort_compat import encode_audio, load_onnx_models, onnx_files, ort

pytestmark = pytest.mark.gpu

STOP = (151643, 151645)  # decoder.py:53


def tokenize(L, vocab, text):
    """llama.py:738-743 (add_special False, parse_special True)."""
    b = text.encode("utf-8")
    buf = (ctypes.c_int32 * (len(b) + 32))()
    n = L.llama_tokenize(vocab, b, len(b), buf, len(buf), False, True)
    return [buf[i] for i in range(n)]


def piece(L, vocab, t):
    """llama.py:745-748."""
    b = ctypes.create_string_buffer(256)
    n = L.llama_token_to_piece(vocab, t, b, 256, 0, True)
    return b.raw[:n] if n > 0 else b""


def test_reference_path_through_both_dropins_equals_api(tmp_path):
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.prompt_utils import prompt_texts
    from fun_asr_gguf.synthetic import synth_audio
    from fun_asr_gguf._native import load as load_native
    rt = ort()
    ep, cp, _ = onnx_files(tmp_path, "fp32")
    gg = tmp_path / "decoder.q8_0.gguf"
    model_gguf(gg)
    L = bind()
    L.llama_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                 ctypes.c_int32, ctypes.c_bool, ctypes.c_bool]
    L.llama_token_to_piece.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_bool]
    audio = synth_audio(16000 * 6 + 321, 11)
    n_predict = 16
    # ---- ModelManager.initialize: ORT sessions + LlamaModel / LlamaContext (model_manager.py:36-100)
    es, cs = load_onnx_models(rt, ep, cp)
    model = L.llama_model_load_from_file(str(gg).encode(), L.llama_model_default_params())
    cparams = L.llama_context_default_params()
    cparams.n_ctx, cparams.n_batch, cparams.n_ubatch, cparams.flash_attn_type = 512, 512, 512, 1
    ctx = L.llama_init_from_model(model, cparams)
    assert model and ctx
    vocab = L.llama_model_get_vocab(model)
    eos = L.llama_vocab_eos(vocab)
    api = None
    try:
        # ---- decode_stream: encode + CTC, prompt, LLM (decoder.py:132-246)
        audio_embd, enc = encode_audio(rt, audio, es)
        ids = cs.run(None, {"enc_output": enc})[0]
        assert ids.shape == enc.shape[:2]
        pre_txt, suf_txt = prompt_texts()
        pre, suf = tokenize(L, vocab, pre_txt), tokenize(L, vocab, suf_txt)
        table = np.zeros((LLM_V["n_vocab"], LLM_V["n_embd"]), np.float32)  # get_token_embeddings_gguf (fp16 product)
        lib = load_native()
        assert lib.fa_gguf_read_tensor(str(gg).encode(), b"token_embd.weight", 1, table.ctypes.data, table.size) == 0
        full = np.ascontiguousarray(np.concatenate([table[pre], audio_embd, table[suf]], 0), np.float32)
        L.llama_memory_clear(L.llama_get_memory(ctx), True)
        n = full.shape[0]
        b = L.llama_batch_init(n, full.shape[1], 1)
        ctypes.memmove(b.embd, full.ctypes.data, full.nbytes)
        b.n_tokens = n
        for i in range(n):
            b.pos[i], b.n_seq_id[i], b.logits[i] = i, 1, 1 if i == n - 1 else 0
            b.seq_id[i][0] = 0
        tok_ptr = b.token
        b.token = ctypes.cast(None, ctypes.POINTER(ctypes.c_int32))
        assert L.llama_decode(ctx, b) == 0
        b.token = tok_ptr
        L.llama_batch_free(b)
        bt = L.llama_batch_init(1, 0, 1)
        smpl = L.llama_sampler_chain_init(True)
        L.llama_sampler_chain_add(smpl, L.llama_sampler_init_greedy())  # temperature 0 (llama.py:604-605)
        dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
        text, pos = "", n
        for _ in range(n_predict):  # decoder.py:91-114
            t = L.llama_sampler_sample(smpl, ctx, -1)
            bt.n_tokens = 1
            bt.token[0], bt.pos[0], bt.n_seq_id[0], bt.logits[0] = t, pos, 1, 1
            bt.seq_id[0][0] = 0
            if L.llama_decode(ctx, bt) != 0:
                break
            pos += 1
            if t == eos or t in STOP:
                break
            text += dec.decode(piece(L, vocab, t), final=False)
        text += dec.decode(b"", final=True)
        L.llama_sampler_free(smpl)
        L.llama_batch_free(bt)
        # ---- the public API on the same files
        api = create_asr_engine(ep, cp, str(gg), "synthetic", verbose=False, model="tiny", max_batch=1, n_ctx=512,
                                n_predict=n_predict)
        r = api.transcribe(audio, temperature=0.0, verbose=False)
        assert r.text == text.strip() and len(text.strip()) > 0
    finally:
        if api is not None:
            api.cleanup()
        L.llama_free(ctx)
        L.llama_model_free(model)
        del es, cs
