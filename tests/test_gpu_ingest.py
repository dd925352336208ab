"""Real-weight ingestion through the public API on the GPU:
  * decoder from a GGUF (fa_load_gguf replaces llama_model_load_from_file + get_token_embeddings_gguf,
    llama.py:352-391, 751-796): q8_0 bytes and logits bit-identical to the same weights made on device;
  * encoder / CTC from ONNX files laid out as the reference's export + quantise scripts produce them
    (01-Export-Encoder-Adaptor-CTC.py:107-135, 02-Quantize-ONNX.py:13-48; reader parity unpinned: no real file)
    and from a safetensors state dict: encoder outputs bit-identical to the synthetic-weight engine;
  * the GGUF's tokenizer drives the prompt (PromptBuilder.build_prompt, prompt_utils.py:16-54): prefix / suffix
    ids equal the HuggingFace `tokenizers` golden of the same text.
The GGUF is written by tests/gguf_io.py with the tokenizer metadata of tests/golden/tokenizer_qwen2_synth.gguf
and the synthetic q8_0 tensors of oracle/synth.py (vocabulary 711 = the tokenizer's).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gguf_io import GGML_F32, GGML_Q8_0, write_gguf
from onnx_io import write_onnx
from oracle import synth

pytestmark = pytest.mark.gpu

LLM_V = dict(synth.LLM_TINY, n_vocab=711)
TOK = json.load(open(os.path.join(GOLDEN, "tokenizer_golden.json")))


@pytest.fixture(scope="module")
def gguf_path(tmp_path_factory):
    from fun_asr_gguf.vocab import read_gguf_metadata
    kv = {k: v for k, v in read_gguf_metadata(os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf")).items()
          if k.startswith("tokenizer.")}
    kv.update({"qwen3.block_count": LLM_V["n_layer"], "qwen3.embedding_length": LLM_V["n_embd"],
               "qwen3.attention.head_count": LLM_V["n_head"], "qwen3.attention.head_count_kv": LLM_V["n_head_kv"]})
    W = synth.make_weights(synth.llm_tensors(LLM_V), seed=0)
    p = tmp_path_factory.mktemp("gguf") / "decoder.q8_0.gguf"
    write_gguf(str(p), kv, [(n, w, GGML_Q8_0 if w.ndim == 2 else GGML_F32) for n, w in W.items()])
    return str(p)


def _engine(seed):
    from fun_asr_gguf import _native
    e = _native.Engine(synth.ENC_TINY, dict(LLM_V, n_ctx=256, max_seqs=2), max_batch=1, max_samples=16000 * 4)
    e.synthetic_weights(seed)
    return e


def test_fa_load_gguf_bit_identical_to_device_weights(gguf_path):
    a, b = _engine(0), _engine(5)
    try:
        b.load_gguf(gguf_path)
        for name in ("token_embd.weight", "blk.0.attn_q.weight", "blk.1.ffn_down.weight", "blk.1.attn_output.weight"):
            n = int(np.prod([s for nm, s, _, _ in synth.llm_tensors(LLM_V) if nm == name][0]))
            assert (a.get_tensor_q8_0(name, n) == b.get_tensor_q8_0(name, n)).all(), name
        ids = np.array(TOK["cases"][0]["ids"], np.int32)
        prompt = a.embd_rows(ids)
        assert (b.embd_rows(ids) == prompt).all()
        outs = []
        for e in (a, b):
            e.llm_reset(0)
            t, lg = e.llm_prefill(0, prompt, want_logits=True)
            outs.append((t, lg, e.llm_generate([0], 12)[0].tolist()))
        assert outs[0][0] == outs[1][0] and (outs[0][1] == outs[1][1]).all() and outs[0][2] == outs[1][2]
    finally:
        a.close()
        b.close()


def test_api_onnx_encoder_and_gguf_tokenizer(gguf_path, tmp_path):
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.prompt_utils import prompt_texts
    from fun_asr_gguf.synthetic import synth_audio
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), seed=0)
    enc_sd = {k: v for k, v in W.items() if k.startswith(("audio_encoder.", "audio_adaptor."))}
    ctc_sd = {k: v for k, v in W.items() if k.startswith(("ctc_decoder.", "ctc_proj."))}
    enc_p, ctc_p = tmp_path / "Fun-ASR-Nano-Encoder-Adaptor.fp32.onnx", tmp_path / "Fun-ASR-Nano-CTC.fp32.onnx"
    write_onnx(str(enc_p), enc_sd, prefix="hybrid_model.")
    write_onnx(str(ctc_p), ctc_sd)
    from safetensors.numpy import save_file
    st_p = tmp_path / "model.safetensors"
    # model.pt naming (HybridSenseVoice.load_weights, model_definition.py:231-238): ctc.ctc_lo.* -> ctc_proj.ctc_lo.*
    save_file({k.replace("ctc_proj.ctc_lo", "ctc.ctc_lo"): np.ascontiguousarray(v) for k, v in W.items()}, str(st_p))
    kw = dict(verbose=False, model="tiny", synthetic_seed=3, max_batch=2, n_ctx=512, n_predict=16, ignore_eos=True)
    api = create_asr_engine(str(enc_p), str(ctc_p), gguf_path, "synthetic", **kw)
    api_st = create_asr_engine(str(st_p), "synthetic", gguf_path, "synthetic", **kw)
    ref = _engine(0)
    try:
        audio = synth_audio(16000 * 3 + 555, 9)
        want = ref.encode([audio], want_enc=True)
        for e in (api, api_st):
            got = e.models.engine.encode([audio], want_enc=True)
            assert (got["enc"][0] == want["enc"][0]).all() and (got["audio_embd"][0] == want["audio_embd"][0]).all()
            assert (got["ctc_ids"][0] == want["ctc_ids"][0]).all()
        # the GGUF tokenizer builds the prompt: ids = the HF tokenizers golden of the same text
        pre, suf, _ = api.models.prompt_builder.build_ids()
        assert pre == next(c["ids"] for c in TOK["cases"] if c["text"] == prompt_texts()[0])
        assert suf == next(c["ids"] for c in TOK["cases"] if c["text"] == prompt_texts()[1])
        assert api.models.eos_token == TOK["eos"]
        r = api.transcribe(audio, temperature=0.0, verbose=False)
        d = api.transcribe_batch([audio], temperature=0.0)[0]
        assert d.n_gen == 16 and r.text == d.text and isinstance(r.text, str)
    finally:
        api.cleanup()
        api_st.cleanup()
        ref.close()


def test_incomplete_model_files_fail_init(tmp_path):
    """A model file that leaves any tensor of its part of the graph unfilled fails initialisation (the reference's ORT /
    llama.cpp loaders raise, model_manager.py:98-100 -> asr_engine.py:135) and names the missing tensors."""
    import logging
    from fun_asr_gguf import create_asr_engine
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), seed=0)
    enc_sd = {k: v for k, v in W.items() if k.startswith(("audio_encoder.", "audio_adaptor."))}
    ctc_sd = {k: v for k, v in W.items() if k.startswith(("ctc_decoder.", "ctc_proj."))}
    drop_enc, drop_ctc = "audio_encoder.encoders.1.feed_forward.w_2.bias", "ctc_decoder.blocks.0.norm1.weight"
    assert drop_enc in enc_sd and drop_ctc in ctc_sd
    enc_p, ctc_p = tmp_path / "enc.onnx", tmp_path / "ctc.onnx"
    enc_bad, ctc_bad = tmp_path / "enc_bad.onnx", tmp_path / "ctc_bad.onnx"
    write_onnx(str(enc_p), enc_sd, prefix="hybrid_model.")
    write_onnx(str(ctc_p), ctc_sd)
    write_onnx(str(enc_bad), {k: v for k, v in enc_sd.items() if k != drop_enc}, prefix="hybrid_model.")
    write_onnx(str(ctc_bad), {k: v for k, v in ctc_sd.items() if k != drop_ctc})
    # a GGUF missing one decoder matrix
    Wl = synth.make_weights(synth.llm_tensors(LLM_V), seed=0)
    g_bad = tmp_path / "bad.gguf"
    from fun_asr_gguf.vocab import read_gguf_metadata
    kv = {k: v for k, v in read_gguf_metadata(os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf")).items()
          if k.startswith("tokenizer.")}
    write_gguf(str(g_bad), kv,
               [(n, w, GGML_Q8_0 if w.ndim == 2 else GGML_F32) for n, w in Wl.items() if n != "blk.1.ffn_up.weight"])
    kw = dict(verbose=False, model="tiny", max_batch=1, n_ctx=256, n_predict=4)
    ok = create_asr_engine(str(enc_p), str(ctc_p), "synthetic", "synthetic", **kw)  # complete files load
    ok.cleanup()
    for args, missing in (((str(enc_bad), str(ctc_p), "synthetic", "synthetic"), drop_enc),
                          ((str(enc_p), str(ctc_bad), "synthetic", "synthetic"), drop_ctc),
                          (("synthetic", "synthetic", str(g_bad), "synthetic"), "blk.1.ffn_up.weight")):
        records = []
        h = logging.Handler()
        h.emit = records.append
        logging.getLogger("fun_asr_gguf").addHandler(h)
        try:
            with pytest.raises(RuntimeError):
                create_asr_engine(*args, **kw)
        finally:
            logging.getLogger("fun_asr_gguf").removeHandler(h)
        assert any(missing in r.getMessage() or (r.exc_info and missing in str(r.exc_info[1])) for r in records), missing
