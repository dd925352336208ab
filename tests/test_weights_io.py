"""Weight ingestion on the host (no GPU): the ONNX initializer reader (fun_asr_gguf.onnx_weights, parity unpinned:
no ONNX file or `onnx` package exists here) on files the repo's own protobuf writer produces in the layouts the
reference's export / quantise scripts give them, and GGUF metadata + tensor reading (tests/gguf_io.py writer,
native fa_gguf_read_tensor)."""
import os

import numpy as np

from gguf_io import GGML_F32, GGML_Q8_0, write_gguf
from onnx_io import write_onnx
from oracle import q8, synth


def _enc_sd():
    return synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), only=lambda n: n.startswith(
        ("audio_encoder.encoders0.", "audio_encoder.tp_norm", "ctc_decoder.blocks.0.", "ctc_proj.")))


def test_onnx_reader_fp32_roundtrip(tmp_path):
    from fun_asr_gguf.onnx_weights import state_dict_from_onnx
    sd = _enc_sd()
    p = tmp_path / "Fun-ASR-Nano-Encoder-Adaptor.fp32.onnx"
    write_onnx(str(p), sd, prefix="hybrid_model.")
    got = state_dict_from_onnx(str(p))
    assert sorted(got) == sorted(sd)
    for k, v in sd.items():
        assert got[k].shape == v.shape and (got[k] == v).all(), k


def test_onnx_reader_fp16_and_int8(tmp_path):
    from fun_asr_gguf.onnx_weights import state_dict_from_onnx
    sd = _enc_sd()
    p16 = tmp_path / "Fun-ASR-Nano-CTC.fp16.onnx"
    write_onnx(str(p16), sd, dtype="fp16")
    got = state_dict_from_onnx(str(p16))
    for k, v in sd.items():
        assert (got[k] == v.astype(np.float16).astype(np.float32)).all(), k
    p8 = tmp_path / "Fun-ASR-Nano-CTC.int8.onnx"
    write_onnx(str(p8), sd, dtype="int8")
    got = state_dict_from_onnx(str(p8))
    assert sorted(got) == sorted(sd)
    for k, v in sd.items():
        if v.ndim == 2:
            step = (np.maximum(v.max(1), 0) - np.minimum(v.min(1), 0)) / 255.0  # per output channel
            assert (np.abs(got[k] - v) <= step[:, None] * 0.5001 + 1e-7).all(), k
        else:
            assert (got[k] == v).all(), k


def test_gguf_writer_reader_roundtrip(tmp_path):
    from fun_asr_gguf._native import gguf_read_tensor
    from fun_asr_gguf.vocab import read_gguf_metadata
    rng = np.random.default_rng(0)
    w = (rng.standard_normal((64, 96)) * 0.1).astype(np.float32)
    n = (rng.standard_normal(96)).astype(np.float32)
    p = tmp_path / "t.gguf"
    write_gguf(str(p), {"qwen3.embedding_length": 96, "tokenizer.ggml.tokens": ["a", "b"],
                        "tokenizer.ggml.token_type": [1, 3]}, [("blk.0.ffn_up.weight", w, GGML_Q8_0),
                                                               ("output_norm.weight", n, GGML_F32)])
    kv = read_gguf_metadata(str(p))
    assert kv["tokenizer.ggml.tokens"] == ["a", "b"] and kv["tokenizer.ggml.token_type"] == [1, 3]
    d, q = q8.quantize_q8_0(w)
    assert (gguf_read_tensor(str(p), "blk.0.ffn_up.weight", w.size).reshape(w.shape) == q8.dequant_f32(d, q)).all()
    assert (gguf_read_tensor(str(p), "output_norm.weight", n.size) == n).all()
