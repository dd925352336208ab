"""The onnxruntime-compatible session module (fun-asr-gguf_amd/ort_compat/onnxruntime) on the GPU: the call sequence
of the reference's nano_onnx.load_onnx_models + encode_audio and of decoder.py:27's CTC run (restated below; the
reference module cannot travel to the GPU box, tests/test_ort_compat.py runs it against this module in the build
container) over encoder / CTC ONNX files laid out as the reference's export writes them (tests/onnx_io.py), against
  * the engine's own encode of the same clip (adaptor rows and encoder rows bit for bit; past the valid frames zero,
    EncoderExportWrapperPaddable's sweeps, model_definition.py:269-311),
  * the CPU oracle's CTC head over the same padded encoder rows (oracle/encoder.ctc_logits, unmasked like
    model_definition.py:336): ids equal wherever the top-2 margin exceeds 1e-3,
  * fa_ctc_head over a clip's own rows = the ids the engine's encode computes for it, bit for bit,
in the f32 and the fp16 export."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
from onnx_io import write_onnx
from oracle import encoder as oenc, synth

pytestmark = pytest.mark.gpu

ORT_DIR = os.path.join(ROOT, "fun-asr-gguf_amd", "ort_compat")


def ort():
    if ORT_DIR not in sys.path:
        sys.path.insert(0, ORT_DIR)
    import onnxruntime
    assert onnxruntime.__file__.startswith(ORT_DIR)
    return onnxruntime


def onnx_files(tmp_path, dtype):
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), seed=0)
    enc_sd = {k: v for k, v in W.items() if k.startswith(("audio_encoder.", "audio_adaptor."))}
    ctc_sd = {k: v for k, v in W.items() if k.startswith(("ctc_decoder.", "ctc_proj."))}
    e, c = tmp_path / f"Fun-ASR-Nano-Encoder-Adaptor.{dtype}.onnx", tmp_path / f"Fun-ASR-Nano-CTC.{dtype}.onnx"
    write_onnx(str(e), enc_sd, prefix="hybrid_model.", dtype=dtype)
    write_onnx(str(c), ctc_sd, dtype=dtype)
    return str(e), str(c), W


def load_onnx_models(rt, encoder_path, ctc_path, padding_secs=60):
    """nano_onnx.py:21-76: options, providers, both sessions, warm-up runs."""
    so = rt.SessionOptions()
    so.add_session_config_entry("session.intra_op.allow_spinning", "0")
    so.graph_optimization_level = rt.GraphOptimizationLevel.ORT_ENABLE_ALL
    providers = ["CPUExecutionProvider"]
    if "DmlExecutionProvider" in rt.get_available_providers():
        providers.insert(0, "DmlExecutionProvider")
    es = rt.InferenceSession(encoder_path, sess_options=so, providers=providers)
    cs = rt.InferenceSession(ctc_path, sess_options=so, providers=providers)
    n = int(16000 * padding_secs)
    dt = np.float16 if "float16" in es.get_inputs()[0].type else np.float32
    names = [x.name for x in es.get_inputs()]
    es.run(None, {names[0]: np.zeros((1, 1, n), dt), names[1]: np.array([n], np.int64)})
    ci = cs.get_inputs()[0]
    cs.run(None, {ci.name: np.zeros((1, n // 160 // 6, 512), np.float16 if "float16" in ci.type else np.float32)})
    return es, cs


def encode_audio(rt, audio, es, padding_secs=60):
    """nano_onnx.py:78-133 (pad to padding_secs unless the provider is the CPU EP, ilens, crop to target_len)."""
    names = [x.name for x in es.get_inputs()]
    dt = np.float16 if "float16" in es.get_inputs()[0].type else np.float32
    actual = len(audio)
    if es.get_providers()[0] == "CPUExecutionProvider":
        padding_secs = 1
    target = int(padding_secs * 16000)
    if actual < target:
        a = np.zeros(target, audio.dtype)
        a[:actual] = audio
        audio = a
    feed = {names[0]: rt.OrtValue.ortvalue_from_numpy(audio.astype(dt).reshape(1, 1, -1), "cpu", 0),
            "ilens": rt.OrtValue.ortvalue_from_numpy(np.array([actual], np.int64), "cpu", 0)}
    outs = es.run_with_ort_values([x.name for x in es.get_outputs()], feed)
    enc = outs[0].numpy()
    t_mel = actual // 160 + 1
    t_lfr = (t_mel + 5) // 6
    o1 = 1 + (t_lfr - 3 + 2) // 2
    tgt = (1 + (o1 - 3 + 2) // 2 - 1) // 2 + 1
    return outs[1].numpy().squeeze(0)[:tgt].astype(np.float32), enc


@pytest.mark.parametrize("dtype", ["fp32", "fp16"])
def test_reference_onnx_call_sequence_on_the_engine(tmp_path, dtype):
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    rt = ort()
    ep, cp, W = onnx_files(tmp_path, dtype)
    es, cs = load_onnx_models(rt, ep, cp)
    fp16 = dtype == "fp16"
    assert es.get_inputs()[0].type == ("tensor(float16)" if fp16 else "tensor(float)")
    ref = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=64, max_seqs=1), max_batch=1,
                         max_samples=16000 * 64)
    try:
        ref.synthetic_weights(0)
        from fun_asr_gguf.onnx_weights import state_dict_from_onnx
        for k, v in state_dict_from_onnx(ep).items():  # the file's values (the fp16 export rounds every initializer)
            ref.set_tensor(k, v)
        ref.set_encoder_fp16(fp16)
        audio = synth_audio(16000 * 10 + 777, 5)
        if fp16:
            audio = audio.astype(np.float16).astype(np.float32)  # the fp16 graph takes fp16 audio (nano_onnx.py:101)
        emb, enc = encode_audio(rt, audio, es)
        want = ref.encode([audio], want_enc=True)
        assert enc.shape == (1, 1001, 512) and enc.dtype == (np.float16 if fp16 else np.float32)
        tl = want["enc"][0].shape[0]
        assert (enc[0, :tl].astype(np.float32) == want["enc"][0]).all() and not enc[0, tl:].any()
        assert (emb == want["audio_embd"][0]).all()
        # decoder.py:27: the CTC graph over the whole padded enc_output
        ids = cs.run(None, {"enc_output": enc})[0]
        assert ids.shape == (1, 1001) and ids.dtype == np.int32
        if not fp16:  # (the fp16 graph's CTC logits are checked through the engine's own encode below)
            lg = oenc.ctc_logits(enc[0].astype(np.float32), W, synth.ENC_TINY, None)
            top2 = np.sort(lg, -1)[:, -2:]
            nontie = (top2[:, 1] - top2[:, 0]) > 1e-3
            assert nontie[:tl].sum() > tl // 2
            assert (ids[0][nontie] == np.argmax(lg, -1)[nontie]).all()
        # the CTC graph over the clip's own rows: the ids of the engine's encode, bit for bit
        ids2 = cs.run(["indices"], {"enc_output": want["enc"][0][None].astype(enc.dtype)})[0][0]
        assert (ids2 == want["ctc_ids"][0]).all()
    finally:
        ref.close()
        del es, cs


def test_session_refuses_incomplete_graph(tmp_path):
    rt = ort()
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), seed=0)
    sd = {k: v for k, v in W.items() if k.startswith(("ctc_decoder.", "ctc_proj.")) and "blocks.0.norm2" not in k}
    p = tmp_path / "Fun-ASR-Nano-CTC.fp32.onnx"
    write_onnx(str(p), sd)
    with pytest.raises(ValueError, match="norm2"):
        rt.InferenceSession(str(p), providers=["CPUExecutionProvider"])


def test_int8_ctc_session_runs_the_int8_graph(tmp_path):
    """Fun-ASR-Nano-CTC.int8.onnx (the reference README's default CTC model): the session hands the file's dynamic-quant
    weights to the engine as stored, so decoder.py:27's ctc_sess.run computes the int8 graph (oracle/ctc_int8.py over the
    same quantized weights: ids equal wherever the oracle's top-2 margin exceeds 0.25, the int8 noise floor of
    tests/test_gpu_ctc_int8.py), not an f32 graph of dequantised weights."""
    from fun_asr_gguf.onnx_weights import state_dict_from_onnx, u8dq_from_onnx
    from oracle import ctc_int8 as oi8
    rt = ort()
    _, c, _ = onnx_files(tmp_path, "int8")
    cs = rt.InferenceSession(c, providers=["CPUExecutionProvider"])
    assert cs._eng.ctc_int8_active()
    g = np.load(os.path.join(ROOT, "tests", "golden", "encoder_tiny_3s.npz"))
    enc = g["enc"][: int(g["t_lfr_valid"])].astype(np.float32)
    ids = cs.run(None, {cs.get_inputs()[0].name: enc[None]})[0][0]
    sd = state_dict_from_onnx(c)
    Q = {k[: -len(".weight")]: v for k, v in u8dq_from_onnx(c).items()}
    ref_ids, lg = oi8.ctc_ids_int8(enc, sd, Q, synth.ENC_TINY)
    top2 = np.sort(lg, -1)[:, -2:]
    bad = (ids != ref_ids) & ((top2[:, 1] - top2[:, 0]) > 0.25)
    assert ids.shape == ref_ids.shape and bad.sum() == 0 and (ids != ref_ids).mean() < 0.1
