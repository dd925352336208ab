"""CPU checks of the onnxruntime-compatible session module (fun-asr-gguf_amd/ort_compat/onnxruntime): the surface the
reference's nano_onnx.py uses (SessionOptions, GraphOptimizationLevel, get_available_providers, OrtValue), graph
recognition and engine dimensions from the ONNX initializers, and failures before any device work. When /root/reference is
present, its own nano_onnx.load_onnx_models runs against the module in a subprocess up to the engine creation (which
needs a GPU: the session's run path is tests/test_gpu_ort_compat.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from onnx_io import write_onnx
from oracle import synth

ORT_DIR = os.path.join(ROOT, "fun-asr-gguf_amd", "ort_compat")
REF = "/root/reference/fun_asr_gguf"


def ort():
    if ORT_DIR not in sys.path:
        sys.path.insert(0, ORT_DIR)
    import onnxruntime
    assert onnxruntime.__file__.startswith(ORT_DIR)
    return onnxruntime


def test_session_surface():
    rt = ort()
    so = rt.SessionOptions()
    so.add_session_config_entry("session.intra_op.allow_spinning", "0")
    assert so.get_session_config_entry("session.intra_op.allow_spinning") == "0"
    so.graph_optimization_level = rt.GraphOptimizationLevel.ORT_ENABLE_ALL
    assert rt.get_available_providers()[0] == rt.PROVIDER and "DmlExecutionProvider" not in rt.get_available_providers()
    a = np.arange(6, dtype=np.float32).reshape(1, 2, 3)
    v = rt.OrtValue.ortvalue_from_numpy(a, "cpu", 0)
    assert v.numpy() is a and v.shape() == [1, 2, 3]
    with pytest.raises(ValueError):
        rt.OrtValue.ortvalue_from_numpy(a, "cuda", 0)


@pytest.mark.parametrize("cfg", [synth.ENC_FULL, synth.ENC_TINY])
def test_engine_dimensions_from_initializers(cfg):
    rt = ort()
    names = synth.encoder_tensors(cfg)
    sd = {n: np.zeros(shape, np.float32) for n, shape, _, _ in names}
    e = rt._config({k: v for k, v in sd.items() if k.startswith(("audio_encoder.", "audio_adaptor."))}, "encoder")
    assert (e["n_blocks"], e["n_tp_blocks"], e["adaptor_blocks"], e["d_llm"]) == (
        cfg["n_blocks"], cfg["n_tp_blocks"], cfg["adaptor_blocks"], cfg["d_llm"])
    c = rt._config({k: v for k, v in sd.items() if k.startswith(("ctc_decoder.", "ctc_proj."))}, "ctc")
    assert (c["ctc_blocks"], c["ctc_vocab"]) == (cfg["ctc_blocks"], cfg["ctc_vocab"])


def test_session_errors_before_device_work(tmp_path):
    rt = ort()
    with pytest.raises(FileNotFoundError):
        rt.InferenceSession(str(tmp_path / "absent.onnx"))
    p = tmp_path / "other.onnx"
    write_onnx(str(p), {"some_model.linear.weight": np.ones((4, 4), np.float32)})
    with pytest.raises(ValueError, match="neither"):
        rt.InferenceSession(str(p))
    with pytest.raises(TypeError):
        rt.InferenceSession(b"\x08\x07")


_REF_SCRIPT = r'''
import importlib.util, logging, os, sys
ref, ort_dir, enc, ctc = sys.argv[1:5]
sys.path.insert(0, ort_dir)
spec = importlib.util.spec_from_file_location("ref_nano_onnx", os.path.join(ref, "nano_onnx.py"))
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
import onnxruntime
assert m.onnxruntime is onnxruntime and onnxruntime.__file__.startswith(ort_dir)
try:
    m.load_onnx_models(enc, ctc)
    print("RESULT loaded")
except RuntimeError as e:
    print("RESULT " + str(e).splitlines()[0])
'''


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is only present in the build container")
def test_reference_nano_onnx_reaches_the_engine(tmp_path):
    """The reference's unmodified nano_onnx.py imports this module as onnxruntime and builds its sessions through it; on
    a machine without a GPU the engine creation is where it stops."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: tests/test_gpu_ort_compat.py runs the sessions")
    except Exception:
        pass
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY), seed=0)
    e, c = tmp_path / "Fun-ASR-Nano-Encoder-Adaptor.fp32.onnx", tmp_path / "Fun-ASR-Nano-CTC.fp32.onnx"
    write_onnx(str(e), {k: v for k, v in W.items() if k.startswith(("audio_encoder.", "audio_adaptor."))},
               prefix="hybrid_model.")
    write_onnx(str(c), {k: v for k, v in W.items() if k.startswith(("ctc_decoder.", "ctc_proj."))})
    r = subprocess.run([sys.executable, "-c", _REF_SCRIPT, REF, ORT_DIR, str(e), str(c)], capture_output=True,
                       text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert r.returncode == 0 and line, r.stderr[-3000:]
    assert "fa_engine_create" in line[0]
