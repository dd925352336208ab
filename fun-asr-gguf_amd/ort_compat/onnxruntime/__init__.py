"""onnxruntime-compatible session API for the two Fun-ASR graphs, served by the MI355X engine.

The reference runs its encoder and CTC head through onnxruntime (nano_onnx.py:21-133, core/decoder.py:27):
`InferenceSession(path, sess_options, providers)`, `get_inputs / get_outputs / get_providers`, `run` and
`run_with_ort_values` with `OrtValue.ortvalue_from_numpy`. With this directory first on PYTHONPATH, `import onnxruntime`
in the reference's unmodified code gets this module, and each session runs on its own HIP engine
(fun_asr_gguf._native.Engine): the weights come from the ONNX file's initializers (fun_asr_gguf.onnx_weights, no `onnx`
package), every tensor of the graph's part must be present (the reference's ORT session fails to load otherwise), and
  * Fun-ASR-Nano-Encoder-Adaptor.*.onnx  inputs audio [1, 1, N] (f32, or f16 for the fp16 export) + ilens [1] int64
      -> enc_output [1, T, 512], adaptor_output [1, T, 1024]: fa_encode of the ilens valid samples, rows past the valid
      frames / target_len zero (EncoderExportWrapperPaddable's sweeps, model_definition.py:269-311);
  * Fun-ASR-Nano-CTC.*.onnx  enc_output [1, T, 512] -> indices [1, T] int32: fa_ctc_head (model_definition.py:335-337).
The fp16 export (fp16 initializers, 02-Quantize-ONNX.py:13-27) selects the engine's fp16 graph. Only these two graphs
are served; any other model raises at session creation, as would a file ORT cannot parse. INTEGRATION.md §5.
"""
import os
import sys

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # fun-asr-gguf_amd
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from fun_asr_gguf import _native  # noqa: E402
from fun_asr_gguf.core.model_manager import CTC_GROUPS, ENCODER_GROUPS, require_loaded  # noqa: E402
from fun_asr_gguf.model_config import ENC_FULL, ENC_TINY, LLM_TINY  # noqa: E402
from fun_asr_gguf.onnx_weights import read_onnx, state_dict_from_onnx, u8dq_from_onnx  # noqa: E402

__version__ = "1.20.0+mi355x"
PROVIDER = "MI355XExecutionProvider"
MAX_SECONDS = float(os.environ.get("FUNASR_ORT_MAX_SECONDS", "64"))  # longest clip an encoder session accepts


class GraphOptimizationLevel:
    ORT_DISABLE_ALL = 0
    ORT_ENABLE_BASIC = 1
    ORT_ENABLE_EXTENDED = 2
    ORT_ENABLE_ALL = 99


class SessionOptions:
    """Accepted and recorded; the engine has no graph-level options to set."""

    def __init__(self):
        self.graph_optimization_level = GraphOptimizationLevel.ORT_ENABLE_ALL
        self.intra_op_num_threads = 0
        self.inter_op_num_threads = 0
        self.log_severity_level = 2
        self._entries = {}

    def add_session_config_entry(self, key, value):
        self._entries[key] = value

    def get_session_config_entry(self, key):
        return self._entries[key]


def get_available_providers():
    return [PROVIDER, "CPUExecutionProvider"]


def get_device():
    return "GPU"


class NodeArg:
    def __init__(self, name, type_, shape):
        self.name, self.type, self.shape = name, type_, shape

    def __repr__(self):
        return f"NodeArg(name='{self.name}', type='{self.type}', shape={self.shape})"


class OrtValue:
    """Host array holder (ortvalue_from_numpy with device 'cpu', as the reference uses it)."""

    def __init__(self, array):
        self._a = np.asarray(array)

    @staticmethod
    def ortvalue_from_numpy(array, device_type="cpu", device_id=0):
        if device_type != "cpu":
            raise ValueError("OrtValue: only host ('cpu') arrays are accepted; the engine copies them to HBM")
        return OrtValue(array)

    def numpy(self):
        return self._a

    def shape(self):
        return list(self._a.shape)

    def is_tensor(self):
        return True

    def device_name(self):
        return "cpu"


def _count(sd, prefix):
    """Distinct block indices under prefix ('audio_encoder.encoders.' -> 49)."""
    return len({k[len(prefix):].split(".", 1)[0] for k in sd if k.startswith(prefix)})


def _config(sd, kind):
    if kind == "encoder":
        cfg = dict(ENC_FULL, ctc_blocks=ENC_TINY["ctc_blocks"], ctc_vocab=ENC_TINY["ctc_vocab"])
        cfg.update(n_blocks=_count(sd, "audio_encoder.encoders0.") + _count(sd, "audio_encoder.encoders."),
                   n_tp_blocks=_count(sd, "audio_encoder.tp_encoders."),
                   adaptor_blocks=_count(sd, "audio_adaptor.blocks."))
        w = sd.get("audio_adaptor.linear2.weight")
        if w is not None:
            cfg["d_llm"] = int(w.shape[0])
    else:
        cfg = dict(ENC_TINY, ctc_blocks=_count(sd, "ctc_decoder.blocks."))
        w = sd.get("ctc_proj.ctc_lo.weight")
        if w is None:
            raise ValueError("CTC graph without ctc_proj.ctc_lo.weight")
        cfg["ctc_vocab"] = int(w.shape[0])
    return cfg


def _arr(v):
    return v.numpy() if isinstance(v, OrtValue) else np.asarray(v)


class InferenceSession:
    def __init__(self, path_or_bytes, sess_options=None, providers=None, provider_options=None, **kwargs):
        if not isinstance(path_or_bytes, (str, os.PathLike)):
            raise TypeError("InferenceSession: pass the model file path (in-memory models are not served)")
        path = os.fspath(path_or_bytes)
        if not os.path.exists(path):
            raise FileNotFoundError(f"[ONNXRuntimeError] : NO_SUCHFILE : Load model from {path} failed. File doesn't exist")
        inits, _ = read_onnx(path)
        sd = state_dict_from_onnx(path)
        if any(k.startswith("audio_encoder.") for k in sd):
            self._kind, groups = "encoder", ENCODER_GROUPS
        elif any(k.startswith("ctc_decoder.") for k in sd):
            self._kind, groups = "ctc", CTC_GROUPS
        else:
            raise ValueError(f"{path}: neither the Fun-ASR encoder-adaptor graph nor its CTC graph")
        self._fp16 = any(a.dtype == np.float16 for a in inits.values())
        self._path, self._options = path, sess_options or SessionOptions()
        self._providers = [PROVIDER, "CPUExecutionProvider"]
        self._cfg = _config(sd, self._kind)
        device = int(os.environ.get("FUNASR_ORT_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        self._eng = _native.Engine(self._cfg, dict(LLM_TINY, n_ctx=64, max_seqs=1), max_batch=1,
                                   max_samples=int(16000 * MAX_SECONDS), device=device)
        try:
            self._eng.synthetic_weights(0)  # the other part of the graph (never run) gets defined values
            self._eng.set_encoder_fp16(self._fp16)
            for g in groups:
                self._eng.mark_unset(g)
            for k, v in sd.items():
                if k.startswith(groups):
                    self._eng.set_tensor(k, v)
            if self._kind == "ctc":  # Fun-ASR-Nano-CTC.int8.onnx: its dynamic-quant weights as stored (int8 graph)
                for k, (q, sc, zp) in u8dq_from_onnx(path, inits).items():
                    if k.startswith(groups):
                        self._eng.set_tensor_u8dq(k, q, sc, zp)
            for g in groups:
                require_loaded(self._eng, g, path)
        except Exception:
            self._eng.close()
            raise
        ft = "tensor(float16)" if self._fp16 else "tensor(float)"
        d, dl = self._cfg["d_model"], self._cfg["d_llm"]
        if self._kind == "encoder":
            self._inputs = [NodeArg("audio", ft, [1, 1, "audio_len"]), NodeArg("ilens", "tensor(int64)", [1])]
            self._outputs = [NodeArg("enc_output", ft, [1, "enc_len", d]), NodeArg("adaptor_output", ft, [1, "enc_len", dl])]
        else:
            self._inputs = [NodeArg("enc_output", ft, [1, "enc_len", d])]
            self._outputs = [NodeArg("indices", "tensor(int32)", [1, "enc_len"])]

    # ---- introspection (nano_onnx.py:54-104)
    def get_inputs(self):
        return list(self._inputs)

    def get_outputs(self):
        return list(self._outputs)

    def get_providers(self):
        return list(self._providers)

    def get_provider_options(self):
        return {p: {} for p in self._providers}

    def get_session_options(self):
        return self._options

    # ---- execution
    def _encoder(self, feed):
        audio = _arr(feed["audio"] if "audio" in feed else feed[self._inputs[0].name])
        if audio.ndim != 3 or audio.shape[0] != 1 or audio.shape[1] != 1:
            raise ValueError(f"audio must be [1, 1, N], got {list(audio.shape)}")
        n_phys = audio.shape[2]
        n = int(_arr(feed["ilens"]).reshape(-1)[0]) if "ilens" in feed else n_phys
        if not 1 <= n <= n_phys:
            raise ValueError(f"ilens {n} outside [1, {n_phys}]")
        pcm = np.ascontiguousarray(audio[0, 0, :n], np.float32)
        r = self._eng.encode([pcm], want_enc=True)
        t_phys = (n_phys // 160 + 1 + 5) // 6  # T_lfr of the padded input (model_definition.py:286-290)
        dt = np.float16 if self._fp16 else np.float32
        enc = np.zeros((1, t_phys, self._cfg["d_model"]), dt)
        rows = r["enc"][0][:t_phys]
        enc[0, :rows.shape[0]] = rows  # frames past the valid ones: zero (the wrapper's final sweep)
        ad = np.zeros((1, t_phys, self._cfg["d_llm"]), dt)
        emb = r["audio_embd"][0][:t_phys]
        ad[0, :emb.shape[0]] = emb  # rows >= target_len: zero (final_output, model_definition.py:306-309)
        return {"enc_output": enc, "adaptor_output": ad}

    def _ctc(self, feed):
        x = _arr(feed["enc_output"] if "enc_output" in feed else feed[self._inputs[0].name])
        if x.ndim != 3 or x.shape[0] != 1 or x.shape[2] != self._cfg["d_model"]:
            raise ValueError(f"enc_output must be [1, T, {self._cfg['d_model']}], got {list(x.shape)}")
        return {"indices": self._eng.ctc_head(x[0].astype(np.float32))[None, :]}

    def run(self, output_names, input_feed, run_options=None):
        out = self._encoder(input_feed) if self._kind == "encoder" else self._ctc(input_feed)
        names = output_names or [o.name for o in self._outputs]
        return [out[nm] for nm in names]

    def run_with_ort_values(self, output_names, input_feed, run_options=None):
        return [OrtValue(a) for a in self.run(output_names, input_feed, run_options)]

    def end_profiling(self):
        return ""

    def __del__(self):
        eng = getattr(self, "_eng", None)
        if eng is not None:
            try:
                eng.close()
            except Exception:
                pass
