"""Engine initialisation (ModelManager.initialize, /root/reference/fun_asr_gguf/core/model_manager.py:36-100).

Creates the device-bound native engine and fills its weights:
  * "synthetic" -> the repo's deterministic synthetic weights (oracle/synth.py spec);
  * encoder/CTC: the reference's ONNX files (fun_asr_gguf.onnx_weights: initializers of
    Fun-ASR-Nano-Encoder-Adaptor.*.onnx and Fun-ASR-Nano-CTC.*.onnx), or a PyTorch/safetensors state dict
    (model.pt keys audio_encoder.*, audio_adaptor.*, ctc_decoder.*, ctc.ctc_lo.* -> ctc_proj.ctc_lo.*, as
    HybridSenseVoice.load_weights, model_definition.py:231-238), loaded with weights_only=True;
  * decoder: a GGUF file (q8_0/f16/f32 tensors + tokenizer metadata) through fa_load_gguf.
Any failure returns False (the reference swallows init exceptions the same way, :98-100): a model path that does
not exist, and a model file that leaves any tensor of its part of the graph unfilled (the engine keeps a per-tensor
loaded mark: fa_weights_mark_unset / fa_tensor_names), are failures, never a silent synthetic fallback.
"""
import logging
import os
import time

from .. import _native
from ..model_config import MODELS
from ..nano_ctc import load_ctc_tokens
from ..prompt_utils import PromptBuilder
from ..vocab import CTCSyntheticTokens, GGUFVocab, SyntheticVocab

log = logging.getLogger("fun_asr_gguf")


def _is_synthetic(p):
    return p is None or str(p).startswith("synthetic")


ENCODER_GROUPS = ("audio_encoder.", "audio_adaptor.")
CTC_GROUPS = ("ctc_decoder.", "ctc_proj.")
LLM_GROUPS = ("token_embd.", "blk.", "output_norm.")


def state_dict_file(path):
    """model.pt / safetensors -> {engine tensor name: f32 array} for the encoder, adaptor and CTC parts
    (HybridSenseVoice state_dict keys; ctc.ctc_lo.* -> ctc_proj.ctc_lo.*). torch.load with weights_only=True."""
    if str(path).endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(path)
    else:
        import torch
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if "state_dict" in sd:
            sd = sd["state_dict"]
        sd = {k: v.float().numpy() for k, v in sd.items() if hasattr(v, "float")}
    out = {}
    for k, v in sd.items():
        if k.startswith(ENCODER_GROUPS + ("ctc_decoder.",)):
            out[k] = v
        elif k.startswith("ctc.ctc_lo."):
            out[k.replace("ctc.ctc_lo", "ctc_proj.ctc_lo")] = v
    if not out:
        raise ValueError(f"{path}: no encoder / adaptor / CTC tensors found")
    return out


def onnx_state_dict(path):
    """Initializers of an encoder-adaptor or CTC ONNX file (onnx_weights.state_dict_from_onnx)."""
    from ..onnx_weights import state_dict_from_onnx
    sd = state_dict_from_onnx(path)
    if not sd:
        raise ValueError(f"{path}: no encoder / adaptor / CTC initializers found")
    return sd


def require_loaded(engine, prefix, path):
    """Raise naming the tensors under `prefix` that the model file at `path` left unfilled."""
    missing = engine.tensor_names(prefix, only_unset=True)
    if missing:
        shown = ", ".join(missing[:8]) + (f", ... ({len(missing)} in all)" if len(missing) > 8 else "")
        log.error("%s does not fill %d %s* tensors: %s", path, len(missing), prefix, shown)
        raise ValueError(f"{path}: model file does not hold {len(missing)} tensor(s) under '{prefix}': {shown}")


class ModelManager:
    def __init__(self, config):
        self.config = config
        self.engine = None
        self.vocab = None
        self.eos_token = None
        self.ctc_id2token = None
        self.prompt_builder = None
        self.hotwords = []
        self.hotword_source = None
        self.enc_cfg = None
        self.llm_cfg = None
        self._initialized = False

    def initialize(self, verbose=True):
        if self._initialized:
            return True
        try:
            t0 = time.perf_counter()
            c = self.config
            for role, p in (("encoder", c.encoder_onnx_path), ("ctc", getattr(c, "ctc_onnx_path", None)),
                            ("decoder", c.decoder_gguf_path), ("tokens", c.tokens_path)):
                if not _is_synthetic(p) and not os.path.exists(str(p)):
                    raise FileNotFoundError(f"{role} model file not found: {p}")
            enc_cfg, llm_cfg = MODELS[c.model]
            self.enc_cfg = dict(enc_cfg)
            self.llm_cfg = dict(llm_cfg, n_ctx=c.n_ctx, max_seqs=max(1, c.max_batch))
            gguf_kv = None
            if not _is_synthetic(c.decoder_gguf_path):
                from ..vocab import read_gguf_metadata
                gguf_kv = read_gguf_metadata(c.decoder_gguf_path)
                self.llm_cfg["n_vocab"] = len(gguf_kv["tokenizer.ggml.tokens"])
            # segments up to segment_size + 2 s (orchestrator short path) fit one encode
            self.engine = _native.Engine(self.enc_cfg, self.llm_cfg, max_batch=max(1, c.max_batch),
                                         max_samples=c.sample_rate * 64, device=c.device)
            self.engine.synthetic_weights(c.synthetic_seed)
            self.engine.set_encoder_fp16(c.encoder_fp16())
            # encoder/adaptor + CTC weights: the reference's ONNX files (initializers read without `onnx`), or a
            # model.pt / safetensors state dict (HybridSenseVoice.load_weights, model_definition.py:231-238).
            # Fail loudly like the reference (a missing file makes the ORT session raise, model_manager.py:98-100):
            # a path that does not exist, or a file that leaves any tensor of its part of the graph unfilled.
            expect = []
            for role, p in (("encoder", c.encoder_onnx_path), ("ctc", getattr(c, "ctc_onnx_path", None))):
                if _is_synthetic(p):
                    continue
                groups = ENCODER_GROUPS if role == "encoder" else CTC_GROUPS
                if str(p).endswith(".onnx"):
                    sd = onnx_state_dict(p)
                else:
                    sd = state_dict_file(p)
                if role == "encoder" and any(k.startswith(CTC_GROUPS) for k in sd):
                    groups = groups + CTC_GROUPS  # one model.pt holds the whole HybridSenseVoice
                for g in groups:
                    self.engine.mark_unset(g)
                for k, v in sd.items():
                    self.engine.set_tensor(k, v)
                if role == "ctc" and str(p).endswith(".onnx"):
                    # Fun-ASR-Nano-CTC.int8.onnx (the README's default CTC model): its weights as stored, so the CTC
                    # head runs the int8-dynamic graph's arithmetic rather than an f32 graph of dequantised weights
                    from ..onnx_weights import u8dq_from_onnx
                    for k, (q, sc, zp) in u8dq_from_onnx(p).items():
                        if k.startswith(CTC_GROUPS):
                            self.engine.set_tensor_u8dq(k, q, sc, zp)
                expect += [(g, p) for g in groups]
            for g, p in expect:
                require_loaded(self.engine, g, p)
            if gguf_kv is not None:
                for g in LLM_GROUPS:
                    self.engine.mark_unset(g)
                self.engine.load_gguf(c.decoder_gguf_path)
                for g in LLM_GROUPS:
                    require_loaded(self.engine, g, c.decoder_gguf_path)
                self.vocab = GGUFVocab(c.decoder_gguf_path)
            else:
                self.vocab = SyntheticVocab(self.llm_cfg["n_vocab"])
            self.eos_token = self.vocab.eos
            if _is_synthetic(c.tokens_path):
                self.ctc_id2token = CTCSyntheticTokens(self.enc_cfg["ctc_vocab"])
            else:
                self.ctc_id2token = load_ctc_tokens(c.tokens_path)  # raises on a missing file (nano_ctc.py:12-36)
            self.prompt_builder = PromptBuilder(self.vocab, self.engine)
            if c.hotwords_path and os.path.exists(c.hotwords_path):
                # phoneme hotword retrieval (hotword/manager.py + hot_phoneme.py), reloaded when hot.txt changes
                from ..hotword import HotwordSource
                self.hotword_source = HotwordSource(c.hotwords_path, c.similar_threshold)
                self.hotwords = list(self.hotword_source.corrector.hotwords)
            self._initialized = True
            if verbose:
                print(f"✓ 模型加载完成 (耗时: {time.perf_counter() - t0:.2f}s)")
            return True
        except Exception as e:  # same contract as the reference: report and return False
            log.exception("initialize failed")
            if self.engine is not None:  # a half-initialised engine would hold its HBM until process exit
                self.engine.close()
                self.engine = None
            if verbose:
                print(f"✗ 初始化失败: {e}")
            return False

    def match_hotwords(self, ctc_text, k):
        """CTCDecoder.decode's hotword step (decoder.py:39-44): PhonemeCorrector.correct(ctc_text, k) -> the
        hotwords of its matches and similars (fun_asr_gguf.hotword)."""
        if self.hotword_source is None or not ctc_text:
            return []
        return self.hotword_source.hotwords_for(ctc_text, k)

    def cleanup(self):
        if self.engine is not None:
            self.engine.close()
        self.engine = None
        self._initialized = False
