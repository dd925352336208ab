"""Engine initialisation (ModelManager.initialize, /root/reference/fun_asr_gguf/core/model_manager.py:36-100).

Creates the device-bound native engine and fills its weights:
  * "synthetic" (or a missing path) -> the repo's deterministic synthetic weights (oracle/synth.py spec);
  * encoder/CTC: the reference's ONNX files (fun_asr_gguf.onnx_weights: initializers of
    Fun-ASR-Nano-Encoder-Adaptor.*.onnx and Fun-ASR-Nano-CTC.*.onnx), or a PyTorch/safetensors state dict
    (model.pt keys audio_encoder.*, audio_adaptor.*, ctc_decoder.*, ctc.ctc_lo.* -> ctc_proj.ctc_lo.*, as
    HybridSenseVoice.load_weights, model_definition.py:231-238), loaded with weights_only=True;
  * decoder: a GGUF file (q8_0/f16/f32 tensors + tokenizer metadata) through fa_load_gguf.
Any failure returns False (the reference swallows init exceptions the same way, :98-100).
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


def load_encoder_state_dict(engine, path):
    if str(path).endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(path)
    else:
        import torch
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if "state_dict" in sd:
            sd = sd["state_dict"]
        sd = {k: v.float().numpy() for k, v in sd.items() if hasattr(v, "float")}
    n = 0
    for k, v in sd.items():
        if k.startswith(("audio_encoder.", "audio_adaptor.", "ctc_decoder.")):
            name = k
        elif k.startswith("ctc.ctc_lo."):
            name = k.replace("ctc.ctc_lo", "ctc_proj.ctc_lo")
        else:
            continue
        engine.set_tensor(name, v)
        n += 1
    return n


def load_encoder_onnx(engine, path):
    """Initializers of an encoder-adaptor or CTC ONNX file (onnx_weights.state_dict_from_onnx) -> engine tensors."""
    from ..onnx_weights import state_dict_from_onnx
    sd = state_dict_from_onnx(path)
    if not sd:
        raise ValueError(f"{path}: no encoder / adaptor / CTC initializers found")
    for k, v in sd.items():
        engine.set_tensor(k, v)
    return len(sd)


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
            # model.pt / safetensors state dict (HybridSenseVoice.load_weights, model_definition.py:231-238)
            for p in (c.encoder_onnx_path, getattr(c, "ctc_onnx_path", None)):
                if _is_synthetic(p) or not os.path.exists(str(p)):
                    continue
                if str(p).endswith(".onnx"):
                    load_encoder_onnx(self.engine, p)
                else:
                    load_encoder_state_dict(self.engine, p)
            if gguf_kv is not None:
                self.engine.load_gguf(c.decoder_gguf_path)
                self.vocab = GGUFVocab(c.decoder_gguf_path)
            else:
                self.vocab = SyntheticVocab(self.llm_cfg["n_vocab"])
            self.eos_token = self.vocab.eos
            if _is_synthetic(c.tokens_path) or not os.path.exists(c.tokens_path):
                self.ctc_id2token = CTCSyntheticTokens(self.enc_cfg["ctc_vocab"])
            else:
                self.ctc_id2token = load_ctc_tokens(c.tokens_path)
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
