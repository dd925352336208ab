"""Result / config / timing types of the public API.

Field names, defaults and semantics mirror /root/reference/fun_asr_gguf/nano_dataclass.py
(RecognitionResult :22-33, RecognitionStream :36-77, Timings :80-109, TranscriptionResult :112-127,
ASREngineConfig :132-165, CTCResult :170-184, Statistics :189-221, DecodeResult :224-249,
LLMDecodeResult :252-268). Additive fields only (marked "MI355X").
"""
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np


@dataclass
class RecognitionResult:
    """sherpa-onnx style result: text, per-char start times (s), per-char tokens."""
    text: str = ""
    timestamps: List[float] = field(default_factory=list)
    tokens: List[str] = field(default_factory=list)


@dataclass
class RecognitionStream:
    """sherpa-onnx style stream carrying one waveform (float32, 16 kHz)."""
    sample_rate: int = 16000
    audio_data: Optional[np.ndarray] = None
    _result: Optional[RecognitionResult] = field(default=None, init=False, repr=False)

    def accept_waveform(self, sample_rate: int, audio: np.ndarray):
        self.sample_rate = sample_rate
        self.audio_data = np.asarray(audio).astype(np.float32)

    @property
    def result(self) -> RecognitionResult:
        if self._result is None:
            self._result = RecognitionResult()
        return self._result

    def set_result(self, text: str, timestamps: List[float] = None, tokens: List[str] = None):
        self._result = RecognitionResult(text=text, timestamps=timestamps or [], tokens=tokens or [])


@dataclass
class Timings:
    """Stage wall times in seconds (filled from host timers around device-synchronising calls)."""
    encode: float = 0.0
    load_audio: float = 0.0
    ctc: float = 0.0
    prepare: float = 0.0
    inject: float = 0.0
    llm_generate: float = 0.0
    align: float = 0.0
    total: float = 0.0
    ctc_infer: float = 0.0
    ctc_decode: float = 0.0
    ctc_cast: float = 0.0
    ctc_argmax: float = 0.0
    ctc_loop: float = 0.0
    hotword_verify: float = 0.0


@dataclass
class TranscriptionResult:
    text: str = ""
    segments: List[Dict[str, Any]] = field(default_factory=list)
    ctc_text: str = ""
    hotwords: List[str] = field(default_factory=list)
    timings: Timings = field(default_factory=Timings)


@dataclass
class ASREngineConfig:
    encoder_onnx_path: str
    ctc_onnx_path: str
    decoder_gguf_path: str
    tokens_path: str
    hotwords_path: Optional[str] = None
    enable_ctc: bool = True
    n_predict: int = 512
    n_threads: Optional[int] = None
    n_threads_batch: Optional[int] = None
    n_ubatch: int = 512
    similar_threshold: float = 0.6
    max_hotwords: int = 10
    sample_rate: int = 16000
    # MI355X additions
    device: int = 0
    max_batch: int = 1
    n_ctx: int = 2048
    model: str = "full"            # "full" (Fun-ASR-Nano dims) or "tiny" (test dims)
    synthetic_seed: int = 0
    ignore_eos: bool = False       # benchmark protocol: pin the decode length (no stop tokens, no breaker)
    # encoder graph precision: "auto" follows the reference's file naming (*.fp16.onnx -> the float16 graph of
    # 02-Quantize-ONNX.py; anything else fp32), or "fp32" / "fp16" explicitly
    encoder_precision: str = "auto"

    def encoder_fp16(self) -> bool:
        if self.encoder_precision in ("fp16", "fp32"):
            return self.encoder_precision == "fp16"
        if self.encoder_precision != "auto":
            raise ValueError(f"encoder_precision must be auto, fp32 or fp16, not {self.encoder_precision!r}")
        return ".fp16." in os.path.basename(str(self.encoder_onnx_path))


@dataclass
class CTCResult:
    text: str
    start: float
    end: float
    score: float = 1.0


@dataclass
class Statistics:
    audio_duration: float = 0.0
    n_input_tokens: int = 0
    n_prefix_tokens: int = 0
    n_audio_tokens: int = 0
    n_suffix_tokens: int = 0
    n_generated_tokens: int = 0
    tps_in: float = 0.0
    tps_out: float = 0.0

    def __str__(self) -> str:
        return (f"  音频长度: {self.audio_duration:6.2f}s\n"
                f"  Decoder输入: {self.tps_in:6.0f} tokens/s (总: {self.n_input_tokens}, prefix:{self.n_prefix_tokens}, "
                f"audio:{self.n_audio_tokens}, suffix:{self.n_suffix_tokens})\n"
                f"  Decoder输出: {self.tps_out:6.0f} tokens/s (总: {self.n_generated_tokens})")


@dataclass
class DecodeResult:
    text: str = ""
    ctc_results: List = field(default_factory=list)
    aligned: List[Dict[str, Any]] = field(default_factory=list)
    audio_embd: Optional[np.ndarray] = None
    n_prefix: int = 0
    n_suffix: int = 0
    n_gen: int = 0
    timings: Timings = field(default_factory=Timings)
    hotwords: List[str] = field(default_factory=list)
    is_aborted: bool = False


@dataclass
class LLMDecodeResult:
    text: str = ""
    n_gen: int = 0
    t_inject: float = 0.0
    t_gen: float = 0.0
    is_aborted: bool = False


__all__ = ["RecognitionResult", "RecognitionStream", "TranscriptionResult", "DecodeResult", "LLMDecodeResult",
           "ASREngineConfig", "Timings", "CTCResult", "Statistics"]
