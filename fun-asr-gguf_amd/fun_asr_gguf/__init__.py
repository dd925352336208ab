"""fun_asr_gguf (MI355X-native): drop-in for lpyjmj/Fun-ASR-GGUF's Python API on the per-segment hot path.

Exports mirror /root/reference/fun_asr_gguf/__init__.py:49-87. Compute runs in libfunasr_hip.so
(hand-written gfx950 HIP kernels behind a C-ABI, include/funasr_hip.h); there is no CPU fallback.
"""
import logging
import os


def setup_logging(level: int = logging.WARNING, log_file: str = os.path.join("logs", "latest.log")):
    root_logger = logging.getLogger("fun_asr_gguf")
    root_logger.setLevel(logging.DEBUG)
    root_logger.handlers.clear()
    if log_file and os.environ.get("FUNASR_LOG_FILE", "0") == "1":
        d = os.path.dirname(log_file)
        if d:
            os.makedirs(d, exist_ok=True)
        h = logging.FileHandler(log_file, mode="w", encoding="utf-8")
        h.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
        root_logger.addHandler(h)
    return root_logger


logger = setup_logging()

from .asr_engine import FunASREngine, create_asr_engine  # noqa: E402
from .nano_dataclass import (ASREngineConfig, DecodeResult, RecognitionResult, RecognitionStream,  # noqa: E402
                             Statistics, Timings, TranscriptionResult)

__all__ = ["logger", "setup_logging", "FunASREngine", "create_asr_engine", "RecognitionResult", "RecognitionStream",
           "TranscriptionResult", "DecodeResult", "Timings", "ASREngineConfig", "Statistics"]
