"""Public facade: FunASREngine / create_asr_engine with the reference's signatures and defaults
(/root/reference/fun_asr_gguf/asr_engine.py:15-136). Additive keyword arguments only:
device, max_batch, n_ctx, model, synthetic_seed, ignore_eos; transcribe() also accepts a numpy waveform and
ranks= (torch.distributed) for multi-GPU segment sharding; transcribe_batch() decodes many clips at once."""
from typing import List, Optional

from .core.model_manager import ModelManager
from .core.orchestrator import TranscriptionOrchestrator
from .nano_dataclass import ASREngineConfig, DecodeResult, RecognitionStream, TranscriptionResult


class FunASREngine:
    def __init__(self, encoder_onnx_path: str, ctc_onnx_path: str, decoder_gguf_path: str, tokens_path: str,
                 hotwords_path: str = None, enable_ctc: bool = True, n_predict: int = 512, n_threads: int = None,
                 similar_threshold: float = 0.6, max_hotwords: int = 10, **mi355x):
        self.config = ASREngineConfig(encoder_onnx_path=encoder_onnx_path, ctc_onnx_path=ctc_onnx_path,
                                      decoder_gguf_path=decoder_gguf_path, tokens_path=tokens_path,
                                      hotwords_path=hotwords_path, enable_ctc=enable_ctc, n_predict=n_predict,
                                      n_threads=n_threads, similar_threshold=similar_threshold,
                                      max_hotwords=max_hotwords, **mi355x)
        self.models = ModelManager(self.config)
        self.orchestrator = TranscriptionOrchestrator(self.models)
        self.sample_rate = self.config.sample_rate

    def initialize(self, verbose: bool = True) -> bool:
        return self.models.initialize(verbose=verbose)

    def transcribe(self, audio_path, language: Optional[str] = None, context: Optional[str] = None,
                   verbose: bool = True, segment_size: float = 60.0, overlap: float = 2.0,
                   start_second: Optional[float] = None, duration: Optional[float] = None, srt: bool = False,
                   temperature: float = 0.4, top_p: float = 1.0, top_k: int = 50, ranks=None) -> TranscriptionResult:
        return self.orchestrator.transcribe(audio_path, language=language, context=context, verbose=verbose,
                                            segment_size=segment_size, overlap=overlap, start_second=start_second,
                                            duration=duration, srt=srt, temperature=temperature, top_p=top_p,
                                            top_k=top_k, ranks=ranks)

    def transcribe_batch(self, clips: List, language=None, context=None, temperature: float = 0.4, top_p=1.0,
                         top_k=50, ranks=None) -> Optional[List[DecodeResult]]:
        """Many independent clips (each <= segment_size + 2 s) as encoder batches + one decoder batch.
        ranks (an initialised torch.distributed): the clips are assigned longest-first across the ranks, every rank
        decodes its share, results are gathered to rank 0 (the list there, None on the other ranks)."""
        from .audio import load_audio
        pcm = [load_audio(c, self.sample_rate) for c in clips]
        if ranks is not None:
            from .parallel import sharded_decode
            return sharded_decode(self.orchestrator, pcm, language, context, False, temperature, top_p, top_k, ranks)
        return self.orchestrator.decode_segments(pcm, language, context, False, temperature, top_p, top_k)

    def create_stream(self, hotwords: Optional[str] = None) -> RecognitionStream:
        return RecognitionStream(sample_rate=self.sample_rate)

    def decode_stream(self, stream: RecognitionStream, language: Optional[str] = None, context: Optional[str] = None,
                      verbose: bool = True, reporter=None, temperature: float = 0.3, top_p: float = 1.0,
                      top_k: int = 50) -> DecodeResult:
        return self.orchestrator.decoder.decode_stream(stream, language, context, verbose, reporter,
                                                       temperature=temperature, top_p=top_p, top_k=top_k)

    def cleanup(self):
        self.models.cleanup()


def create_asr_engine(encoder_onnx_path: str, ctc_onnx_path: str, decoder_gguf_path: str, tokens_path: str,
                      hotwords_path: str = None, enable_ctc: bool = True, similar_threshold: float = 0.6,
                      max_hotwords: int = 10, verbose: bool = True, **mi355x) -> FunASREngine:
    engine = FunASREngine(encoder_onnx_path=encoder_onnx_path, ctc_onnx_path=ctc_onnx_path,
                          decoder_gguf_path=decoder_gguf_path, tokens_path=tokens_path, hotwords_path=hotwords_path,
                          enable_ctc=enable_ctc, similar_threshold=similar_threshold, max_hotwords=max_hotwords,
                          **mi355x)
    if not engine.initialize(verbose=verbose):
        raise RuntimeError("Failed to initialize ASR engine")
    return engine
