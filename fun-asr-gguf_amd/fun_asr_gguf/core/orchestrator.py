"""Short/long strategy, segmentation and merge (TranscriptionOrchestrator,
/root/reference/fun_asr_gguf/core/orchestrator.py:20-189).

Long audio is cut into [t, t+segment) windows with step segment-overlap (:123-136). The reference decodes
them one after another; here the segments of one file decode together on the engine's sequence slots with continuous
batching (core/scheduler.py), or are sharded across ranks by fun_asr_gguf.parallel. Results are merged
with the same difflib rule (text_merge.py). timings.total excludes audio loading (:62, :72).
"""
import os
import time
from typing import Optional

import numpy as np

from ..audio import load_audio
from ..nano_dataclass import RecognitionStream, TranscriptionResult
from ..srt_utils import generate_srt_file
from ..text_merge import merge_transcription_results
from .decoder import StreamDecoder

TIMING_FIELDS = ("encode", "ctc", "prepare", "inject", "llm_generate", "align", "ctc_infer", "ctc_decode",
                 "hotword_verify", "ctc_cast", "ctc_argmax", "ctc_loop")


def segment_windows(duration, segment_size, overlap):
    out, step, cur = [], segment_size - overlap, 0.0
    while cur < duration:
        end = min(cur + segment_size, duration)
        out.append((cur, end))
        if end >= duration:
            break
        cur += step
    return out


def segment_results_entry(d_res, duration):
    return {"text": d_res.text, "segments": d_res.aligned, "duration": duration, "hotwords": d_res.hotwords,
            "ctc_text": "".join(r.text for r in d_res.ctc_results) if d_res.ctc_results else ""}


class TranscriptionOrchestrator:
    def __init__(self, models):
        self.models = models
        self.decoder = StreamDecoder(models)

    def transcribe(self, audio_path, language=None, context=None, verbose=True, segment_size=60.0, overlap=2.0,
                   start_second=None, duration=None, srt=False, temperature=0.3, top_p=1.0, top_k=50,
                   ranks=None) -> TranscriptionResult:
        result = TranscriptionResult()
        sr = self.models.config.sample_rate
        t = time.perf_counter()
        audio = load_audio(audio_path, sr, start_second=start_second, duration=duration)
        result.timings.load_audio = time.perf_counter() - t
        base = start_second if start_second else 0.0
        dur = len(audio) / sr
        t_proc = time.perf_counter()
        if dur <= segment_size + 2.0:
            self._short(audio, result, language, context, verbose, base, temperature, top_p, top_k)
        else:
            self._long(audio, result, language, context, verbose, segment_size, overlap, base, temperature, top_p,
                       top_k, ranks)
        result.timings.total = time.perf_counter() - t_proc
        if srt and result.segments and isinstance(audio_path, (str, os.PathLike)):
            generate_srt_file(result.segments, os.path.splitext(str(audio_path))[0] + ".srt")
        if verbose and result.text:
            print(result.text)
        return result

    def _short(self, audio, result, language, context, verbose, base, temperature, top_p, top_k):
        st = RecognitionStream()
        st.accept_waveform(self.models.config.sample_rate, audio)
        d = self.decoder.decode_stream(st, language, context, verbose, None, temperature, top_p, top_k)
        for f in TIMING_FIELDS:
            setattr(result.timings, f, getattr(d.timings, f))
        result.text = d.text
        result.segments = [{"char": s["char"], "start": s["start"] + base} for s in (d.aligned or [])]
        result.hotwords = d.hotwords
        if d.ctc_results:
            result.ctc_text = "".join(r.text for r in d.ctc_results)

    def decode_segments(self, chunks, language, context, verbose, temperature, top_p, top_k, n_predicts=None):
        """Decode a list of PCM chunks with continuous batching over the engine's max_batch sequence slots
        (core/scheduler.py: a finished sequence's slot is refilled with the next waiting chunk); -> [DecodeResult]
        in input order."""
        from .scheduler import ContinuousBatcher
        if not chunks:
            return []
        self.batcher = ContinuousBatcher(self.decoder)
        return self.batcher.run(chunks, language, context, temperature, top_p, top_k, n_predicts=n_predicts)

    def _long(self, audio, result, language, context, verbose, segment_size, overlap, base, temperature, top_p,
              top_k, ranks):
        sr = self.models.config.sample_rate
        dur = len(audio) / sr
        wins = segment_windows(dur, segment_size, overlap)
        chunks = [audio[int(s * sr):int(e * sr)] for s, e in wins]
        if ranks is not None:
            from ..parallel import sharded_decode
            d_results = sharded_decode(self, chunks, language, context, verbose, temperature, top_p, top_k, ranks)
        else:
            d_results = self.decode_segments(chunks, language, context, verbose, temperature, top_p, top_k)
        if d_results is None:  # non-root rank
            return
        seg_results = []
        for (s, e), d in zip(wins, d_results):
            seg_results.append(segment_results_entry(d, e - s))
            for f in TIMING_FIELDS:
                setattr(result.timings, f, getattr(result.timings, f) + getattr(d.timings, f))
        text, segs = merge_transcription_results(seg_results, [s + base for s, _ in wins], overlap)
        result.text, result.segments = text, segs
        hw = set()
        for r in seg_results:
            hw.update(r["hotwords"])
        result.hotwords = list(hw)
        result.ctc_text = "".join(r["ctc_text"] for r in seg_results if r["ctc_text"])
