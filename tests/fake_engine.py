"""Host stand-in for fun_asr_gguf._native.Engine (no GPU): the surface StreamDecoder / TranscriptionOrchestrator use
(encode, ctc_collapse, embd_rows, llm_reset / llm_prefill(_batch) / llm_generate), deterministic in each clip's own samples
and independent of how clips are batched, so a sharded run must equal a single-rank run exactly. Lets the real
orchestration code (windows, LPT sharding, record gather, merge) run in multi-process CPU tests."""
import numpy as np

from fun_asr_gguf.core.model_manager import ModelManager
from fun_asr_gguf.nano_dataclass import ASREngineConfig
from fun_asr_gguf.prompt_utils import PromptBuilder
from fun_asr_gguf.vocab import CTCSyntheticTokens, SyntheticVocab

N_VOCAB, CTC_VOCAB = 4096, 3001


def _frames(n):
    return ((max(n, 16000) // 160 + 1) + 5) // 6


class FakeEngine:
    """max_seqs: slot range like the native engine's KV cache ('seq out of range' beyond it). loop_below: sampling
    temperatures below it emit one repeated token (the repetition breaker cuts such a decode), like a looping model."""

    def __init__(self, max_seqs=None, loop_below=None):
        self.last = []
        self.seqs = {}
        self.max_seqs = max_seqs
        self.loop_below = loop_below

    def _slot(self, s):
        if self.max_seqs is not None and not 0 <= s < self.max_seqs:
            raise RuntimeError(f"fa_llm_reset: seq out of range ({s} of {self.max_seqs})")

    def encode(self, clips, want_enc=False, resident=None, independent=False):
        self._idle("encode")
        self.n_encodes = getattr(self, "n_encodes", 0) + 1
        self.last = [np.asarray(c, np.float32) for c in clips]
        out = dict(audio_embd=[], ctc_ids=[])
        for c in self.last:
            T = _frames(len(c))
            frames = np.resize(c, T * 160)[: T * 160].reshape(T, 160)
            key = (np.abs(frames).sum(1) * 1e4).astype(np.int64)
            ids = np.where(key % 3 == 0, CTC_VOCAB - 1, key % 50).astype(np.int32)  # blanks + 50 symbols
            tgt = max(1, T // 8)
            out["audio_embd"].append(np.full((tgt, 1024), float(key.sum() % 97) / 97, np.float32))
            out["ctc_ids"].append(ids)
        return out

    def ctc_collapse(self, blank, B):
        res = []
        for c in self.last[:B]:
            ids = self.encode_ids(c)
            keep = [(int(t), i) for i, t in enumerate(ids) if t != blank and (i == 0 or t != ids[i - 1])]
            res.append((np.array([k for k, _ in keep], np.int32), np.array([f for _, f in keep], np.int32)))
        return res

    def encode_ids(self, c):
        T = _frames(len(c))
        frames = np.resize(c, T * 160)[: T * 160].reshape(T, 160)
        key = (np.abs(frames).sum(1) * 1e4).astype(np.int64)
        return np.where(key % 3 == 0, CTC_VOCAB - 1, key % 50)

    def embd_rows(self, ids, fp16_round=True):
        return np.repeat(np.asarray(ids, np.float32)[:, None] / N_VOCAB, 1024, 1)

    def llm_reset(self, s):
        self._idle("llm_reset")
        self._slot(s)
        self.seqs.pop(s, None)

    def llm_prefill(self, s, embd, **samp):
        self._idle("llm_prefill")
        self._slot(s)
        h = int(np.abs(embd).sum() * 1000) % 100003
        self.seqs[s] = h
        return 1000 + h % 20

    def llm_prefill_batch(self, seqs, embds, **samp):
        return [self.llm_prefill(s, e, **samp) for s, e in zip(seqs, embds)]

    def llm_generate(self, seqs, n, **samp):
        out = np.zeros((len(seqs), n), np.int32)
        for r, s in enumerate(seqs):
            self._slot(s)
            if self.loop_below is not None and samp.get("temperature", 0.0) < self.loop_below:
                out[r, :] = 1000
                continue
            for k in range(n):
                self.seqs[s] = (self.seqs[s] * 1103515245 + 12345) % 2147483647
                out[r, k] = 1000 + self.seqs[s] % 40
        return out

    def llm_generate_begin(self, seqs, n, **samp):
        self._idle("llm_generate_begin")
        self._pending = self.llm_generate(seqs, n, **samp)
        self.max_width = max(getattr(self, "max_width", 0), len(seqs))

    def llm_generate_end(self):
        if getattr(self, "_pending", None) is None:
            raise RuntimeError("no generate call in flight")
        out, self._pending = self._pending, None
        return out

    def _idle(self, what):
        # the native engine refuses every other decoder call while a generate call is in flight
        if getattr(self, "_pending", None) is not None:
            raise RuntimeError(f"{what}: a generate call is in flight")


def fake_models(max_batch=4, n_predict=24, ignore_eos=True, loop_below=None):
    cfg = ASREngineConfig(encoder_onnx_path="synthetic", ctc_onnx_path="synthetic", decoder_gguf_path="synthetic",
                          tokens_path="synthetic", n_predict=n_predict, max_batch=max_batch, ignore_eos=ignore_eos)
    m = ModelManager(cfg)
    m.engine = FakeEngine(max_seqs=max_batch, loop_below=loop_below)
    m.vocab = SyntheticVocab(N_VOCAB)
    m.eos_token = m.vocab.eos
    m.ctc_id2token = CTCSyntheticTokens(CTC_VOCAB)
    m.prompt_builder = PromptBuilder(m.vocab, m.engine)
    m._initialized = True
    return m


def fake_api(max_batch=4, n_predict=24, ignore_eos=True, loop_below=None):
    from fun_asr_gguf import FunASREngine
    api = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=n_predict, max_batch=max_batch,
                       ignore_eos=ignore_eos)
    m = fake_models(max_batch, n_predict, ignore_eos, loop_below)
    api.models = m
    api.orchestrator.models = m
    api.orchestrator.decoder.models = m
    api.orchestrator.decoder.llm_decoder.models = m
    return api
