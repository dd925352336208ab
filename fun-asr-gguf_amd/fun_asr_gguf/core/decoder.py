"""Per-segment hot path: encode -> CTC -> prompt -> LLM -> align
(StreamDecoder.decode_stream, /root/reference/fun_asr_gguf/core/decoder.py:132-246).

Differences in *mechanism* only (results are the reference's):
  * encoder + CTC head + CTC argmax + greedy collapse run on the GPU in one fa_encode call;
  * the LLM loop samples on the device and returns tokens in chunks (no per-token host round trip);
    stop / repetition-breaker decisions are then replayed on the host in token order exactly as the
    reference's loop takes them (decoder.py:91-114), so tokens the device produced after a stop are
    discarded and never reach the output;
  * decode_streams() runs several segments as one encoder batch + one continuous decoder batch.
"""
import codecs
import time
from typing import List, Optional

import numpy as np

from concurrent.futures import Future, ThreadPoolExecutor

from ..nano_ctc import align_timestamps, ctc_pair_rows, tokens_of
from ..nano_dataclass import DecodeResult, LLMDecodeResult, RecognitionStream, Timings

STOP_TOKENS = (151643, 151645)          # decoder.py:53
ABORT_MARK = "====解码有误，强制熔断===="   # decoder.py:210
GEN_CHUNK = 32


class PieceStream:
    """ASRStreamDecoder (llama.py:661-690): incremental UTF-8 decode of token pieces."""

    def __init__(self, vocab, reporter=None):
        self.vocab = vocab
        self.reporter = reporter
        self.dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
        self.generated_text = ""
        self.tokens_generated = 0
        self.tokens = []

    def push(self, tid):
        piece = self.dec.decode(self.vocab.token_to_bytes(tid), final=False)
        self.tokens.append(piece)
        self.tokens_generated += 1
        self.generated_text += piece
        if self.reporter:
            self.reporter.stream(piece)
        return piece

    def flush(self):
        rem = self.dec.decode(b"", final=True)
        self.tokens.append(rem)
        self.generated_text += rem
        return rem


class _SeqState:
    def __init__(self, vocab, n_predict, eos, ignore_eos, reporter):
        self.ps = PieceStream(vocab, reporter)
        self.n_predict = n_predict
        self.eos = eos
        self.ignore_eos = ignore_eos
        self.sampled = 0
        self.done = False
        self.aborted = False

    def feed(self, tokens):
        for t in tokens:
            if self.done:
                return
            self.sampled += 1
            t = int(t)
            if not self.ignore_eos and (t == self.eos or t in STOP_TOKENS):
                self.done = True
                return
            self.ps.push(t)
            # pinned-length benchmark protocol (ignore_eos) also disables the repetition breaker: synthetic
            # weights loop by construction and the protocol fixes the decode length
            if not self.ignore_eos and len(self.ps.tokens) > 30 and len(set(self.ps.tokens[-30:])) <= 3:
                self.aborted = True
                self.done = True
                return
            if self.sampled >= self.n_predict:
                self.done = True

    def remaining(self):
        return 0 if self.done else self.n_predict - self.sampled


def invariant_width(eng):
    """Largest decode batch width whose tokens equal decoding each sequence alone (fa_llm_invariant_width)."""
    f = getattr(eng, "llm_invariant_width", None)
    return f() if f is not None else 1


class PromptRows:
    """One prompt, [prefix rows | audio rows | suffix rows], whose audio rows are the adaptor output of clip `clip` of
    the engine's encode generation `enc_gen`, still in HBM. The reference concatenates the three on the host
    (core/decoder.py:199: np.concatenate([p_embd, audio_embd.astype(np.float32), s_embd])); prefill_group has the
    engine assemble them on the device instead (fa_llm_prefill_rows: no host concatenation, no upload of the audio
    rows), bit for bit the same rows. np.asarray(prompt) is that concatenation (the host path, e.g. after another
    encode replaced the rows)."""
    __slots__ = ("pre", "audio", "suf", "clip", "enc_gen")

    def __init__(self, pre, audio, suf, clip, enc_gen):
        self.pre, self.audio, self.suf, self.clip, self.enc_gen = pre, audio, suf, int(clip), int(enc_gen)

    @property
    def n_audio(self):
        return len(self.audio)

    @property
    def shape(self):
        return (len(self.pre) + len(self.audio) + len(self.suf), self.audio.shape[1])

    def __len__(self):
        return self.shape[0]

    def __array__(self, dtype=None, copy=None):
        a = np.concatenate([self.pre, np.asarray(self.audio, np.float32), self.suf], 0)
        return a if dtype is None else a.astype(dtype, copy=False)


def prefill_group(eng, seqs, embds, samp):
    """Prefill `embds` into slots `seqs` -> first tokens. One prompt: llama_decode of its batch. Several: their
    prompts share forwards (one weight pass per forward, fa_llm_prefill_batch); within the engine's invariant width
    that batch is row-local, so every sequence gets exactly its single-sequence prefill (the reference decodes every
    segment alone, core/decoder.py:70-123); wider groups agree to the q8_0 noise floor. PromptRows of the encode the
    engine still holds are assembled on the device (fa_llm_prefill_rows), with the same results."""
    if all(isinstance(e, PromptRows) for e in embds) and hasattr(eng, "llm_prefill_rows") \
            and len({e.enc_gen for e in embds}) == 1 and embds[0].enc_gen == eng.encode_generation():
        return eng.llm_prefill_rows(list(seqs), embds, **samp)
    embds = [np.asarray(e, np.float32) for e in embds]
    if len(embds) == 1:
        return [eng.llm_prefill(seqs[0], embds[0], **samp)]
    return eng.llm_prefill_batch(list(seqs), embds, **samp)


class LLMDecoder:
    def __init__(self, models):
        self.models = models

    def _sampling(self, temperature, top_p, top_k):
        seed = int(np.random.randint(0, 2 ** 31 - 1))  # decoder.py:89: fresh seed per call
        return dict(temperature=temperature, top_p=top_p, top_k=top_k, seed=seed)

    def slot_capacity(self):
        """Sequence slots of the engine (its KV cache holds max_seqs sequences; a host stand-in: config.max_batch)."""
        eng = self.models.engine
        cap = getattr(eng, "llm_cfg", None)
        cap = cap.get("max_seqs") if isinstance(cap, dict) else getattr(eng, "max_seqs", None)
        if not cap:
            cap = getattr(getattr(self.models, "config", None), "max_batch", None)
        return max(1, int(cap or 1 << 30))  # no stated capacity (a bare stand-in): one group

    def decode_many(self, embds, n_predict, temperature=0.3, top_p=1.0, top_k=50, reporter=None, stream_output=False):
        """Prefill every sequence, then decode them as one continuous batch. -> [LLMDecodeResult]
        More sequences than the engine has slots run as consecutive groups of slot_capacity()."""
        cap = self.slot_capacity()
        if len(embds) > cap:
            out = []
            for i in range(0, len(embds), cap):
                n_p = n_predict[i:i + cap] if isinstance(n_predict, (list, tuple)) else n_predict
                out += self.decode_many(embds[i:i + cap], n_p, temperature, top_p, top_k, reporter, stream_output)
            return out
        eng = self.models.engine
        cfg = self.models.config
        samp = self._sampling(temperature, top_p, top_k)
        states, res = [], []
        t0 = time.perf_counter()
        for s in range(len(embds)):
            eng.llm_reset(s)
        firsts = prefill_group(eng, list(range(len(embds))), embds, samp)
        t_inject = (time.perf_counter() - t0) / len(embds)
        for s, first in enumerate(firsts):
            r = LLMDecodeResult()
            r.t_inject = t_inject
            n_p = n_predict[s] if isinstance(n_predict, (list, tuple)) else n_predict
            st = _SeqState(self.models.vocab, n_p, self.models.eos_token, cfg.ignore_eos,
                           reporter if stream_output and len(embds) == 1 else None)
            st.feed([first])
            states.append(st)
            res.append(r)
        t_gen = time.perf_counter()
        stop_ids = np.array(sorted({self.models.eos_token} | set(STOP_TOKENS)), np.int64)
        active = [s for s, st in enumerate(states) if not st.done]
        chunk = min(GEN_CHUNK, max(states[s].remaining() for s in active)) if active else 0
        in_flight = False
        try:
            if active:
                eng.llm_generate_begin(active, chunk, **samp)
                in_flight = True
            while active:
                toks = eng.llm_generate_end()
                in_flight = False
                # the sequences this chunk leaves unfinished, from the token ids alone (stop ids, n_predict), go into
                # the next chunk, which is enqueued BEFORE the host detokenises this one (the host work overlaps the
                # GPU's); a sequence the repetition breaker cuts during feed() rides along one chunk, tokens ignored
                nxt, left_after = [], []
                for row, s in enumerate(active):
                    st = states[s]
                    left = st.remaining()
                    if left <= 0:
                        continue
                    used = toks[row][:min(chunk, left)]
                    if not st.ignore_eos and np.isin(used, stop_ids).any():
                        continue
                    if left > chunk:
                        nxt.append(s)
                        left_after.append(left - chunk)
                nchunk = min(GEN_CHUNK, max(left_after)) if nxt else 0
                if nxt:
                    eng.llm_generate_begin(nxt, nchunk, **samp)
                    in_flight = True
                for row, s in enumerate(active):
                    states[s].feed(toks[row])
                active, chunk = nxt, nchunk
        finally:
            # host code between begin and end (detokenising, the reporter) may raise: land the chunk in flight so
            # the engine is not left refusing every later call with "a generate call is in flight"
            if in_flight:
                try:
                    eng.llm_generate_end()
                except Exception:
                    pass
        dt = time.perf_counter() - t_gen
        for st, r in zip(states, res):
            st.ps.flush()
            r.text = st.ps.generated_text
            r.n_gen = st.ps.tokens_generated
            r.t_gen = dt
            r.is_aborted = st.aborted
        return res

    def decode(self, full_embd, n_input_tokens, n_predict, stream_output=False, reporter=None, temperature=0.3,
               top_p=1.0, top_k=50):
        return self.decode_many([full_embd], n_predict, temperature, top_p, top_k, reporter, stream_output)[0]

    def decode_with_retry(self, embds, n_predict, temperature=0.3, top_p=1.0, top_k=50, reporter=None,
                          stream_output=False, attempts=6):
        """The reference's retry policy (decoder.py:201-211) per sequence: an attempt cut by the repetition
        breaker is decoded again at temperature + 0.3, up to 6 attempts in all; the final attempt's text keeps the
        abort marker when it was cut too. Sequences still pending retry together as one batch."""
        B = len(embds)
        temps = [temperature] * B
        final = [None] * B
        pending = list(range(B))
        for attempt in range(attempts):
            n_p = [n_predict[b] for b in pending] if isinstance(n_predict, (list, tuple)) else n_predict
            rs = self.decode_many([embds[b] for b in pending], n_p, temps[pending[0]], top_p, top_k, reporter,
                                  stream_output)
            nxt = []
            for b, r in zip(pending, rs):
                if r.is_aborted and attempt < attempts - 1:
                    temps[b] += 0.3
                    nxt.append(b)
                else:
                    if r.is_aborted:
                        r.text += ABORT_MARK
                    final[b] = r
            if not nxt:
                break
            pending = nxt
        return final


_TOKEN_POOL = None


def _token_pool():
    """One background thread that builds the CTC Token lists (tens of thousands of objects per 32-clip batch) while the
    main thread waits on the GPU in prefill / generate (ctypes releases the GIL inside the engine calls)."""
    global _TOKEN_POOL
    if _TOKEN_POOL is None:
        _TOKEN_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ctc-tokens")
    return _TOKEN_POOL


def _pair_tokens(ids, frames, id2token):
    return tokens_of(*ctc_pair_rows(ids, frames, id2token))


_BLANK = {}


def _blank_of(id2token):
    """The CTC blank id = the largest id of the vocabulary (tokens.txt's last line, decoder.py:27); cached per table
    (max over 60k keys costs ~1 ms per call)."""
    if not id2token:
        return 0
    key = (id(id2token), len(id2token))
    hit = _BLANK.get(key)
    if hit is None or hit[0] is not id2token:  # (holding the table keeps its id from being reused)
        if len(_BLANK) > 8:
            _BLANK.clear()
        hit = _BLANK[key] = (id2token, max(id2token.keys()))
    return hit[1]


class StreamDecoder:
    def __init__(self, models):
        self.models = models
        self.llm_decoder = LLMDecoder(models)

    def decode_stream(self, stream: RecognitionStream, language=None, context=None, verbose=True, reporter=None,
                      temperature=0.3, top_p=1.0, top_k=50) -> DecodeResult:
        return self.decode_streams([stream], language, context, verbose, reporter, temperature, top_p, top_k)[0]

    def front(self, streams: List[RecognitionStream], language=None, context=None, resident=None, independent=False):
        """Steps 1-3 for a group of streams: encode (+ CTC head / argmax) as one device batch (independent: every clip
        its single-clip encode, in concurrent lanes), CTC collapse + host token map + hotwords, prompt rows. -> list of
        dicts (embd, ctc_results, hotwords, n_p, n_s, audio_embd, timings)."""
        m = self.models
        eng = m.engine
        B = len(streams)
        timings = [Timings() for _ in range(B)]
        # 1. encode (+ CTC head + argmax) — one device batch
        t = time.perf_counter()
        clips = None if resident is not None else [s.audio_data for s in streams]
        out = eng.encode(clips, resident=resident, independent=True) if independent and B > 1 else \
            eng.encode(clips, resident=resident)
        dt = time.perf_counter() - t
        for tm in timings:
            tm.encode = dt
            tm.ctc_infer = 0.0  # fused into the encode call
        # 2. CTC collapse on device + host token map + hotwords
        t = time.perf_counter()
        ctc_results, hotwords = [[] for _ in range(B)], [[] for _ in range(B)]
        if m.config.enable_ctc:
            pairs = eng.ctc_collapse(_blank_of(m.ctc_id2token), B)
            # the hotword step needs the CTC text before the prompt; without a hotword source the prompt does not depend
            # on it, and the whole host decode of the pairs runs off the critical path (back() collects the Tokens)
            need_text = getattr(m, "hotword_source", None) is not None
            for b in range(B):
                if need_text or len(pairs[b][0]) <= 64:
                    texts, starts = ctc_pair_rows(pairs[b][0], pairs[b][1], m.ctc_id2token)
                    hotwords[b] = m.match_hotwords("".join(texts), m.config.max_hotwords)
                    ctc_results[b] = _token_pool().submit(tokens_of, texts, starts) if len(texts) > 64 else \
                        tokens_of(texts, starts)
                else:
                    ctc_results[b] = _token_pool().submit(_pair_tokens, pairs[b][0], pairs[b][1], m.ctc_id2token)
        dt = time.perf_counter() - t
        for tm in timings:
            tm.ctc = tm.ctc_decode = dt / B
        # 3. prompt
        t = time.perf_counter()
        jobs = []
        gen = out.get("enc_gen", -1)
        for b in range(B):
            pe, se, n_p, n_s, _ = m.prompt_builder.build_prompt(hotwords[b], language, context)
            # the prompt rows stay unassembled while the engine holds this encode (PromptRows); else the reference's
            # host concatenation
            embd = PromptRows(pe, out["audio_embd"][b], se, b, gen) if gen >= 0 else \
                np.concatenate([pe, out["audio_embd"][b].astype(np.float32), se], 0)
            jobs.append(dict(embd=embd, ctc_results=ctc_results[b], hotwords=hotwords[b], n_p=n_p, n_s=n_s,
                             audio_embd=out["audio_embd"][b], timings=timings[b]))
        dt = time.perf_counter() - t
        for tm in timings:
            tm.prepare = dt / B
        return jobs

    @staticmethod
    def back(stream, job, r):
        """Step 5 for one stream: alignment of the LLM text to the CTC tokens -> DecodeResult."""
        text = r.text.strip()
        tm = job["timings"]
        if isinstance(job["ctc_results"], Future):
            job["ctc_results"] = job["ctc_results"].result()
        tm.inject, tm.llm_generate = r.t_inject, r.t_gen
        t = time.perf_counter()
        aligned = align_timestamps(job["ctc_results"], text) if job["ctc_results"] else None
        tm.align = time.perf_counter() - t
        toks = [a["char"] for a in aligned] if aligned else []
        ts = [a["start"] for a in aligned] if aligned else []
        if stream is not None:
            stream.set_result(text=text, timestamps=ts, tokens=toks)
        return DecodeResult(text=text, ctc_results=job["ctc_results"], aligned=aligned, audio_embd=job["audio_embd"],
                            n_prefix=job["n_p"], n_suffix=job["n_s"], n_gen=r.n_gen, timings=tm,
                            hotwords=job["hotwords"], is_aborted=r.is_aborted)

    def decode_streams(self, streams: List[RecognitionStream], language=None, context=None, verbose=True,
                       reporter=None, temperature=0.3, top_p=1.0, top_k=50, resident=None,
                       n_predicts=None) -> List[DecodeResult]:
        """One group of streams: encode batch, then all sequences decode together (no admission).
        resident: handle from engine.upload() holding these streams' PCM in HBM (benchmark path).
        n_predicts: per-stream decode-length caps (default config.n_predict)."""
        jobs = self.front(streams, language, context, resident)
        # 4. LLM with the reference's retry policy (decoder.py:201-211), per sequence
        n_p = list(n_predicts) if n_predicts is not None else self.models.config.n_predict
        final = self.llm_decoder.decode_with_retry([j["embd"] for j in jobs], n_p,
                                                   temperature, top_p, top_k, reporter, verbose)
        return [self.back(st, j, r) for st, j, r in zip(streams, jobs, final)]
