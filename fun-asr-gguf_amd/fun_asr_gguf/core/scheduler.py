"""Continuous batching of many segments / clips on one engine (configs[2]: "encoder batching + decoder continuous
batch").

The reference decodes segments one after another (core/orchestrator.py:139-171; per segment
StreamDecoder.decode_stream, core/decoder.py:132-246). Here the engine's sequence slots (max_batch of them) decode
together, and a slot freed by a finished sequence (stop token, n_predict, repetition breaker) is refilled with the
next waiting clip: clips are encoded (+ CTC + prompt) ahead of need in full encoder batches, and a free slot takes
the next encoded clip's prompt as a prefill between decode chunks; it joins the running decode at the next chunk. The per-segment
rules are the reference's: stop ids and the breaker replayed on the host in token order (decoder.py:91-114), a cut
attempt retried at temperature + 0.3 up to 6 attempts (decoder.py:201-211; retries run as one group after the
queue drains, since one generate call shares one sampler setting).

Results per clip do not depend on grouping or admission order when max_batch <= the engine's invariant width
(fa_llm_invariant_width): every clip is then encoded alone, prefilled alone and decodes with its single-sequence
arithmetic, so a batch gives exactly the one-segment-at-a-time results of the reference's loop, and a segment set
sharded over N GPUs gives exactly the 1-GPU results. Wider batches (padded encoder batches, shared prefill forwards,
the M > 6 decode kernels) agree to the fp32 / q8_0 noise floors.
"""
import time
import warnings
from typing import List, Optional

import numpy as np

from ..nano_dataclass import LLMDecodeResult, RecognitionStream
from .decoder import ABORT_MARK, GEN_CHUNK, STOP_TOKENS, _SeqState, invariant_width, prefill_group

RETRY_ATTEMPTS = 6  # decoder.py:201-211: the first attempt + 5 retries


class _Job:
    __slots__ = ("idx", "stream", "front", "state", "res", "t0", "slot")

    def __init__(self, idx, stream, front):
        self.idx, self.stream, self.front = idx, stream, front
        self.state = self.res = self.t0 = self.slot = None


class ContinuousBatcher:
    """decode_segments with slot reuse. Clips are encoded ahead of need in full encoder batches; admit_min free slots
    trigger an admission (a prefill of that many prompts) while encoded clips wait."""

    def __init__(self, decoder, admit_min=None):
        self.decoder = decoder
        self.models = decoder.models
        self.admit_min = admit_min
        self.stats = {}

    def _begin(self, eng, jobs, n_waiting, n_free, admit_min, samp, landed=0):
        # while clips wait: a chunk that ends when enough slots have reached their length cap for the next admission
        # (stop tokens can end sequences sooner: seen at the chunk's end); otherwise up to GEN_CHUNK steps
        rem = sorted(j.state.remaining() - landed for j in jobs)  # landed: steps fed to no state yet
        need = min(admit_min, n_waiting) - n_free if n_waiting else 0
        chunk = rem[min(need, len(rem)) - 1] if need > 0 else rem[-1]
        chunk = max(1, min(GEN_CHUNK, chunk))
        eng.llm_generate_begin([j.slot for j in jobs], chunk, **samp)
        self.n_chunks += 1
        return list(jobs), chunk

    @staticmethod
    def _continues(j, row, chunk, stop_ids):
        st = j.state
        if st.done:
            return False
        left = st.remaining()
        if left <= chunk:
            return False
        return st.ignore_eos or not np.isin(row[:chunk], stop_ids).any()

    def run(self, chunks: List[np.ndarray], language=None, context=None, temperature=0.3, top_p=1.0, top_k=50,
            n_predicts: Optional[List[int]] = None, reporter=None):
        """chunks: PCM clips (each <= segment_size + 2 s). n_predicts: per-clip decode-length caps (default
        config.n_predict each; the variable-length benchmark protocol pins them). -> [DecodeResult] in input order."""
        m = self.models
        eng = m.engine
        cfg = m.config
        sr = cfg.sample_rate
        S = max(1, cfg.max_batch)
        admit_min = self.admit_min or max(1, S // 8)
        n_pred = list(n_predicts) if n_predicts is not None else [cfg.n_predict] * len(chunks)
        samp = self.decoder.llm_decoder._sampling(temperature, top_p, top_k)
        stop_ids = np.array(sorted({m.eos_token} | set(STOP_TOKENS)), np.int64)
        queue = list(range(len(chunks)))
        free = list(range(S))
        active = []          # jobs decoding, in slot-admission order
        done = {}            # idx -> (job, LLMDecodeResult)
        retry = []           # jobs cut by the breaker: retried after the queue drains
        # within the engine's invariant width every clip is encoded and prefilled alone and decodes with its
        # single-sequence arithmetic: results are exactly the one-clip-at-a-time results, whatever the grouping
        alone = S <= invariant_width(eng)
        invariance_lost = False
        rec = getattr(eng, "llm_decode_recoveries", None)
        fallbacks0 = rec()[1] if rec else 0
        n_admit = n_encode_batches = 0
        t_enc = t_pre = t_wait = 0.0
        self.n_chunks = 0
        t_run = time.perf_counter()

        ready = []  # encoded clips (front done) waiting for a slot
        enc_cap = eng.max_batch if hasattr(eng, "max_batch") else S

        def check_width():
            # a fused fan-in timeout is re-run on the fused layer (exact); only when that times out too does the chunk
            # run on the 5-launch layer (fa_llm_decode_recoveries counts it), and after three such chunks in a row the
            # engine keeps that layer (fa_llm_invariant_width 6 -> 1). Either way results from there on are no longer
            # bit-identical to one-clip decoding. Re-read before every admission and decode chunk; say so once, in
            # stats and a warning
            nonlocal alone, invariance_lost
            fell_back = bool(rec) and rec()[1] > fallbacks0
            if alone and (S > invariant_width(eng) or fell_back):
                alone, invariance_lost = False, True
                warnings.warn(f"decode batches of {S}: a decode chunk ran on the 5-launch layer (fused-layer timeouts; "
                              f"invariant width now {invariant_width(eng)}): results from here on agree with one-clip "
                              "decoding to the q8_0 noise floor, not bit for bit", RuntimeWarning)

        def encode_ahead(need):
            # clips are encoded ahead of their admission in encoder batches of the engine's full capacity (a padded
            # batch of 32 runs ~2.5x the per-clip rate of a batch of 8); within the invariant width as independent
            # clips (each its single-clip encode, in concurrent lanes)
            nonlocal n_encode_batches, t_enc
            while len(ready) < need and queue:
                k = min(enc_cap, len(queue))
                idxs = [queue.pop(0) for _ in range(k)]
                streams = []
                for i in idxs:
                    st = RecognitionStream()
                    st.accept_waveform(sr, chunks[i])
                    streams.append(st)
                t = time.perf_counter()
                fronts = self.decoder.front(streams, language, context, independent=alone)
                t_enc += time.perf_counter() - t
                n_encode_batches += 1
                ready.extend(_Job(i, st, f) for i, st, f in zip(idxs, streams, fronts))

        def admit(k):
            nonlocal n_admit, t_pre
            check_width()
            encode_ahead(k)
            jobs = [ready.pop(0) for _ in range(min(k, len(ready)))]
            slots = [free.pop(0) for _ in jobs]
            t = time.perf_counter()
            for q in slots:
                eng.llm_reset(q)
            firsts = prefill_group(eng, slots, [j.front["embd"] for j in jobs], samp)
            dt = time.perf_counter() - t
            t_pre += dt
            now = time.perf_counter()
            for j, q, first in zip(jobs, slots, firsts):
                j.slot = q
                j.state = _SeqState(m.vocab, n_pred[j.idx], m.eos_token, cfg.ignore_eos, None)
                j.res = LLMDecodeResult()
                j.res.t_inject = dt / len(jobs)
                j.t0 = now
                j.state.feed([first])
                if j.state.done:
                    finish(j)
                else:
                    active.append(j)
            n_admit += len(jobs)

        def finish(j):
            st = j.state
            st.ps.flush()
            j.res.text, j.res.n_gen = st.ps.generated_text, st.ps.tokens_generated
            j.res.t_gen, j.res.is_aborted = time.perf_counter() - j.t0, st.aborted
            free.append(j.slot)
            if st.aborted:
                retry.append(j)
            else:
                done[j.idx] = (j, j.res)

        def waiting():
            return len(ready) + len(queue)

        def want_admit():
            if not waiting() or not free:
                return 0
            if len(free) >= min(admit_min, waiting()) or not active:
                return min(len(free), waiting())
            return 0

        pending = None  # (jobs, chunk) of the generate call in flight
        try:
            while True:
                if pending is None:
                    k = want_admit()
                    if k:
                        admit(k)
                        continue
                    if not active:
                        break
                    check_width()
                    pending = self._begin(eng, active, waiting(), len(free), admit_min, samp)
                jobs, chunk = pending
                t = time.perf_counter()
                toks = eng.llm_generate_end()
                t_wait += time.perf_counter() - t
                pending = None
                check_width()
                # sequences this chunk leaves unfinished, decided from the token ids alone (stop ids, n_predict), get
                # the next chunk enqueued BEFORE the host detokenises this one (host work overlaps the GPU's) -- unless
                # the slots it frees are due for an admission (a prefill cannot run while a chunk is in flight). A
                # sequence the repetition breaker cuts during feed() rides along one chunk; its tokens are ignored.
                cont = [j for row, j in enumerate(jobs) if self._continues(j, toks[row], chunk, stop_ids)]
                n_free = len(free) + len(jobs) - len(cont)
                if cont and not (waiting() and n_free >= min(admit_min, waiting())):
                    pending = self._begin(eng, cont, waiting(), n_free, admit_min, samp, landed=chunk)
                cs = set(id(j) for j in cont)
                for row, j in enumerate(jobs):
                    j.state.feed(toks[row][:chunk])
                    if pending is None or id(j) not in cs:
                        if j.state.done:
                            finish(j)
                active = [j for j in jobs if (pending is not None and id(j) in cs) or not j.state.done]
        finally:
            if pending is not None:  # host code raised between begin and end: land the chunk, keep the engine usable
                try:
                    eng.llm_generate_end()
                except Exception:
                    pass
        # the reference retries a cut segment at temperature + 0.3, up to 6 attempts (decoder.py:201-211)
        if retry:
            embds = [j.front["embd"] for j in retry]
            rs = self.decoder.llm_decoder.decode_with_retry(embds, [n_pred[j.idx] for j in retry],
                                                            temperature + 0.3, top_p, top_k, None, False,
                                                            attempts=RETRY_ATTEMPTS - 1)
            for j, r in zip(retry, rs):
                done[j.idx] = (j, r)
        self.stats = dict(admissions=n_admit, encode_batches=n_encode_batches, retried=len(retry), chunks=self.n_chunks,
                          slots=S, batch_invariant=not invariance_lost and S <= invariant_width(eng),
                          encode_s=round(t_enc, 4), prefill_s=round(t_pre, 4), generate_wait_s=round(t_wait, 4),
                          total_s=round(time.perf_counter() - t_run, 4))
        out = []
        for i in range(len(chunks)):
            j, r = done[i]
            out.append(self.decoder.back(j.stream, j.front, r))
        return out


__all__ = ["ContinuousBatcher", "ABORT_MARK"]
