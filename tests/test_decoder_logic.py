"""Host logic of the LLM loop against the reference's rules, with a scripted fake engine (no GPU):
stop tokens, repetition breaker and the retry policy of /root/reference/fun_asr_gguf/core/decoder.py:84-123,
201-211, replayed by fun_asr_gguf.core.decoder over device-sampled token chunks.

The expected results come from `ref_attempt` / `ref_retry` below, a line-by-line restatement of the reference
loop driven by the same token stream the sampler would have produced (the reference samples one token, feeds
it, then checks stop -> push piece -> breaker; decoder.py:91-114).
"""
import codecs

import numpy as np
import pytest

from fun_asr_gguf.core.decoder import ABORT_MARK, GEN_CHUNK, LLMDecoder

EOS = 151645
STOP = (151643, 151645)


class FakeVocab:
    """Pieces: 1000+i -> one ASCII letter; 2000/2001 -> the two halves of the UTF-8 bytes of '中'."""

    def token_to_bytes(self, t):
        if t == 2000:
            return "中".encode()[:1]
        if t == 2001:
            return "中".encode()[1:]
        if 1000 <= t < 1026:
            return bytes([ord("a") + t - 1000])
        return b"?"


class FakeEngine:
    """Token streams per (logical sequence, attempt); the logical id rides in embd[0, 0], the attempt is the
    temperature step above the base (retries add 0.3)."""

    def __init__(self, scripts, base_temp):
        self.scripts = scripts
        self.base = base_temp
        self.slot = {}
        self.calls = []

    def llm_reset(self, s):
        self.slot.pop(s, None)

    def _stream(self, seq, temp):
        att = int(round((temp - self.base) / 0.3))
        sc = self.scripts[seq]
        return list(sc[min(att, len(sc) - 1)]) + [1000 + (seq % 20)] * 600

    def llm_prefill(self, s, embd, temperature=0.0, **kw):
        seq = int(embd[0, 0])
        st = self._stream(seq, temperature)
        self.slot[s] = [st, 1]
        self.calls.append(("prefill", seq, temperature))
        return st[0]

    def llm_prefill_batch(self, seqs, embds, temperature=0.0, **kw):
        return [self.llm_prefill(s, e, temperature) for s, e in zip(seqs, embds)]

    def llm_generate(self, seqs, n, temperature=0.0, **kw):
        out = np.zeros((len(seqs), n), np.int32)
        for r, s in enumerate(seqs):
            st, p = self.slot[s]
            out[r] = st[p:p + n]
            self.slot[s][1] = p + n
        self.calls.append(("generate", tuple(seqs), n))
        return out

    def llm_generate_begin(self, seqs, n, temperature=0.0, **kw):
        assert getattr(self, "_pending", None) is None, "one generate call in flight"
        self._pending = self.llm_generate(seqs, n, temperature=temperature, **kw)

    def llm_generate_end(self):
        out, self._pending = self._pending, None
        return out


class FakeModels:
    def __init__(self, scripts, n_predict, base_temp, ignore_eos=False):
        self.engine = FakeEngine(scripts, base_temp)
        self.vocab = FakeVocab()
        self.eos_token = EOS

        class C:
            pass

        self.config = C()
        self.config.n_predict = n_predict
        self.config.ignore_eos = ignore_eos


def ref_attempt(tokens, n_predict, vocab):
    """decoder.py:84-123 (ASRStreamDecoder llama.py:661-690) over a given sampled-token stream."""
    dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
    pieces, text, n_gen, aborted = [], "", 0, False
    for i in range(n_predict):
        t = tokens[i]
        if t == EOS or t in STOP:
            break
        piece = dec.decode(vocab.token_to_bytes(t), final=False)
        pieces.append(piece)
        n_gen += 1
        text += piece
        if len(pieces) <= 30:
            continue
        if len(set(pieces[-30:])) <= 3:
            aborted = True
            break
    text += dec.decode(b"", final=True)
    return text, n_gen, aborted


def ref_retry(streams_of_seq, n_predict, vocab):
    """decoder.py:201-211: up to 6 attempts, +0.3 per retry, marker kept only by a final aborted attempt."""
    for att in range(6):
        text, n_gen, aborted = ref_attempt(streams_of_seq(att), n_predict, vocab)
        if not aborted:
            break
        text += ABORT_MARK
    return text, n_gen, aborted


def _letters(s):
    return [1000 + ord(c) - ord("a") for c in s]


REPEAT = _letters("ab") * 40                 # 2 unique pieces: breaker fires at piece 31
NORMAL = _letters("thequickbrownfoxjumpsoverthelazydog" * 3)


def make_scripts():
    return {
        0: [_letters("hello") + [2000, 2001] + NORMAL[:33] + [EOS] + NORMAL],   # EOS after a chunk boundary
        1: [REPEAT, REPEAT, NORMAL[:50] + [151643]],                           # aborted twice, then ok
        2: [REPEAT],                                                           # aborted 6 times: marker
        3: [NORMAL * 10],                                                      # runs to n_predict
        4: [[151645] + NORMAL],                                                # stop at the first token
        5: [_letters("x") * 27 + _letters("wyz") + NORMAL],                    # 5 unique at piece 31: goes on
        6: [_letters("x") * 29 + _letters("yz") + NORMAL],                     # 3 unique at piece 31: breaker
    }


@pytest.mark.parametrize("n_predict", [40, 100, 512])
def test_stop_breaker_retry_match_reference_loop(n_predict):
    scripts = make_scripts()
    T0 = 0.4
    models = FakeModels(scripts, n_predict, T0)
    dec = LLMDecoder(models)
    embds = [np.full((3, 8), s, np.float32) for s in sorted(scripts)]
    got = dec.decode_with_retry(embds, n_predict, temperature=T0, top_p=1.0, top_k=50)
    for s in sorted(scripts):
        want = ref_retry(lambda att: models.engine._stream(s, T0 + 0.3 * att), n_predict, models.vocab)
        r = got[s]
        assert (r.text, r.n_gen, r.is_aborted) == want, (s, r.text, want)
    # retries decode at +0.3 per attempt, only the aborted sequences
    temps = sorted({round(t, 6) for kind, seq, t in models.engine.calls if kind == "prefill" and seq == 2})
    assert temps == [round(T0 + 0.3 * i, 6) for i in range(6)]
    first_cut = {q for q in scripts if ref_attempt(models.engine._stream(q, T0), n_predict, models.vocab)[2]}
    assert {1, 2, 6} <= first_cut
    assert {seq for kind, seq, t in models.engine.calls if kind == "prefill" and t > T0 + 0.1} == first_cut
    # device chunks never exceed GEN_CHUNK tokens per call
    assert all(c[2] <= GEN_CHUNK for c in models.engine.calls if c[0] == "generate")


def test_marker_only_on_final_failed_attempt():
    scripts = make_scripts()
    dec = LLMDecoder(FakeModels(scripts, 200, 0.3))
    r = dec.decode_with_retry([np.full((2, 4), 1, np.float32), np.full((2, 4), 2, np.float32)], 200, temperature=0.3)
    assert not r[0].is_aborted and ABORT_MARK not in r[0].text
    assert r[1].is_aborted and r[1].text.endswith(ABORT_MARK) and r[1].text.count(ABORT_MARK) == 1


def test_ignore_eos_pinned_length_protocol():
    """Benchmark protocol: EOS and the breaker are off, every sequence decodes n_predict tokens."""
    scripts = make_scripts()
    dec = LLMDecoder(FakeModels(scripts, 253, 0.0, ignore_eos=True))
    res = dec.decode_many([np.full((2, 4), s, np.float32) for s in sorted(scripts)], 253, temperature=0.0)
    assert [r.n_gen for r in res] == [253] * len(scripts)
    assert not any(r.is_aborted for r in res)


def test_deferred_ctc_tokens_equal_decode_ctc_pairs():
    """front() builds each clip's CTC Token list on a background thread (long lists) and back() collects it: the results
    carry exactly decode_ctc_pairs' tokens for the clip's collapsed pairs (reference nano_ctc.py:38-116)."""
    import numpy as np
    from fake_engine import fake_models
    from fun_asr_gguf.core.decoder import StreamDecoder
    from fun_asr_gguf.nano_ctc import Token, decode_ctc_pairs
    from fun_asr_gguf.nano_dataclass import RecognitionStream
    m = fake_models(max_batch=4, n_predict=8)
    dec = StreamDecoder(m)
    rng = np.random.default_rng(3)
    clips = [(rng.standard_normal(int(16000 * s)) * 0.1).astype(np.float32) for s in (30.0, 0.5, 12.0)]
    streams = []
    for c in clips:
        st = RecognitionStream()
        st.accept_waveform(16000, c)
        streams.append(st)
    rs = dec.decode_streams(streams, verbose=False, temperature=0.0)
    blank = max(m.ctc_id2token.keys())
    m.engine.encode(clips)
    pairs = m.engine.ctc_collapse(blank, len(clips))
    assert max(len(p[0]) for p in pairs) > 64  # the background path ran
    for r, (ids, fr) in zip(rs, pairs):
        _, want = decode_ctc_pairs(ids, fr, m.ctc_id2token)
        assert isinstance(r.ctc_results, list) and all(type(t) is Token for t in r.ctc_results)
        assert r.ctc_results == want
