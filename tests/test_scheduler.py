"""Continuous batching (core/scheduler.py) and the decode loop's failure handling, on the host fake engine (no GPU):
clips with mixed decode lengths through max_batch slots give each clip exactly its single-clip result (the fake
engine is batch-independent by construction, like the native engine within its invariant width), freed slots are
refilled while others decode, and an exception in host code between generate_begin and _end leaves the engine
usable (the native engine refuses every decoder call while a chunk is in flight)."""
import numpy as np
import pytest

from fake_engine import fake_api, fake_models
from fun_asr_gguf.core.decoder import ABORT_MARK
from fun_asr_gguf.synthetic import synth_audio


def _clips(n):
    return [synth_audio(16000 * (3 + (i * 7) % 11) + 371 * i, 100 + i) for i in range(n)]


def test_continuous_batch_equals_per_clip_with_mixed_lengths():
    api = fake_api(max_batch=4, n_predict=64)
    clips = _clips(11)
    n_pred = [5, 40, 12, 33, 7, 60, 21, 9, 50, 17, 28]
    orch = api.orchestrator
    got = orch.decode_segments(clips, None, None, False, 0.0, 1.0, 50, n_predicts=n_pred)
    stats = dict(orch.batcher.stats)
    eng = api.models.engine
    assert eng.max_width <= 4 and stats["admissions"] == 11
    assert stats["encode_batches"] >= 3  # freed slots were refilled while other clips were decoding
    for c, n, g in zip(clips, n_pred, got):
        alone = orch.decode_segments([c], None, None, False, 0.0, 1.0, 50, n_predicts=[n])[0]
        assert g.n_gen == n and alone.n_gen == n
        assert g.text == alone.text and g.aligned == alone.aligned and g.ctc_results == alone.ctc_results


def test_continuous_batch_admission_order_independent():
    api = fake_api(max_batch=3, n_predict=30)
    clips = _clips(7)
    n_pred = [30, 4, 25, 6, 18, 11, 3]
    a = api.orchestrator.decode_segments(clips, None, None, False, 0.0, 1.0, 50, n_predicts=n_pred)
    perm = [6, 2, 0, 5, 1, 4, 3]
    b = api.orchestrator.decode_segments([clips[i] for i in perm], None, None, False, 0.0, 1.0, 50,
                                         n_predicts=[n_pred[i] for i in perm])
    for k, i in enumerate(perm):
        assert b[k].text == a[i].text and b[k].n_gen == a[i].n_gen


def test_reporter_exception_leaves_engine_usable():
    from fun_asr_gguf.core.decoder import LLMDecoder
    m = fake_models(max_batch=1, n_predict=80)
    dec = LLMDecoder(m)
    embd = np.full((10, 1024), 0.25, np.float32)

    class Boom:  # fails while detokenising the first landed chunk, after the next chunk was enqueued
        n = 0

        def stream(self, piece):
            self.n += 1
            if self.n == 5:
                raise ValueError("reporter failed")

    with pytest.raises(ValueError):
        dec.decode_many([embd], 80, temperature=0.0, reporter=Boom(), stream_output=True)
    r = dec.decode_many([embd], 80, temperature=0.0)[0]  # no "a generate call is in flight"
    assert r.n_gen == 80


def test_more_breaker_retries_than_slots():
    """Every clip loops at the first attempts' temperatures, so all 5 are cut by the repetition breaker and retried
    (decoder.py:201-211) on an engine with 2 sequence slots: the retries run in groups that fit the slots (the fake
    engine refuses a slot out of range, as fa_llm_reset does)."""
    api = fake_api(max_batch=2, n_predict=40, ignore_eos=False, loop_below=0.5)
    clips = _clips(5)
    got = api.orchestrator.decode_segments(clips, None, None, False, 0.0, 1.0, 50)
    st = api.orchestrator.batcher.stats
    assert st["retried"] == 5 and api.models.engine.max_width <= 2
    for g in got:  # attempts at 0.0 and 0.3 loop; the one at 0.6 decodes
        assert not g.is_aborted and g.n_gen == 40
    # a model that loops at every temperature: all 6 attempts cut, the marker text is kept (decoder.py:210)
    api = fake_api(max_batch=2, n_predict=40, ignore_eos=False, loop_below=100.0)
    got = api.orchestrator.decode_segments(clips[:3], None, None, False, 0.0, 1.0, 50)
    for g in got:
        assert g.is_aborted and g.text.endswith(ABORT_MARK)


def test_decode_many_splits_by_slot_capacity():
    from fun_asr_gguf.core.decoder import LLMDecoder
    m = fake_models(max_batch=3, n_predict=12)
    dec = LLMDecoder(m)
    embds = [np.full((10, 1024), 0.1 * (i + 1), np.float32) for i in range(7)]
    rs = dec.decode_many(embds, [12, 5, 7, 12, 3, 9, 11], temperature=0.0)
    assert [r.n_gen for r in rs] == [12, 5, 7, 12, 3, 9, 11] and m.engine.max_width <= 3
    for e, r in zip(embds, rs):
        assert dec.decode_many([e], r.n_gen, temperature=0.0)[0].text == r.text


def test_invariant_width_drop_is_reported():
    """A fused fan-in recovery drops the native engine's invariant width (6 -> 1) for good: the batcher re-reads it
    before every admission and chunk, and says that later batches are no longer bit-identical to one-clip decoding."""
    api = fake_api(max_batch=4, n_predict=64)
    eng = api.models.engine
    calls = {"n": 0}

    def width():
        calls["n"] += 1
        return 6 if calls["n"] < 4 else 1

    eng.llm_invariant_width = width
    with pytest.warns(RuntimeWarning, match="invariant width"):
        api.orchestrator.decode_segments(_clips(9), None, None, False, 0.0, 1.0, 50,
                                         n_predicts=[5, 40, 12, 33, 7, 60, 21, 9, 50])
    assert api.orchestrator.batcher.stats["batch_invariant"] is False
    eng.llm_invariant_width = lambda: 6
    api.orchestrator.decode_segments(_clips(5), None, None, False, 0.0, 1.0, 50)
    assert api.orchestrator.batcher.stats["batch_invariant"] is True
