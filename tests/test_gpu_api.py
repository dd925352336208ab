"""GPU end-to-end through the public API (create_asr_engine -> FunASREngine.transcribe), tiny synthetic model.

Covers the long-audio strategy of the reference (orchestrator.py:123-189): windows of segment_size with step
segment_size - overlap, every segment through encode -> CTC -> prompt -> LLM -> align, then the difflib merge
(text_merge.py:14-114). Here the segments of one file go through the device as ONE batch; the test pins
  * the windows against oracle.ctc.segments_info (restated from orchestrator.py:123-136),
  * the merged text / char timestamps against oracle.ctc.merge_results applied to the per-segment results,
  * each segment's CTC ids (device, padded batch) against the oracle encoder on the unpadded chunk, exact on
    frames whose top-1/top-2 logit margin exceeds 1e-3 (the encoder tolerance of test_gpu_parity.py),
  * determinism (temperature 0: greedy) and the short path (duration <= segment_size + 2, orchestrator.py:65).
The decoder runs with ignore_eos (pinned decode length, no breaker/retry), so the result is deterministic.
"""
import numpy as np
import pytest

from oracle import ctc as octc, encoder as oenc, synth

pytestmark = pytest.mark.gpu

SR = 16000
N_PRED = 24


@pytest.fixture(scope="module")
def api_engine():
    from fun_asr_gguf import create_asr_engine
    eng = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="tiny",
                            max_batch=4, n_ctx=512, n_predict=N_PRED, ignore_eos=True)
    yield eng
    eng.cleanup()


def _audio(seconds, seed):
    from fun_asr_gguf.synthetic import synth_audio
    return synth_audio(int(seconds * SR), seed)


def test_long_audio_segments_batched_and_merged(api_engine):
    audio = _audio(14.0, 7)
    seg, ov = 6.0, 2.0
    res = api_engine.transcribe(audio, segment_size=seg, overlap=ov, temperature=0.0, verbose=False)
    wins = octc.segments_info(len(audio) / SR, seg, ov)
    assert wins == [(0.0, 6.0), (4.0, 10.0), (8.0, 14.0)]
    chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
    per = api_engine.transcribe_batch(chunks, temperature=0.0)
    assert all(d.n_gen == N_PRED for d in per)
    seg_results = [{"text": d.text, "segments": d.aligned or []} for d in per]
    text, segs = octc.merge_results(seg_results, [s for s, _ in wins], ov)
    assert res.text == text
    assert [(c["char"], round(c["start"], 6)) for c in res.segments] == [(c["char"], round(c["start"], 6)) for c in segs]
    assert res.text and len(res.segments) > 0
    starts = [c["start"] for c in res.segments]
    assert min(starts) >= 0.0 and max(starts) <= len(audio) / SR + 1.0
    # deterministic at temperature 0
    res2 = api_engine.transcribe(audio, segment_size=seg, overlap=ov, temperature=0.0, verbose=False)
    assert res2.text == res.text and res2.segments == res.segments
    # the CTC text the engine reports is the concatenation of the segments' CTC texts
    assert res.ctc_text == "".join("".join(t.text for t in d.ctc_results) for d in per if d.ctc_results)


def test_long_audio_segment_ctc_ids_vs_oracle(api_engine):
    """Device CTC ids of the padded 3-segment batch == oracle encoder on each unpadded chunk (non-tie frames)."""
    audio = _audio(14.0, 7)
    wins = octc.segments_info(len(audio) / SR, 6.0, 2.0)
    chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
    out = api_engine.models.engine.encode(chunks)
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY))
    for b, c in enumerate(chunks):
        ref = oenc.encode(c, W, synth.ENC_TINY)
        lg = np.sort(ref["ctc_logits"], axis=-1)
        margin = lg[:, -1] - lg[:, -2]
        ids = out["ctc_ids"][b]
        assert ids.shape == ref["ctc_ids"].shape
        bad = (ids != ref["ctc_ids"]) & (margin > 1e-3)
        assert bad.sum() == 0, f"segment {b}: {int(bad.sum())} non-tie CTC ids differ"
        emb = out["audio_embd"][b]
        assert emb.shape == ref["audio_embd"].shape
        assert float(np.abs(emb - ref["audio_embd"]).max()) <= 5e-5 * max(1.0, float(np.abs(ref["audio_embd"]).max()))


def test_short_path_equals_single_decode_stream(api_engine):
    audio = _audio(7.5, 3)  # <= segment_size + 2: one segment, reference short path
    res = api_engine.transcribe(audio, segment_size=6.0, overlap=2.0, temperature=0.0, verbose=False)
    st = api_engine.create_stream()
    st.accept_waveform(SR, audio)
    d = api_engine.decode_stream(st, temperature=0.0, verbose=False)
    assert res.text == d.text
    assert res.segments == [{"char": a["char"], "start": a["start"]} for a in (d.aligned or [])]
