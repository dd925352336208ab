"""GPU parity at the BENCHMARKED sizes (BASELINE.json configs[0..4]): the full 70-block encoder, the full Qwen3-0.6B
q8_0 decoder (28 layers, vocab 151936) and the 300 s long-audio path, on the synthetic weights of oracle/synth.py.

Oracles:
  * reference goldens generated from /root/reference's model_definition.py (tests/golden/make_golden.py):
    encoder_full_60s (configs[1] clip, T_lfr 1001) and encoder_full_10s (configs[0] clip);
  * oracle/cref (C++/OpenMP restatement, pinned in tests/test_cref.py to those goldens and to the numpy oracle)
    for the decoder at full dims and for clips no golden holds (batch of 32, C4 segments);
  * oracle/encoder_fp16 (numpy) for the fp16 graph (configs[4]).
Tolerances as test_gpu_parity.py: encoder fp32 max-abs/max <= 1e-4 and cosine >= 0.999999 at full depth (SURVEY §8(c),
experience/03 ONNX_Export_Optimization_Experience.md:68-73; measured 1.6e-5 bf16x3, 1.7e-6 exact f32); CTC ids
exact where the top-1/top-2 margin exceeds 1e-3; decoder teacher-forced logits cosine >= 0.9995 with equal argmax
where the oracle's top-2 margin exceeds 0.25 (q8_0 activation rounding noise, tests/test_oracle_golden.py).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import cref, ctc as octc, synth

pytestmark = pytest.mark.gpu

SR = 16000
ENC_ATOL = 1e-4
ENC_COS = 0.999999
TIE_MARGIN = 0.25


def _cos(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-6, float(np.abs(b).max())))


def _check_step(gpu, ref):
    assert _cos(gpu, ref) > 0.9995
    s = np.sort(ref)
    if s[-1] - s[-2] > TIE_MARGIN:
        assert int(np.argmax(gpu)) == int(np.argmax(ref))


@pytest.fixture(scope="module")
def eng():
    from fun_asr_gguf import _native
    e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_FULL, n_ctx=512, max_seqs=32), max_batch=32,
                       max_samples=SR * 62)
    e.synthetic_weights(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def cenc():
    e = cref.CEncoder(synth.ENC_FULL)
    yield e
    e.close()


@pytest.fixture(scope="module")
def cllm():
    m = cref.CQwen3(synth.LLM_FULL, n_ctx=512, max_seqs=1)
    yield m
    m.close()


@pytest.fixture(scope="module")
def g60():
    from fun_asr_gguf.synthetic import synth_audio
    g = dict(np.load(os.path.join(GOLDEN, "encoder_full_60s.npz")))
    a = synth_audio(960000, int(g["audio_seed"]))
    assert hashlib.sha256(a.tobytes()).digest() == g["audio_sha256"].tobytes(), "synthetic audio changed"
    g["audio"] = a
    return g


def _check_encoder(out_enc, out_emb, out_ids, ref_enc, ref_emb, ref_ids, margin, tag):
    e_enc, c_enc, e_emb, c_emb = _rel(out_enc, ref_enc), _cos(out_enc, ref_enc), None, None
    assert out_emb.shape == ref_emb.shape, tag
    e_emb, c_emb = _rel(out_emb, ref_emb), _cos(out_emb, ref_emb)
    print(f"{tag}: enc max-abs/max {e_enc:.2e} cos {c_enc:.8f}; adaptor max-abs/max {e_emb:.2e} cos {c_emb:.8f}")
    assert e_enc < ENC_ATOL and c_enc > ENC_COS, tag
    assert e_emb < ENC_ATOL and c_emb > ENC_COS, tag
    bad = (out_ids != ref_ids) & (margin > 1e-3)
    assert bad.sum() == 0, f"{tag}: {int(bad.sum())} non-tie CTC ids differ"


def test_encoder_60s_vs_reference_golden(eng, g60):
    """configs[1] clip: T_lfr 1001 (key splits, XCD tile order and K-split GEMMs of the one-clip shapes)."""
    out = eng.encode([g60["audio"]], want_enc=True)
    T = int(g60["t_lfr_valid"])
    assert T == 1001 and out["enc"][0].shape[0] == T and int(out["target_len"][0]) == 126
    rows = g60["enc_rows"]
    _check_encoder(out["enc"][0][rows], out["audio_embd"][0], out["ctc_ids"][0], g60["enc"], g60["adaptor"],
                   g60["ctc_ids"], g60["ctc_margin"], "60 s")


def test_encoder_60s_exact_f32_gemm_mode(eng, g60):
    """fa_set_encoder_gemm(0): the exact-f32 MFMA GEMMs (v_mfma_f32_32x32x2_f32, K-split few-tile shapes) against the
    same golden as the default bf16x3 split-operand GEMMs above; both modes agree to the golden bar."""
    eng.set_encoder_gemm("f32")
    try:
        out = eng.encode([g60["audio"]], want_enc=True)
    finally:
        eng.set_encoder_gemm("bf16x3")
    out3 = eng.encode([g60["audio"]], want_enc=True)
    rows = g60["enc_rows"]
    _check_encoder(out["enc"][0][rows], out["audio_embd"][0], out["ctc_ids"][0], g60["enc"], g60["adaptor"],
                   g60["ctc_ids"], g60["ctc_margin"], "60 s exact f32")
    e32, e3 = _rel(out["enc"][0][rows], g60["enc"]), _rel(out3["enc"][0][rows], g60["enc"])
    print(f"60 s encoder max-abs/max vs golden: exact f32 {e32:.2e}, bf16x3 {e3:.2e}")
    assert e3 < ENC_ATOL and _rel(out3["audio_embd"][0], out["audio_embd"][0]) < ENC_ATOL


def test_encoder_batch32_vs_oracle(eng, cenc):
    """configs[2]: 32 clips in one encoder batch (32 x 1001 rows: the 128x128-tile GEMM path), ragged lengths
    included; clips 0, 5, 17 and 31 against the oracle run of each clip alone (CPU-EP policy, unpadded)."""
    from fun_asr_gguf.synthetic import synth_audio
    lens = [960000] * 32
    lens[5], lens[17], lens[31] = 661234, 192000, 959999
    clips = [synth_audio(n, 1000 + i) for i, n in enumerate(lens)]
    out = eng.encode(clips, want_enc=True)
    for b in (0, 5, 17, 31):
        r = cenc.encode(clips[b])
        _check_encoder(out["enc"][b], out["audio_embd"][b], out["ctc_ids"][b], r["enc"], r["audio_embd"],
                       r["ctc_ids"], r["ctc_margin"], f"clip {b}")


def test_encoder_fp16_60s_vs_oracle(eng, g60):
    """configs[4] encoder: the float16 graphs (02-Quantize-ONNX.py:13-27) at 60 s against oracle/encoder_fp16, and
    within fp16 accuracy of the fp32 reference golden."""
    from oracle import encoder_fp16 as oe16
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_FULL))
    eng.set_encoder_fp16(True)
    try:
        out = eng.encode([g60["audio"]], want_enc=True)
    finally:
        eng.set_encoder_fp16(False)
    r = oe16.encode(g60["audio"], W, synth.ENC_FULL)
    del W
    enc, emb = out["enc"][0], out["audio_embd"][0]
    assert (emb.astype(np.float16).astype(np.float32) == emb).all()
    assert _rel(enc, r["enc"]) < 1e-2 and _cos(enc, r["enc"]) > 0.9999
    assert _rel(emb, r["audio_embd"]) < 1e-2 and _cos(emb, r["audio_embd"]) > 0.9999
    assert _cos(emb, g60["adaptor"]) > 0.999
    lg = r["ctc_logits"]
    top2 = np.sort(lg, -1)[:, -2:]
    nontie = (top2[:, 1] - top2[:, 0]) > 0.05
    assert ((out["ctc_ids"][0] != r["ctc_ids"]) & nontie).sum() == 0


def _prompt(cllm, audio_rows, seed):
    rng = np.random.default_rng(seed)
    return np.concatenate([cllm.embed_prompt(rng.integers(0, 151933, 73)), audio_rows.astype(np.float32),
                           cllm.embed_prompt(rng.integers(0, 151933, 5))], 0)


@pytest.mark.parametrize("clip", ["10s", "60s"])
def test_llm_full_prefill_and_steps_teacher_forced(eng, cllm, g60, clip):
    """configs[0]/[1] decoder at full dims: 73 + target_len + 5 prefill rows (99 / 204), then 6 steps; every
    step's full-vocab logits against the oracle fed the same token, and the device's greedy pick (argmax-partial
    reduction of the 151936-wide LM head) equal to the argmax of its own logits."""
    audio_rows = g60["adaptor"] if clip == "60s" else np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))["adaptor"]
    p = _prompt(cllm, audio_rows, 1 if clip == "60s" else 2)
    assert p.shape[0] == (204 if clip == "60s" else 99)
    eng.llm_reset(0)
    tok, lg = eng.llm_prefill(0, p, want_logits=True)
    ref = cllm.forward(p, 0)
    _check_step(lg, ref)
    assert tok == int(np.argmax(lg))
    pos = p.shape[0]
    for _ in range(6):
        nxt = int(eng.llm_generate([0], 1)[0][0])
        lg = eng.llm_logits(0)
        ref = cllm.forward(cllm.embed_tokens([tok]), pos)
        _check_step(lg, ref)
        assert nxt == int(np.argmax(lg))
        tok, pos = nxt, pos + 1
    assert eng.llm_n_past(0) == p.shape[0] + 6


def test_llm_full_prefill_batch_tiled_gemm(eng, cllm, g60):
    """configs[2] prefill: four 204-row prompts in one forward (816 rows: the 128x128-tile q8_0 GEMM for q|k|v, o,
    gate|up with the SwiGLU q8_0 epilogue, and down; the prefill attention of every row over its own sequence) against
    the oracle run of each prompt alone (first and last sequence), then one decode step of all four."""
    prompts = [_prompt(cllm, g60["adaptor"], 10 + i) for i in range(4)]
    for s in range(4):
        eng.llm_reset(s)
    toks = eng.llm_prefill_batch([0, 1, 2, 3], prompts)
    for s in (0, 3):
        lg = eng.llm_logits(s)
        _check_step(lg, cllm.forward(prompts[s], 0))
        assert toks[s] == int(np.argmax(lg))
    step = eng.llm_generate([0, 1, 2, 3], 1)
    lg = eng.llm_logits(3)
    _check_step(lg, cllm.forward(cllm.embed_tokens([toks[3]]), prompts[3].shape[0]))  # the oracle holds prompt 3
    assert int(step[3][0]) == int(np.argmax(lg))


@pytest.mark.parametrize("n_seq", [5, 32])
def test_llm_full_batched_decode_rows(eng, cllm, n_seq):
    """configs[2] continuous batch at full dims: M = 32 (int8 MFMA GEMMs + the batched LM head with its argmax
    partials) and M = 5 (fused GEMV, 2 tokens per block); sampled rows against the oracle run of that sequence
    alone, two steps."""
    rng = np.random.default_rng(40 + n_seq)
    lens = [int(n) for n in rng.integers(6, 48, n_seq)]
    prompts = [cllm.embed_prompt(rng.integers(0, 151933, n)) for n in lens]
    firsts = []
    for s, p in enumerate(prompts):
        eng.llm_reset(s)
        firsts.append(eng.llm_prefill(s, p))
    seqs = list(range(n_seq))
    steps = [eng.llm_generate(seqs, 1)[:, 0]]
    logits1 = {s: eng.llm_logits(s) for s in (0, n_seq // 3, n_seq - 1)}
    steps.append(eng.llm_generate(seqs, 1)[:, 0])
    logits2 = {s: eng.llm_logits(s) for s in logits1}
    for s in logits1:
        cllm.forward(prompts[s], 0)
        r1 = cllm.forward(cllm.embed_tokens([firsts[s]]), lens[s])
        _check_step(logits1[s], r1)
        assert int(steps[0][s]) == int(np.argmax(logits1[s]))
        r2 = cllm.forward(cllm.embed_tokens([int(steps[0][s])]), lens[s] + 1)
        _check_step(logits2[s], r2)
        assert int(steps[1][s]) == int(np.argmax(logits2[s]))


def test_sampler_full_vocab_membership(eng, cllm, g60):
    """Default transcribe() sampling (temperature 0.4, top_k 50; asr_engine.py:65) on the 151936-wide LM head:
    every draw in the top-k set of that step's logits (and in the top-p prefix when top_p < 1)."""
    p = _prompt(cllm, g60["adaptor"], 3)
    eng.llm_reset(0)
    eng.llm_prefill(0, p, temperature=0.4, top_k=50, seed=5)
    for step in range(8):
        top_p = 1.0 if step % 2 == 0 else 0.7
        t = int(eng.llm_generate([0], 1, temperature=0.4, top_k=50, top_p=top_p, seed=99 + step)[0][0])
        lg = eng.llm_logits(0).astype(np.float64)
        order = np.argsort(-lg, kind="stable")[:50]
        assert lg[t] >= lg[order[-1]]
        if top_p < 1:
            v = lg[order]
            w = np.exp(v - v[0])
            cum = np.cumsum(w / w.sum())
            n = int(np.searchsorted(cum, top_p - 1e-6)) + 1
            assert lg[t] >= v[n - 1]


def _pin_segment_decode(api, cllm, prompt, seg_text, n_gen=253):
    """One segment's decoder pinned token by token: its prompt rows (prefix | audio rows of the segment | suffix)
    prefilled alone on the engine, then n_gen - 1 greedy steps. (a) The detokenised tokens equal the segment's text
    from the public path (the batch gave it exactly its single-sequence arithmetic, DESIGN §1 batch invariance);
    (b) the prefill logits and every step's logits, teacher-forced on the GPU's own tokens, pass the oracle's
    per-step bar (cref at full dims: cosine >= 0.9995, argmax equal where its top-2 margin > 0.25)."""
    from fun_asr_gguf.core.decoder import PieceStream
    eng = api.models.engine
    eng.llm_reset(0)
    tok, lg = eng.llm_prefill(0, prompt, want_logits=True, temperature=0.0)
    ref = cllm.forward(prompt, 0)
    _check_step(lg, ref)
    toks, pos, worst = [tok], prompt.shape[0], _cos(lg, ref)
    for _ in range(n_gen - 1):
        nxt = int(eng.llm_generate([0], 1, temperature=0.0)[0][0])
        lg = eng.llm_logits(0)
        ref = cllm.forward(cllm.embed_tokens([toks[-1]]), pos)
        _check_step(lg, ref)
        worst = min(worst, _cos(lg, ref))
        toks.append(nxt)
        pos += 1
    ps = PieceStream(api.models.vocab)
    for t in toks:
        ps.push(t)
    ps.flush()
    assert ps.generated_text.strip() == seg_text
    return worst


def test_c4_300s_long_audio_full_model(cenc, cllm):
    """configs[3]: one 300 s file, segment 60 / overlap 4 -> 6 segments through the public transcribe() long path
    (one device batch), 253 greedy tokens per segment (pinned length). Pinned: the windows (oracle of
    orchestrator.py:123-136), every segment's CTC ids / audio rows against the oracle encoder on the unpadded
    chunk, the merged text + char timestamps = the reference merge rule (oracle.ctc.merge_results, pinned to
    text_merge.py goldens) applied to the per-segment results, and the decoded text of the first and the last
    segment token by token against the oracle decoder (_pin_segment_decode: all 253 steps teacher-forced)."""
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.synthetic import synth_audio
    api = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="full",
                            max_batch=6, n_ctx=512, n_predict=253, ignore_eos=True)
    try:
        audio = synth_audio(300 * SR, 4000)
        res = api.transcribe(audio, segment_size=60.0, overlap=4.0, temperature=0.0, verbose=False)
        wins = octc.segments_info(300.0, 60.0, 4.0)
        assert wins == [(0.0, 60.0), (56.0, 116.0), (112.0, 172.0), (168.0, 228.0), (224.0, 284.0), (280.0, 300.0)]
        chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
        per = api.transcribe_batch(chunks, temperature=0.0)
        assert [d.n_gen for d in per] == [253] * 6
        seg_results = [{"text": d.text, "segments": d.aligned or []} for d in per]
        text, segs = octc.merge_results(seg_results, [s for s, _ in wins], 4.0)
        assert res.text == text and len(text) > 0
        assert [(c["char"], round(c["start"], 6)) for c in res.segments] == \
               [(c["char"], round(c["start"], 6)) for c in segs]
        out = api.models.engine.encode(chunks, want_enc=True)
        for b, c in enumerate(chunks):
            r = cenc.encode(c)
            _check_encoder(out["enc"][b], out["audio_embd"][b], out["ctc_ids"][b], r["enc"], r["audio_embd"],
                           r["ctc_ids"], r["ctc_margin"], f"segment {b}")
        pe, se, n_p, n_s, _ = api.models.prompt_builder.build_prompt([], None, None)
        assert all((d.n_prefix, d.n_suffix) == (n_p, n_s) for d in per)
        for b in (0, 5):
            prompt = np.concatenate([pe, per[b].audio_embd.astype(np.float32), se], 0)
            worst = _pin_segment_decode(api, cllm, prompt, per[b].text)
            print(f"C4 segment {b}: 253 steps teacher-forced, worst logits cosine {worst:.6f}")
    finally:
        api.cleanup()


# configs[4]'s hotword / context prompt (bench.py C5_CONTEXT / C5_HOTWORDS)
C5_CONTEXT = "这是一段关于人工智能的会议"
C5_HOTWORDS = ["通义千问", "语音识别", "魔搭社区", "大模型"]


def test_c5_300s_fp16_hotword_prompt_full_path(cllm):
    """configs[4] end to end: the 300 s file through the public transcribe() long path with the fp16 encoder graph
    (encoder_precision="fp16") and the hotword / context prompt. The prompt text comes from the reference's
    prompt_texts (prompt_utils.py:16-54) for C5_HOTWORDS (supplied by a hotword source from the CTC text, the
    reference's decoder.py:39-44 step) and C5_CONTEXT, tokenized by the product's GGUF tokenizer (fa_tokenize on the
    synthetic Qwen2 BPE vocabulary: 73 prefix + 5 suffix tokens). Pinned:
      * every segment's fp16 audio rows against oracle/encoder_fp16 on the unpadded chunk;
      * the merged text + char timestamps = oracle.ctc.merge_results of the per-segment results;
      * the first and last segments' decodes token by token against cref (_pin_segment_decode, 253 steps)."""
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.prompt_utils import prompt_texts
    from fun_asr_gguf.synthetic import synth_audio
    from fun_asr_gguf.vocab import GGUFVocab
    from oracle import encoder_fp16 as oe16

    class _C5Hotwords:  # the hotword source's interface (model_manager.match_hotwords)
        def __init__(self):
            self.texts = []

        def hotwords_for(self, ctc_text, k):
            self.texts.append(ctc_text)
            return list(C5_HOTWORDS)[:k]

    api = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="full",
                            max_batch=6, n_ctx=512, n_predict=253, ignore_eos=True, encoder_precision="fp16")
    try:
        m = api.models
        vocab = GGUFVocab(os.path.join(GOLDEN, "tokenizer_qwen2_synth.gguf"))
        m.prompt_builder.vocab = vocab  # prompt tokenisation only; the LLM's own ids detokenise on m.vocab
        m.hotword_source = _C5Hotwords()
        pt, st = prompt_texts(C5_HOTWORDS, None, C5_CONTEXT)
        pre_ids, suf_ids = vocab.tokenize(pt), vocab.tokenize(st)
        assert (len(pre_ids), len(suf_ids)) == (73, 5)
        audio = synth_audio(300 * SR, 4000)
        res = api.transcribe(audio, segment_size=60.0, overlap=4.0, context=C5_CONTEXT, temperature=0.0,
                             verbose=False)
        wins = octc.segments_info(300.0, 60.0, 4.0)
        chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
        per = api.transcribe_batch(chunks, context=C5_CONTEXT, temperature=0.0)
        assert len(m.hotword_source.texts) >= 12 and all(m.hotword_source.texts)  # CTC text reached the source
        for d in per:
            assert (d.n_prefix, d.n_suffix, d.n_gen) == (73, 5, 253) and list(d.hotwords) == C5_HOTWORDS
        seg_results = [{"text": d.text, "segments": d.aligned or []} for d in per]
        text, segs = octc.merge_results(seg_results, [s for s, _ in wins], 4.0)
        assert res.text == text and len(text) > 0
        assert [(c["char"], round(c["start"], 6)) for c in res.segments] == \
               [(c["char"], round(c["start"], 6)) for c in segs]
        W = synth.make_weights(synth.encoder_tensors(synth.ENC_FULL))
        for b, c in enumerate(chunks):
            r = oe16.encode(c, W, synth.ENC_FULL)
            emb = per[b].audio_embd
            assert emb.shape == r["audio_embd"].shape, b
            assert (emb.astype(np.float16).astype(np.float32) == emb).all(), b
            e, cs = _rel(emb, r["audio_embd"]), _cos(emb, r["audio_embd"])
            print(f"C5 segment {b}: fp16 audio rows max-abs/max {e:.2e} cos {cs:.7f}")
            assert e < 1e-2 and cs > 0.9999, b
        del W
        pe, se, n_p, n_s, _ = m.prompt_builder.build_prompt(C5_HOTWORDS, None, C5_CONTEXT)
        assert (n_p, n_s) == (73, 5)
        assert np.array_equal(pe, cllm.embed_prompt(pre_ids)) and np.array_equal(se, cllm.embed_prompt(suf_ids))
        for b in (0, 5):
            prompt = np.concatenate([pe, per[b].audio_embd.astype(np.float32), se], 0)
            worst = _pin_segment_decode(api, cllm, prompt, per[b].text)
            print(f"C5 segment {b}: 253 steps teacher-forced, worst logits cosine {worst:.6f}")
    finally:
        api.cleanup()


def test_llm_full_vs_hf_anchor(eng):
    """The GPU decoder at full dims against the independent anchor (tests/golden/qwen3_full_hf.npz: HF Qwen3 on the
    configs[1] prompt, 204 rows): prefill last-row logits, then 12 decode steps through the production step (the
    fused two-launch layer, graph-replayed) teacher-forced on HF's greedy ids (fa_llm_set_token) at positions
    204-215. Bars in tests/hf_full.py (the q8_0 activation noise floor)."""
    import hf_full
    g, adaptor = hf_full.load()
    p = hf_full.prompt(g, adaptor, lambda ids: eng.embd_rows(np.asarray(ids, np.int32)))
    eng.llm_reset(0)
    _, lg = eng.llm_prefill(0, p, want_logits=True)
    cos = [hf_full.check(g, 0, lg)]
    for i, t in enumerate(g["greedy"]):
        eng.llm_set_token(0, int(t))
        eng.llm_generate([0], 1)
        cos.append(hf_full.check(g, i + 1, eng.llm_logits(0)))
    print("GPU vs HF full-dims cosines", np.round(cos, 6))


def _bench_prompts(eng, adaptor, n):
    """configs[2] prompts: n x (73 prefix + 126 adaptor rows + 5 suffix) = n x 204 rows, each its own prefix ids."""
    out = []
    for i in range(n):
        rng = np.random.default_rng(500 + i)
        out.append(np.concatenate([eng.embd_rows(rng.integers(0, 151933, 73).astype(np.int32)), adaptor,
                                   eng.embd_rows(rng.integers(0, 151933, 5).astype(np.int32))], 0).astype(np.float32))
    return out


def test_llm_full_c3_bench_shape_vs_oracle(eng, cllm, g60):
    """configs[2] at its benchmarked shape: 32 x 204 rows = 6528 rows prefilled by one fa_llm_prefill_batch (the tiled
    q8_0 GEMM and query-tiled prefill attention), then 8 decode steps at M = 32 (int8 MFMA GEMMs, batched attention,
    the batched LM head) at n_past 204-211; prompts 0, 15 and 31 against the oracle run of that prompt alone."""
    prompts = _bench_prompts(eng, g60["adaptor"].astype(np.float32), 32)
    seqs = list(range(32))
    for s in seqs:
        eng.llm_reset(s)
    firsts = eng.llm_prefill_batch(seqs, prompts)
    lg0 = {s: eng.llm_logits(s) for s in (0, 15, 31)}
    steps, lgs = [], []
    for _ in range(8):
        steps.append(eng.llm_generate(seqs, 1)[:, 0])
        lgs.append({s: eng.llm_logits(s) for s in (0, 15, 31)})
    for s in (0, 15, 31):
        ref = cllm.forward(prompts[s], 0)
        _check_step(lg0[s], ref)
        assert firsts[s] == int(np.argmax(lg0[s]))
        tok, pos = firsts[s], 204
        for k in range(8):
            ref = cllm.forward(cllm.embed_tokens([tok]), pos)
            _check_step(lgs[k][s], ref)
            assert int(steps[k][s]) == int(np.argmax(lgs[k][s]))
            tok, pos = int(steps[k][s]), pos + 1


def _single_runs(eng, prompts, K):
    """Each prompt decoded alone in slot 0 (the reference decodes every segment alone): first token + K greedy steps,
    logits of every step."""
    out = []
    for p in prompts:
        eng.llm_reset(0)
        t, lg = eng.llm_prefill(0, p, want_logits=True)
        toks, lgs = [t], [lg]
        for _ in range(K):
            toks.append(int(eng.llm_generate([0], 1)[0][0]))
            lgs.append(eng.llm_logits(0))
        out.append((toks, np.stack(lgs)))
    return out


def test_llm_full_invariant_width_batch_equals_single(eng, g60):
    """Within the engine's invariant width (6: the two-launch layer gives every token its own grid slab, the LM head is
    the fused GEMV) a batch of full-dims sequences, each prefilled alone, decodes with exactly the arithmetic of each
    sequence alone: bit-identical logits and tokens over 16 free-running greedy steps. This is what makes C4's
    6-segment batch (and any rank's share of segments) give the reference's one-segment-at-a-time results."""
    from fun_asr_gguf.core.decoder import prefill_group
    W = eng.llm_invariant_width()
    assert W >= 6
    prompts = _bench_prompts(eng, g60["adaptor"].astype(np.float32), W)
    K = 16
    single = _single_runs(eng, prompts, K)
    seqs = list(range(W))
    for s in seqs:
        eng.llm_reset(s)
    firsts = prefill_group(eng, seqs, prompts, dict(temperature=0.0))
    toks = [list(firsts)]
    for k in range(K):
        toks.append([int(t) for t in eng.llm_generate(seqs, 1)[:, 0]])
        if k == K - 1:
            for s in seqs:
                assert np.array_equal(eng.llm_logits(s), single[s][1][K]), f"seq {s}: logits differ from alone"
    for s in seqs:
        assert [t[s] for t in toks] == single[s][0], f"seq {s}: tokens differ from decoding it alone"


@pytest.mark.parametrize("M", [2, 3, 5])
def test_llm_full_small_batch_lm_head_equals_single(eng, g60, M):
    """Batches of 2-5 full-dims sequences (the 151936-row LM head on k_lm_head_s, the small-batch MFMA form whose
    every logit sums in the batch-1 GEMV's order) give bit-identical logits and tokens to each sequence decoded alone
    (width 6 is test_llm_full_invariant_width_batch_equals_single)."""
    from fun_asr_gguf.core.decoder import prefill_group
    prompts = _bench_prompts(eng, g60["adaptor"].astype(np.float32), M)
    K = 4
    single = _single_runs(eng, prompts, K)
    seqs = [2 * i + 1 for i in range(M)]  # non-contiguous slots
    for s in seqs:
        eng.llm_reset(s)
    firsts = prefill_group(eng, seqs, prompts, dict(temperature=0.0))
    assert list(firsts) == [single[i][0][0] for i in range(M)]
    for k in range(K):
        toks = [int(t) for t in eng.llm_generate(seqs, 1)[:, 0]]
        for i, s in enumerate(seqs):
            assert toks[i] == single[i][0][k + 1], f"M={M} seq {i} step {k}: token differs from alone"
            assert np.array_equal(eng.llm_logits(s), single[i][1][k + 1]), f"M={M} seq {i} step {k}: logits differ"


def test_llm_full_batch32_vs_single_streams_bound(eng, g60):
    """Above the invariant width (configs[2]: 32 streams at M = 32 on the int8 MFMA GEMMs with producer-side
    quantisation and the batched LM head, prefilled as one 6528-row batch) a stream's logits differ from decoding it
    alone by f32 summation order, amplified by q8_0 activation rounding flips: 32 streams x 16 steps, teacher-forced
    on each stream's single-stream tokens (fa_llm_set_token). Bound: cosine >= 0.9995 per vector and the same argmax
    wherever the single-stream top-2 margin exceeds 0.15 (two q8_0 noise floors, tests/hf_full.py)."""
    prompts = _bench_prompts(eng, g60["adaptor"].astype(np.float32), 32)
    K = 16
    single = _single_runs(eng, prompts, K)
    seqs = list(range(32))
    for s in seqs:
        eng.llm_reset(s)
    eng.llm_prefill_batch(seqs, prompts)
    worst_cos, diffs, flips = 1.0, [], []
    for k in range(K + 1):
        if k > 0:
            for s in seqs:
                eng.llm_set_token(s, single[s][0][k - 1])
            eng.llm_generate(seqs, 1)
        for s in seqs:
            lg, ref = eng.llm_logits(s), single[s][1][k]
            c = _cos(lg, ref)
            worst_cos = min(worst_cos, c)
            diffs.append(float(np.abs(lg - ref).max()))
            top2 = np.sort(ref)[-2:]
            if int(np.argmax(lg)) != int(np.argmax(ref)):
                flips.append(float(top2[1] - top2[0]))
            assert c >= 0.9995, f"seq {s} step {k}: cosine {c}"
            if top2[1] - top2[0] > 0.15:
                assert int(np.argmax(lg)) == int(np.argmax(ref)), f"seq {s} step {k}: argmax at margin {top2[1] - top2[0]}"
    d = np.array(diffs)
    print(f"batch-32 vs single: worst cos {worst_cos:.6f}, max|diff| p50 {np.median(d):.4f} p99 "
          f"{np.quantile(d, 0.99):.4f} max {d.max():.4f}; bit-identical vectors {(d == 0).mean():.3f}; argmax flips "
          f"{len(flips)} / {d.size} at margins {np.round(sorted(flips), 4).tolist()[:12]}")


def test_c4_batch_of_6_equals_sequential_segments():
    """configs[3] on one GPU: the six segments of the 300 s file decoded as one continuous batch (max_batch 6, the
    invariant width) give exactly the text and char timestamps of six one-segment calls (the reference decodes the
    segments one after another, orchestrator.py:139-171)."""
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.synthetic import synth_audio
    api = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="full",
                            max_batch=6, n_ctx=512, n_predict=253, ignore_eos=True)
    try:
        audio = synth_audio(300 * SR, 4000)
        wins = octc.segments_info(300.0, 60.0, 4.0)
        chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
        w0 = api.models.engine.llm_invariant_width()
        batch = api.transcribe_batch(chunks, temperature=0.0)
        ones = [api.transcribe_batch([c], temperature=0.0)[0] for c in chunks]
        diag = []
        for k, (b, one) in enumerate(zip(batch, ones)):
            if b.text != one.text or b.aligned != one.aligned:
                pre = next((i for i, (x, y) in enumerate(zip(b.text, one.text)) if x != y), min(len(b.text), len(one.text)))
                diag.append(f"segment {k}: texts agree on {pre} of {len(one.text)} chars; audio rows equal "
                            f"{np.array_equal(b.audio_embd, one.audio_embd)}; ctc equal {b.ctc_results == one.ctc_results}")
        w1 = api.models.engine.llm_invariant_width()
        assert not diag and w0 == w1 == 6, f"invariant width {w0} -> {w1}; " + "; ".join(diag)
        assert all(b.n_gen == one.n_gen == 253 for b, one in zip(batch, ones))
    finally:
        api.cleanup()


def test_encoder_batch_vs_alone_f32_order(eng):
    """The padded encoder batch (configs[3]'s six segments in one encode) against each segment encoded alone: equal to
    the fp32 bar (a different GEMM tiling / key-split order, not other math); reports how far from bit-identical."""
    from fun_asr_gguf.synthetic import synth_audio
    audio = synth_audio(300 * SR, 4000)
    wins = octc.segments_info(300.0, 60.0, 4.0)
    chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
    out = eng.encode(chunks, want_enc=True)
    worst, same = 0.0, []
    for b, c in enumerate(chunks):
        one = eng.encode([c], want_enc=True)
        worst = max(worst, _rel(out["audio_embd"][b], one["audio_embd"][0]))
        same.append(bool(np.array_equal(out["audio_embd"][b], one["audio_embd"][0])))
        assert _rel(out["enc"][b], one["enc"][0]) < ENC_ATOL
    print(f"encoder batch-6 vs alone: audio_embd max-abs/max {worst:.2e}, bit-identical per segment {same}")
    # independent-clip mode (fa_set_encode_mode(1): each clip's single-clip encode in a concurrent lane): bit-identical
    # to encoding each clip alone, CTC collapse included
    ind = eng.encode(chunks, want_enc=True, independent=True)
    pairs = eng.ctc_collapse(60514, len(chunks))
    for b, c in enumerate(chunks):
        one = eng.encode([c], want_enc=True)
        p1 = eng.ctc_collapse(60514, 1)[0]
        assert np.array_equal(ind["audio_embd"][b], one["audio_embd"][0]), f"segment {b}: audio rows"
        assert np.array_equal(ind["enc"][b], one["enc"][0]) and np.array_equal(ind["ctc_ids"][b], one["ctc_ids"][0])
        assert np.array_equal(pairs[b][0], p1[0]) and np.array_equal(pairs[b][1], p1[1]), f"segment {b}: collapse"


def test_continuous_batching_slot_reuse_equals_per_clip():
    """configs[2]'s continuous batch with slot reuse, within the invariant width (N2): 10 ragged clips (3-20 s) with
    mixed decode lengths (5-40 tokens) on 4 sequence slots through decode_segments (core/scheduler.py: a finished
    clip's slot is refilled with the next clip, prefilled between decode chunks, while the other slots are mid-decode).
    Every clip's text, n_gen, CTC tokens and char timestamps equal decoding that clip alone bit for bit (the reference
    decodes every segment alone: orchestrator.py:139-171 -> core/decoder.py:132-246)."""
    from fun_asr_gguf import create_asr_engine
    from fun_asr_gguf.synthetic import synth_audio
    api = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="full",
                            max_batch=4, n_ctx=512, n_predict=40, ignore_eos=True)
    try:
        secs = [3.0, 17.5, 8.2, 20.0, 5.1, 12.7, 3.9, 15.3, 9.6, 6.4]
        n_pred = [5, 40, 12, 33, 7, 38, 21, 9, 26, 17]
        clips = [synth_audio(int(s * SR), 900 + i) for i, s in enumerate(secs)]
        orch = api.orchestrator
        got = orch.decode_segments(clips, None, None, False, 0.0, 1.0, 50, n_predicts=n_pred)
        st = dict(orch.batcher.stats)
        assert st["admissions"] == 10 > st["slots"] == 4 and st["batch_invariant"], st
        for i, (c, n, g) in enumerate(zip(clips, n_pred, got)):
            one = orch.decode_segments([c], None, None, False, 0.0, 1.0, 50, n_predicts=[n])[0]
            assert g.n_gen == one.n_gen == n, (i, g.n_gen, one.n_gen)
            assert g.ctc_results == one.ctc_results, f"clip {i}: CTC tokens"
            assert g.text == one.text, f"clip {i}: text"
            assert g.aligned == one.aligned, f"clip {i}: char timestamps"
        assert api.models.engine.llm_invariant_width() == 6
    finally:
        api.cleanup()


def test_llm_full_slot_reuse_above_width_bound(eng, cllm, g60):
    """Slot reuse above the invariant width (configs[2] shape): 40 ragged prompts on 32 slots. Slots 0-31 are prefilled
    as one batch; the first 8 clips stop after 8 steps, and their slots take clips 32-39 (one 8-prompt admission
    prefill while 24 sequences are mid-decode, slots reset and reused with their stale K/V rows still in the cache);
    then every slot decodes together, in admission order. 16 steps per clip, teacher-forced on each clip's single-stream
    tokens: the batch-32 bound of test_llm_full_batch32_vs_single_streams_bound (cosine >= 0.9995, equal argmax where
    the single-stream top-2 margin exceeds 0.15). The two clips on the first and last reused slot (32 on slot 0, 39 on
    slot 7: the stale K/V rows of clips 0 and 7 still in their caches past the new prompts) are also checked
    teacher-forced against the oracle (cref) fed the same tokens, not only against the GPU's own single-stream run."""
    adaptor = g60["adaptor"].astype(np.float32)
    base = _bench_prompts(eng, adaptor, 40)
    prompts = [p[:204 - 3 * (i % 7)] if i % 7 else p for i, p in enumerate(base)]  # ragged: 186-204 rows
    K = 16
    single = _single_runs(eng, prompts, K)
    n_steps = [8] * 8 + [K] * 32
    slot_of, k_of, order = {}, {}, []
    for s in range(32):
        eng.llm_reset(s)
    eng.llm_prefill_batch(list(range(32)), prompts[:32])
    for c in range(32):
        slot_of[c], k_of[c] = c, 0
        order.append(c)
    worst = 1.0
    kept = {32: [], 39: []}  # reused slots' logits per step, for the oracle check

    def check(c):
        nonlocal worst
        lg, ref = eng.llm_logits(slot_of[c]), single[c][1][k_of[c]]
        if c in kept:
            kept[c].append(lg)
        cs = _cos(lg, ref)
        worst = min(worst, cs)
        assert cs >= 0.9995, f"clip {c} step {k_of[c]}: cosine {cs}"
        top2 = np.sort(ref)[-2:]
        if top2[1] - top2[0] > 0.15:
            assert int(np.argmax(lg)) == int(np.argmax(ref)), f"clip {c} step {k_of[c]}: argmax"

    for c in order:
        check(c)
    admitted = False
    while order:
        for c in order:
            eng.llm_set_token(slot_of[c], single[c][0][k_of[c]])
        eng.llm_generate([slot_of[c] for c in order], 1)
        for c in order:
            k_of[c] += 1
            check(c)
        order = [c for c in order if k_of[c] < n_steps[c]]
        if not admitted and len(order) == 24:  # clips 0-7 finished: their slots take clips 32-39
            freed = sorted(set(range(32)) - {slot_of[c] for c in order})
            assert freed == list(range(8))
            for s in freed:
                eng.llm_reset(s)
            eng.llm_prefill_batch(freed, prompts[32:40])
            for c, s in zip(range(32, 40), freed):
                slot_of[c], k_of[c] = s, 0
                check(c)
                order.append(c)
            admitted = True
    assert admitted and all(k_of[c] == n_steps[c] for c in range(40))
    print(f"slot reuse above the width: worst cosine {worst:.6f}")
    for c, lgs in kept.items():
        assert len(lgs) == K + 1 and slot_of[c] in (0, 7)
        toks = single[c][0]
        _check_step(lgs[0], cllm.forward(prompts[c], 0))
        for k in range(K):
            _check_step(lgs[k + 1], cllm.forward(cllm.embed_tokens([toks[k]]), prompts[c].shape[0] + k))


def test_long_prompt_prefilled_alone_in_row_local_batch(monkeypatch):
    """A prompt above the row-local limit (FUNASR_PF_ROW_LOCAL_MAX; default 1024 rows, above which the tiled forward is
    faster: scripts/prof_prefill_long.py) prefills on the tiled forward when alone, so a row-local batch prefills it
    alone too: every prompt's first token, and the logits of the next decode step (a batch of 3 within the invariant
    width), equal its single-prompt run bit for bit."""
    from fun_asr_gguf import _native
    monkeypatch.setenv("FUNASR_PF_ROW_LOCAL_MAX", "100")
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_FULL, n_ctx=512, max_seqs=4), max_batch=1, max_samples=SR * 2)
    try:
        e.synthetic_weights(0)
        rng = np.random.default_rng(5)
        prompts = [(rng.standard_normal((n, 1024)) * 0.05).astype(np.float32) for n in (204, 80, 150)]
        single = []
        for p in prompts:
            e.llm_reset(0)
            t, lg = e.llm_prefill(0, p, want_logits=True)
            t1 = int(e.llm_generate([0], 1)[0][0])
            single.append((int(t), lg, t1, e.llm_logits(0)))
        for s in range(3):
            e.llm_reset(s)
        toks = e.llm_prefill_batch([0, 1, 2], prompts)
        assert [int(t) for t in toks] == [x[0] for x in single]
        assert np.array_equal(e.llm_logits(1), single[1][1])  # the row-local part of the batch (its last forward)
        nxt = e.llm_generate([0, 1, 2], 1)[:, 0]
        for s in range(3):
            assert int(nxt[s]) == single[s][2] and np.array_equal(e.llm_logits(s), single[s][3]), f"prompt {s}"
    finally:
        e.close()


def test_prefill_rows_assembled_on_device_equal_host_prompts(eng):
    """fa_llm_prefill_rows (prompt rows assembled in HBM from the caller's prefix / suffix rows and the last encode's
    adaptor rows, core/decoder.PromptRows) against the reference's host concatenation (core/decoder.py:199) through
    fa_llm_prefill / fa_llm_prefill_batch: first tokens and last-row logits bit-identical for one prompt, a row-local
    batch of 3 (from a padded-batch encode and from independent-clip lanes, whose adaptor rows sit at another row
    stride) and a tiled batch of 8 (above the invariant width); a later encode invalidates the rows (loud failure,
    and prefill_group falls back to the host rows)."""
    from fun_asr_gguf.core.decoder import PromptRows, prefill_group
    from fun_asr_gguf.synthetic import synth_audio
    rng = np.random.default_rng(77)
    clips = [synth_audio(int(s * SR), 700 + i) for i, s in enumerate((9.5, 4.2, 7.0, 3.1, 5.5, 6.6, 2.2, 8.8))]
    pre = [eng.embd_rows(rng.integers(0, 151933, 73).astype(np.int32)) for _ in range(2)]
    suf = eng.embd_rows(rng.integers(0, 151933, 5).astype(np.int32))

    def run(n, independent=False):
        out = eng.encode(clips[:n], independent=independent)
        gen = out["enc_gen"]
        assert gen >= 0 and gen == eng.encode_generation()
        rows = [PromptRows(pre[b % 2], out["audio_embd"][b], suf, b, gen) for b in range(n)]
        host = [np.concatenate([pre[b % 2], out["audio_embd"][b], suf], 0) for b in range(n)]
        assert all(np.array_equal(np.asarray(r), h) for r, h in zip(rows, host))
        seqs = list(range(n))
        for s in seqs:
            eng.llm_reset(s)
        if n == 1:
            t_host, lg_host = eng.llm_prefill(0, host[0], want_logits=True)
            t_host, lg_host = [t_host], [lg_host]
        else:
            t_host = eng.llm_prefill_batch(seqs, host)
            lg_host = [eng.llm_logits(s) for s in seqs]
        for s in seqs:
            eng.llm_reset(s)
        t_dev = eng.llm_prefill_rows(seqs, rows)
        assert [int(t) for t in t_dev] == [int(t) for t in t_host], f"batch {n}: first tokens"
        for s in seqs:
            assert np.array_equal(eng.llm_logits(s), lg_host[s]), f"batch {n}: logits of prompt {s}"
        return rows

    run(1)
    run(3)
    run(3, independent=True)  # lane layout (the scheduler's front(independent=alone)): clip b's rows at b * tl_max
    rows = run(8)
    eng.encode(clips[:1])  # replaces the adaptor rows the PromptRows point at
    for s in range(8):
        eng.llm_reset(s)
    with pytest.raises(RuntimeError, match="adaptor rows"):
        eng.llm_prefill_rows(list(range(8)), rows)
    for s in range(8):
        eng.llm_reset(s)
    t_fb = prefill_group(eng, list(range(8)), rows, dict(temperature=0.0))  # host fallback
    for s in range(8):
        eng.llm_reset(s)
    t_ref = eng.llm_prefill_batch(list(range(8)), [np.asarray(r) for r in rows])
    assert [int(t) for t in t_fb] == [int(t) for t in t_ref]
    bad = PromptRows(pre[0], rows[0].audio, suf, 5, eng.encode_generation())  # clip 5 of a 1-clip encode
    eng.llm_reset(0)
    with pytest.raises(RuntimeError, match="out of range"):
        eng.llm_prefill_rows([0], [bad])


def test_write_after_barrier_gemm_staging_bit_identical(monkeypatch):
    """The 256x256 / 128x128 bf16x3 tiles' write-after-barrier staging (FUNASR_BF3_256_S=1, the default) keeps every
    product's MFMA order: a batch of eight 60 s clips (M = 8008: the encoder GEMMs and the CTC projection with its fused
    argmax on the 256x256 tile) encodes bit-identically with the earlier load-then-store schedule."""
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    clips = [synth_audio(SR * 60, 300 + i) for i in range(8)]
    outs = []
    for sched in ("0", "1"):
        monkeypatch.setenv("FUNASR_BF3_256_S", sched)
        e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=8,
                           max_samples=SR * 62)
        try:
            e.synthetic_weights(0)
            outs.append(e.encode(clips, want_enc=True))
        finally:
            e.close()
    for b in range(len(clips)):
        assert np.array_equal(outs[0]["enc"][b], outs[1]["enc"][b]), f"clip {b}: encoder rows"
        assert np.array_equal(outs[0]["audio_embd"][b], outs[1]["audio_embd"][b]), f"clip {b}: adaptor rows"
        assert np.array_equal(outs[0]["ctc_ids"][b], outs[1]["ctc_ids"][b]), f"clip {b}: CTC ids"


def test_encoder_activation_planes_bit_identical(monkeypatch):
    """bf16x3 encoder: the SANM blocks' GEMM inputs written as bf16 hi / lo planes by their producers (layernorm, the
    attention epilogue, the ffn1 epilogue) instead of f32 rows split by the GEMM's staging. The split is the same, so
    every product is: a batch of eight 60 s clips (the 256x256 tile) and one 60 s clip (the few-tile shapes) encode
    bit-identically with f32 rows (FUNASR_ENC_PLANES=0), with planes at every size (=2) staged by registers or by
    LDS-DMA (k_gemm_bf3_256d, FUNASR_BF3_DMA=1), as persistent blocks (FUNASR_BF3_PERSIST=1), and with the default (=1:
    planes below the 256x256 tile's sizes)."""
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    clips = [synth_audio(SR * 60, 400 + i) for i in range(8)]
    outs = []
    modes = (("0", "1", "0"), ("2", "1", "0"), ("2", "0", "0"), ("0", "1", "1"), ("2", "1", "1"), ("2", "0", "1"),
             ("1", "0", "0"))  # 2: planes at every size; 1 (default): below enc_planes_max_rows
    for planes, dma, persist in modes:  # ..., and as persistent blocks (FUNASR_BF3_PERSIST=1)
        monkeypatch.setenv("FUNASR_ENC_PLANES", planes)
        monkeypatch.setenv("FUNASR_BF3_DMA", dma)
        monkeypatch.setenv("FUNASR_BF3_PERSIST", persist)
        e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=8,
                           max_samples=SR * 62)
        try:
            e.synthetic_weights(0)
            outs.append((e.encode(clips, want_enc=True), e.encode(clips[3:4], want_enc=True)))
        finally:
            e.close()
    for v in range(1, len(modes)):
        for k in range(2):
            for b in range(len(outs[0][k]["enc"])):
                assert np.array_equal(outs[0][k]["enc"][b], outs[v][k]["enc"][b]), f"mode {v} call {k} clip {b}: encoder"
                assert np.array_equal(outs[0][k]["audio_embd"][b], outs[v][k]["audio_embd"][b]), f"mode {v} {k} {b}"
                assert np.array_equal(outs[0][k]["ctc_ids"][b], outs[v][k]["ctc_ids"][b]), f"mode {v} {k} {b}: CTC ids"


@pytest.mark.parametrize("fp16", [False, True])
def test_encoder_attention_xcd_order_bit_identical(monkeypatch, fp16):
    """The encoder attention's XCD-aware block order (FUNASR_ATTN_XCD=1, off by default: the query tiles of one (key split,
    head, clip) group dispatched to one XCD so its L2 fetches their K/V rows once) is a permutation of the same blocks:
    eight 60 s clips (no key splits) and one 60 s clip (key splits) encode bit-identically with the dispatch order, in
    the bf16x3 and the fp16 graphs."""
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    clips = [synth_audio(SR * 60, 500 + i) for i in range(8)]
    outs = []
    for xo in ("0", "1"):
        monkeypatch.setenv("FUNASR_ATTN_XCD", xo)
        e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=8,
                           max_samples=SR * 62)
        try:
            e.synthetic_weights(0)
            e.set_encoder_fp16(fp16)
            outs.append((e.encode(clips, want_enc=True), e.encode(clips[5:6], want_enc=True)))
        finally:
            e.close()
    for k in range(2):
        for b in range(len(outs[0][k]["enc"])):
            assert np.array_equal(outs[0][k]["enc"][b], outs[1][k]["enc"][b]), f"call {k} clip {b}: encoder rows"
            assert np.array_equal(outs[0][k]["audio_embd"][b], outs[1][k]["audio_embd"][b]), f"call {k} clip {b}"



@pytest.mark.parametrize("fp16", [False, True])
def test_encoder_attention_split_merge_launch_bit_identical(monkeypatch, fp16):
    """The one-clip encoder attention's key splits merged by their own launch (k_attn_merge, FUNASR_ATTN_MERGE=1, the
    default: every tile's partials read by 8 blocks) run the last-arriving split's merge arithmetic: one 60 s clip
    (eight key splits) and a batch of two (no splits) encode bit-identically with the in-launch merge, in the bf16x3 and
    the fp16 graphs; and with 1 and 32 query slices per merge block."""
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    clips = [synth_audio(SR * 60, 600 + i) for i in range(2)]
    outs = []
    for merge, ms in (("0", "8"), ("1", "8"), ("1", "1"), ("1", "32")):
        monkeypatch.setenv("FUNASR_ATTN_MERGE", merge)
        monkeypatch.setenv("FUNASR_ATTN_MS", ms)
        e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=2,
                           max_samples=SR * 62)
        try:
            e.synthetic_weights(0)
            e.set_encoder_fp16(fp16)
            outs.append((e.encode(clips[:1], want_enc=True), e.encode(clips, want_enc=True)))
        finally:
            e.close()
    for v in range(1, len(outs)):
        for k in range(2):
            for b in range(len(outs[0][k]["enc"])):
                assert np.array_equal(outs[0][k]["enc"][b], outs[v][k]["enc"][b]), f"mode {v} call {k} clip {b}: encoder"
                assert np.array_equal(outs[0][k]["audio_embd"][b], outs[v][k]["audio_embd"][b]), f"mode {v} {k} {b}"
                assert np.array_equal(outs[0][k]["ctc_ids"][b], outs[v][k]["ctc_ids"][b]), f"mode {v} {k} {b}: CTC"


@pytest.mark.parametrize("fp16", [False, True])
def test_encoder_ffn2_k_split_matches_unsplit(monkeypatch, fp16):
    """One clip's ffn2 on 128x128 tiles with K split over 8 blocks and a split-order reduce launch (FUNASR_BF3_SK /
    FUNASR_F16_SK = 1, the default) against the unsplit K-group tile (= 0): only the f32 summation order of the split
    differs, so the 60 s clip's encoder rows agree to the encoder's f32 bar (fp16 graph: its own bar, the rounding to
    fp16 after every op lets one-ulp flips travel), and the split path is deterministic."""
    from fun_asr_gguf import _native
    from fun_asr_gguf.synthetic import synth_audio
    clip = [synth_audio(SR * 60, 700)]
    outs = []
    for v in ("0", "1", "1"):
        monkeypatch.setenv("FUNASR_BF3_SK", v)
        monkeypatch.setenv("FUNASR_F16_SK", v)
        e = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=1,
                           max_samples=SR * 62)
        try:
            e.synthetic_weights(0)
            e.set_encoder_fp16(fp16)
            outs.append(e.encode(clip, want_enc=True))
        finally:
            e.close()
    assert np.array_equal(outs[1]["enc"][0], outs[2]["enc"][0]), "split path not deterministic"
    a, b = outs[0]["enc"][0], outs[1]["enc"][0]
    if fp16:
        assert _rel(b, a) < 1e-2 and _cos(b, a) > 0.9999
    else:
        assert _rel(b, a) < ENC_ATOL and _cos(b, a) > ENC_COS
