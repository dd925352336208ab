"""Pin the C++/OpenMP restatement (oracle/cref) before trusting it as the full-size oracle of the GPU parity tests
and as bench.py's CPU baseline: against the reference goldens (generated from /root/reference's own
model_definition.py, tests/golden/make_golden.py) and against the numpy oracle.

Bars: encoder fp32 max-abs / max <= 1e-5 vs the reference (same bar as the numpy oracle meets); CTC ids exact on
non-tie frames; synthetic q8_0 tensors byte-identical; decoder logits cosine >= 0.9995 vs the numpy oracle with
equal argmax where its top-2 margin exceeds 0.25 (q8_0 activation rounding noise, test_qwen3_q8_noise_floor).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import cref, encoder as oenc, q8, qwen3 as oqw, synth


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-6, float(np.abs(b).max())))


def _cos(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


@pytest.fixture(scope="module")
def cenc_tiny():
    e = cref.CEncoder(synth.ENC_TINY)
    yield e
    e.close()


@pytest.mark.parametrize("tag", ["tiny_3s", "tiny_pad2s"])
def test_cref_encoder_tiny_vs_reference_golden(cenc_tiny, tag):
    g = np.load(os.path.join(GOLDEN, f"encoder_{tag}.npz"))
    valid = int(g["valid"])
    r = cenc_tiny.encode(g["audio"][:valid])
    T = int(g["t_lfr_valid"])
    assert _rel(r["enc"][:T], g["enc"][:T]) < 1e-5
    assert r["target_len"] == int(g["target_len"])
    assert _rel(r["audio_embd"], g["adaptor"]) < 1e-5
    nontie = g["ctc_margin"] > 1e-3
    assert ((r["ctc_ids"][:T] != g["ctc_ids"]) & nontie).sum() == 0


def test_cref_encoder_ragged_vs_numpy_oracle(cenc_tiny):
    """valid < physical length (padded clip) and a clip under 1 s, against oracle.encoder.encode."""
    from fun_asr_gguf.synthetic import synth_audio
    W = synth.make_weights(synth.encoder_tensors(synth.ENC_TINY))
    for n, valid, seed in ((16000 * 2 + 77, 16000 + 5, 1), (9000, 9000, 2)):
        a = synth_audio(n, seed)
        a[valid:] = 0
        r = cenc_tiny.encode(a, valid)
        o = oenc.encode(a, W, synth.ENC_TINY, valid=valid)
        assert _rel(r["enc"], o["enc"]) < 1e-5
        assert _rel(r["adaptor"], o["adaptor"]) < 1e-5
        s = np.sort(o["ctc_logits"], -1)
        marg = s[:, -1] - s[:, -2]
        assert ((r["ctc_ids"] != o["ctc_ids"]) & (marg > 1e-3)).sum() == 0
        assert np.abs(r["ctc_margin"] - marg).max() < 1e-3


@pytest.mark.slow
def test_cref_encoder_full_10s_vs_reference_golden():
    g = np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))
    e = cref.CEncoder(synth.ENC_FULL)
    r = e.encode(g["audio"])
    e.close()
    T = int(g["t_lfr_valid"])
    assert _rel(r["enc"][:T], g["enc"][:T]) < 1e-5
    assert _rel(r["audio_embd"], g["adaptor"]) < 1e-5
    assert ((r["ctc_ids"][:T] != g["ctc_ids"]) & (g["ctc_margin"] > 1e-3)).sum() == 0


def test_cref_decoder_tiny_vs_numpy_oracle():
    cfg = synth.LLM_TINY
    W = synth.make_weights(synth.llm_tensors(cfg))
    m = oqw.Qwen3Q8(W, cfg, n_ctx=256)
    c = cref.CQwen3(cfg, n_ctx=256)
    for name, shape, _, _ in synth.llm_tensors(cfg):
        if len(shape) == 2:
            d, q = q8.quantize_q8_0(W[name])
            assert (c.tensor_q8(name, int(np.prod(shape))) == q8.pack_q8_0(d, q).ravel()).all(), name
    ids = np.array([0, 7, 4095, 1234], np.int32)
    assert (c.embed_prompt(ids) == m.embed_prompt(ids)).all()
    assert (c.embed_tokens(ids) == m.embed_tokens(ids)).all()
    rng = np.random.default_rng(3)
    p = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 30)),
                        (rng.standard_normal((21, 1024)) * 0.5).astype(np.float32)], 0)
    a, b = c.forward(p, 0), m.forward(p, 0)
    assert _cos(a, b) > 0.9995
    pos, tok = p.shape[0], int(np.argmax(b))
    for _ in range(6):
        a = c.forward(m.embed_tokens([tok]), pos)
        b = m.forward(m.embed_tokens([tok]), pos)
        assert _cos(a, b) > 0.9995
        s = np.sort(b)
        if s[-1] - s[-2] > 0.25:
            assert int(np.argmax(a)) == int(np.argmax(b))
        tok, pos = int(np.argmax(b)), pos + 1


def test_cref_decoder_full_vs_hf():
    """cref's decoder at full dims (28 layers, vocab 151936, GQA 16/8, RoPE theta 1e6 at positions 204-215) against
    HF Qwen3 on the configs[1] prompt, teacher-forced on HF's greedy ids (tests/hf_full.py for the bars)."""
    import hf_full
    g, adaptor = hf_full.load()
    c = cref.CQwen3(synth.LLM_FULL, n_ctx=512)
    try:
        hf_full.check(g, 0, c.forward(hf_full.prompt(g, adaptor, c.embed_prompt), 0))
        pos = 204
        for i, t in enumerate(g["greedy"]):
            hf_full.check(g, i + 1, c.forward(c.embed_tokens([int(t)]), pos))
            pos += 1
    finally:
        c.close()
