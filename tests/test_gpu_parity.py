"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle and the reference goldens.

Tolerances (written here, per SURVEY §8(c) / experience/03 ONNX_Export_Optimization_Experience.md:68-73):
  encoder/adaptor fp32: max-abs <= ENC_ATOL_* relative to the tensor's max, cosine >= 0.99999 (tiny configs), >= 0.999999
  at full depth (ENC_ATOL_FULL)
  CTC ids: exact on frames whose top-1/top-2 logit margin exceeds 1e-3 (non-tie frames)
  decoder (q8_0 integer-dot numerics on both sides): logits cosine >= 0.9999, greedy ids equal
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import ctc as octc, encoder as oenc, frontend as ofe, q8 as oq8, qwen3 as oqw, synth

pytestmark = pytest.mark.gpu

ENC_ATOL_TINY = 5e-5
ENC_ATOL_FULL = 1e-4  # max-abs <= 1e-4 of the max, cosine >= 0.999999 at full depth


def _cos(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-6, float(np.abs(b).max())))


@pytest.fixture(scope="module")
def tiny_engine():
    from fun_asr_gguf import _native
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=512, max_seqs=8), max_batch=4,
                         max_samples=16000 * 4)
    eng.synthetic_weights(0)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def enc_w_tiny():
    return synth.make_weights(synth.encoder_tensors(synth.ENC_TINY))


@pytest.fixture(scope="module")
def llm_tiny_oracle():
    return oqw.Qwen3Q8(synth.make_weights(synth.llm_tensors(synth.LLM_TINY)), synth.LLM_TINY, n_ctx=512)


def test_synthetic_f32_weights_bit_exact(tiny_engine, enc_w_tiny):
    """Device hash of every f32 encoder / norm tensor == the numpy spec (oracle/synth.py), bit for bit (two IEEE
    roundings for the offset-1 LayerNorm weights: no fused multiply-add)."""
    for name, w in enc_w_tiny.items():
        assert (tiny_engine.get_tensor_f32(name, w.size) == w.ravel()).all(), name
    for name, shape, scale, off in synth.llm_tensors(synth.LLM_TINY):
        if len(shape) == 1 and name.startswith(("blk.1.", "output_norm")):
            assert (tiny_engine.get_tensor_f32(name, shape[0]) == synth.gen(name, shape[0], scale, off, 0)).all(), name


def test_synthetic_q8_weights_bit_exact(tiny_engine):
    """Device hash + device ggml quantiser == numpy hash + reference quantiser, byte for byte."""
    cfg = synth.LLM_TINY
    for name, shape, scale, off in synth.llm_tensors(cfg):
        if name not in ("token_embd.weight", "blk.1.attn_k.weight", "blk.0.ffn_down.weight", "blk.1.attn_output.weight"):
            continue
        w = synth.gen(name, int(np.prod(shape)), scale, off, 0).reshape(shape)
        d, q = oq8.quantize_q8_0(w)
        want = oq8.pack_q8_0(d, q).ravel()
        got = tiny_engine.get_tensor_q8_0(name, int(np.prod(shape)))
        assert (got == want).all(), name


@pytest.mark.parametrize("tag", ["tiny_3s", "tiny_pad2s"])
def test_encoder_tiny_vs_reference_golden(tiny_engine, enc_w_tiny, tag):
    g = np.load(os.path.join(GOLDEN, f"encoder_{tag}.npz"))
    valid = int(g["valid"])
    audio = g["audio"][:valid]  # the golden is the padded==unpadded reference result for the valid part
    out = tiny_engine.encode([audio], want_enc=True, debug_lfr=True)
    T = int(g["t_lfr_valid"])
    lfr_emb = g["lfr"][:T] * np.float32(512 ** 0.5) + ofe.sinusoidal_pe(g["lfr"].shape[0], 560)[:T]
    assert _rel(out["lfr_embedded"][:T], lfr_emb) < 1e-4  # same bar as the oracle vs reference
    enc = out["enc"][0][:T]
    assert _rel(enc, g["enc"][:T]) < ENC_ATOL_TINY and _cos(enc, g["enc"][:T]) > 0.99999
    emb = out["audio_embd"][0]
    assert emb.shape[0] == int(g["target_len"])
    assert _rel(emb, g["adaptor"]) < ENC_ATOL_TINY
    ids = out["ctc_ids"][0][:T]
    nontie = g["ctc_margin"] > 1e-3
    assert ((ids != g["ctc_ids"]) & nontie).sum() == 0


def test_encoder_padded_batch_equals_unpadded(tiny_engine, enc_w_tiny):
    """Ragged batch (incl. a < 1 s clip, CPU-EP 1 s padding policy) vs per-clip oracle runs."""
    from fun_asr_gguf.synthetic import synth_audio
    lens = [41234, 8000, 16000 * 3 + 7, 15999]
    clips = [synth_audio(n, 20 + i) for i, n in enumerate(lens)]
    out = tiny_engine.encode(clips, want_enc=True)
    for i, c in enumerate(clips):
        n = len(c)
        phys = max(n, 16000)
        a = np.zeros(phys, np.float32)
        a[:n] = c
        r = oenc.encode(a, enc_w_tiny, synth.ENC_TINY, valid=n)
        tl = r["counts"]["t_lfr_phys"]
        assert out["enc"][i].shape[0] == tl
        assert _rel(out["enc"][i], r["enc"]) < ENC_ATOL_TINY, i
        assert _rel(out["audio_embd"][i], r["audio_embd"]) < ENC_ATOL_TINY, i
        lg = r["ctc_logits"]
        top2 = np.sort(lg, -1)[:, -2:]
        nontie = (top2[:, 1] - top2[:, 0]) > 1e-3
        assert ((out["ctc_ids"][i] != r["ctc_ids"]) & nontie).sum() == 0, i


# fp16 encoder graph (C5): GPU vs oracle/encoder_fp16 (same fp16 rounding points; differences are f32
# accumulation order, i.e. occasional 1-ulp fp16 flips), and loosely vs the fp32 reference golden.
FP16_REL, FP16_COS = 1e-2, 0.99995


def test_encoder_fp16_graph_vs_oracle(tiny_engine, enc_w_tiny):
    from oracle import encoder_fp16 as oe16
    g = np.load(os.path.join(GOLDEN, "encoder_tiny_3s.npz"))
    valid = int(g["valid"])
    audio = g["audio"][:valid]
    tiny_engine.set_encoder_fp16(True)
    try:
        out = tiny_engine.encode([audio], want_enc=True)
    finally:
        tiny_engine.set_encoder_fp16(False)
    r = oe16.encode(audio, enc_w_tiny, synth.ENC_TINY)
    T = int(g["t_lfr_valid"])
    enc, emb = out["enc"][0][:T], out["audio_embd"][0]
    assert (emb.astype(np.float16).astype(np.float32) == emb).all()  # fp16 values
    assert _rel(enc, r["enc"][:T]) < FP16_REL and _cos(enc, r["enc"][:T]) > FP16_COS
    assert _rel(emb, r["audio_embd"]) < FP16_REL and _cos(emb, r["audio_embd"]) > FP16_COS
    assert _cos(emb, g["adaptor"]) > 0.9995  # fp32 reference, fp16 accuracy
    lg = r["ctc_logits"][:T]
    top2 = np.sort(lg, -1)[:, -2:]
    nontie = (top2[:, 1] - top2[:, 0]) > 0.05
    assert ((out["ctc_ids"][0][:T] != r["ctc_ids"][:T]) & nontie).sum() == 0
    # the engine is back on the fp32 graph: bit-for-bit the result it gave before the switch
    out32 = tiny_engine.encode([audio], want_enc=True)
    assert _rel(out32["audio_embd"][0], g["adaptor"]) < ENC_ATOL_TINY


def test_encoder_fp16_graph_padded_batch(tiny_engine, enc_w_tiny):
    """fp16 graph on a ragged batch (incl. a < 1 s clip): each clip equals its own unpadded fp16-oracle run."""
    from fun_asr_gguf.synthetic import synth_audio
    from oracle import encoder_fp16 as oe16
    lens = [16000 * 2 + 321, 9000]
    clips = [synth_audio(n, 40 + i) for i, n in enumerate(lens)]
    tiny_engine.set_encoder_fp16(True)
    try:
        out = tiny_engine.encode(clips, want_enc=True)
    finally:
        tiny_engine.set_encoder_fp16(False)
    for i, c in enumerate(clips):
        n = len(c)
        a = np.zeros(max(n, 16000), np.float32)
        a[:n] = c
        r = oe16.encode(a, enc_w_tiny, synth.ENC_TINY, valid=n)
        assert _rel(out["enc"][i], r["enc"]) < FP16_REL and _cos(out["enc"][i], r["enc"]) > FP16_COS, i
        assert _rel(out["audio_embd"][i], r["audio_embd"]) < FP16_REL, i


def test_ctc_collapse_matches_reference_rule(tiny_engine):
    from fun_asr_gguf.synthetic import synth_audio
    clips = [synth_audio(30000, 5), synth_audio(20000, 6)]
    out = tiny_engine.encode(clips)
    blank = synth.ENC_TINY["ctc_vocab"] - 1
    col = tiny_engine.ctc_collapse(blank, 2)
    for b in range(2):
        want = octc.collapse(out["ctc_ids"][b], blank)
        assert [int(x) for x in col[b][0]] == [t for t, _ in want]
        assert [int(x) for x in col[b][1]] == [s for _, s in want]


def test_embedding_rows(tiny_engine, llm_tiny_oracle):
    ids = np.array([0, 5, 4095, 17, 2048], np.int32)
    assert (tiny_engine.embd_rows(ids, True) == llm_tiny_oracle.embed_prompt(ids)).all()
    assert (tiny_engine.embd_rows(ids, False) == llm_tiny_oracle.embed_tokens(ids)).all()


# q8_0 activation rounding makes the logits jump by ~0.05 under 1e-7 input noise (measured on the oracle
# itself: tests/test_oracle_golden.py::test_qwen3_q8_noise_floor), so decoder parity is teacher-forced:
# per-step logits cosine >= 0.9995 and equal argmax wherever the oracle's top-2 margin exceeds TIE_MARGIN.
TIE_MARGIN = 0.25


def _check_step(gpu, ref):
    assert _cos(gpu, ref) > 0.9995
    s = np.sort(ref)
    if s[-1] - s[-2] > TIE_MARGIN:
        assert int(np.argmax(gpu)) == int(np.argmax(ref))


def test_llm_prefill_and_decode_teacher_forced_tiny(tiny_engine, llm_tiny_oracle):
    m = llm_tiny_oracle
    rng = np.random.default_rng(3)
    prompt = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 30)),
                             (rng.standard_normal((21, 1024)) * 0.5).astype(np.float32)], 0)
    tiny_engine.llm_reset(0)
    tok, lg = tiny_engine.llm_prefill(0, prompt, want_logits=True)
    m.reset()
    ref = m.forward(prompt, 0)
    _check_step(lg, ref)
    assert tok == int(np.argmax(lg))
    pos = prompt.shape[0]
    for _ in range(12):
        nxt = tiny_engine.llm_generate([0], 1)[0][0]
        lg_new = tiny_engine.llm_logits(0)
        ref = m.forward(m.embed_tokens([tok]), pos)  # the token the GPU fed at this step
        _check_step(lg_new, ref)
        assert nxt == int(np.argmax(lg_new))
        tok, pos = int(nxt), pos + 1
    assert tiny_engine.llm_n_past(0) == prompt.shape[0] + 12


def test_llm_long_context_split_attention(tiny_engine, llm_tiny_oracle):
    """400-token context: the decode/prefill attention cuts keys over 13 blocks and combines their partials
    (last-arriving block); teacher-forced against the oracle at every step."""
    m = llm_tiny_oracle
    rng = np.random.default_rng(5)
    prompt = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 150)),
                             (rng.standard_normal((250, 1024)) * 0.5).astype(np.float32)], 0)
    tiny_engine.llm_reset(1)
    tok, lg = tiny_engine.llm_prefill(1, prompt, want_logits=True)
    m.reset()
    ref = m.forward(prompt, 0)
    _check_step(lg, ref)
    pos = prompt.shape[0]
    for _ in range(5):
        nxt = tiny_engine.llm_generate([1], 1)[0][0]
        lg_new = tiny_engine.llm_logits(1)
        ref = m.forward(m.embed_tokens([tok]), pos)
        _check_step(lg_new, ref)
        tok, pos = int(nxt), pos + 1


@pytest.mark.parametrize("n_seq", [6, 8])
def test_llm_batched_decode_teacher_forced(tiny_engine, llm_tiny_oracle, n_seq):
    """n_seq sequences decode as one batch: M=6 on the fused GEMV with 2 tokens per block (3 blocks rows), M=8
    with every GEMM (and the lm_head + argmax partials) on the int8 MFMA path; each row's logits are checked
    against the oracle run of that sequence alone."""
    m = llm_tiny_oracle
    rng = np.random.default_rng(6)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (7, 19, 33, 12, 70, 45, 26, 9)[:n_seq]]
    toks = []
    for s_, p in enumerate(prompts):
        tiny_engine.llm_reset(s_)
        toks.append(tiny_engine.llm_prefill(s_, p))
    seqs = list(range(len(prompts)))
    fed = [[t] for t in toks]  # tokens fed so far per sequence (first = the prefill's sampled token)
    for _ in range(3):
        nxt = tiny_engine.llm_generate(seqs, 1)[:, 0]
        for s_, p in enumerate(prompts):
            lg = tiny_engine.llm_logits(s_)
            m.reset()
            m.forward(p, 0)
            for k, t in enumerate(fed[s_]):
                ref = m.forward(m.embed_tokens([t]), p.shape[0] + k)
            _check_step(lg, ref)
            assert int(nxt[s_]) == int(np.argmax(lg))
        for s_ in seqs:
            fed[s_].append(int(nxt[s_]))


def test_llm_batch20_lean_attention_chunked_combine(llm_tiny_oracle):
    """20 sequences decode as one M=20 batch: 6 key splits x 20 x 8 blocks > 3 per CU, so the lean (128-VGPR)
    attention variant runs, and contexts past 160 keys give 5-6 active splits, merged in two chunks of 4; the
    split-K GEMMs and the batched LM head at M=20. Rows checked against the oracle run of that sequence alone."""
    from fun_asr_gguf import _native
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=320, max_seqs=20), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    m = llm_tiny_oracle
    rng = np.random.default_rng(8)
    lens = [int(n) for n in rng.integers(3, 280, 20)]
    lens[0], lens[1] = 250, 200  # at least two contexts with 6 and 5 active splits
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in lens]
    toks = []
    for s_, p in enumerate(prompts):
        eng.llm_reset(s_)
        toks.append(eng.llm_prefill(s_, p))
    nxt = eng.llm_generate(list(range(20)), 1)[:, 0]
    for s_ in (0, 1, 5, 9, 14, 19):
        lg = eng.llm_logits(s_)
        m.reset()
        m.forward(prompts[s_], 0)
        ref = m.forward(m.embed_tokens([toks[s_]]), prompts[s_].shape[0])
        _check_step(lg, ref)
        assert int(nxt[s_]) == int(np.argmax(lg))
    eng.close()


@pytest.mark.parametrize("ob", ["1", "0"])
def test_llm_batch32_wide_attention_long_contexts(monkeypatch, ob):
    """M = 32 decode: the wide attention launch (one 16-wave block per (token, kv head), no key splits) over contexts of
    3 .. 651 keys in one launch -- with the o projection, residual and normalising epilogue in the same launch
    (k_attn_ob, FUNASR_ATTN_OB=1, the default: a 32-block head fan-in, MFMA o tiles, last-arriver head sum) and as the
    separate o GEMM (=0). Rows checked teacher-forced against the oracle run of each sequence alone, over two steps; no
    in-launch hand-off timed out."""
    from fun_asr_gguf import _native
    monkeypatch.setenv("FUNASR_ATTN_OB", ob)
    m = oqw.Qwen3Q8(synth.make_weights(synth.llm_tensors(synth.LLM_TINY)), synth.LLM_TINY, n_ctx=700)
    rng = np.random.default_rng(32)
    lens = [int(n) for n in rng.integers(3, 300, 32)]
    lens[0], lens[1], lens[2], lens[3] = 510, 515, 600, 650
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in lens]
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=700, max_seqs=32), max_batch=1, max_samples=16000)
    try:
        eng.synthetic_weights(0)
        toks = []
        for s_, p in enumerate(prompts):
            eng.llm_reset(s_)
            toks.append(eng.llm_prefill(s_, p))
        steps, lgs = [], []
        for k in range(2):
            steps.append(eng.llm_generate(list(range(32)), 1)[:, 0])
            lgs.append({s_: eng.llm_logits(s_) for s_ in (0, 1, 2, 3, 7, 19, 31)})
        assert eng.llm_decode_recoveries() == (0, 0)
    finally:
        eng.close()
    for s_ in (0, 1, 2, 3, 7, 19, 31):
        m.reset()
        m.forward(prompts[s_], 0)
        fed = [toks[s_], int(steps[0][s_])]
        for k in range(2):
            ref = m.forward(m.embed_tokens([fed[k]]), lens[s_] + k)
            _check_step(lgs[k][s_], ref)
            assert int(steps[k][s_]) == int(np.argmax(lgs[k][s_]))


def test_llm_continuous_batch_equals_single(tiny_engine, llm_tiny_oracle):
    """A sequence decoded inside a batch gives the tokens it gives alone on the same layer structure: the two-launch
    fused layer (a batch of 3 runs one grid slab per token; the batch-1 run completes the residual in the LM head's
    prologue, the batch in psum_rows: same order) and the 5-launch layer (fa_set_decode_fused(0))."""
    rng = np.random.default_rng(4)
    prompts = [llm_tiny_oracle.embed_prompt(rng.integers(0, 4096, n)) for n in (9, 17, 5)]
    try:
        for mode in (1, 0):
            tiny_engine.set_decode_fused(mode)
            singles = []
            for p in prompts:
                tiny_engine.llm_reset(0)
                t = tiny_engine.llm_prefill(0, p)
                singles.append([t] + list(tiny_engine.llm_generate([0], 10)[0]))
            firsts = []
            for s_, p in enumerate(prompts):
                tiny_engine.llm_reset(s_)
                firsts.append(tiny_engine.llm_prefill(s_, p))
            batch = tiny_engine.llm_generate([0, 1, 2], 10)
            for s_ in range(3):
                assert [firsts[s_]] + list(batch[s_]) == singles[s_], (mode, s_)
    finally:
        tiny_engine.set_decode_fused(True)


@pytest.mark.parametrize("M", [2, 6, 8])
def test_two_launch_layer_small_batches(llm_tiny_oracle, monkeypatch, M):
    """Decode batches of 2..8 sequences on the two-launch layer (one grid slab per token; sequences at different
    positions, non-contiguous ids) against the 5-launch layer and teacher-forced against the oracle; a token's logits
    equal its batch-1 logits on the same layer (bit-identical up to M = 6, the engine's fused-path width: the LM head is
    the batch-1 GEMV or the small-batch MFMA LM head, which sums every logit in the GEMV's order: per-token arithmetic
    does not depend on the batch)."""
    from fun_asr_gguf import _native
    m = llm_tiny_oracle
    monkeypatch.setenv("FUNASR_FUSED_MAX_M", "8")  # the default stops at the measured crossover (6)
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=512, max_seqs=16), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    rng = np.random.default_rng(30 + M)
    seqs = [1 + 2 * i for i in range(M - 1)] + [0]
    prompts = [m.embed_prompt(rng.integers(0, 4096, 6 + 11 * i)) for i in range(M)]
    runs = {}
    for mode in (1, 0):
        eng.set_decode_fused(mode)
        firsts = []
        for q, p in zip(seqs, prompts):
            eng.llm_reset(q)
            firsts.append(eng.llm_prefill(q, p))
        toks, lgs = [], []
        for _ in range(3):
            toks.append([int(t[0]) for t in eng.llm_generate(seqs, 1)])
            lgs.append([eng.llm_logits(q) for q in seqs])
        runs[mode] = (firsts, toks, lgs)
    # batch-1 reference on the same (two-launch) layer for the last sequence
    eng.set_decode_fused(1)
    q, p = seqs[-1], prompts[-1]
    eng.llm_reset(q)
    first1 = eng.llm_prefill(q, p)
    single = []
    for k in range(3):
        single.append((int(eng.llm_generate([q], 1)[0][0]), eng.llm_logits(q)))
    eng.close()
    (f1, t1, l1), (f0, t0, l0) = runs[1], runs[0]
    assert first1 == f1[-1]
    if [t[-1] for t in t1] == [tk for tk, _ in single]:
        for k in range(3):  # M <= 6: the batch-1 LM head's arithmetic; above, the batched MFMA LM head (f32 order)
            if M <= 6:
                assert np.array_equal(l1[k][-1], single[k][1])
            else:
                assert _cos(l1[k][-1], single[k][1]) > 0.999999
    for i in range(M):
        m.reset()
        m.forward(prompts[i], 0)
        fed = [f1[i]] + [t1[k][i] for k in range(3)]
        for k in range(3):
            ref = m.forward(m.embed_tokens([fed[k]]), prompts[i].shape[0] + k)
            _check_step(l1[k][i], ref)
            if fed[:k + 1] == ([f0[i]] + [t0[j][i] for j in range(3)])[:k + 1]:
                # M > 5: the 5-launch layer runs the MFMA GEMMs with producer-side quantisation (the same
                # integers except at exact .5 ties), so it sits within the q8_0 noise floor of the fused layer
                assert _cos(l1[k][i], l0[k][i]) > (0.99999 if M <= 5 else 0.9995)


@pytest.mark.slow
def test_encoder_full_10s_vs_reference_golden():
    from fun_asr_gguf import _native
    g = np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))
    eng = _native.Engine(synth.ENC_FULL, dict(synth.LLM_TINY, n_ctx=64), max_batch=1, max_samples=160000)
    eng.synthetic_weights(0)
    out = eng.encode([g["audio"]], want_enc=True)
    eng.close()
    T = int(g["t_lfr_valid"])
    assert _rel(out["enc"][0], g["enc"][:T]) < ENC_ATOL_FULL and _cos(out["enc"][0], g["enc"][:T]) > 0.999999
    assert _rel(out["audio_embd"][0], g["adaptor"]) < ENC_ATOL_FULL and _cos(out["audio_embd"][0], g["adaptor"]) > 0.999999
    nontie = g["ctc_margin"] > 1e-3
    assert ((out["ctc_ids"][0] != g["ctc_ids"]) & nontie).sum() == 0


def test_fused_decode_layer_vs_five_launch_layer(tiny_engine, llm_tiny_oracle):
    """The fused batch-1 layer (attention + split o projection, gate|up + split down projection, in-launch fan-ins)
    against the 5-launch layer on the same steps: logits equal up to f32 summation order, same greedy token where the
    margin is not a tie; teacher-forced against the oracle too; over a long context (12 active key splits). The
    two-launch fused layer (q|k|v GEMV inside the attention launch, default) and the three-launch one (the q|k|v GEMV
    as its own launch) compute the same arithmetic: bit-identical logits and tokens."""
    m = llm_tiny_oracle
    rng = np.random.default_rng(12)
    prompt = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 40)),
                             (rng.standard_normal((330, 1024)) * 0.5).astype(np.float32)], 0)
    runs = []
    for fused in (1, 0, 2):
        tiny_engine.set_decode_fused(fused)
        tiny_engine.llm_reset(0)
        tok = tiny_engine.llm_prefill(0, prompt)
        lgs, toks = [], [tok]
        for _ in range(8):
            toks.append(int(tiny_engine.llm_generate([0], 1)[0][0]))
            lgs.append(tiny_engine.llm_logits(0))
        runs.append((toks, lgs))
    tiny_engine.set_decode_fused(True)
    (tf, lf), (tu, lu), (t3, l3) = runs
    assert t3 == tf
    for k in range(8):
        assert np.array_equal(l3[k], lf[k])
    m.reset()
    m.forward(prompt, 0)
    for k in range(8):
        if tf[:k + 1] != tu[:k + 1]:
            break  # a tie flipped the fed token: later steps are different sequences
        assert _cos(lf[k], lu[k]) > 0.99999
        ref = m.forward(m.embed_tokens([tf[k]]), prompt.shape[0] + k)
        _check_step(lf[k], ref)
        s = np.sort(lu[k])
        if s[-1] - s[-2] > 1e-3:
            assert tf[k + 1] == tu[k + 1]


@pytest.mark.parametrize("t_min_m,apf_min_m", [(512, 512), (32, 512), (512, 16)])
def test_llm_prefill_batch_equals_per_sequence(llm_tiny_oracle, monkeypatch, t_min_m, apf_min_m):
    """fa_llm_prefill_batch: three prompts of different lengths in one forward (each row attends its own sequence's
    keys) against prefilling each alone: same first token (non-tie margins), logits within the q8_0 noise floor (the
    batch takes other GEMM shapes, so f32 summation orders differ), positions advanced, and the first decode step
    teacher-forced against the oracle. t_min_m = 32 sends the batch (68 rows) and the 35-row prompt through the
    128x128-tile q8_0 GEMM (FUNASR_GEMM_T_MIN_M, read at engine creation); apf_min_m = 16 sends the batch and the
    75- and 21-row prompts through the query-tiled prefill attention (k_attn_prefill; the 75-row prompt spans two
    64-row tiles) while the 12-row prompt stays on the per-row kernel."""
    from fun_asr_gguf import _native
    monkeypatch.setenv("FUNASR_GEMM_T_MIN_M", str(t_min_m))
    monkeypatch.setenv("FUNASR_ATTN_PREFILL_MIN_M", str(apf_min_m))
    monkeypatch.setenv("FUNASR_FUSED_MAX_M", "1")  # invariant width 1: the batch takes the shared-forward kernels
    m = llm_tiny_oracle
    rng = np.random.default_rng(21)
    prompts = [np.concatenate([m.embed_prompt(rng.integers(0, 4096, n)),
                               (rng.standard_normal((5, 1024)) * 0.3).astype(np.float32)], 0) for n in (7, 70, 16)]
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=128, max_seqs=4), max_batch=1, max_samples=16000)
    try:
        e.synthetic_weights(0)
        single = []
        for s, p in enumerate(prompts):
            e.llm_reset(s)
            t = e.llm_prefill(s, p, temperature=0.0)
            single.append((t, e.llm_logits(s)))
        for s in range(3):
            e.llm_reset(s)
        toks = e.llm_prefill_batch([0, 1, 2], prompts, temperature=0.0)
        for s in range(3):
            lg = e.llm_logits(s)
            assert _cos(lg, single[s][1]) > 0.9995
            srt = np.sort(single[s][1])
            if srt[-1] - srt[-2] > 0.25:
                assert toks[s] == single[s][0], s
            assert e.llm_n_past(s) == prompts[s].shape[0]
        m.reset()
        _check_step(e.llm_logits(1), m.forward(prompts[1], 0))
        step = e.llm_generate([0, 1, 2], 1)
        _check_step(e.llm_logits(1), m.forward(m.embed_tokens([toks[1]]), prompts[1].shape[0]))
        assert step.shape == (3, 1)
    finally:
        e.close()


def test_llm_prefill_batch_continuation_query_tiles(llm_tiny_oracle, monkeypatch):
    """Query-tiled prefill attention (k_attn_prefill) on prompts that continue a cached prefix (tiles start at n_past
    > 0, keys [0, pos] from the cache) and on tiles cut at 64 rows: prefilling [p0 | p1] in two batched calls equals one
    per-sequence prefill of the whole prompt (cosine within the q8_0 noise floor) and the oracle's teacher-forced
    logits."""
    from fun_asr_gguf import _native
    monkeypatch.delenv("FUNASR_ATTN_PREFILL_MIN_M", raising=False)
    monkeypatch.setenv("FUNASR_FUSED_MAX_M", "1")  # invariant width 1: the batch takes the shared-forward kernels
    m = llm_tiny_oracle
    rng = np.random.default_rng(5)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (90, 20, 70)]
    cut = [33, 7, 64]
    cfg = dict(synth.LLM_TINY, n_ctx=128, max_seqs=4)
    e = _native.Engine(synth.ENC_TINY, cfg, max_batch=1, max_samples=16000)  # per-row attention (default threshold)
    try:
        e.synthetic_weights(0)
        single = []
        for s, p in enumerate(prompts):
            e.llm_reset(s)
            e.llm_prefill(s, p, temperature=0.0)
            single.append(e.llm_logits(s))
    finally:
        e.close()
    monkeypatch.setenv("FUNASR_ATTN_PREFILL_MIN_M", "8")  # read at engine creation
    e = _native.Engine(synth.ENC_TINY, cfg, max_batch=1, max_samples=16000)
    try:
        e.synthetic_weights(0)
        e.llm_prefill_batch([0, 1, 2], [p[:c] for p, c in zip(prompts, cut)], temperature=0.0)
        e.llm_prefill_batch([2, 0, 1], [prompts[2][cut[2]:], prompts[0][cut[0]:], prompts[1][cut[1]:]], temperature=0.0)
        for s in range(3):
            assert e.llm_n_past(s) == prompts[s].shape[0]
            assert _cos(e.llm_logits(s), single[s]) > 0.9995
        m.reset()
        _check_step(e.llm_logits(0), m.forward(prompts[0], 0))
    finally:
        e.close()


@pytest.mark.parametrize("f16", ["0", "1"])
def test_llm_prefill_query_tiles_f16_mfma_vs_oracle(llm_tiny_oracle, monkeypatch, f16):
    """The query-tiled prefill attention on f16 MFMAs (k_attn_prefill_h: the cache's fp16 K / V exact, q split into f16
    hi + lo, P split into f16 hi + lo; FUNASR_ATTN_PF_F16=1, the default) and on exact-f32 MFMAs (=0): a four-prompt
    batch above the invariant width (tiles cut at 64 rows, one prompt continuing a cached prefix) against the oracle's
    teacher-forced logits, and the two kernels' logits within the q8_0 noise floor of each other."""
    from fun_asr_gguf import _native
    monkeypatch.setenv("FUNASR_ATTN_PF_F16", f16)
    monkeypatch.setenv("FUNASR_ATTN_PREFILL_MIN_M", "8")
    monkeypatch.setenv("FUNASR_FUSED_MAX_M", "1")  # invariant width 1: the batch takes the shared-forward kernels
    m = llm_tiny_oracle
    rng = np.random.default_rng(44)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (100, 9, 66, 40)]
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=160, max_seqs=4), max_batch=1, max_samples=16000)
    try:
        e.synthetic_weights(0)
        for s in range(4):
            e.llm_reset(s)
        e.llm_prefill_batch([0, 1], [prompts[0][:30], prompts[1]], temperature=0.0)
        e.llm_prefill_batch([2, 0, 3], [prompts[2], prompts[0][30:], prompts[3]], temperature=0.0)
        for s in (0, 2, 3):
            m.reset()
            _check_step(e.llm_logits(s), m.forward(prompts[s], 0))
    finally:
        e.close()


def test_llm_prefill_large_q_norm_takes_exact_f32_attention(monkeypatch):
    """The f16-MFMA prefill attention holds q * d^-0.5 * 2^8 as f16: a q_norm weight above ~234 could overflow it. The
    engine bounds |q| by max|q_norm| * sqrt(head_dim) after every weight change and then runs the exact-f32 prefill
    attention (tiled batches) and the per-row path (row-local prefill). With q_norm scaled to ~300 the default run
    equals a FUNASR_ATTN_PF_F16=0 run bit for bit, its logits are finite, and they match the oracle teacher-forced."""
    from fun_asr_gguf import _native
    from oracle import qwen3 as oq
    monkeypatch.setenv("FUNASR_ATTN_PREFILL_MIN_M", "8")
    W = synth.make_weights(synth.llm_tensors(synth.LLM_TINY))
    names = [n for n in W if n.endswith("attn_q_norm.weight")]
    for n in names:
        W[n] = (W[n] * 300.0).astype(np.float32)
    m = oq.Qwen3Q8(W, synth.LLM_TINY, n_ctx=160)
    rng = np.random.default_rng(45)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (70, 9, 40)]
    runs = []
    for f16 in ("1", "0"):
        monkeypatch.setenv("FUNASR_ATTN_PF_F16", f16)
        for fmax in ("6", "1"):  # row-local batch (invariant width 6), shared-forward tiles (width 1)
            monkeypatch.setenv("FUNASR_FUSED_MAX_M", fmax)
            e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=160, max_seqs=3), max_batch=1,
                               max_samples=16000)
            try:
                e.synthetic_weights(0)
                for n in names:
                    e.set_tensor(n, W[n])
                for q in range(3):
                    e.llm_reset(q)
                e.llm_prefill_batch([0, 1, 2], prompts, temperature=0.0)
                runs.append([e.llm_logits(q) for q in range(3)])
            finally:
                e.close()
    for a, b in ((runs[0], runs[2]), (runs[1], runs[3])):
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
    for r in runs[:2]:
        assert all(np.isfinite(x).all() for x in r)
        for q in (0, 2):
            m.reset()
            _check_step(r[q], m.forward(prompts[q], 0))


def test_llm_generate_begin_end_equals_generate(llm_tiny_oracle):
    """fa_llm_generate_begin / _end (the host works while the chunk runs) give the tokens of fa_llm_generate, chunk
    after chunk, and the other LLM calls refuse while a chunk is in flight."""
    from fun_asr_gguf import _native
    m = llm_tiny_oracle
    rng = np.random.default_rng(9)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (9, 14, 11)]
    runs = []
    for split in (False, True):
        e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=128, max_seqs=4), max_batch=1, max_samples=16000)
        try:
            e.synthetic_weights(0)
            for s in range(3):
                e.llm_reset(s)
            e.llm_prefill_batch([0, 1, 2], prompts, temperature=0.0)
            if not split:
                runs.append(e.llm_generate([0, 1, 2], 12))
                runs.append(e.llm_generate([0, 2], 7))
            else:
                e.llm_generate_begin([0, 1, 2], 12)
                with pytest.raises(RuntimeError):
                    e.llm_prefill(3, prompts[0])
                runs.append(e.llm_generate_end())
                e.llm_generate_begin([0, 2], 7)
                runs.append(e.llm_generate_end())
                assert e.llm_n_past(0) == prompts[0].shape[0] + 19 and e.llm_n_past(1) == prompts[1].shape[0] + 12
        finally:
            e.close()
    np.testing.assert_array_equal(runs[0], runs[2])
    np.testing.assert_array_equal(runs[1], runs[3])


def test_two_launch_layer_long_context():
    """The two-launch layer past the positions the other tests reach: n_past ~1300 gives each wave of a key split
    more than 4 groups, so the AB launch runs several lean passes (the three-launch layer runs 8-group passes there:
    the same math in another f32 order). Teacher-forced against the oracle and close to the three-launch layer; the
    granule epochs keep working across mode switches (1 -> 2 -> 1 on one engine)."""
    from fun_asr_gguf import _native
    cfg = dict(synth.LLM_TINY, n_ctx=1400, max_seqs=2)
    eng = _native.Engine(synth.ENC_TINY, cfg, max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    m = oqw.Qwen3Q8(synth.make_weights(synth.llm_tensors(synth.LLM_TINY)), synth.LLM_TINY, n_ctx=1400)
    rng = np.random.default_rng(21)
    prompt = np.concatenate([m.embed_prompt(rng.integers(0, 4096, 40)),
                             (rng.standard_normal((1260, 1024)) * 0.5).astype(np.float32)], 0)
    runs = []
    for mode in (1, 2, 1):
        eng.set_decode_fused(mode)
        eng.llm_reset(0)
        tok = eng.llm_prefill(0, prompt)
        lgs, toks = [], [tok]
        for _ in range(5):
            toks.append(int(eng.llm_generate([0], 1)[0][0]))
            lgs.append(eng.llm_logits(0))
        runs.append((toks, lgs))
    eng.close()
    (t1, l1), (t2, l2), (t1b, l1b) = runs
    assert t1b == t1 and all(np.array_equal(a, b) for a, b in zip(l1, l1b))  # the epochs after a mode switch
    m.reset()
    m.forward(prompt, 0)
    for k in range(5):
        if t1[:k + 1] != t2[:k + 1]:
            break
        assert _cos(l1[k], l2[k]) > 0.99999
        ref = m.forward(m.embed_tokens([t1[k]]), prompt.shape[0] + k)
        _check_step(l1[k], ref)


def test_two_launch_layer_l2_prefetch_bit_identical(monkeypatch):
    """The batch-1 attention launch's L2 prefetch blocks (FUNASR_L2PF, default 16 per kv head) only move lines into
    the L2 of the XCDs that read them next: tokens and logits of 48 greedy steps (graph-replayed chunk and single
    eager steps, n_past 300-348, both layers: layer 0 prefetches layer 1's attention inputs, the last layer only its
    FFN weights) equal the run without them bit for bit."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(5)
    prompt = (rng.standard_normal((300, 1024)) * 0.5).astype(np.float32)
    runs = []
    for pf in ("0", "16", "4"):
        monkeypatch.setenv("FUNASR_L2PF", pf)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=512, max_seqs=2), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            eng.set_decode_fused(1)
            eng.llm_reset(1)
            toks = [eng.llm_prefill(1, prompt)]
            toks += [int(t) for t in eng.llm_generate([1], 40)[0]]
            lgs = [eng.llm_logits(1)]
            for _ in range(8):
                toks.append(int(eng.llm_generate([1], 1)[0][0]))
                lgs.append(eng.llm_logits(1))
            runs.append((toks, lgs))
        finally:
            eng.close()
    for toks, lgs in runs[1:]:
        assert toks == runs[0][0]
        assert all(np.array_equal(a, b) for a, b in zip(lgs, runs[0][1]))


def test_batched_decode_gemm_l2_prefetch_bit_identical(monkeypatch):
    """The batched-decode split-K GEMMs' L2 prefetch slabs (FUNASR_GEMM_PF: o -> gate|up, gate|up -> down,
    down -> next q|k|v, q|k|v -> o) only move lines: a batch of 12 sequences decodes 24 graph-replayed steps and one
    eager step with the same tokens and logits as without them."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(8)
    prompts = [(rng.standard_normal((40 + 9 * q, 1024)) * 0.5).astype(np.float32) for q in range(12)]
    runs = []
    for pf in ("0", "15"):
        monkeypatch.setenv("FUNASR_GEMM_PF", pf)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=12), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            for q in range(12):
                eng.llm_reset(q)
                eng.llm_prefill(q, prompts[q])
            toks = eng.llm_generate(list(range(12)), 24)
            toks1 = eng.llm_generate(list(range(12)), 1)
            runs.append((toks, toks1, [eng.llm_logits(q) for q in range(12)]))
        finally:
            eng.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][2], runs[1][2]))


@pytest.mark.parametrize("n_seq", [12, 32])
def test_batched_decode_ffn_one_launch_bit_identical(monkeypatch, n_seq):
    """gate|up + SwiGLU and the down projection of a batched-decode layer in one launch (FUNASR_GU_DOWN=1, an A/B
    form: the down blocks wait per K split for their act tiles) keep the two launches' per-tile arithmetic and split
    order: the same tokens and logits over 24 graph-replayed steps and one eager step."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(9)
    prompts = [(rng.standard_normal((30 + 5 * q, 1024)) * 0.5).astype(np.float32) for q in range(n_seq)]
    runs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("FUNASR_GU_DOWN", fuse)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=n_seq), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            for q in range(n_seq):
                eng.llm_reset(q)
                eng.llm_prefill(q, prompts[q])
            toks = eng.llm_generate(list(range(n_seq)), 24)
            toks1 = eng.llm_generate(list(range(n_seq)), 1)
            runs.append((toks, toks1, [eng.llm_logits(q) for q in range(n_seq)], eng.llm_decode_recoveries()))
        finally:
            eng.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][2], runs[1][2]))
    assert runs[1][3] == (0, 0)  # no hand-off timed out


def test_batched_decode_attention_lds_prefetch_bit_identical(monkeypatch):
    """The 16-wave batched-decode attention pulls each next pass's K/V rows into LDS by LDS-DMA while the current pass
    computes (FUNASR_ATTN_LDSPF=1; off by default, it measured slower): the same bytes reach the same arithmetic, so 32 sequences of 30-510
    keys decode with the same tokens and logits as with register loads per pass."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(10)
    lens = [30 + 15 * q for q in range(32)]
    prompts = [(rng.standard_normal((n, 1024)) * 0.5).astype(np.float32) for n in lens]
    runs = []
    for pf in ("0", "1"):
        monkeypatch.setenv("FUNASR_ATTN_LDSPF", pf)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=560, max_seqs=32), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            for q in range(32):
                eng.llm_reset(q)
                eng.llm_prefill(q, prompts[q])
            toks = eng.llm_generate(list(range(32)), 24)
            toks1 = eng.llm_generate(list(range(32)), 1)
            runs.append((toks, toks1, [eng.llm_logits(q) for q in range(32)]))
        finally:
            eng.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][2], runs[1][2]))


@pytest.mark.parametrize("M", [3, 4, 6])
def test_fused_ffn_one_slab_bit_identical(monkeypatch, M):
    """Small decode batches with the fused FFN as ONE slab of M tokens per block (FUNASR_FFN_WIDE=1: every block's
    gate|up and down weight rows read once for the batch, one block per CU) keep each token's batch-1 arithmetic: the
    same tokens and logits as the token-pair slabs over 20 graph-replayed steps and one eager step, and no fan-in timed
    out."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(60 + M)
    prompts = [(rng.standard_normal((20 + 9 * q, 1024)) * 0.5).astype(np.float32) for q in range(M)]
    runs = []
    for wide in ("0", "1"):
        monkeypatch.setenv("FUNASR_FFN_WIDE", wide)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=M), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            for q in range(M):
                eng.llm_reset(q)
                eng.llm_prefill(q, prompts[q])
            toks = eng.llm_generate(list(range(M)), 20)
            toks1 = eng.llm_generate(list(range(M)), 1)
            runs.append((toks, toks1, [eng.llm_logits(q) for q in range(M)], eng.llm_decode_recoveries()))
        finally:
            eng.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][2], runs[1][2]))
    assert runs[1][3] == (0, 0)


@pytest.mark.parametrize("M", [1, 6, 32])
def test_poisoned_allocations_decode_bit_identical(monkeypatch, M):
    """Every allocation of the engine starts filled with 0xFF bytes (NaN patterns as fp16 / f32; FUNASR_ALLOC_FILL)
    instead of whatever earlier buffers left: prefill, 8 graph-replayed steps, 4 single-step calls give the same tokens
    and logits bit for bit as an engine on zero-filled memory. Round 6 found the decode attention re-reading the fresh
    cache row pos (the clamp target of masked keys) before its owner wave stored it: a masked key's p = 0 times a NaN V
    poisoned the head's output when the memory held such bytes (tests/test_gpu_llama_compat.py failed after other
    tests' engines had freed theirs)."""
    from fun_asr_gguf import _native
    rng = np.random.default_rng(80 + M)
    prompts = [(rng.standard_normal((23 + 7 * q, 1024)) * 0.5).astype(np.float32) for q in range(M)]
    runs = []
    for fill in ("0:100000:0", "0:100000:255"):
        monkeypatch.setenv("FUNASR_ALLOC_FILL", fill)
        eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=M), max_batch=1,
                             max_samples=16000)
        try:
            eng.synthetic_weights(0)
            for q in range(M):
                eng.llm_reset(q)
                eng.llm_prefill(q, prompts[q])
            toks = [eng.llm_generate(list(range(M)), 8)]
            for _ in range(4):
                toks.append(eng.llm_generate(list(range(M)), 1))
            runs.append((np.concatenate(toks, 1), [eng.llm_logits(q) for q in range(M)]))
        finally:
            eng.close()
    assert np.array_equal(runs[0][0], runs[1][0])
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][1], runs[1][1]))


def test_two_launch_layer_mixed_batch_widths(llm_tiny_oracle):
    """Sequences decoded under a changing batch schedule (widths 5, 2, 3, 1, 4 ...; a sequence takes different token
    slots from call to call, so every slot's granules and ticket lines see launches of other widths in between) give
    exactly the tokens they give alone on the two-launch layer (per-token arithmetic is batch-independent up to 5 rows,
    where the LM head is the fused GEMV for every width)."""
    from fun_asr_gguf import _native
    m = llm_tiny_oracle
    eng = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=6), max_batch=1, max_samples=16000)
    eng.synthetic_weights(0)
    rng = np.random.default_rng(77)
    prompts = [m.embed_prompt(rng.integers(0, 4096, 5 + 7 * i)) for i in range(5)]
    n_steps = 6
    singles = []
    for p in prompts:
        eng.llm_reset(0)
        t = eng.llm_prefill(0, p)
        singles.append([t] + list(eng.llm_generate([0], n_steps)[0]))
    got = {}
    for q, p in enumerate(prompts):
        eng.llm_reset(q)
        got[q] = [eng.llm_prefill(q, p)]
    schedule = [[0, 1, 2, 3, 4], [3, 1], [4, 0, 2], [2], [1, 4, 3, 0], [0, 2, 4, 1, 3], [3, 1], [4, 0, 2],
                [1, 3, 0, 2, 4], [0], [3, 4, 1, 2], [4, 2], [1, 3, 0], [2, 4, 3, 1, 0]]
    for seqs in schedule:
        seqs = [q for q in seqs if len(got[q]) <= n_steps]
        if not seqs:
            continue
        out = eng.llm_generate(seqs, 1)
        for q, t in zip(seqs, out):
            got[q].append(int(t[0]))
    eng.close()
    for q in range(5):
        assert len(got[q]) == n_steps + 1, (q, len(got[q]))
        assert got[q] == singles[q], q


def test_fused_timeout_recovery_keeps_fused_layer():
    """A fan-in timeout in the fused decode layer (forced: fa_set_debug bit 1 makes one block withhold its q|k|v
    hand-off in the next chunk; every wait is bounded at 10 ms) is not an error to the caller: fa_llm_generate_end
    re-runs the chunk on the fused layer from the same positions and tokens. The tokens and logits equal an undisturbed
    run, and the invariant width stays 6 (DESIGN §3 decode step). With bit 2 too the re-run times out as well: that
    chunk runs on the 5-launch layer (tokens and logits equal a 5-launch run of it), the next chunk is fused again, and
    three such chunks in a row keep the 5-launch layer (width 1); a clean fused chunk between fallbacks resets that count
    (fallback, clean, fallback, clean, fallback keeps width 6)."""
    from fun_asr_gguf import _native
    from oracle import qwen3 as oq
    cfg = dict(synth.LLM_TINY, n_ctx=256, max_seqs=2)
    m = oq.Qwen3Q8(synth.make_weights(synth.llm_tensors(synth.LLM_TINY)), synth.LLM_TINY, n_ctx=256)
    rng = np.random.default_rng(77)
    prompt = m.embed_prompt(rng.integers(0, 4096, 40))

    def run(debug=0, fused=1, chunks=1):
        eng = _native.Engine(synth.ENC_TINY, cfg, max_batch=1, max_samples=16000)
        try:
            eng.synthetic_weights(0)
            eng.set_decode_fused(fused)
            eng.llm_reset(0)
            first = eng.llm_prefill(0, prompt)
            toks = []
            sched = debug if isinstance(debug, list) else [debug] * chunks
            for dbg in sched:  # per chunk: 0 undisturbed, else the fa_set_debug bits set before it
                if dbg:
                    eng.lib.fa_set_debug(eng.h, dbg)
                toks += [int(t) for t in eng.llm_generate([0], 3)[0]]
            lg = eng.llm_logits(0)
            more = [int(t) for t in eng.llm_generate([0], 2)[0]]  # undisturbed chunk after the recovery
            return first, toks, lg, more, eng.llm_invariant_width(), eng.llm_decode_recoveries()
        finally:
            eng.close()

    f_ok, t_ok, l_ok, m_ok, w_ok, r_ok = run()
    assert w_ok == 6 and r_ok == (0, 0)
    f1, t1, l1, m1, w1, r1 = run(debug=2)
    assert r1 == (1, 0) and w1 == 6, (r1, w1)
    assert f1 == f_ok and t1 == t_ok and m1 == m_ok and np.array_equal(l1, l_ok)
    # the re-run times out too: this chunk on the 5-launch layer, then the fused layer again
    f2, t2, l2, m2, w2, r2 = run(debug=6)
    assert r2 == (1, 1) and w2 == 6, (r2, w2)
    e5 = _native.Engine(synth.ENC_TINY, cfg, max_batch=1, max_samples=16000)
    try:
        e5.synthetic_weights(0)
        e5.set_decode_fused(0)
        e5.llm_reset(0)
        assert e5.llm_prefill(0, prompt) == f2
        assert [int(t) for t in e5.llm_generate([0], 3)[0]] == t2
        assert np.array_equal(e5.llm_logits(0), l2)
    finally:
        e5.close()
    # three fallbacks in a row: the engine keeps the 5-launch layer
    *_, w3, r3 = run(debug=6, chunks=3)
    assert r3 == (3, 3) and w3 == 1, (r3, w3)
    # ... but not with clean fused chunks between them (the count is of consecutive fallbacks)
    *_, w4, r4 = run(debug=[6, 0, 6, 0, 6])
    assert r4 == (3, 3) and w4 == 6, (r4, w4)


def test_llm_prefill_batch_row_local_exact(llm_tiny_oracle):
    """Within the invariant width fa_llm_prefill_batch is row-local: every prompt gets exactly the arithmetic of its own
    fa_llm_prefill (K-in-block GEMMs, one key split, f16-MFMA query tiles whose rows depend only on their own keys,
    never the row-count-dependent fused-GEMV path), so
    first tokens and logits are bit-identical, for short prompts (<= 6 rows) and for prompts continuing a cached prefix."""
    from fun_asr_gguf import _native
    m = llm_tiny_oracle
    rng = np.random.default_rng(33)
    prompts = [m.embed_prompt(rng.integers(0, 4096, n)) for n in (5, 90, 37, 12)]
    cut = [2, 41, 20, 6]
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=128, max_seqs=4), max_batch=1, max_samples=16000)
    try:
        e.synthetic_weights(0)
        assert e.llm_invariant_width() >= 4
        single = []
        for s, p in enumerate(prompts):  # each alone, in two calls (prefix, then the rest)
            e.llm_reset(s)
            e.llm_prefill(s, p[:cut[s]], temperature=0.0)
            t = e.llm_prefill(s, p[cut[s]:], temperature=0.0)
            single.append((t, e.llm_logits(s)))
        for s in range(4):
            e.llm_reset(s)
        e.llm_prefill_batch([0, 1, 2, 3], [p[:c] for p, c in zip(prompts, cut)], temperature=0.0)
        toks = e.llm_prefill_batch([3, 1, 0, 2], [prompts[q][cut[q]:] for q in (3, 1, 0, 2)], temperature=0.0)
        for k, q in enumerate((3, 1, 0, 2)):
            assert toks[k] == single[q][0], q
            assert np.array_equal(e.llm_logits(q), single[q][1]), q
        m.reset()
        _check_step(e.llm_logits(1), m.forward(prompts[1], 0))
    finally:
        e.close()
