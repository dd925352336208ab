"""GPU sampler chain (D6; LlamaSampler, /root/reference/fun_asr_gguf/llama.py:599-605): top_k -> top_p (min_keep 1)
-> temp -> dist, through fa_llm_prefill / fa_llm_generate on the tiny synthetic decoder.

The reference draws with llama.cpp's mt19937 seeded from np.random on every call (core/decoder.py:89), so no
draw is reproducible there: the contract is the candidate set and the distribution. Checked here:
  * membership: every drawn token lies in the top-k set, and in the top-p prefix (sorted by logit, softmax mass
    at temperature 1 over the top-k) -- exact sets, ties at the boundary value admitted;
  * distribution: chi-square of >= 3000 draws (one per seed) against softmax(top-k logits / T), p > 1e-4;
  * the wide path (top_k <= 0: no top-k cut) with and without top_p;
  * fresh draws: the counter is (seed, sequence, position), so two generate calls with one seed, or two
    sequences with one seed and one position, do not repeat each other (chunked calls reused draws).
"""
import numpy as np
import pytest

from oracle import qwen3 as oqw, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from fun_asr_gguf import _native
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=512, max_seqs=4), max_batch=1, max_samples=16000)
    e.synthetic_weights(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def prompt():
    m = oqw.Qwen3Q8(synth.make_weights(synth.llm_tensors(synth.LLM_TINY)), synth.LLM_TINY, n_ctx=64)
    rng = np.random.default_rng(11)
    return m.embed_prompt(rng.integers(0, 4096, 12))


def _topk_set(lg, k):
    kth = np.sort(lg)[-k]
    return set(np.nonzero(lg >= kth)[0].tolist())


def _topp_set(lg, k, p):
    """llama.cpp top_p over the top-k candidates sorted by logit; ties at the cut value admitted."""
    order = np.argsort(-lg.astype(np.float64), kind="stable")[:k]
    v = lg[order].astype(np.float64)
    w = np.exp(v - v[0])
    cum = np.cumsum(w / w.sum())
    n = int(np.searchsorted(cum, p - 1e-6)) + 1
    cut = v[min(n, k) - 1]
    return set(order[v >= cut].tolist())


def test_topk_topp_membership_decode_steps(eng, prompt):
    eng.llm_reset(0)
    eng.llm_prefill(0, prompt, temperature=1.0, top_k=5, seed=1)
    for step in range(24):
        k, p = (5, 1.0) if step % 2 == 0 else (50, 0.3)
        tok = int(eng.llm_generate([0], 1, temperature=1.3, top_k=k, top_p=p, seed=100 + step)[0][0])
        lg = eng.llm_logits(0)
        assert tok in _topk_set(lg, k), (step, tok)
        if p < 1:
            assert tok in _topp_set(lg, k, p), (step, tok)


def _chi2_ok(counts, probs, n):
    from scipy.stats import chi2
    exp = probs * n
    stat = float(((counts - exp) ** 2 / exp).sum())
    return chi2.sf(stat, len(probs) - 1) > 1e-4, stat


@pytest.mark.parametrize("top_k", [8, 0])
def test_draw_distribution_chi_square(eng, prompt, top_k):
    """top_k = 8: fast path (sorted candidates in LDS); top_k = 0: wide path (whole row, token-id order)."""
    eng.llm_reset(0)
    _, lg = eng.llm_prefill(0, prompt, want_logits=True, temperature=0.0)
    lg = lg.astype(np.float64)
    order = np.argsort(-lg, kind="stable")
    k8 = order[:8]
    T = max(0.05, (lg[k8[0]] - lg[k8[-1]]) / 2.0)  # top-1 : top-8 odds of e^2
    if top_k > 0:
        p = np.exp((lg[k8] - lg[k8[0]]) / T)
        p /= p.sum()
        buckets = list(k8)
    else:
        z = np.exp((lg - lg.max()) / T)
        z /= z.sum()
        buckets = list(order[:6])
        p = np.concatenate([z[buckets], [1.0 - z[buckets].sum()]])
    n = 3000
    counts = np.zeros(len(p))
    for seed in range(n):
        eng.llm_reset(0)
        t = eng.llm_prefill(0, prompt, temperature=T, top_k=top_k, top_p=1.0, seed=seed)
        if t in buckets:
            counts[buckets.index(t)] += 1
        else:
            assert top_k == 0, t  # the fast path never leaves the top-k
            counts[-1] += 1
    ok, stat = _chi2_ok(counts, p, n)
    assert ok, (stat, counts, p * n)


def test_wide_path_top_p_membership(eng, prompt):
    eng.llm_reset(0)
    _, lg = eng.llm_prefill(0, prompt, want_logits=True, temperature=0.0)
    allowed = _topp_set(lg, lg.size, 0.5)
    for seed in range(200):
        eng.llm_reset(0)
        t = eng.llm_prefill(0, prompt, temperature=0.7, top_k=0, top_p=0.5, seed=seed)
        assert t in allowed


def test_fresh_draws_across_calls_and_sequences(eng, prompt):
    for s in (0, 1):
        eng.llm_reset(s)
        eng.llm_prefill(s, prompt, temperature=0.0)
    samp = dict(temperature=50.0, top_k=0, top_p=1.0, seed=7)  # near-uniform over the 4096-token vocab
    a = eng.llm_generate([0, 1], 32, **samp)
    b = eng.llm_generate([0, 1], 32, **samp)  # same seed, next 32 positions
    assert not np.array_equal(a[0], b[0]) and not np.array_equal(a[1], b[1])
    assert not np.array_equal(a[0], a[1])  # same seed, same positions, different sequences
    assert len(set(a[0].tolist() + b[0].tolist())) > 48


def test_batched_membership_mfma_lm_head(prompt):
    """8 sequences per step: the LM head runs on the MFMA GEMM (32-row argmax partials), so the fast path's chunk
    gather walks 32-row chunks instead of the GEMV's; every row's draw stays in its own top-k / top-p set."""
    from fun_asr_gguf import _native
    e = _native.Engine(synth.ENC_TINY, dict(synth.LLM_TINY, n_ctx=256, max_seqs=8), max_batch=1, max_samples=16000)
    try:
        e.synthetic_weights(0)
        rng = np.random.default_rng(4)
        for s in range(8):
            e.llm_reset(s)
            e.llm_prefill(s, prompt[: 4 + s] + (rng.standard_normal((4 + s, 1024)) * 0.05).astype(np.float32),
                          temperature=0.0)
        for step in range(6):
            k, p = (5, 1.0) if step % 2 == 0 else (50, 0.3)
            toks = e.llm_generate(list(range(8)), 1, temperature=1.3, top_k=k, top_p=p, seed=300 + step)
            for s in range(8):
                lg = e.llm_logits(s)
                t = int(toks[s][0])
                assert t in _topk_set(lg, k), (step, s, t)
                if p < 1:
                    assert t in _topp_set(lg, k, p), (step, s, t)
    finally:
        e.close()
