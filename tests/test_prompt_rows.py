"""Host logic of the device-assembled prompt rows (core/decoder.PromptRows, prefill_group): the object is the
reference's host concatenation (core/decoder.py:199) when materialised, and prefill_group hands it to
fa_llm_prefill_rows only while the engine still holds that encode; otherwise the host rows go through
fa_llm_prefill / fa_llm_prefill_batch. The row codes the binding builds (distinct prefix / suffix arrays uploaded once,
audio rows as -1 - (clip << 16 | t)) are checked against a stand-in for the C call."""
import ctypes

import numpy as np

from fun_asr_gguf.core.decoder import PromptRows, prefill_group


class _Stub:
    def __init__(self, gen):
        self.gen, self.calls = gen, []

    def encode_generation(self):
        return self.gen

    def llm_prefill_rows(self, seqs, prompts, **samp):
        self.calls.append(("rows", list(seqs)))
        return [7] * len(seqs)

    def llm_prefill(self, seq, embd, **samp):
        assert isinstance(embd, np.ndarray)
        self.calls.append(("one", embd.shape))
        return 5

    def llm_prefill_batch(self, seqs, embds, **samp):
        assert all(isinstance(e, np.ndarray) for e in embds)
        self.calls.append(("batch", [e.shape for e in embds]))
        return [6] * len(seqs)


def _prompts(gen, n=3):
    rng = np.random.default_rng(0)
    pre = rng.standard_normal((4, 8)).astype(np.float32)
    suf = rng.standard_normal((2, 8)).astype(np.float32)
    return [PromptRows(pre, rng.standard_normal((3 + b, 8)).astype(np.float32), suf, b, gen) for b in range(n)], pre, suf


def test_prompt_rows_materialise_as_the_reference_concatenation():
    ps, pre, suf = _prompts(4)
    for p in ps:
        want = np.concatenate([pre, p.audio, suf], 0)
        assert p.shape == want.shape and len(p) == want.shape[0]
        assert np.array_equal(np.asarray(p), want) and np.asarray(p, np.float32).dtype == np.float32
        assert np.array_equal(np.ascontiguousarray(p, dtype=np.float32), want)


def test_prefill_group_routes_by_encode_generation():
    ps, _, _ = _prompts(4)
    eng = _Stub(4)
    assert prefill_group(eng, [0, 1, 2], ps, {}) == [7, 7, 7] and eng.calls == [("rows", [0, 1, 2])]
    eng = _Stub(5)  # another encode ran since: the host rows
    assert prefill_group(eng, [0, 1, 2], ps, {}) == [6, 6, 6]
    assert eng.calls == [("batch", [(9, 8), (10, 8), (11, 8)])]
    eng = _Stub(5)
    assert prefill_group(eng, [3], ps[:1], {}) == [5] and eng.calls == [("one", (9, 8))]
    eng = _Stub(4)  # mixed with a plain array: the host rows
    assert prefill_group(eng, [0, 1], [ps[0], np.asarray(ps[1])], {}) == [6, 6]


def test_prefill_rows_binding_codes(monkeypatch):
    from fun_asr_gguf import _native
    seen = {}

    class _Lib:
        def fa_llm_prefill_rows(self, h, seqs, n_seqs, host, n_host, rs, n, gen, s, tok):
            cast = lambda p, t, k: np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(t)), (k,)).copy()
            nn = cast(n, ctypes.c_int32, n_seqs)
            seen.update(n=nn, codes=cast(rs, ctypes.c_int32, int(nn.sum())), n_host=n_host, gen=gen,
                        host=cast(host, ctypes.c_float, n_host * 8).reshape(n_host, 8))
            return 0

    eng = object.__new__(_native.Engine)
    eng.lib, eng.h = _Lib(), None
    ps, pre, suf = _prompts(9)
    assert eng.llm_prefill_rows([0, 1, 2], ps) == [0, 0, 0]
    assert seen["gen"] == 9 and list(seen["n"]) == [9, 10, 11]
    assert seen["n_host"] == 6 and np.array_equal(seen["host"], np.concatenate([pre, suf]))  # shared rows once
    c = seen["codes"]
    assert list(c[:9]) == [0, 1, 2, 3, -1, -2, -3, 4, 5]
    assert list(c[13:17]) == [-1 - (1 << 16), -2 - (1 << 16), -3 - (1 << 16), -4 - (1 << 16)]
    assert list(c[-2:]) == [4, 5]
