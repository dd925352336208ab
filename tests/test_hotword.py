"""Hotword phoneme retrieval (fun_asr_gguf.hotword), pinned to the reference's own hotword modules
(tests/golden/hotword_golden.json from make_hotword_golden.py: pypinyin is absent, so a fixed pinyin table with its
interface, tests/golden/fake_pinyin.py, fills its slot for both sides; and the reference's no-pypinyin degraded mode).
numba is absent: the reference's pure-Python FastRAG distance (rag_fast.py:291-313) is restated below as the oracle of
the native DP."""
import numpy as np
import pytest

from fun_asr_gguf import hotword as hwm


def ref_python_distance(main, sub):
    """rag_fast.FastRAG._python_distance (:291-313), verbatim algorithm."""
    n, m = len(sub), len(main)
    if n == 0 or m == 0:
        return float(n)
    dp = [[0.0] * (m + 1) for _ in range(n + 1)]
    for i in range(1, n + 1):
        dp[i][0] = float(i)
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            cost = 0.0 if sub[i - 1] == main[j - 1] else 1.0
            dp[i][j] = min(dp[i - 1][j] + 1.0, dp[i][j - 1] + 1.0, dp[i - 1][j - 1] + cost)
    return min(dp[n][j] for j in range(1, m + 1))


def test_native_fastrag_distance_matches_reference_dp():
    from fun_asr_gguf._native import fuzzy_substring_distance
    rng = np.random.default_rng(0)
    for _ in range(300):
        m, n = int(rng.integers(0, 40)), int(rng.integers(0, 9))
        a = rng.integers(1, 6, m)
        b = rng.integers(1, 6, n)
        assert fuzzy_substring_distance(a, b) == ref_python_distance(list(a), list(b))


def test_degraded_mode_is_the_references(monkeypatch):
    """Without pypinyin the reference's get_phoneme_info yields one phoneme per character with no word-start / end
    flags (algo_phoneme.py:194-195): FastRAG still ranks candidates, but the boundary-constrained fine search
    (algo_calc.py:401-499) can start only at position 0 and end nowhere, so correct() finds nothing."""
    monkeypatch.setattr(hwm, "pinyin", None)
    c = hwm.PhonemeCorrector(threshold=1.0, similar_threshold=0.6)
    assert c.update_hotwords("# comment\n阿里巴巴\n通义千问\n\nMI355X\n") == 3
    text = "今天阿里巴吧发布了通义千问和 MI355 芯片"
    coarse = dict(c.fast_rag.search(hwm.get_phoneme_info(text), top_k=100))
    assert coarse["通义千问"] == 1.0 and coarse["阿里巴巴"] == 0.75 and coarse["MI355X"] == 0.833
    r = c.correct(text, k=10)
    assert r == hwm.CorrectionResult(text, [], [])


PY = {"张": ("zh", "ang", "1"), "三": ("s", "an", "1"), "章": ("zh", "ang", "1"), "山": ("sh", "an", "1"),
      "赞": ("z", "an", "4"), "是": ("sh", "i", "4"), "我": ("", "uo", "3"), "好": ("h", "ao", "3")}


INITS = ["b", "p", "m", "f", "d", "t", "n", "l", "g", "k", "h", "j", "q", "x", "zh", "ch", "sh", "r", "z", "c", "s", ""]
FINS = ["a", "o", "e", "ai", "ei", "ao", "ou", "an", "en", "ang", "eng", "i", "u", "in", "ing", "uo"]


class _FakePinyin:
    """A fixed table standing in for pypinyin's pinyin(fragment, style=...) (absent in this image); characters off
    the table get a syllable derived from their code point."""
    INITIALS, FINALS, TONE3 = 0, 1, 2

    @staticmethod
    def pinyin(frag, style=0, **kw):
        out = []
        for ch in frag:
            o = ord(ch)
            i, f, t = PY.get(ch, (INITS[o % len(INITS)], FINS[(o // 7) % len(FINS)], str(1 + o % 4)))
            out.append([i if style == 0 else f if style == 1 else f"{i}{f}{t}"])
        return out


def test_pinyin_path_similar_phonemes(monkeypatch):
    monkeypatch.setattr(hwm, "pinyin", _FakePinyin.pinyin)
    monkeypatch.setattr(hwm, "Style", _FakePinyin)
    ph = hwm.get_phoneme_info("我是张三abc12")
    assert [p.value for p in ph] == ["uo", "3", "sh", "i", "4", "zh", "ang", "1", "s", "an", "1", "a", "b", "c", "1", "2"]
    assert [(p.char_start, p.is_word_start, p.is_word_end) for p in ph[:3]] == [(0, True, False), (0, False, True),
                                                                              (1, True, False)]
    c = hwm.PhonemeCorrector(threshold=0.8, similar_threshold=0.6)
    c.update_hotwords("张三")
    # 章山: zh ang 1 | sh an 1 vs zh ang 1 | s an 1 -> one similar-initial pair (s/sh, cost 0.5): 1 - 0.5/6
    r = c.correct("我是章山", k=5)
    assert r.similars == [("章山", "张三", pytest.approx(1 - 0.5 / 6))]
    assert r.text == "我是张三" and r.matchs[0][:2] == ("章山", "张三")


def test_engine_hotword_list_into_prompt(tmp_path, monkeypatch):
    """ModelManager.match_hotwords -> PromptBuilder: a hotword found in the CTC text reaches the prompt
    (decoder.py:39-44, prompt_utils.py:36-38), through the real StreamDecoder on the host fake engine."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fake_engine import fake_models
    from fun_asr_gguf.core.decoder import StreamDecoder
    from fun_asr_gguf.hotword import HotwordSource
    from fun_asr_gguf.nano_dataclass import RecognitionStream
    from fun_asr_gguf.synthetic import synth_audio
    monkeypatch.setattr(hwm, "pinyin", _FakePinyin.pinyin)
    monkeypatch.setattr(hwm, "Style", _FakePinyin)
    m = fake_models(max_batch=1, n_predict=8)
    st = RecognitionStream()
    st.accept_waveform(16000, synth_audio(16000 * 4, 1))
    d0 = StreamDecoder(m).decode_stream(st, verbose=False, temperature=0.0)
    ctc = "".join(t.text for t in d0.ctc_results)
    assert len(ctc) >= 6 and d0.hotwords == []
    hot = tmp_path / "hot.txt"
    hot.write_text(ctc[2:5] + "\n" + "无关热词\n", encoding="utf-8")
    m.hotword_source = HotwordSource(str(hot), 0.6)
    d1 = StreamDecoder(m).decode_stream(st, verbose=False, temperature=0.0)
    assert d1.hotwords == [ctc[2:5]]
    assert d1.n_prefix > d0.n_prefix  # the prompt grew by the 热词列表 line


def _approx(a, b):
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_approx(x, y) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        return abs(float(a) - float(b)) <= 1e-9
    return a == b


@pytest.mark.parametrize("mode", ["pinyin_table", "degraded"])
def test_hotword_path_vs_reference_golden(monkeypatch, mode):
    """Pinned to the reference's own hotword modules (tests/golden/hotword_golden.json, make_hotword_golden.py): the
    phoneme sequences (algo_phoneme.get_phoneme_info), the boundary-constrained fine search
    (algo_calc.fuzzy_substring_search_constrained), FastRAG.search and PhonemeCorrector.correct on a hot.txt, with the
    same fixed pinyin table standing in for pypinyin, and in the reference's no-pypinyin degraded mode."""
    import json
    import os
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import fake_pinyin
    gold = json.load(open(os.path.join(GOLDEN, "hotword_golden.json"), encoding="utf-8"))
    g = gold[mode]
    if mode == "pinyin_table":
        monkeypatch.setattr(hwm, "pinyin", fake_pinyin.pinyin)
        monkeypatch.setattr(hwm, "Style", fake_pinyin.Style)
    else:
        monkeypatch.setattr(hwm, "pinyin", None)
    for t, ph in g["phonemes"].items():
        assert [list(p.info) for p in hwm.get_phoneme_info(t)] == ph, t
    for case in g["search"]:
        hwi = [p.info[:5] for p in hwm.get_phoneme_info(case["hotword"])]
        inp = [p.info for p in hwm.get_phoneme_info(case["text"])]
        got = [list(r) for r in hwm.fuzzy_substring_search_constrained(hwi, inp, case["threshold"])]
        assert _approx(got, case["result"]), (case["hotword"], case["text"], got, case["result"])
    lines = [ln.strip() for ln in gold["hot"].splitlines() if ln.strip() and not ln.strip().startswith("#")]
    rag = hwm.FastRAG(threshold=0.5)
    rag.add_hotwords({hw: hwm.get_phoneme_info(hw) for hw in lines})
    for t, res in g["fastrag"].items():
        got = [list(r) for r in rag.search(hwm.get_phoneme_info(t), top_k=10)]
        assert _approx(got, res), (t, got, res)
    correctors = {}
    for case in g["correct"]:
        key = (case["threshold"], case["similar_threshold"])
        if key not in correctors:
            correctors[key] = hwm.PhonemeCorrector(threshold=key[0], similar_threshold=key[1])
            assert correctors[key].update_hotwords(gold["hot"]) == case["n_hotwords"]
        r = correctors[key].correct(case["text"], k=10)
        assert r.text == case["out"], (key, case["text"], r.text, case["out"])
        assert _approx([list(x) for x in r.matchs], case["matchs"]), (key, case["text"], r.matchs, case["matchs"])
        assert _approx([list(x) for x in r.similars], case["similars"]), (key, case["text"], r.similars, case["similars"])
