"""Hotword phoneme retrieval: what the reference's CTCDecoder asks of its corrector,
`corrector.correct(ctc_text, k=max_hotwords)` (/root/reference/fun_asr_gguf/core/decoder.py:39-44), restated:

  * phonemes: get_phoneme_info (hotword/algo_phoneme.py:190-291): CJK runs -> pinyin initial / final / tone
    (pypinyin, Style INITIALS / FINALS / TONE3 with neutral tone 5), ASCII letter / digit runs split at camel-case
    and letter-digit boundaries into one phoneme per character, everything else skipped; each phoneme keeps
    (value, lang, word start, word end, is tone, char start, char end). Without pypinyin the reference degrades
    to one phoneme per character of the text (algo_phoneme.py:194-195), and so does this module.
  * coarse retrieval: FastRAG (hotword/rag_fast.py:110-318): integer phoneme codes, an inverted index on the
    first two codes of every hotword, candidate expansion through SIMILAR_PHONEMES for Chinese, a length filter,
    the fuzzy-substring edit distance (numba there; native fa_fuzzy_substring_distance here), score
    1 - dist / len >= threshold, top 100.
  * fine matching: fuzzy_substring_search_constrained (hotword/algo_calc.py:401-499): DP over phoneme tuples with
    0.5-cost similar phonemes and tones, LCS-based cost for English, starts on word starts, ends on word ends;
    then PhonemeCorrector._find_matches / _resolve_and_replace / correct (hot_phoneme.py:85-221).
  * the engine's hotword list: every hotword of `matchs` and `similars`. The reference builds it as list(set(...))
    (hash order, not reproducible across processes); here it is ordered by first appearance (matchs, similars).
Thresholds as ModelManager (model_manager.py:82-88): threshold 1.0, similar_threshold = config.similar_threshold.
The hot.txt watchdog thread (manager.py) becomes an mtime check per call.
Parity: pinned to the reference's own hotword modules (algo_phoneme / algo_calc / rag_fast / hot_phoneme imported
by tests/golden/make_hotword_golden.py with a fixed pinyin table in pypinyin's module slot, and in the reference's
no-pypinyin degraded mode): phonemes, the constrained fine search, FastRAG.search and PhonemeCorrector.correct equal
the reference's outputs (tests/test_hotword.py::test_hotword_path_vs_reference_golden). pypinyin itself stays
absent (its tables are not restated: any implementation with its interface plugs in as `pinyin` / `Style`).
"""
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, NamedTuple, Tuple

import numpy as np

try:  # optional, as in the reference's degraded mode
    from pypinyin import Style, pinyin
except ImportError:  # pragma: no cover - absent in this image
    pinyin, Style = None, None

SIMILAR_PHONEMES = [{'an', 'ang'}, {'en', 'eng'}, {'in', 'ing'}, {'ian', 'iang'}, {'uan', 'uang'}, {'z', 'zh'},
                    {'c', 'ch'}, {'s', 'sh'}, {'l', 'n'}, {'f', 'h'}, {'ai', 'ei'}, {'o', 'uo'}, {'e', 'ie'},
                    {'p', 't'}, {'p', 'b'}, {'t', 'd'}, {'k', 'g'}]  # algo_calc.py:11-35


@dataclass(frozen=True)
class Phoneme:
    value: str
    lang: str
    is_word_start: bool = False
    is_word_end: bool = False
    char_start: int = 0
    char_end: int = 0

    @property
    def is_tone(self):
        return self.value.isdigit()

    @property
    def info(self):
        return (self.value, self.lang, self.is_word_start, self.is_word_end, self.is_tone, self.char_start,
                self.char_end)


def _is_zh(c):
    return '一' <= c <= '鿿'


def _process_zh(text, pos, seq):
    end = pos + 1
    while end < len(text) and _is_zh(text[end]):
        end += 1
    frag = text[pos:end]
    try:
        ini = pinyin(frag, style=Style.INITIALS, strict=False, errors="ignore")
        fin = pinyin(frag, style=Style.FINALS, strict=False, errors="ignore")
        ton = pinyin(frag, style=Style.TONE3, neutral_tone_with_five=True, errors="ignore")
        for i in range(min(len(frag), len(ini), len(fin), len(ton))):
            idx = pos + i
            a, b, t = ini[i][0], fin[i][0], ton[i][0]
            items = []
            if a:
                items.append(Phoneme(a, 'zh', True, False, idx, idx + 1))
            if b:
                items.append(Phoneme(b, 'zh', not a, False, idx, idx + 1))
            if t and t[-1].isdigit():
                items.append(Phoneme(t[-1], 'zh', False, True, idx, idx + 1))
            seq.extend(items or [Phoneme(frag[i], 'zh', True, True, idx, idx + 1)])
    except Exception:
        seq.extend(Phoneme(c, 'zh', True, True, pos + i, pos + i + 1) for i, c in enumerate(frag))
    return end


def _process_en_num(text, pos, seq):
    start = pos
    while pos < len(text):
        c = text[pos]
        if not ('a' <= c.lower() <= 'z' or '0' <= c <= '9'):
            break
        if pos > start:
            p = text[pos - 1]
            if (p.islower() and c.isupper()) or (p.isalpha() and c.isdigit()) or (p.isdigit() and c.isalpha()):
                break
        pos += 1
    tok = text[start:pos].lower()
    lang = 'num' if tok.isdigit() else 'en'
    seq.extend(Phoneme(c, lang, i == 0, i == len(tok) - 1, start + i, start + i + 1) for i, c in enumerate(tok))
    return pos


def get_phoneme_info(text: str) -> List[Phoneme]:
    """algo_phoneme.get_phoneme_info (ascii_split_char=True)."""
    if not pinyin:
        return [Phoneme(c, 'zh', char_start=i, char_end=i + 1) for i, c in enumerate(text)]
    seq, pos = [], 0
    while pos < len(text):
        c = text[pos]
        if _is_zh(c):
            pos = _process_zh(text, pos, seq)
        elif 'a' <= c.lower() <= 'z' or '0' <= c <= '9':
            pos = _process_en_num(text, pos, seq)
        else:
            pos += 1
    return seq


# ---- coarse retrieval (rag_fast.py)
class FastRAG:
    def __init__(self, threshold=0.6):
        self.threshold = threshold
        self.code = {}
        self.index: Dict[int, List[Tuple[str, np.ndarray]]] = {}
        self.count = 0

    def _enc(self, vals):
        """PhonemeEncoder.encode_sequence (rag_fast.py:88-104): codes from 1, new values get the next code."""
        for v in vals:
            if v not in self.code:
                self.code[v] = len(self.code) + 1
        return np.array([self.code[v] for v in vals], np.int32)

    def add_hotwords(self, hotwords: Dict[str, List[Phoneme]]):
        for hw, ph in hotwords.items():
            if not ph:
                continue
            codes = self._enc([p.value for p in ph])
            for c in {int(codes[i]) for i in range(min(len(codes), 2))}:
                self.index.setdefault(c, []).append((hw, codes))
            self.count += 1

    def candidates(self, ph: List[Phoneme]):
        codes = set()
        for p in ph:
            c = self.code.get(p.value)
            if c is not None:
                codes.add(c)
            if p.lang != 'zh':
                continue
            for s in SIMILAR_PHONEMES:
                if p.value in s:
                    codes.update(self.code[v] for v in s if v in self.code)
        out, seen = [], set()
        for c in codes:
            for hw, hc in self.index.get(c, []):
                if hw not in seen:
                    out.append((hw, hc))
                    seen.add(hw)
        return out

    def search(self, ph: List[Phoneme], top_k=10):
        if not ph:
            return []
        from ._native import fuzzy_substring_distance
        inp = self._enc([p.value for p in ph])  # encoded before the candidate lookup, as rag_fast.py:239-240
        res = []
        for hw, hc in self.candidates(ph):
            if len(hc) > len(inp) + 3:
                continue
            score = 1.0 - fuzzy_substring_distance(inp, hc) / len(hc)
            if score >= self.threshold:
                res.append((hw, round(score, 3)))
        res.sort(key=lambda x: x[1], reverse=True)
        return res[:top_k]


# ---- fine matching (algo_calc.py)
def _lcs_length(a, b):
    if not a or not b:
        return 0
    prev = [0] * (len(b) + 1)
    for i in range(1, len(a) + 1):
        cur = [0] * (len(b) + 1)
        for j in range(1, len(b) + 1):
            cur[j] = prev[j - 1] + 1 if a[i - 1] == b[j - 1] else max(prev[j], cur[j - 1])
        prev = cur
    return prev[len(b)]


def _tuple_cost(t1, t2):
    if t1[1] != t2[1]:
        return 1.0
    if t1[0] == t2[0]:
        return 0.0
    if t1[1] == 'zh':
        if t1[4]:
            return 0.5
        pair = {t1[0], t2[0]}
        if any(pair.issubset(s) for s in SIMILAR_PHONEMES):
            return 0.5
    if t1[1] == 'en':
        ml = max(len(t1[0]), len(t2[0]))
        if ml > 0:
            return 1.0 - _lcs_length(t1[0], t2[0]) / ml
    return 1.0


def fuzzy_substring_search_constrained(hw, inp, threshold=0.6):
    """algo_calc.py:401-499: [(score, start phoneme, end phoneme)] best per end position, score descending."""
    n, m = len(hw), len(inp)
    if n == 0 or m == 0:
        return []
    INF = float('inf')
    dp = [[INF] * (m + 1) for _ in range(n + 1)]
    path = [[(0, 0)] * (m + 1) for _ in range(n + 1)]
    for j in range(m + 1):
        if j == 0 or (j < m and inp[j][2]):
            dp[0][j] = 0.0
            path[0][j] = (0, j)
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            dm = dp[i - 1][j - 1] + _tuple_cost(hw[i - 1], inp[j - 1])
            dd = dp[i - 1][j] + 1.0
            di = dp[i][j - 1] + 1.0
            v = min(dm, dd, di)
            dp[i][j] = v
            path[i][j] = path[i - 1][j - 1] if v == dm else (path[i - 1][j] if v == dd else path[i][j - 1])
    res = []
    for j in range(1, m + 1):
        if not inp[j - 1][3]:
            continue
        d = dp[n][j]
        if d >= n * 0.8:
            continue
        score = 1.0 - d / n
        if score >= threshold:
            res.append((score, path[n][j][1], j))
    res.sort(key=lambda x: x[0], reverse=True)
    used = {}
    for sc, s, e in res:
        if e not in used or sc > used[e][0]:
            used[e] = (sc, s, e)
    return sorted(used.values(), key=lambda x: x[0], reverse=True)


class MatchResult(NamedTuple):
    start: int
    end: int
    score: float
    hotword: str


class CorrectionResult(NamedTuple):
    text: str
    matchs: List[Tuple[str, str, float]]
    similars: List[Tuple[str, str, float]]


class PhonemeCorrector:
    """hot_phoneme.PhonemeCorrector (:36-221)."""

    def __init__(self, threshold=0.7, similar_threshold=None):
        self.threshold = threshold
        self.similar_threshold = similar_threshold if similar_threshold is not None else threshold - 0.2
        self.hotwords: Dict[str, List[Phoneme]] = {}
        self.fast_rag = FastRAG(min(self.threshold, self.similar_threshold) - 0.1)
        self._lock = threading.Lock()

    def update_hotwords(self, text: str) -> int:
        lines = [ln.strip() for ln in text.splitlines() if ln.strip() and not ln.strip().startswith('#')]
        hws = {}
        for hw in lines:
            ph = get_phoneme_info(hw)
            if ph:
                hws[hw] = ph
        with self._lock:
            self.hotwords = hws
            self.fast_rag = FastRAG(min(self.threshold, self.similar_threshold) - 0.1)
            self.fast_rag.add_hotwords(hws)
        return len(hws)

    def _find_matches(self, text, fast, inp):
        matches, similars = [], []
        thr = min(self.threshold, self.similar_threshold) - 0.1
        for hw, _ in fast:
            hwc = [p.info[:5] for p in self.hotwords[hw]]
            for score, s, e in fuzzy_substring_search_constrained(hwc, inp, thr):
                cs, ce = inp[s][5], inp[e - 1][6]
                if score >= self.threshold:
                    matches.append(MatchResult(cs, ce, score, hw))
                if score >= self.similar_threshold:
                    similars.append((text[cs:ce], hw, score))
        similars.sort(key=lambda x: (x[2], len(x[1])), reverse=True)
        out, seen = [], set()
        for o, hw, sc in similars:
            if hw not in seen:
                out.append((o, hw, sc))
                seen.add(hw)
        return matches, out

    def _resolve_and_replace(self, text, matches):
        """hot_phoneme.py:138-171: score first, then span length; no overlap with an accepted span."""
        matches.sort(key=lambda x: (x.score, x.end - x.start), reverse=True)
        final, occupied = [], []
        for m in matches:
            if m.score < self.threshold:
                continue
            if any(not (m.end <= a or m.start >= b) for a, b in occupied):
                continue
            if text[m.start:m.end] != m.hotword:
                final.append(m)
            occupied.append((m.start, m.end))
        final.sort(key=lambda x: x.start, reverse=True)
        chars = list(text)
        for m in final:
            chars[m.start:m.end] = list(m.hotword)
        return "".join(chars), [(text[m.start:m.end], m.hotword, m.score) for m in final]

    def correct(self, text: str, k: int = 10) -> CorrectionResult:
        if not text or not self.hotwords:
            return CorrectionResult(text, [], [])
        inp_ph = get_phoneme_info(text)
        if not inp_ph:
            return CorrectionResult(text, [], [])
        with self._lock:
            fast = self.fast_rag.search(inp_ph, top_k=100)
            matches, similars = self._find_matches(text, fast, [p.info for p in inp_ph])
        new_text, final = self._resolve_and_replace(text, matches)
        return CorrectionResult(new_text, final, similars[:k])


class HotwordSource:
    """hot.txt -> PhonemeCorrector, reloaded when the file changes (the reference's watchdog, manager.py:95-117)."""

    def __init__(self, path, similar_threshold=0.6):
        self.path = path
        self.corrector = PhonemeCorrector(threshold=1.0, similar_threshold=similar_threshold)
        self._mtime = None
        self.refresh()

    def refresh(self):
        try:
            mt = os.path.getmtime(self.path)
        except OSError:
            return
        if mt != self._mtime:
            self._mtime = mt
            with open(self.path, encoding="utf-8") as f:
                self.corrector.update_hotwords(f.read())

    def hotwords_for(self, ctc_text, k):
        """CTCDecoder.decode's hotword list (decoder.py:39-44): hotwords of matchs, then of similars."""
        self.refresh()
        if not ctc_text or not self.corrector.hotwords:
            return []
        res = self.corrector.correct(ctc_text, k=k)
        out = []
        for _, hw, _ in list(res.matchs) + list(res.similars):
            if hw not in out:
                out.append(hw)
        return out
