"""A fixed pinyin table with pypinyin's call interface (pinyin(fragment, style=..., **kw) -> [[str], ...] and a Style
namespace with INITIALS / FINALS / TONE3), standing in for pypinyin, which is absent from this image. Test data only:
the same table feeds the reference's hotword modules (tests/golden/make_hotword_golden.py) and fun_asr_gguf.hotword
(tests/test_hotword.py), so both see identical phonemes. Characters off the table get a syllable derived from their
code point."""

PY = {"张": ("zh", "ang", "1"), "三": ("s", "an", "1"), "章": ("zh", "ang", "1"), "山": ("sh", "an", "1"),
      "赞": ("z", "an", "4"), "是": ("sh", "i", "4"), "我": ("", "uo", "3"), "好": ("h", "ao", "3"),
      "阿": ("", "a", "1"), "里": ("l", "i", "3"), "巴": ("b", "a", "1"), "吧": ("b", "a", "5"),
      "通": ("t", "ong", "1"), "义": ("", "i", "4"), "千": ("q", "ian", "1"), "问": ("", "uen", "4"),
      "同": ("t", "ong", "2"), "一": ("", "i", "1"), "钱": ("q", "ian", "2"), "文": ("", "uen", "2"),
      "芯": ("x", "in", "1"), "片": ("p", "ian", "4"), "心": ("x", "in", "1"), "天": ("t", "ian", "1"),
      "今": ("j", "in", "1"), "发": ("f", "a", "1"), "布": ("b", "u", "4"), "了": ("l", "e", "5"),
      "和": ("h", "e", "2"), "年": ("n", "ian", "2"), "南": ("n", "an", "2"), "京": ("j", "ing", "1"),
      "蓝": ("l", "an", "2"), "经": ("j", "ing", "1"), "市": ("sh", "i", "4"), "长": ("zh", "ang", "3"),
      "江": ("j", "iang", "1"), "大": ("d", "a", "4"), "桥": ("q", "iao", "2"), "人": ("r", "en", "2"),
      "工": ("g", "ong", "1"), "智": ("zh", "i", "4"), "能": ("n", "eng", "2"), "只": ("zh", "i", "3")}

INITS = ["b", "p", "m", "f", "d", "t", "n", "l", "g", "k", "h", "j", "q", "x", "zh", "ch", "sh", "r", "z", "c", "s", ""]
FINS = ["a", "o", "e", "ai", "ei", "ao", "ou", "an", "en", "ang", "eng", "i", "u", "in", "ing", "uo"]


class Style:
    INITIALS, FINALS, TONE3 = 0, 1, 2


def pinyin(frag, style=0, **kw):
    out = []
    for ch in frag:
        o = ord(ch)
        i, f, t = PY.get(ch, (INITS[o % len(INITS)], FINS[(o // 7) % len(FINS)], str(1 + o % 4)))
        out.append([i if style == Style.INITIALS else f if style == Style.FINALS else f"{i}{f}{t}"])
    return out
