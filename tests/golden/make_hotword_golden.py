"""Golden vectors for the hotword path from the REFERENCE's own modules, run in this container.

Run (container only, needs /root/reference):  python tests/golden/make_hotword_golden.py

Imported from /root/reference/fun_asr_gguf/hotword by file path, without the package __init__ (it pulls in the
watchdog-based manager and the other correctors): algo_phoneme.py, algo_calc.py, rag_fast.py, hot_phoneme.py.
pypinyin is absent: its module slot is filled with tests/golden/fake_pinyin.py (a fixed table with pypinyin's call
interface), and the reference's degraded mode is run too by setting algo_phoneme.pinyin = None (its own
`if not pinyin` branches, algo_phoneme.py:175, 204). numba is absent: rag_fast.py runs its pure-Python distance
(rag_fast.py:21-26, 291-313). Output: tests/golden/hotword_golden.json.
"""
import importlib
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/fun_asr_gguf/hotword"
sys.path.insert(0, HERE)
import fake_pinyin  # noqa: E402

HOT = "# 热词\n张三\n阿里巴巴\n通义千问\nMI355X\n南京市长江大桥\n人工智能\nHelloWorld\n芯片\n"
TEXTS = ["我是章山", "今天阿里巴吧发布了通义千问和 MI355 芯片", "同一钱文是人工只能", "南京市长江大桥", "蓝经市长江大桥好",
         "hello world 2024年", "我好", "", "abc", "张三张三赞山", "MI 355 x 和 mi355x"]
PAIRS = [("张三", "我是章山", 0.5), ("通义千问", "今天阿里巴吧发布了通义千问和", 0.6), ("阿里巴巴", "今天阿里巴吧发布了", 0.5),
         ("MI355X", "和 MI355 芯片", 0.4), ("南京市长江大桥", "蓝经市长江大桥好", 0.6), ("人工智能", "人工只能", 0.5),
         ("HelloWorld", "hello world 2024", 0.5), ("张三", "张三张三赞山", 0.6)]


def ref_modules():
    sys.modules["pypinyin"] = fake_pinyin
    pkg = types.ModuleType("ref_hotword")
    pkg.__path__ = [REF]
    import logging
    pkg.logger = logging.getLogger("ref_hotword")
    sys.modules["ref_hotword"] = pkg
    return {n: importlib.import_module("ref_hotword." + n) for n in ("algo_phoneme", "algo_calc", "rag_fast", "hot_phoneme")}


def run(mods):
    ap, ac, rf, hp = mods["algo_phoneme"], mods["algo_calc"], mods["rag_fast"], mods["hot_phoneme"]
    out = {"phonemes": {t: [list(p.info) for p in ap.get_phoneme_info(t)] for t in TEXTS}}
    out["search"] = []
    for hw, text, th in PAIRS:
        hwi = [p.info[:5] for p in ap.get_phoneme_info(hw)]
        inp = [p.info for p in ap.get_phoneme_info(text)]
        out["search"].append({"hotword": hw, "text": text, "threshold": th,
                              "result": [list(r) for r in ac.fuzzy_substring_search_constrained(hwi, inp, th)]})
    lines = [ln.strip() for ln in HOT.splitlines() if ln.strip() and not ln.strip().startswith("#")]
    rag = rf.FastRAG(threshold=0.5)
    rag.add_hotwords({hw: ap.get_phoneme_info(hw) for hw in lines})
    out["fastrag"] = {t: [list(r) for r in rag.search(ap.get_phoneme_info(t), top_k=10)] for t in TEXTS if t}
    out["correct"] = []
    for th, sim in ((1.0, 0.6), (0.8, 0.6), (0.7, None)):
        c = hp.PhonemeCorrector(threshold=th, similar_threshold=sim)
        n = c.update_hotwords(HOT)
        for t in TEXTS:
            r = c.correct(t, k=10)
            out["correct"].append({"threshold": th, "similar_threshold": sim, "n_hotwords": n, "text": t,
                                   "out": r.text, "matchs": [list(x) for x in r.matchs],
                                   "similars": [list(x) for x in r.similars]})
    return out


def main():
    mods = ref_modules()
    gold = {"hot": HOT, "texts": TEXTS, "pinyin_table": run(mods)}
    mods["algo_phoneme"].pinyin = None  # the reference's degraded mode (no pypinyin)
    gold["degraded"] = run(mods)
    json.dump(gold, open(os.path.join(HERE, "hotword_golden.json"), "w"), ensure_ascii=False, indent=0)
    print("hotword_golden.json written:", {k: len(v["correct"]) for k, v in gold.items() if isinstance(v, dict)})


if __name__ == "__main__":
    main()
