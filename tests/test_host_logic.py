"""Host-side product logic vs the reference's own outputs (tests/golden/ctc_align_merge.json, produced by
importing nano_ctc.py / text_merge.py from /root/reference). CPU only: fa_align_timestamps is host code."""
import json
import os
import tempfile

import numpy as np

from conftest import GOLDEN

G = json.load(open(os.path.join(GOLDEN, "ctc_align_merge.json"), encoding="utf-8"))


def test_load_ctc_tokens_matches_reference():
    from fun_asr_gguf.nano_ctc import load_ctc_tokens
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "tokens.txt")
        open(p, "w", encoding="utf-8").write(G["tokens_txt"])
        got = load_ctc_tokens(p)
    assert {str(k): v for k, v in got.items()} == G["id2token"]


def test_ctc_collapse_and_decode_match_reference():
    from fun_asr_gguf.nano_ctc import collapse_ids, decode_ctc_pairs
    id2 = {int(k): v for k, v in G["id2token"].items()}
    blank = max(id2)
    for c in G["decode"]:
        ids, fr = collapse_ids(np.array(c["ids"], np.int64), blank)
        text, toks = decode_ctc_pairs(ids, fr, id2)
        assert text == c["text"]
        assert [[t.text, t.start] for t in toks] == c["tokens"]


def test_native_align_bit_identical_to_reference():
    from fun_asr_gguf.nano_ctc import Token, align_timestamps
    for c in G["align"]:
        got = align_timestamps([Token(t, s) for t, s in c["ctc"]], c["llm"])
        assert got == c["aligned"]


def test_native_align_large_random_vs_oracle():
    """Sizes of a dense 60 s segment (~390 x 350 chars), mixed case, vs the oracle restatement."""
    from fun_asr_gguf.nano_ctc import Token, align_timestamps
    from oracle.ctc import align_timestamps as ref_align
    rng = np.random.default_rng(0)
    alpha = list("你好世界的是在有人我他这中大来上个国到说们为子和你地出道也时年aAbBcC，。")
    toks = [("".join(rng.choice(alpha, size=rng.integers(1, 3))), round(float(i * 0.15), 3)) for i in range(300)]
    text = "".join(rng.choice(alpha, size=350))
    got = align_timestamps([Token(t, s) for t, s in toks], text)
    assert got == ref_align(toks, text)


def test_merge_matches_reference():
    from fun_asr_gguf.text_merge import merge_transcription_results
    import copy
    for c in G["merge"]:
        text, segs = merge_transcription_results(copy.deepcopy(c["results"]), c["offsets"], c["overlap"])
        assert text == c["text"] and segs == c["segments"]


def test_segment_windows_match_reference_rule():
    from fun_asr_gguf.core.orchestrator import segment_windows
    from oracle.ctc import segments_info
    for d, s, o in [(300, 60, 4), (300, 60, 2), (61.9, 60, 2), (125.5, 60, 4), (1000, 30, 0.5)]:
        assert segment_windows(d, s, o) == segments_info(d, s, o)
    assert segment_windows(300, 60, 4) == [(0.0, 60.0), (56.0, 116.0), (112.0, 172.0), (168.0, 228.0),
                                          (224.0, 284.0), (280.0, 300)]


def test_lpt_assignment_balanced_and_complete():
    from fun_asr_gguf.parallel import lpt_assign
    lens = [60, 60, 60, 60, 60, 20]
    a = lpt_assign(lens, 8)
    assert sorted(i for x in a for i in x) == list(range(6))
    a4 = lpt_assign(lens, 4)
    loads = sorted(sum(lens[i] for i in x) for x in a4)
    assert loads == [60, 60, 80, 120]


def test_srt_writer():
    from fun_asr_gguf.srt_utils import generate_srt_file
    segs = [{"char": c, "start": i * 0.3} for i, c in enumerate("你好。世界！abc")]
    with tempfile.TemporaryDirectory() as td:
        p = generate_srt_file(segs, os.path.join(td, "a.srt"))
        s = open(p, encoding="utf-8").read()
    assert s.startswith("1\n00:00:00,000 --> ") and "你好。" in s and "世界！" in s


def test_init_fails_loudly_on_missing_model_files(tmp_path):
    """A model path that does not exist fails initialisation (model_manager.py:98-100 returns False, asr_engine.py:135
    raises) instead of running on synthetic weights; checked before any device work, so this runs without a GPU."""
    import pytest
    from fun_asr_gguf import FunASREngine, create_asr_engine
    missing = str(tmp_path / "Fun-ASR-Nano-Encoder-Adaptor.typo.onnx")
    for args in ((missing, "synthetic", "synthetic", "synthetic"), ("synthetic", missing, "synthetic", "synthetic"),
                 ("synthetic", "synthetic", str(tmp_path / "q8.gguf"), "synthetic"),
                 ("synthetic", "synthetic", "synthetic", str(tmp_path / "tokens.txt"))):
        eng = FunASREngine(*args, model="tiny")
        assert eng.initialize(verbose=False) is False
        assert eng.models.engine is None
        with pytest.raises(RuntimeError):
            create_asr_engine(*args, verbose=False, model="tiny")
