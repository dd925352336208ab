"""Merge of overlapping long-audio segment results (host step after the multi-GPU gather).

Semantics of /root/reference/fun_asr_gguf/text_merge.py:14-114: for each new segment, find the longest
common substring (difflib.SequenceMatcher.find_longest_match, >= 2 chars) between the merged tail whose
global start >= offset - 1 s and the new segment's head whose local start <= overlap + 1 s; cut the
merged list at the (last) matching element and append the new segment from its match; otherwise append
the new chars later than last + 0.1 s. Finally drop immediately repeated punctuation.
"""
import difflib
from typing import Any, Dict, List, Tuple

PUNCS = frozenset("，。！？；,.!?; ")


def merge_transcription_results(results: List[Dict[str, Any]], segment_offsets: List[float],
                                overlap_s: float) -> Tuple[str, List[Dict[str, Any]]]:
    if not results:
        return "", []
    if len(results) == 1:
        off = segment_offsets[0]
        return results[0]["text"], [{"char": s["char"], "start": s["start"] + off}
                                    for s in (results[0].get("segments") or [])]
    merged: List[Dict[str, Any]] = []
    for k, res in enumerate(results):
        off = segment_offsets[k]
        cur = [(s["char"], s["start"], s["start"] + off) for s in (res.get("segments") or [])]
        if k == 0:
            merged.extend({"char": c, "start": g} for c, _, g in cur)
            continue
        if not cur:
            continue
        tail = [s for s in merged if s["start"] >= off - 1.0]
        head_idx = [i for i, (_, st, _) in enumerate(cur) if st <= overlap_s + 1.0]
        a = "".join(s["char"] for s in tail)
        b = "".join(cur[i][0] for i in head_idx)
        m = difflib.SequenceMatcher(None, a, b).find_longest_match(0, len(a), 0, len(b))
        if m.size >= 2:
            anchor = tail[m.a]
            for i in range(len(merged) - 1, -1, -1):
                if merged[i]["start"] == anchor["start"] and merged[i]["char"] == anchor["char"]:
                    merged = merged[:i]
                    break
            start_at = head_idx[m.b]
            merged.extend({"char": c, "start": g} for c, _, g in cur[start_at:])
        else:
            last = merged[-1]["start"] if merged else off
            merged.extend({"char": c, "start": g} for c, _, g in cur if g > last + 0.1)
    out: List[Dict[str, Any]] = []
    for s in merged:
        if out and s["char"] in PUNCS and out[-1]["char"] == s["char"]:
            continue
        out.append(s)
    return "".join(s["char"] for s in out), out
