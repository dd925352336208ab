"""CTC vocabulary, greedy decode and char alignment (host side of SURVEY §8(a) A9/A14).

load_ctc_tokens   same file semantics as nano_ctc.py:12-36 (reference): "<b64 token> <id>" per line,
                  base64-decoded once at load; an undecodable token keeps its raw text.
decode_ctc_pairs  nano_ctc.py:38-116 on the device-collapsed (id, first_frame) pairs produced by the
                  k_ctc_collapse kernel (repeats/blank already removed on the GPU); token start time
                  max((frame*60 - 240)/1000, 0).
align_timestamps  nano_ctc.py:118-232 through the native fa_align_timestamps (bit-identical DP).
"""
import base64
import ctypes
import os
from dataclasses import dataclass
from itertools import repeat

import numpy as np

from . import _native


@dataclass(slots=True)  # the reference's fields, order, eq and repr (nano_ctc.py:7-10); slots: ~2x faster to build
class Token:
    text: str
    start: float


def load_ctc_tokens(filename):
    id2token = {}
    if not os.path.exists(filename):
        return id2token
    with open(filename, encoding="utf-8") as f:
        for line in f:
            parts = line.strip().split()
            if not parts:
                continue
            t, i = (" ", parts[0]) if len(parts) == 1 else (parts[0], parts[1])
            try:
                id2token[int(i)] = base64.b64decode(t).decode("utf-8")
            except Exception:
                id2token[int(i)] = t
    return id2token


def ctc_pair_rows(ids, frames, id2token):
    """(texts, starts) of the collapsed pairs, empty tokens dropped: the Token fields of decode_ctc_pairs as two lists.
    start = max((frame * 60 - 240) / 1000, 0) in float64 (exactly the reference's Python arithmetic)."""
    ids = ids.tolist() if hasattr(ids, "tolist") else list(ids)
    texts = list(map(id2token.get, ids, repeat("")))
    starts = np.maximum((np.asarray(frames, np.int64) * 60 - 240) / 1000.0, 0.0).tolist()
    if "" in texts:
        keep = [k for k, x in enumerate(texts) if x]
        texts, starts = [texts[k] for k in keep], [starts[k] for k in keep]
    return texts, starts


def tokens_of(texts, starts):
    return list(map(Token, texts, starts))


def decode_ctc_pairs(ids, frames, id2token):
    """(text, [Token]) from collapsed pairs; blank and empty tokens never appear in the output."""
    texts, starts = ctc_pair_rows(ids, frames, id2token)
    return "".join(texts), tokens_of(texts, starts)


def collapse_ids(ids, blank_id):
    """Host form of the collapse rule (used for ids already on the host)."""
    ids = np.asarray(ids)
    if ids.size == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    keep = np.ones(ids.size, bool)
    keep[1:] = ids[1:] != ids[:-1]
    keep &= ids != blank_id
    fr = np.nonzero(keep)[0]
    return ids[fr].astype(np.int32), fr.astype(np.int32)


def align_timestamps(ctc_results, llm_text):
    if not ctc_results or not llm_text:
        return []
    chars, starts = [], []
    for item in ctc_results:
        for i, ch in enumerate(item.text):
            chars.append(ch)
            starts.append(item.start + i * 0.08)
    llm_chars = list(llm_text)
    if not chars:  # every CTC token empty: the reference DP aligns nothing -> all starts 0.0
        return [{"char": c, "start": 0.0} for c in llm_chars]
    keys = {}
    ck = np.array([keys.setdefault(c.lower(), len(keys)) for c in chars], np.int32)
    lk = np.array([keys.setdefault(c.lower(), len(keys)) for c in llm_chars], np.int32)
    st = np.array(starts, np.float64)
    out = np.empty(len(llm_chars), np.float64)
    lib = _native.load()
    rc = lib.fa_align_timestamps(ck.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p), len(chars),
                                 lk.ctypes.data_as(ctypes.c_void_p), len(llm_chars), out.ctypes.data_as(ctypes.c_void_p),
                                 None)
    if rc != 0:
        raise RuntimeError("fa_align_timestamps failed")
    return [{"char": c, "start": float(s)} for c, s in zip(llm_chars, out.tolist())]
