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
    texts = [item.text for item in ctc_results]
    chars = list("".join(texts))
    if len(chars) == len(texts) and "" not in texts:  # one char per token (the common case): the starts as they are
        starts = [item.start for item in ctc_results]
    else:  # char i of a token starts at start + i * 0.08 (nano_ctc.py:128-131)
        starts = []
        for item in ctc_results:
            starts.extend([item.start + i * 0.08 for i in range(len(item.text))])
    llm_chars = list(llm_text)
    if not chars:  # every CTC token empty: the reference DP aligns nothing -> all starts 0.0
        return [{"char": c, "start": 0.0} for c in llm_chars]
    # the DP compares lower-cased chars for equality only: one id per distinct lower-cased char, over both strings
    low = {}
    cid = {c: low.setdefault(c.lower(), len(low)) for c in set(chars).union(llm_chars)}
    ck = np.fromiter(map(cid.__getitem__, chars), np.int32, len(chars))
    lk = np.fromiter(map(cid.__getitem__, llm_chars), np.int32, len(llm_chars))
    st = np.array(starts, np.float64)
    out = np.empty(len(llm_chars), np.float64)
    lib = _native.load()
    rc = lib.fa_align_timestamps(ck.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p), len(chars),
                                 lk.ctypes.data_as(ctypes.c_void_p), len(llm_chars), out.ctypes.data_as(ctypes.c_void_p),
                                 None)
    if rc != 0:
        raise RuntimeError("fa_align_timestamps failed")
    return [{"char": c, "start": float(s)} for c, s in zip(llm_chars, out.tolist())]
