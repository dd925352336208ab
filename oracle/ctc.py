"""CTC greedy collapse + char alignment + segment merge restatements — TEST INFRASTRUCTURE ONLY.

decode_ctc        <- /root/reference/fun_asr_gguf/nano_ctc.py:38-116
align_timestamps  <- nano_ctc.py:118-232 (Needleman-Wunsch, tie order diag > up > left)
merge_results     <- text_merge.py:14-114
segments_info     <- core/orchestrator.py:123-136
"""
import difflib


def collapse(ids, blank_id):
    """Greedy collapse (:65-104): runs of equal ids -> (id, first frame); drop blank."""
    out = []
    n = len(ids)
    if n == 0:
        return out
    cur, start = int(ids[0]), 0
    for i in range(1, n):
        if int(ids[i]) != cur:
            out.append((cur, start))
            cur, start = int(ids[i]), i
    out.append((cur, start))
    return [(t, s) for t, s in out if t != blank_id]


def decode_ctc(ids, id2token):
    """Returns (text, [(token_text, start_seconds)])."""
    blank = max(id2token.keys()) if id2token else 0
    res = []
    for tid, s in collapse(ids, blank):
        txt = id2token.get(tid, "")
        if not txt:
            continue
        res.append((txt, max((s * 60 + -240) / 1000.0, 0.0)))
    return "".join(t for t, _ in res), res


def align_timestamps(ctc_results, llm_text):
    if not ctc_results or not llm_text:
        return []
    cc = []
    for text, start in ctc_results:
        for i, ch in enumerate(text):
            cc.append((ch, start + i * 0.08))
    lc = list(llm_text)
    n, m = len(cc) + 1, len(lc) + 1
    score = [[0.0] * m for _ in range(n)]
    trace = [[0] * m for _ in range(n)]
    for i in range(n):
        score[i][0] = -float(i)
    for j in range(m):
        score[0][j] = -float(j)
    for i in range(1, n):
        a = cc[i - 1][0].lower()
        row, prev = score[i], score[i - 1]
        tr = trace[i]
        for j in range(1, m):
            d = prev[j - 1] + (1.0 if a == lc[j - 1].lower() else -1.0)
            u = prev[j] - 1.0
            l = row[j - 1] - 1.0
            best = max(d, u, l)
            row[j] = best
            tr[j] = 1 if best == d else (2 if best == u else 3)
    al = [None] * len(lc)
    i, j = n - 1, m - 1
    while i > 0 or j > 0:
        if i > 0 and j > 0 and trace[i][j] == 1:
            al[j - 1] = cc[i - 1]
            i -= 1
            j -= 1
        elif i > 0 and (j == 0 or trace[i][j] == 2):
            i -= 1
        elif j > 0 and (i == 0 or trace[i][j] == 3):
            al[j - 1] = None
            j -= 1
    anchors = [(k, it[1]) for k, it in enumerate(al) if it is not None]

    def interp(t):
        pa = na = None
        for a in anchors:
            if a[0] < t:
                pa = a
            elif a[0] > t:
                na = a
                break
        if pa and na:
            return pa[1] + (t - pa[0]) * ((na[1] - pa[1]) / (na[0] - pa[0]))
        if pa:
            return pa[1] + 0.05
        if na:
            return max(0, na[1] - 0.05)
        return 0.0

    return [{"char": ch, "start": (al[k][1] if al[k] else interp(k))} for k, ch in enumerate(lc)]


def segments_info(duration, segment_size, overlap):
    out, step, cur = [], segment_size - overlap, 0.0
    while cur < duration:
        end = min(cur + segment_size, duration)
        out.append((cur, end))
        if end >= duration:
            break
        cur += step
    return out


def merge_results(results, offsets, overlap_s):
    if not results:
        return "", []
    if len(results) == 1:
        return results[0]["text"], [{"char": s["char"], "start": s["start"] + offsets[0]}
                                     for s in (results[0].get("segments") or [])]
    full = []
    puncs = set("，。！？；,.!?; ")
    for i, res in enumerate(results):
        off = offsets[i]
        cur = [dict(s) for s in (res.get("segments") or [])]
        for s in cur:
            s["_g"] = s["start"] + off
        if i == 0:
            full.extend({"char": s["char"], "start": s["_g"]} for s in cur)
            continue
        if not cur:
            continue
        bseg = [s for s in full if s["start"] >= off - 1.0]
        btxt = "".join(s["char"] for s in bseg)
        cseg = [s for s in cur if s["start"] <= overlap_s + 1.0]
        ctxt = "".join(s["char"] for s in cseg)
        mt = difflib.SequenceMatcher(None, btxt, ctxt).find_longest_match(0, len(btxt), 0, len(ctxt))
        if mt.size >= 2:
            tgt = bseg[mt.a]
            gi = -1
            for k in range(len(full) - 1, -1, -1):
                if full[k]["start"] == tgt["start"] and full[k]["char"] == tgt["char"]:
                    gi = k
                    break
            if gi != -1:
                full = full[:gi]
            ms = cseg[mt.b]
            mi = next((k for k, s in enumerate(cur) if s is ms), -1)
            add = cur[mi:] if mi != -1 else cur
            full.extend({"char": s["char"], "start": s["_g"]} for s in add)
        else:
            last = full[-1]["start"] if full else off
            full.extend({"char": s["char"], "start": s["_g"]} for s in cur if s["_g"] > last + 0.1)
    clean = []
    for s in full:
        if clean and s["char"] in puncs and clean[-1]["char"] == s["char"]:
            continue
        clean.append(s)
    return "".join(s["char"] for s in clean), clean
