"""SRT export from char timestamps (reference srt_utils.py:10-74 uses the absent `srt` package; this
writes the same kind of subtitle file with the stdlib: lines cut at sentence punctuation or 2 s gaps)."""

_BREAK = set("。！？!?；;")


def _fmt(t):
    t = max(0.0, float(t))
    h, r = divmod(int(t * 1000 + 0.5), 3600_000)
    m, r = divmod(r, 60_000)
    s, ms = divmod(r, 1000)
    return f"{h:02d}:{m:02d}:{s:02d},{ms:03d}"


def group_lines(segments, max_chars=24, gap=2.0):
    lines, cur = [], []
    for i, s in enumerate(segments):
        if cur and (s["start"] - cur[-1]["start"] > gap):
            lines.append(cur)
            cur = []
        cur.append(s)
        if s["char"] in _BREAK or len(cur) >= max_chars:
            lines.append(cur)
            cur = []
    if cur:
        lines.append(cur)
    return lines


def generate_srt_file(segments, path, max_chars=24):
    lines = group_lines(segments, max_chars)
    with open(path, "w", encoding="utf-8") as f:
        for k, ln in enumerate(lines):
            start = ln[0]["start"]
            nxt = lines[k + 1][0]["start"] if k + 1 < len(lines) else ln[-1]["start"] + 0.5
            end = max(nxt, ln[-1]["start"] + 0.2)
            text = "".join(s["char"] for s in ln).strip()
            f.write(f"{k + 1}\n{_fmt(start)} --> {_fmt(end)}\n{text}\n\n")
    return path
