"""Per-kernel means of every counter in a rocprofv3 --pmc pass (rocpd sqlite), for the kernels whose name contains one
of the given substrings (default: all with >= 3 dispatches). With the SQ stall set (MI355X_MICROARCH.md, PMC table):
WAIT_ANY = waves parked on s_waitcnt / barriers, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY = issuing; the three
add up to WAVE_CYCLES, so their shares are printed too.
Usage: python scripts/pmc_kernels.py <results.db> [substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db, keys = sys.argv[1], sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute("select name, counter_name, counter_value from pmc_events").fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    for name, cn, v in rows:
        if keys and not any(k in name for k in keys):
            continue
        agg[name][cn].append(float(v))
    for name, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
        n = max(len(v) for v in cs.values())
        if not keys and n < 3:
            continue
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        line = f"{name[:110]}\n  dispatches {n}: " + ", ".join(f"{k} {v:.4g}" for k, v in sorted(m.items()))
        w = m.get("SQ_WAVE_CYCLES")
        if w:
            line += "\n  shares of WAVE_CYCLES: " + ", ".join(
                f"{k[3:]} {m[k] / w:.3f}" for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in m)
        print(line)


if __name__ == "__main__":
    main()
