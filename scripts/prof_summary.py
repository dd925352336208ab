"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) or *_kernel_stats.csv: per-kernel calls,
total/avg duration. Usage: python scripts/prof_summary.py <results.db|kernel_stats.csv> [top]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def from_db(path, by_grid=False):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    gcols = [x for x in cols if x.startswith("grid")] if by_grid else []
    sel = ", ".join([name_col, "start", "end"] + gcols)
    agg = defaultdict(lambda: [0, 0.0])
    for row in c.execute(f"select {sel} from kernels").fetchall():
        n, s, e = row[:3]
        if gcols:
            n = f"[grid {'x'.join(str(g) for g in row[3:])}] {n}"
        agg[n][0] += 1
        agg[n][1] += (e - s)
    return agg


def from_csv(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        agg[r["Name"]] = [int(r["Calls"]), float(r["TotalDurationNs"])]
    return agg


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 30
    by_grid = "--by-grid" in sys.argv  # split each kernel's rows by launch grid (e.g. prefill vs decode shapes)
    agg = from_db(path, by_grid) if path.endswith(".db") else from_csv(path)
    tot = sum(v[1] for v in agg.values())
    print(f"{'total_ms':>10} {'calls':>8} {'avg_us':>9} {'pct':>6}  kernel")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / 1e6:10.2f} {k:8d} {t / k / 1e3:9.2f} {100 * t / tot:6.2f}  {n[:130]}")
    print(f"{tot / 1e6:10.2f} total kernel ms")


if __name__ == "__main__":
    main()
