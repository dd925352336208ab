"""Launch gaps on one stream from a rocprofv3 kernel-trace database: for the last `n` kernels (the timed region of a
profiling script), the span from the first start to the last end, the summed kernel time, and the gap quantiles
between consecutive kernels (next start - previous end). Usage: python scripts/prof_gaps.py <results.db> [n]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = sorted(c.execute(f"select start, end, {name_col} from kernels").fetchall())[-n:]
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in rows) / 1e3
    gaps = sorted((rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1))
    q = lambda f: gaps[min(len(gaps) - 1, int(f * len(gaps)))]
    print(f"last {len(rows)} kernels: span {span:.1f} us, kernel time {busy:.1f} us ({busy / span:.3f} busy), "
          f"gaps p10 {q(0.1):.2f} p50 {q(0.5):.2f} p90 {q(0.9):.2f} us, sum {sum(gaps):.1f} us")


if __name__ == "__main__":
    main()
