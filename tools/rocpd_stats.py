#!/usr/bin/env python3
"""Per-kernel summary (calls, total / average duration, share) of a rocprofv3 rocpd SQLite
database (`rocprofv3 --kernel-trace -d DIR -o run` writes DIR/run_results.db on this image).
usage: python tools/rocpd_stats.py DB [TOP] [--last-dispatches N]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 40
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    if "--last-dispatches" in sys.argv:
        rows = rows[-int(sys.argv[sys.argv.index("--last-dispatches") + 1]):]
    agg = defaultdict(lambda: [0, 0])
    for name, s, e in rows:
        a = agg[name]
        a[0] += 1
        a[1] += e - s
    tot = sum(v[1] for v in agg.values())
    span = (rows[-1][2] - rows[0][1]) if rows else 0
    print(f"# {len(rows)} dispatches, kernel time {tot / 1e6:.3f} ms, span {span / 1e6:.3f} ms")
    print("  calls   total_ms    avg_us    pct  kernel")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:7d} {t / 1e6:10.3f} {t / n / 1e3:9.2f} {100 * t / tot:6.2f}  {name[:160]}")


if __name__ == "__main__":
    main()
