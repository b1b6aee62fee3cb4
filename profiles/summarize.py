#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) into a
per-kernel stats table: calls, total / average / min / max duration, share.

usage: python profiles/summarize.py <results.db | kernel_trace.csv> [--grid] [--top N] [--after-gap S] [--steps K]
  --grid: one row per (kernel, grid): per-shape rows
  --after-gap S: only the dispatches after the last idle gap of >= S seconds (bench.py --profile sleeps 1 s
                 between its warm-up / capture and the graph replays: the replay-only trace)
  --steps K: also print the per-step kernel time (total / K)
"""
import collections
import csv
import sqlite3
import sys


def load(path):
    rows = []  # (name, dur_ns, grid, start_ns, end_ns)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
        kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
        ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
        q = (f"select s.kernel_name, d.end - d.start, d.grid_size_x, d.grid_size_y, d.workgroup_size_x, d.start, d.end "
             f"from {kd} d join {ks} s on d.kernel_id = s.id")
        for name, dur, gx, gy, wx, t0, t1 in c.execute(q):
            rows.append((name, dur, (gx // max(wx, 1), gy), t0, t1))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                rows.append((r["Kernel_Name"], t1 - t0, (r.get("Grid_Size_X"), r.get("Grid_Size_Y")), t0, t1))
    return rows


def short(name):
    import re
    n = re.sub(r"\(.*", "", name)
    return n[:110]


def main():
    path = sys.argv[1]
    by_grid = "--grid" in sys.argv
    top = 40
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    rows = sorted(load(path), key=lambda r: r[3])
    if "--after-gap" in sys.argv:
        gap = float(sys.argv[sys.argv.index("--after-gap") + 1]) * 1e9
        cut, last_end = 0, None
        for i, r in enumerate(rows):
            if last_end is not None and r[3] - last_end >= gap:
                cut = i
            last_end = r[4] if last_end is None else max(last_end, r[4])
        rows = rows[cut:]
    agg = collections.OrderedDict()
    for name, dur, grid, _, _ in rows:
        key = (short(name), grid) if by_grid else short(name)
        a = agg.setdefault(key, [0, 0, None, 0])
        a[0] += 1
        a[1] += dur
        a[2] = dur if a[2] is None else min(a[2], dur)
        a[3] = max(a[3], dur)
    total = sum(a[1] for a in agg.values())
    print(f"# kernels: {len(rows)} dispatches, total {total / 1e6:.3f} ms")
    if "--steps" in sys.argv:
        k = int(sys.argv[sys.argv.index("--steps") + 1])
        print(f"# per step ({k} steps): {len(rows) / k:.0f} dispatches, {total / k / 1e6:.3f} ms of kernel time")
    print(f"{'calls':>7} {'total_ms':>10} {'avg_us':>10} {'min_us':>9} {'max_us':>9} {'pct':>6}  kernel")
    for key, (n, s, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:7d} {s / 1e6:10.3f} {s / n / 1e3:10.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} {100 * s / total:6.2f}  {key}")


if __name__ == "__main__":
    main()
