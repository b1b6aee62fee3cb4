#!/usr/bin/env python3
"""Critical-path view of the last N graph replays in a rocprofv3 kernel trace (.db).

For the final `--last` dispatches that form the timed replays, reports the wall span,
the GPU-busy time (union of kernel intervals), the idle gaps, the per-queue busy
time, and per kernel: total time and the time during which it was the ONLY kernel
running (a lower bound on its share of the critical path).

usage: python profiles/timeline.py run_results.db [--steps 5] [--top 30]
"""
import argparse
import collections
import sqlite3


def load(path):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    q = (f"select s.kernel_name, d.start, d.end, d.queue_id, d.grid_size_x / max(d.workgroup_size_x, 1) "
         f"from {kd} d join {ks} s on d.kernel_id = s.id order by d.start")
    return [(n, a, b, qid, g) for n, a, b, qid, g in c.execute(q)]


def short(name):
    for p in ("_ZN3lic", "_ZN2at6native"):
        if name.startswith(p):
            name = name[len(p):]
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5, help="timed replays at the end of the trace")
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    rows = load(args.db)
    # the timed replays are the trailing dispatches after the largest host-side gap
    gaps = [(rows[i + 1][1] - rows[i][2], i + 1) for i in range(len(rows) - 1)]
    per = None
    # dispatches per forward: count between the last two big gaps is unreliable under
    # graph replay (no gaps), so take the trailing fraction by kernel count of one
    # eager forward: the number of syntax_recon kernels marks forwards
    marks = [i for i, r in enumerate(rows) if "syntax_recon" in r[0]]
    if len(marks) >= args.steps + 1:
        start = marks[-args.steps - 1] + 1
    else:
        start = 0
    sel = rows[start:]
    t0 = min(r[1] for r in sel)
    t1 = max(r[2] for r in sel)
    ev = []
    for k, (n, a, b, qid, g) in enumerate(sel):
        ev.append((a, 1, k))
        ev.append((b, -1, k))
    ev.sort()
    active = set()
    busy = 0
    alone = collections.defaultdict(float)
    last = t0
    for t, d, k in ev:
        if active:
            busy += t - last
            if len(active) == 1:
                alone[sel[next(iter(active))][0]] += t - last
        last = t
        if d > 0:
            active.add(k)
        else:
            active.discard(k)
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for n, a, b, qid, g in sel:
        tot[n] += b - a
        cnt[n] += 1
    qbusy = collections.defaultdict(float)
    for n, a, b, qid, g in sel:
        qbusy[qid] += b - a
    span = (t1 - t0) / 1e6
    print(f"# {args.steps} replays: span {span:.3f} ms ({span / args.steps:.3f} ms/step), "
          f"GPU busy {busy / 1e6:.3f} ms ({100 * busy / (t1 - t0):.1f} %), idle {(t1 - t0 - busy) / 1e6:.3f} ms, "
          f"{len(sel)} dispatches")
    print("# queue busy ms/step:", {q: round(v / 1e6 / args.steps, 3) for q, v in sorted(qbusy.items())})
    print(f"{'ms/step':>8} {'alone':>8} {'calls':>5}  kernel")
    for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:args.top]:
        print(f"{v / 1e6 / args.steps:8.3f} {alone[n] / 1e6 / args.steps:8.3f} {cnt[n] // args.steps:5d}  {short(n)}")


if __name__ == "__main__":
    main()
