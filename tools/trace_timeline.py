#!/usr/bin/env python3
"""Wall-time view of the timed graph replays in a rocprofv3 kernel trace (CSV).

The forwards are delimited by their first kernel (nchw_to_nhwc: the input conversion) and
their last (psnr_finalize).  For the last --steps forwards: wall span per forward, GPU-busy
time (union of kernel intervals), time with >= 2 kernels in flight, per hardware queue busy
time, and the wall time of the phases: analysis transform (up to quantize_median), hyper +
slice loop (to the last gauss_rate / lrp launch before s_model), synthesis + recon.
usage: python tools/trace_timeline.py TRACE_kernel_trace.csv [--steps 5]"""
import argparse
import collections
import csv


def union(iv):
    iv = sorted(iv)
    tot, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def overlap2(iv):
    ev = sorted([(a, 1) for a, b in iv] + [(b, -1) for a, b in iv])
    n, last, tot = 0, None, 0
    for t, d in ev:
        if n >= 2 and last is not None:
            tot += t - last
        n += d
        last = t
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
            for r in csv.DictReader(open(args.csv))]
    rows.sort(key=lambda r: r[1])
    starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r[0]]
    ends = [i for i, r in enumerate(rows) if "psnr_finalize" in r[0]]
    fw = []
    for s in starts:
        e = next((e for e in ends if e > s), None)
        if e is not None:
            fw.append((s, e))
    fw = fw[-args.steps:]
    agg = collections.defaultdict(float)
    for s, e in fw:
        sel = rows[s:e + 1]
        t0, t1 = sel[0][1], max(r[2] for r in sel)
        iv = [(r[1], r[2]) for r in sel]
        agg["span"] += t1 - t0
        agg["busy"] += union(iv)
        agg["overlap>=2"] += overlap2(iv)
        agg["kernels"] += len(sel)
        agg["kernel_sum"] += sum(b - a for a, b in iv)
        for q in set(r[3] for r in sel):
            agg[f"queue {q} busy"] += union([(r[1], r[2]) for r in sel if r[3] == q])
        qm = next(i for i, r in enumerate(sel) if "quantize_median" in r[0])
        last_rate = max(i for i, r in enumerate(sel) if "gauss_rate" in r[0])
        agg["phase a_model+h_a (to quantize_median)"] += sel[qm][1] - t0
        agg["phase hyper_s + slice loop"] += sel[last_rate][2] - sel[qm][1]
        agg["phase rest (last lrp, s_model, recon)"] += t1 - sel[last_rate][2]
        sl = [(r[1], r[2]) for r in sel[qm:last_rate + 1]]
        agg["slice phase busy"] += union(sl)
        agg["slice phase overlap>=2"] += overlap2(sl)
        agg["slice phase kernels"] += len(sl)
    n = len(fw)
    print(f"{n} forwards")
    for k, v in agg.items():
        unit = "" if "kernels" in k else " us"
        print(f"  {k:45s} {v / n / (1 if 'kernels' in k else 1e3):10.1f}{unit}")


if __name__ == "__main__":
    main()
