#!/usr/bin/env python3
"""Kernel-time shares of a rocprofv3 --kernel-trace --stats run of `bench.py --profile`:
top kernels, the 8x8-px-tile (slice-loop / latent) share, exact-fp32 (`<float,...>`) kernels and
the dispatch count per forward.  usage: python tools/trace_share.py STATS_CSV [TRACE_CSV] [forwards]"""
import csv
import sys


def main():
    stats = list(csv.DictReader(open(sys.argv[1])))
    total = sum(float(r["TotalDurationNs"]) for r in stats)
    print(f"total kernel time {total / 1e6:.2f} ms over {sum(int(r['Calls']) for r in stats)} dispatches")
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f"{float(r['Percentage']):6.2f} %  {int(r['Calls']):6d} x {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:120]}")

    def share(pred):
        return 100.0 * sum(float(r["TotalDurationNs"]) for r in stats if pred(r["Name"])) / total

    small = lambda n: (("8, 8," in n or "<2, 8, 8" in n) and ("conv_split_wd" in n or "conv_halo_split" in n)) or "resunit" in n
    print(f"8x8-px tile kernels (WD / LDS-staged split, fused ResidualUnit): {share(small):.2f} %")
    print(f"exact-fp32 kernels (<float, ...>): {share(lambda n: '<float' in n):.2f} %")
    for r in stats:
        if "<float" in r["Name"] and float(r["Percentage"]) > 1.0:
            print(f"  > 1 %: {float(r['Percentage']):.2f} % {r['Name'][:100]}")
    if len(sys.argv) > 3:
        fw = int(sys.argv[3])
        print(f"dispatches per forward (all, over {fw} forwards): {sum(int(r['Calls']) for r in stats) / fw:.0f}")


if __name__ == "__main__":
    main()
