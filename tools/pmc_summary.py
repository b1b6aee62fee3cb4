#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one directory each) of
tools/conv_bench.py --only wnsa3x3@64 into the JSON that bench.py reads for `roofline.traffic`.
gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md): FETCH_SIZE counts half the bytes of
16 B/lane streaming reads -> x2; WRITE_SIZE exact; both in KB.
usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR LABEL COMMAND OUT.json [ELEM_BYTES=4]"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def per_dispatch(d, counter, kern):
    vals = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kern in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals[row.get("Dispatch_Id")] += float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals, key=lambda v: int(v))]


def main():
    fdir, wdir, kern, label, cmd, out = sys.argv[1:7]
    esz = int(sys.argv[7]) if len(sys.argv) > 7 else 4
    fe = per_dispatch(fdir, "FETCH_SIZE", kern)
    wr = per_dispatch(wdir, "WRITE_SIZE", kern)
    if not fe or not wr:
        sys.exit(f"no {kern} dispatches found")
    fkb, wkb = statistics.median(fe), statistics.median(wr)
    rd, wb = int(fkb * 1024 * 2), int(wkb * 1024)
    alg = (2 * 32 * 64 * 64 * 192 + 192 * 192 * 9) * esz
    rep = {"kernel": label, "command": cmd, "FETCH_SIZE_kb_per_dispatch_median": fkb,
           "WRITE_SIZE_kb_per_dispatch_median": wkb, "dispatches": [len(fe), len(wr)],
           "correction": "gfx950: FETCH_SIZE counts half the bytes of 16 B/lane streaming reads -> x2; WRITE_SIZE exact",
           "hbm_read_bytes": rd, "hbm_write_bytes": wb, "traffic_bytes_per_launch": rd + wb,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round((rd + wb) / alg, 3), "round": os.environ.get("LIC_ROUND", "r03")}
    with open(out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
