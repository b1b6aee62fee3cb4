#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of
tools/conv_bench.py --only wnsa3x3@64) into the per-launch HBM traffic of the bench's
roofline kernel.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
half the bytes of 16 B/lane streaming reads -> x2; WRITE_SIZE is exact.  Units: KB.
usage: python profiles/pmc_summary.py FETCH_DIR WRITE_DIR DTYPE OUT.json"""
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, match="conv_halo_kernel"):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if match in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals, statistics.median(vals)


def main():
    fdir, wdir, dtype, out = sys.argv[1:5]
    fv, f_kb = per_dispatch(f"{fdir}/pmc_counter_collection.csv", "FETCH_SIZE")
    wv, w_kb = per_dispatch(f"{wdir}/pmc_counter_collection.csv", "WRITE_SIZE")
    esz = 2 if dtype == "f16" else 4
    B, H, C = 32, 64, 192
    alg = B * H * H * C * esz * 2 + C * C * 9 * esz   # input + output + weights
    rd, wr = f_kb * 1024 * 2, w_kb * 1024
    res = {"kernel": f"conv_halo_kernel<{dtype}> conv3x3 192->192 s1 @64x64 x32 (tools/conv_bench.py --only wnsa3x3@64)",
           "command": f"rocprofv3 --pmc FETCH_SIZE --output-format csv -- python3 tools/conv_bench.py --dtype "
                      f"{'fp16' if dtype == 'f16' else 'fp32'} --iters 5 --auto-only --only wnsa3x3@64; same with "
                      f"--pmc WRITE_SIZE (separate passes)",
           "FETCH_SIZE_kb_per_dispatch_median": f_kb, "WRITE_SIZE_kb_per_dispatch_median": w_kb,
           "dispatches": [len(fv), len(wv)],
           "correction": "gfx950: FETCH_SIZE counts half the bytes of 16 B/lane streaming reads -> x2; WRITE_SIZE exact",
           "hbm_read_bytes": int(rd), "hbm_write_bytes": int(wr), "traffic_bytes_per_launch": int(rd + wr),
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round((rd + wr) / alg, 3), "round": "r02"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
