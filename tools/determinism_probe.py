#!/usr/bin/env python3
"""Determinism probe for the B=32 fp16 path (the entropy-coder round-trip failure of
round 1): poisons the caching allocator's free blocks with 0xFF bytes (fp16 NaN,
int32 -1) between calls so that any read of uninitialised memory becomes visible,
then compares every intermediate of repeated forwards / compress / decompress calls
bit for bit.  Prints one JSON line; exit status 1 when anything differs.

usage: python tools/determinism_probe.py [--batch 32] [--precision fp16] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def poison(total_mb=6144, random=False):
    """Allocate, fill with 0xFF (or with fresh random finite fp16 values) and free blocks
    of several sizes: later torch.empty calls reuse them, so uninitialised reads see
    NaN / -1 (or values that change from call to call) instead of stale data."""
    keep = []
    sizes = [1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20]
    used = 0
    while used < total_mb << 20:
        for s in sizes:
            t = torch.empty((s,), dtype=torch.uint8, device="cuda")
            if random:
                t.view(torch.float16).normal_()
            else:
                t.fill_(0xFF)
            keep.append(t)
            used += s
    torch.cuda.synchronize()
    del keep


def diff(a: dict, b: dict, chan_axis=None):
    bad = {}
    chan_axis = chan_axis or {}
    for k in a:
        if k not in b or a[k] is None:
            continue
        x, y = a[k], b[k]
        if x.shape != y.shape:
            bad[k] = "shape"
            continue
        if x.dtype.is_floating_point:
            same = torch.equal(x.view(torch.int16 if x.dtype == torch.float16 else torch.int32),
                               y.view(torch.int16 if y.dtype == torch.float16 else torch.int32))
        else:
            same = torch.equal(x, y)
        if not same:
            ne = (x != y) if not x.dtype.is_floating_point else (x.float() != y.float()) | (x.isnan() != y.isnan())
            bad[k] = {"n_diff": int(ne.sum()), "numel": x.numel(),
                      "max_abs": float((x.float() - y.float()).abs().nan_to_num(1e30).max())}
            cax = chan_axis.get(k)
            if cax is not None and x.dim() == 4 and x.shape[cax] == 192:
                per = ne.movedim(cax, 0).reshape(4, 48, -1).sum(dim=(1, 2))
                bad[k]["per_slice"] = [int(v) for v in per]
    return bad


NHWC = {"means": 3, "scales": 3, "y_hat": 3, "indexes": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-poison", action="store_true")
    ap.add_argument("--poison-random", action="store_true", help="fill freed blocks with random finite fp16")
    ap.add_argument("--single-stream", action="store_true", help="run the side-stream branches on the current stream")
    ap.add_argument("--forward-only", action="store_true")
    args = ap.parse_args()
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B, S = args.batch, args.size
    net = net_ga.Net((B, S, S, 3), (B, S, S, 3), False, False, precision=args.precision).to("cuda")
    x = (torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(1)) * 2 - 1).to("cuda")
    if args.single_stream:
        net.__dict__["_lic_single_stream"] = True
    pz = (lambda: None) if args.no_poison else (lambda: poison(random=args.poison_random))
    report = {"workload": f"net_ga {args.precision} B={B} {S}x{S}", "poison": "none" if args.no_poison else ("random" if args.poison_random else "0xff"),
              "single_stream": args.single_stream}

    def fwd():
        net(x, "test", return_intermediates=True)
        torch.cuda.synchronize()
        return {k: v.detach().clone() for k, v in net.last.items() if torch.is_tensor(v)}

    ref = fwd()
    fw = []
    for r in range(args.reps):
        pz()
        fw.append(diff(ref, fwd(), {"means": 1, "scales": 1, "y_hat": 1, "symbols": 1}))
    report["forward_diffs"] = fw
    report["serial_parts"] = os.environ.get("LIC_DEBUG_SERIAL", "")
    if args.forward_only:
        report["ok"] = all(not d for d in fw)
        report["n_bad"] = sum(1 for d in fw if d)
        print(json.dumps(report), flush=True)
        sys.exit(0 if report["ok"] else 1)

    net.update()
    enc = net.compress(x)
    torch.cuda.synchronize()
    c0 = {k: v.clone() for k, v in net.last_coder.items()}
    report["compress_vs_forward_symbols_equal"] = bool(torch.equal(enc["symbols"].permute(0, 3, 1, 2).cpu(),
                                                                   ref["symbols"].cpu()))
    comp = []
    for r in range(args.reps):
        pz()
        e2 = net.compress(x)
        torch.cuda.synchronize()
        comp.append({"diff": diff(c0, net.last_coder, NHWC), "strings_equal": e2["strings"] == enc["strings"]})
    report["compress_diffs"] = comp
    dec = []
    for r in range(args.reps):
        pz()
        err = None
        try:
            d = net.decompress(enc["strings"], enc["shape"], enc["syntax"])
            torch.cuda.synchronize()
            sym_ok = bool(torch.equal(d["symbols"], enc["symbols"]))
        except ValueError as e:
            err, sym_ok = str(e), False
        dd = diff({k: c0[k] for k in ("means", "scales", "z_hat", "y_hat")}, net.last_coder, NHWC)
        dec.append({"error": err, "symbols_equal": sym_ok, "diff_vs_compress": dd})
    report["decompress"] = dec
    ok = (all(not d for d in fw) and all(not c["diff"] and c["strings_equal"] for c in comp)
          and all(d["error"] is None and d["symbols_equal"] and not d["diff_vs_compress"] for d in dec))
    report["ok"] = ok
    print(json.dumps(report), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
