#!/usr/bin/env python3
"""Micro-benchmark of the conv kernels on the a_model / s_model hot shapes.

Times each shape with the automatic kernel choice and with the generic implicit-GEMM
kernel (force_generic), interleaved in one process (HIP events on the launch
stream), and prints TFLOP/s against the dense MFMA peak of the dtype.
usage: python tools/conv_bench.py [--dtype fp16|fp32] [--batch 32] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = {"fp16": 2516.6, "fp32": 157.3, "fp32x3": 2516.6 / 3, "fp32x6": 2516.6 / 6}

# (name, cin, cout, k, stride, pad(t,l,b,r), H_in)   at 256x256 input
SHAPES = [
    ("wnsa3x3@64", 192, 192, 3, 1, (1, 1, 1, 1), 64),
    ("wnsa7x7@64", 192, 192, 7, 1, (3, 3, 3, 3), 64),
    ("rbws_conv2@128", 192, 192, 3, 1, (1, 1, 1, 1), 128),
    ("conv5x5s2@128", 192, 192, 5, 2, (1, 1, 2, 2), 128),
    ("conv5x5s2@32", 192, 192, 5, 2, (1, 1, 2, 2), 32),
    ("rbws3x3s2@64", 192, 192, 3, 2, (1, 1, 1, 1), 64),
    ("qkv1x1@64", 192, 576, 1, 1, (0, 0, 0, 0), 64),
    ("proj1x1@64", 192, 192, 1, 1, (0, 0, 0, 0), 64),
    ("c1x1@128", 192, 192, 1, 1, (0, 0, 0, 0), 128),
    ("rbneck3x3_96@64", 96, 96, 3, 1, (1, 1, 1, 1), 64),
    ("han3x3_64@256", 64, 64, 3, 1, (1, 1, 1, 1), 256),
    # slice loop / hyper shapes on the 16x16 latent
    ("ru3x3_64@16", 64, 64, 3, 1, (1, 1, 1, 1), 16),
    ("wnsa3x3@16", 192, 192, 3, 1, (1, 1, 1, 1), 16),
    ("wnsa7x7@16", 192, 192, 7, 1, (3, 3, 3, 3), 16),
    ("cc3x3_224_128@16", 224, 128, 3, 1, (1, 1, 1, 1), 16),
    ("cc3x3_128_48@16", 128, 48, 3, 1, (1, 1, 1, 1), 16),
    ("cc3x3_336_224@16", 336, 224, 3, 1, (1, 1, 1, 1), 16),
    ("ru1x1_128_64@16", 128, 64, 1, 1, (0, 0, 0, 0), 16),
    ("ru1x1_64_128@16", 64, 128, 1, 1, (0, 0, 0, 0), 16),
    ("lin512_128@16", 512, 128, 1, 1, (0, 0, 0, 0), 16),
    ("lin128_512@16", 128, 512, 1, 1, (0, 0, 0, 0), 16),
    ("in1x1_320_128@16", 320, 128, 1, 1, (0, 0, 0, 0), 16),
    ("proj1x1@64", 192, 192, 1, 1, (0, 0, 0, 0), 64),
    ("gdn1x1@128", 192, 192, 1, 1, (0, 0, 0, 0), 128),
    ("cc3x3_128_32@16", 128, 32, 3, 1, (1, 1, 1, 1), 16),
    ("cc3x3_224_32@16", 224, 32, 3, 1, (1, 1, 1, 1), 16),
    ("cc1x1_128_32@16", 128, 32, 1, 1, (0, 0, 0, 0), 16),
    ("qkv1x1@16", 192, 576, 1, 1, (0, 0, 0, 0), 16),
    ("gdn1x1@32", 192, 192, 1, 1, (0, 0, 0, 0), 32),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated shape names")
    ap.add_argument("--auto-only", action="store_true")
    ap.add_argument("--gdn", default="", choices=["", "gdn", "gdn_r1", "igdn"],
                    help="1x1 shapes through Fn.gdn (x^2 prologue, GDN epilogue; gdn_r1: + residual)")
    args = ap.parse_args()
    import lic_amd.functional as Fn
    from lic_amd.layers import Conv2d
    dt = torch.float16 if args.dtype == "fp16" else torch.float32
    Fn.set_split_mode(Fn.SPLIT_MODES.get(args.dtype, 0))   # fp32 activations, 16-bit split products
    dev = "cuda"
    st = torch.cuda.current_stream()
    for name, ci, co, k, s, pad, H in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        m = Conv2d(ci, co, k, s, 0).to(dev)
        x = Fn.Act(torch.randn(args.batch, H, H, ci, device=dev).to(dt))
        pk = m.packed(dt, pad)
        if args.gdn:
            if k != 1 or ci != co:
                continue
            from lic_amd.layers.gdn import GDN
            g = GDN(ci, inverse=args.gdn == "igdn").to(dev)
            pk = g.packed(dt)
            r1 = Fn.Act(torch.randn(args.batch, H, H, ci, device=dev).to(dt)) if args.gdn == "gdn_r1" else None
            from lic_amd._ffi import EPI_GDN_RSQRT, EPI_GDN_SQRT
            mode = EPI_GDN_SQRT if args.gdn == "igdn" else EPI_GDN_RSQRT
            Fn_conv = lambda x_, pk_, out_, **kw_: Fn.gdn(x_, pk_, mode, out_, r1)
        Ho, Wo = Fn.conv_out_hw(H, H, pk)
        out = Fn.Act.empty(args.batch, Ho, Wo, co, dt, dev)
        flops = 2.0 * args.batch * Ho * Wo * co * ci * k * k
        conv_fn = Fn_conv if args.gdn else Fn.conv
        res = {}
        for variant in (("auto",) * 3 if args.auto_only else ("auto", "generic", "auto", "generic")):
            kw = dict(force_generic=(variant == "generic"))
            for _ in range(2):
                conv_fn(x, pk, out, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                conv_fn(x, pk, out, **kw)
            e1.record(st)
            e1.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / args.iters
            res.setdefault(variant, []).append(t)
        if args.gdn:
            name = f"{args.gdn}:{name}"
        line = f"{name:18s} {flops / 1e9:8.1f} GFLOP"
        for v, ts in res.items():
            t = min(ts)
            tf = flops / t / 1e12
            line += f" | {v:7s} {t * 1e6:8.1f} us {tf:7.1f} TF/s ({100 * tf / PEAK[args.dtype]:5.1f}%)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
