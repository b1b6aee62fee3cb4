#!/usr/bin/env python3
"""Micro-benchmark of lic_conv2d_wgrad (bf16) on config-5 shapes (batch 8, 256x256 input).

Times the whole call (partial kernel + split reduce) with HIP events on the launch stream and
prints TFLOP/s against the dense bf16 MFMA peak.  LIC_WGRAD_TR=0 in the environment selects the
generic split-K kernel instead of the tiled transpose-read one (for A/B runs in two processes).
usage: python tools/wgrad_bench.py [--batch 8] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = 2516.6  # TFLOP/s, dense bf16

# (name, ci, co, k, stride, pad (t, l, b, r), H_in of x)
SHAPES = [
    ("3x3_128@128", 128, 128, 3, 1, (1, 1, 1, 1), 128),
    ("3x3_192@64", 192, 192, 3, 1, (1, 1, 1, 1), 64),
    ("3x3_192@32", 192, 192, 3, 1, (1, 1, 1, 1), 32),
    ("3x3_192@16", 192, 192, 3, 1, (1, 1, 1, 1), 16),
    ("3x3s2_128@256", 128, 128, 3, 2, (1, 1, 1, 1), 256),
    ("5x5s2_192@128", 192, 192, 5, 2, (1, 1, 2, 2), 128),
    ("5x5_192@32", 192, 192, 5, 1, (2, 2, 2, 2), 32),
    ("1x1_192@64", 192, 192, 1, 1, (0, 0, 0, 0), 64),
    ("1x1_192@128", 192, 192, 1, 1, (0, 0, 0, 0), 128),
    ("7x7_256@32", 256, 256, 7, 1, (3, 3, 3, 3), 32),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from lic_amd import autograd as AG
    B = args.batch
    tag = "generic" if os.environ.get("LIC_WGRAD_TR", "1") == "0" else "tiled"
    for name, ci, co, k, s, pad, H in SHAPES:
        pt, pl, pb, pr = pad
        Ho = (H + pt + pb - k) // s + 1
        x = torch.randn(B, H, H, ci, device="cuda").to(torch.bfloat16)
        dz = torch.randn(B, Ho, Ho, co, device="cuda").to(torch.bfloat16)
        dw = torch.empty((co, ci, k, k), dtype=torch.float32, device="cuda")
        tdy, tdx = AG._taps(k, k, pt, pl)

        def run():
            AG.wgrad(x, dz, tdy, tdx, stride=s, dw=dw, strides=(ci * k * k, k * k, 1), co_out=co, ci_out=ci)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        flops = 2.0 * B * Ho * Ho * co * ci * k * k
        tf = flops / us * 1e-6
        print(f"{tag:8s} {name:16s} {us:9.1f} us  {tf:7.1f} TFLOP/s  {tf / PEAK:6.3f} of peak", flush=True)


if __name__ == "__main__":
    main()
