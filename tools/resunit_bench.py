#!/usr/bin/env python3
"""Times one compressai ResidualUnit(128) at the slice loop's 16x16 latent (B=32, fp32x6):
the fused launch (csrc/resunit_split.hip) against the three per-conv launches, HIP events on
the launch stream.  usage: python tools/resunit_bench.py [--batch 32] [--hw 16] [--iters 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--hw", type=int, default=16)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import lic_amd.functional as Fn
    from lic_amd.layers.compressai import _ResidualUnit
    torch.manual_seed(0)
    m = _ResidualUnit(128).cuda()
    X = Fn.Act(torch.randn(args.batch, args.hw, args.hw, 128, device="cuda"))
    packs = [m.conv[i].packed(torch.float32) for i in (0, 2, 4)]
    st = torch.cuda.current_stream()
    flops = 2.0 * args.batch * args.hw * args.hw * (128 * 64 + 64 * 64 * 9 + 64 * 128)

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    with Fn.split_f32(2):
        out = Fn.Act.empty(X.B, X.H, X.W, 128, torch.float32, "cuda")

        def unfused():
            t = m.conv[0].run(X, act=1)
            t = m.conv[2].run(t, act=1)
            m.conv[4].run(t, out, r1=X, act=1, epi=6)

        for name, fn in (("fused", lambda: Fn.resunit(X, *packs, out=out)), ("3 launches", unfused)) * 2:
            us = timed(fn)
            print(f"resunit N=128 B={args.batch} {args.hw}x{args.hw} {name:>11}: {us:8.2f} us "
                  f"({flops / us / 1e6:6.1f} TF/s fp32-equivalent)", flush=True)


if __name__ == "__main__":
    main()
