#!/usr/bin/env python3
"""Micro-benchmark of the fp32x6 WinBasedAttention core at 64x64, batch 32: the fused qkv + window
attention launch (lic_wba_qkv_attn_fwd) against the unfused qkv 1x1 + lic_win_attn_fwd pair, and the
whole WinBasedAttention.run (incl. proj + shortcut) both ways (HIP events on the launch stream).
usage: python tools/wba_bench.py [--batch 32] [--iters 30] [--shift 4]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shift", type=int, default=4)
    args = ap.parse_args()
    import lic_amd.functional as Fn
    from lic_amd.functional import Act
    from lic_amd.layers import win_attention as WA
    dev = "cuda"
    torch.manual_seed(0)
    m = WA.WinBasedAttention(dim=192, num_heads=8, window_size=8, shift_size=args.shift).to(dev)
    x = Act(torch.randn(args.batch, 64, 64, 192, device=dev))
    mk, sc, tab = (1 if args.shift else 0), float(m.attn.scale), m.attn.relative_position_bias_table
    st = torch.cuda.current_stream()

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

    pk = m.attn.qkv.packed(torch.float32)
    qkv = Act.empty(args.batch, 64, 64, 576, torch.float32, dev)
    att = Act.empty(args.batch, 64, 64, 192, torch.float32, dev)

    def unfused():
        Fn.conv(x, pk, qkv)
        Fn.win_attn(qkv, 192, 8, 8, args.shift, tab, 8, 1, mk, False, sc, out=att)

    def fused():
        Fn.wba_qkv_attn(x, pk, 8, 8, args.shift, tab, 8, 1, mk, sc, out=att)

    def block(f):
        def run():
            WA._FUSED = f
            m.run(x)
        return run

    with Fn.split_f32(2):
        for _ in range(2):
            tu, tf = timed(unfused), timed(fused)
            bu, bf = timed(block(False)), timed(block(True))
            print(f"B={args.batch} 64x64 shift {args.shift}: qkv+attention unfused {tu:8.1f} us  fused {tf:8.1f} us | "
                  f"WinBasedAttention.run unfused {bu:8.1f} us  fused {bf:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
