#!/usr/bin/env python3
"""A/B of the fp32x6 weights-direct conv configurations (env switches such as LIC_WD_W4 are read
once per process, so each side of an A/B is its own process).

Times the a_model's big-map fp32x6 convs with HIP events on the launch stream and saves their
outputs; with --ref FILE it also checks that this run's outputs are bitwise equal to FILE's (a
retiling keeps every output element's chunk / tap / product sequence, so A and B must agree bit
for bit).
usage: python tools/wd_ab.py [--small] --save /tmp/a.pt; LIC_LIB=<variant .so> python tools/wd_ab.py [--small] --ref /tmp/a.pt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, cin, cout, k, stride, pad(t,l,b,r), H_in)
SHAPES = [
    ("wnsa3x3@64", 192, 192, 3, 1, (1, 1, 1, 1), 64),
    ("wnsa7x7@64", 192, 192, 7, 1, (3, 3, 3, 3), 64),
    ("rbws_conv2@128", 192, 192, 3, 1, (1, 1, 1, 1), 128),
    ("conv5x5s2@128", 192, 192, 5, 2, (1, 1, 2, 2), 128),
    ("rbws3x3s2@64", 192, 192, 3, 2, (1, 1, 1, 1), 64),
]
# --small: the latent-map launches (8 x 8-pixel tiles, tap groups)
SMALL = [
    ("wnsa3x3@16", 192, 192, 3, 1, (1, 1, 1, 1), 16),
    ("cc3x3_224_128@16", 224, 128, 3, 1, (1, 1, 1, 1), 16),
    ("cc3x3_128_48@16", 128, 48, 3, 1, (1, 1, 1, 1), 16),
    ("ru3x3_64@16", 64, 64, 3, 1, (1, 1, 1, 1), 16),
    ("wnsa7x7@16", 192, 192, 7, 1, (3, 3, 3, 3), 16),
    ("lin128_512@16", 128, 512, 1, 1, (0, 0, 0, 0), 16),
]
PEAK6 = 2516.6 / 6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--save", default="")
    ap.add_argument("--ref", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--small", action="store_true", help="the latent-map shapes instead")
    args = ap.parse_args()
    import lic_amd.functional as Fn
    from lic_amd.layers import Conv2d
    Fn.set_split_mode(Fn.SPLIT_MODES["fp32x6"])
    dev = "cuda"
    st = torch.cuda.current_stream()
    ref = torch.load(args.ref, weights_only=True) if args.ref else {}
    outs, bad = {}, 0
    for name, ci, co, k, s, pad, H in (SMALL if args.small else SHAPES):
        if args.only and name not in args.only.split(","):
            continue
        torch.manual_seed(0)
        m = Conv2d(ci, co, k, s, 0).to(dev)
        x = Fn.Act(torch.randn(args.batch, H, H, ci, device=dev))
        pk = m.packed(torch.float32, pad)
        Ho, Wo = Fn.conv_out_hw(H, H, pk)
        out = Fn.Act.empty(args.batch, Ho, Wo, co, torch.float32, dev)
        for _ in range(2):
            Fn.conv(x, pk, out)
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                Fn.conv(x, pk, out)
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3 / args.iters)
        t = min(ts)
        flops = 2.0 * args.batch * Ho * Wo * co * ci * k * k
        o = out.t.detach().clone().cpu()
        outs[name] = o
        line = f"{name:16s} {t * 1e6:8.1f} us  {flops / t / 1e12:6.1f} TF/s  {flops / t / 1e12 / PEAK6:.3f} of peak/6"
        if name in ref:
            eq = torch.equal(ref[name], o)
            bad += not eq
            line += f"  bitwise vs ref: {'EQUAL' if eq else 'DIFF max %.3e' % (ref[name] - o).abs().max().item()}"
        print(line, flush=True)
    if args.save:
        torch.save(outs, args.save)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
