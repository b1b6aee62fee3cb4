#!/usr/bin/env python3
"""Accuracy of the fp32 convolution modes against a float64 reference: exact fp32-input MFMA
(mfma_mode 0), fp32x3 (1) and fp32x6 (2) on one layer; max / RMS error over the output scale
and the mean signed error (a rounding bias shows there).
usage: python tools/split_accuracy.py [--k 3] [--cin 192] [--batch 8] [--size 64]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--cin", type=int, default=192)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--positive", action="store_true", help="non-negative inputs (post-ReLU / GDN-like)")
    args = ap.parse_args()
    import lic_amd.functional as Fn
    from lic_amd.layers import Conv2d
    torch.manual_seed(5)
    k, c, B, H = args.k, args.cin, args.batch, args.size
    m = Conv2d(c, c, k, 1, 0).to("cuda")
    x = torch.randn(B, c, H, H) * 0.5
    if args.positive:
        x = x.abs()
    p = k // 2
    ref = F.conv2d(F.pad(x.double(), (p, p, p, p)), m.weight.detach().cpu().double(), m.bias.detach().cpu().double())
    X = Fn.Act.from_nchw(x.to("cuda").contiguous(), torch.float32)
    pk = m.packed(torch.float32, (p, p, p, p))
    scale = ref.abs().max().item()
    rep = {"layer": f"conv{k}x{k} {c}->{c} B={B} {H}^2", "scale": scale}
    for mode in (0, 1, 2):
        with Fn.split_f32(mode):
            got = Fn.conv(X, pk).nchw().cpu().double()
        e = got - ref
        rep[f"mode{mode}"] = {"max_rel": e.abs().max().item() / scale, "rms_rel": e.pow(2).mean().sqrt().item() / scale,
                              "mean_rel": e.mean().item() / scale}
    cpu = F.conv2d(F.pad(x, (p, p, p, p)), m.weight.detach().cpu(), m.bias.detach().cpu()).double() - ref
    rep["torch_cpu_fp32"] = {"max_rel": cpu.abs().max().item() / scale, "rms_rel": cpu.pow(2).mean().sqrt().item() / scale,
                             "mean_rel": cpu.mean().item() / scale}
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
