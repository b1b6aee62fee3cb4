#!/usr/bin/env python3
"""End-to-end accuracy of the fp32 modes (exact 'fp32', 'fp32x3', 'fp32x6') against the oracle
run in float64: RMS / max abs error of the latent y (z3), the hyper means / scales and the
slice-loop means, and the symbol flips against the float64 symbols and the fp32 oracle's.
usage: python tools/split_net_accuracy.py [--arch net_ga] [--batch 1]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="net_ga")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    from oracle import ref_cpu as R
    from test_gpu_split import _net
    B = args.batch
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(123 + B)) * 2 - 1
    net0 = _net(args.arch, B, seed=args.seed, precision="fp32")
    P = {k: v.detach().float() for k, v in net0.state_dict().items()}
    ref64 = R.net_forward(x.double(), {k: v.double() for k, v in P.items()}, arch=args.arch)
    ref32 = R.net_forward(x, P, arch=args.arch)
    keys = ("z3", "latent_means", "latent_scales", "means")
    rep = {"arch": args.arch, "batch": B}

    def stats(d):
        out = {}
        for k in keys:
            e = (d[k].double().cpu() - ref64[k])
            out[k] = [float(e.pow(2).mean().sqrt()), float(e.abs().max())]
        out["flips_vs_f64"] = int((d["symbols"].cpu() != ref64["symbols"]).sum())
        out["flips_vs_f32_oracle"] = int((d["symbols"].cpu() != ref32["symbols"]).sum())
        return out
    rep["oracle_fp32"] = stats(ref32)
    for prec in ("fp32", "fp32x3", "fp32x6"):
        net = _net(args.arch, B, seed=args.seed, precision=prec)
        net.load_state_dict(net0.state_dict())
        net = net.to("cuda")
        net(x.to("cuda"), "test", return_intermediates=True)
        torch.cuda.synchronize()
        last = dict(net.last)
        rep[prec] = stats(last)
        del net
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
