#!/usr/bin/env python3
"""Run each slice-loop layer (net_ga, B=32 fp16, 16x16 latents) on the current stream
while other kernels run concurrently on a second stream, and report any output that
is not bit-identical to the op's isolated result.  A kernel whose result depends on
what shares its CUs (a cross-wave LDS race that only shows when waves are slowed
unevenly, an uninitialised read) shows up here and not in op_determinism.py.
usage: python tools/concurrency_stress.py [--reps 10] [--noise conv|same|mix]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--noise", default="mix", choices=["conv", "same", "mix", "none", "wba", "syntax"])
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    from lic_amd.functional import Act
    from lic_amd import functional as Fn
    from lic_amd._ffi import ACT_GELU
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B = args.batch
    net = net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision=args.precision).to("cuda")
    dt = net.dtype
    g = torch.Generator(device="cuda").manual_seed(3)
    X = lambda c, h=16: Act((torch.randn(B, h, h, c, device="cuda", generator=g) * 0.5).to(dt))
    sw = net.atten_scale[0][0]
    blk = sw.non_local_block.block_1
    x192, x128, x224 = X(192), X(128), X(224)
    cs = net.cc_scale_transforms[0]
    msa = blk.msa
    qkv128 = msa.embedding_layer.run(x128)
    tab_fixed = msa.relative_position_params.detach().contiguous().clone()

    def attn(q, tab, valu=False):
        return Fn.win_attn(q, msa.input_dim, msa.n_heads, 8, 0, tab, 1, 225, 0, True, float(msa.scale),
                           force_valu=valu)

    def attn_sync(q, tab):
        y = attn(q, tab)
        torch.cuda.current_stream().synchronize()
        return y
    ops = {
        "swatten_192": lambda: sw.run(x192).t,
        "in_conv_1x1_192_128": lambda: sw.in_conv.run(x192).t,
        "layernorm_128": lambda: Fn.layernorm(x128, blk.ln1.weight, blk.ln1.bias, blk.ln1.eps).t,
        "wmsa_qkv": lambda: blk.msa.embedding_layer.run(x128).t,
        "wmsa_W": lambda: blk.msa.run(x128, residual=x128).t,
        "wmsa_SW": lambda: sw.non_local_block.block_2.msa.run(x128, residual=x128).t,
        "mlp0_gelu": lambda: blk.mlp[0].run(x128, act=ACT_GELU).t,
        "block_1": lambda: blk.run(x128).t,
        "swinblock": lambda: sw.non_local_block.run(x128).t,
        "conv_a_unit": lambda: sw.conv_a[0].run(x128).t,
        "cc_conv3x3_192_224": lambda: cs[0].run(x192, act=ACT_GELU).t,
        "cc_conv3x3_224_128": lambda: cs[2].run(x224, act=ACT_GELU).t,
        "cc_conv3x3_128_48": lambda: cs[4].run(x128).t,
        "hs_conv3x3_192_192": lambda: net.h_mean_s[0].run(x192, act=ACT_GELU).t,
        "wmsa_attn_cached_table": lambda: attn(qkv128, tab_fixed).t,
        "wmsa_attn_temp_table": lambda: attn(qkv128, msa.relative_position_params.contiguous()).t,
        "wmsa_attn_valu_cached": lambda: attn(qkv128, tab_fixed, valu=True).t,
        "wmsa_attn_cached_sync": lambda: attn_sync(qkv128, tab_fixed).t,
    }
    if args.only:
        ops = {k: v for k, v in ops.items() if k in args.only.split(",")}
    # noise: a 64x64 WNSA conv, attention and the syntax head on another stream
    wn = net.a_model.transform[8]
    y64 = Act((torch.randn(B, 64, 64, 192, device="cuda", generator=g) * 0.5).to(dt))
    z3 = X(320)
    xs192 = X(192)

    def noise(name):
        if args.noise in ("conv", "mix"):
            for _ in range(3):
                wn.conv_b[4].run(y64)
        if args.noise in ("same", "mix"):
            for _ in range(4):
                ops[name]() if name != "swatten_192" else sw.run(xs192)
        if args.noise == "wba":
            for _ in range(4):
                wn.conv_b[0].run(y64)
        if args.noise == "syntax":
            for _ in range(6):
                net.syntax_model.run(z3.ch(0, 16))
        if args.noise == "mix":
            for _ in range(3):
                net.syntax_model.run(z3.ch(0, 16))
                wn.conv_b[0].run(y64)

    side = torch.cuda.Stream()
    rep = {}
    for name, fn in ops.items():
        ref = fn().clone()
        torch.cuda.synchronize()
        nbad, worst, ndiff = 0, 0.0, 0
        for r in range(args.reps):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                noise(name)
            outs = [fn() for _ in range(3)]
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            for y in outs:
                a = y.view(torch.int16) if y.dtype == torch.float16 else y.view(torch.int32)
                b = ref.view(torch.int16) if ref.dtype == torch.float16 else ref.view(torch.int32)
                if not torch.equal(a, b):
                    nbad += 1
                    ndiff = max(ndiff, int((a != b).sum()))
                    worst = max(worst, float((y.float() - ref.float()).abs().max()))
        rep[name] = {"bad": nbad, "of": 3 * args.reps, "max_n_diff": ndiff, "max_abs": worst}
        print(name, rep[name], flush=True)
    print(json.dumps({"noise": args.noise, "batch": B, "precision": args.precision, "ops": rep}), flush=True)


if __name__ == "__main__":
    main()
