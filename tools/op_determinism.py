#!/usr/bin/env python3
"""Run each layer of the slice loop (net_ga, B=32 fp16, 16x16 latents) many times on
one fixed input and report any output that is not bit-identical to the first run.
usage: python tools/op_determinism.py [--reps 30] [--batch 32] [--precision fp16]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--big-only", action="store_true")
    ap.add_argument("--wba-stages", action="store_true")
    ap.add_argument("--poison", action="store_true", help="random garbage in freed blocks before every rep")
    ap.add_argument("--steps", action="store_true", help="Win_noShift_Attention intermediates")
    args = ap.parse_args()
    from lic_amd.functional import Act
    from lic_amd._ffi import ACT_GELU
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B = args.batch
    net = net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision=args.precision).to("cuda")
    dt = net.dtype
    g = torch.Generator(device="cuda").manual_seed(3)
    X = lambda c: Act((torch.randn(B, 16, 16, c, device="cuda", generator=g) * 0.5).to(dt))
    sw = net.atten_mean[0][0]
    blk = sw.non_local_block.block_1
    x192, x240, x128 = X(192), X(240), X(128)
    x224 = X(224)
    cm = net.cc_mean_transforms[1]
    from lic_amd import functional as Fn
    wn = net.a_model.transform[8]
    X64 = lambda c: Act((torch.randn(B, 64, 64, c, device="cuda", generator=g) * 0.5).to(dt))
    y64 = X64(192)
    big = {
        "wnsa64_conv3x3_rb": lambda: wn.conv_a[0].conv1.run(y64).t,
        "wnsa64_resblock": lambda: wn.conv_a[0].run(y64).t,
        "wnsa64_conv7x7": lambda: wn.conv_b[7].run(y64).t,
        "wnsa64_conv3x3_b4": lambda: wn.conv_b[4].run(y64).t,
        "wnsa64_conv1x1": lambda: wn.conv_b[1].run(y64).t,
        "wnsa64_wba": lambda: wn.conv_b[0].run(y64).t,
        "wnsa64_full": lambda: wn.run(y64).t,
    }
    wba = wn.conv_b[0]

    def attn_of(q):
        return Fn.win_attn(q, wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                           wba.attn.relative_position_bias_table, wba.num_heads, 1,
                           1 if wba.shift_size > 0 else 0, False, float(wba.attn.scale))

    def wba_chain(sync):
        q = wba.attn.qkv.run(y64)
        if sync:
            torch.cuda.synchronize()
        a = attn_of(q)
        if sync:
            torch.cuda.synchronize()
        return wba.attn.proj.run(a, None, r1=y64).t

    side = torch.cuda.Stream()

    def wba_chain_stream():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            y = wba_chain(False)
        torch.cuda.current_stream().wait_stream(side)
        return y

    def wba_chain_clone():
        # attention on a fresh copy of qkv (fresh allocation, written by a torch copy kernel)
        q = wba.attn.qkv.run(y64)
        from lic_amd.functional import Act as _A
        q2 = _A(q.t.clone())
        return wba.attn.proj.run(attn_of(q2), None, r1=y64).t
    qkv64 = wba.attn.qkv.run(y64)
    att64 = Fn.win_attn(qkv64, wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                        wba.attn.relative_position_bias_table, wba.num_heads, 1, 1 if wba.shift_size > 0 else 0,
                        False, float(wba.attn.scale))
    big.update({
        "wba_qkv": lambda: wba.attn.qkv.run(y64).t,
        "wba_attn": lambda: Fn.win_attn(qkv64, wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                                        wba.attn.relative_position_bias_table, wba.num_heads, 1,
                                        1 if wba.shift_size > 0 else 0, False, float(wba.attn.scale)).t,
        "wba_proj": lambda: wba.attn.proj.run(att64, None, r1=y64).t,
        "wba_chain_sync": lambda: wba_chain(True),
        "wba_chain_stream": lambda: wba_chain_stream(),
        "wba_chain_clone": lambda: wba_chain_clone(),
    })
    cases = dict(big) if args.big_only else {}
    cases.update({} if args.big_only else {
        "swatten_192": lambda: sw.run(x192).t,
        "swatten_240": lambda: net.atten_mean[1][0].run(x240).t,
        "in_conv_1x1_240_128": lambda: net.atten_mean[1][0].in_conv.run(x240).t,
        "layernorm_128": lambda: Fn.layernorm(x128, blk.ln1.weight, blk.ln1.bias, blk.ln1.eps).t,
        "wmsa_W": lambda: blk.msa.run(x128, residual=x128).t,
        "wmsa_SW": lambda: sw.non_local_block.block_2.msa.run(x128, residual=x128).t,
        "block_1": lambda: blk.run(x128).t,
        "swinblock": lambda: sw.non_local_block.run(x128).t,
        "conv_a_unit": lambda: sw.conv_a[0].run(x128).t,
        "cc_conv3x3_240_224": lambda: cm[0].run(x240, act=ACT_GELU).t,
        "cc_conv3x3_224_128": lambda: cm[2].run(x224, act=ACT_GELU).t,
        "cc_conv3x3_128_48": lambda: cm[4].run(x128).t,
        "hs_conv3x3_192_192": lambda: net.h_mean_s[0].run(x192, act=ACT_GELU).t,
    })
    if not args.big_only:
        cases.update(big)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from determinism_probe import poison

    def wnsa_steps():
        """Win_noShift_Attention.run step by step, every intermediate kept."""
        outs = []
        a = y64
        for blk in wn.conv_a:
            a = blk.run(a)
            outs.append(a.t)
        b = y64
        for k in range(9):
            b = wn.conv_b[k].run(b)
            outs.append(b.t)
        outs.append(wn.conv_b[9].run(b, None, gate_a=a, gate_r=y64).t)
        return outs

    if args.wba_stages:
        def stages():
            q = wba.attn.qkv.run(y64)
            a = attn_of(q)
            o = wba.attn.proj.run(a, None, r1=y64)
            torch.cuda.synchronize()
            return [q.t.clone(), a.t.clone(), o.t.clone()]
        ref = stages()
        res = []
        for _ in range(args.reps):
            poison(2048, random=True)
            st = stages()
            nd = [int((u != v).sum()) for u, v in zip(ref, st)]
            info = {}
            if nd[1]:
                ne = ref[1] != st[1]
                idx = ne.nonzero()
                b_, yy, xx, cc = idx.unbind(1)
                info = {"max_abs": float((ref[1].float() - st[1].float()).abs().max()),
                        "images": sorted(set(b_.tolist()))[:8],
                        "windows": sorted(set(((yy // 8) * 8 + xx // 8).tolist()))[:16],
                        "heads": sorted(set((cc // 24).tolist())),
                        "n_pix": int(ne.any(-1).sum()),
                        "ref_vals": ref[1][ne][:4].float().tolist(), "new_vals": st[1][ne][:4].float().tolist()}
            res.append([nd, info])
        # attention re-run on the reference qkv of this process, same buffers
        print(json.dumps({"wba_stage_ndiff[qkv,attn,proj]": res}), flush=True)
        return
    if args.steps:
        ref = [t.clone() for t in wnsa_steps()]
        torch.cuda.synchronize()
        first = []
        for _ in range(args.reps):
            o = wnsa_steps()
            torch.cuda.synchronize()
            bad = [k for k, (u, v) in enumerate(zip(ref, o)) if not torch.equal(u, v)]
            first.append(bad[:4])
        print(json.dumps({"wnsa_steps_first_bad": first}), flush=True)
        return
    rep = {}
    from lic_amd import functional as Fn  # noqa: F811
    for name, fn in cases.items():
        ref = fn().clone()
        torch.cuda.synchronize()
        nbad, worst = 0, 0.0
        for _ in range(args.reps):
            if args.poison:
                poison(2048, random=True)
            y = fn()
            torch.cuda.synchronize()
            if not torch.equal(y.view(torch.int16) if y.dtype == torch.float16 else y, ref.view(torch.int16) if ref.dtype == torch.float16 else ref):
                nbad += 1
                worst = max(worst, float((y.float() - ref.float()).abs().max()))
        rep[name] = {"bad_runs": nbad, "max_abs": worst}
    print(json.dumps({"reps": args.reps, "batch": B, "precision": args.precision, "ops": rep}), flush=True)


if __name__ == "__main__":
    main()
