#!/usr/bin/env python3
"""Diagnose the window-attention result that changes when other kernels share the GPU
(tools/concurrency_stress.py: the 16x16 WMSA attention differs from its isolated result
while a 64x64 WBA runs on another stream).  Reports which noise kernel triggers it and
where (image / window / head / token) the outputs differ."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lic_amd.functional import Act
    from lic_amd import functional as Fn
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B = 32
    net = net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision="fp16").to("cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    X = lambda c, h=16: Act((torch.randn(B, h, h, c, device="cuda", generator=g) * 0.5).half())
    msa = net.atten_scale[0][0].non_local_block.block_1.msa
    x128 = X(128)
    qkv = msa.embedding_layer.run(x128)
    tab = msa.relative_position_params.detach().contiguous().clone()
    ztab = torch.zeros_like(tab)

    def attn(q, t):
        return Fn.win_attn(q, 128, 8, 8, 0, t, 1, 225, 0, True, float(msa.scale)).t

    wn = net.a_model.transform[8]
    wba = wn.conv_b[0]
    y64 = Act((torch.randn(B, 64, 64, 192, device="cuda", generator=g) * 0.5).half())
    qkv64 = wba.attn.qkv.run(y64)
    big = lambda: Fn.win_attn(qkv64, wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                              wba.attn.relative_position_bias_table, wba.num_heads, 1,
                              1 if wba.shift_size > 0 else 0, False, float(wba.attn.scale))
    big4 = lambda: Fn.win_attn(Act(qkv64.t[:15]), wba.dim, wba.num_heads, wba.window_size, wba.shift_size,
                               wba.attn.relative_position_bias_table, wba.num_heads, 1,
                               1 if wba.shift_size > 0 else 0, False, float(wba.attn.scale))
    noises = {
        "wba_full": lambda: wba.run(y64),
        "wba_qkv_conv": lambda: wba.attn.qkv.run(y64),
        "attn8_64x64": big,
        "attn4_64x64_B15": big4,
        "attn4_same16": lambda: attn(qkv, tab),
    }
    side = torch.cuda.Stream()
    rep = {}
    for tname, t in (("table", tab), ("zero_table", ztab)):
        ref = attn(qkv, t).clone()
        torch.cuda.synchronize()
        for nname, nf in noises.items():
            bad, worst, where = 0, 0.0, None
            for r in range(10):
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(4):
                        nf()
                outs = [attn(qkv, t) for _ in range(4)]
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                for y in outs:
                    ne = y.view(torch.int16) != ref.view(torch.int16)
                    if ne.any():
                        bad += 1
                        worst = max(worst, float((y.float() - ref.float()).abs().max()))
                        if where is None:
                            idx = ne.nonzero()
                            b_, yy, xx, cc = idx.unbind(1)
                            win = (yy // 8) * 2 + xx // 8
                            tok = (yy % 8) * 8 + xx % 8
                            where = {"n": int(ne.sum()), "images": sorted(set(b_.tolist()))[:12],
                                     "n_images": len(set(b_.tolist())),
                                     "img_win_head": sorted(set(zip(b_.tolist(), win.tolist(), (cc // 16).tolist())))[:12],
                                     "n_img_win_head": len(set(zip(b_.tolist(), win.tolist(), (cc // 16).tolist()))),
                                     "tokens_per_head": int(ne.any(-1).sum()),
                                     "channels": sorted(set((cc % 16).tolist())),
                                     "ref": ref[ne][:6].float().tolist(), "got": y[ne][:6].float().tolist()}
            rep[f"{tname}/{nname}"] = {"bad": bad, "of": 40, "max_abs": worst, "first": where}
            print(f"{tname}/{nname}", json.dumps(rep[f"{tname}/{nname}"]), flush=True)


if __name__ == "__main__":
    main()
