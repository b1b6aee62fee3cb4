"""Per-workgroup phase stamps of a -DC16_STAMP=1 build of conv16 (csrc/conv16.h).

build: bash tools/build_variant.sh c16stamp "-DC16_STAMP=1" conv16_f16.hip
usage: LIC_LIB=tools/native/liblic_c16stamp.so python tools/conv16_stamps.py [shape ...]
Prints the mean cycles per workgroup in: prologue (first stage's loads), compute (the stages' tap
loops incl. issuing the next stage's LDS-DMA), wait (end-of-stage vmcnt + barrier), epilogue; and the
kernel time with HIP events for the same launch.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402
from lic_amd.layers import Conv2d  # noqa: E402

SHAPES = {"wnsa3x3": (192, 192, 3, 1, (1, 1, 1, 1), 64), "wnsa7x7": (192, 192, 7, 1, (3, 3, 3, 3), 64),
          "rbws_conv2": (192, 192, 3, 1, (1, 1, 1, 1), 128), "conv5x5s2": (192, 192, 5, 2, (1, 1, 2, 2), 128)}


def run(name, B=32):
    ci, co, k, s, pad, H = SHAPES[name]
    m = Conv2d(ci, co, k, s, 0).cuda()
    x = Fn.Act(torch.randn(B, H, H, ci, device="cuda").half())
    pk = m.packed(torch.float16, pad)
    Ho, Wo = Fn.conv_out_hw(H, H, pk)
    big = torch.zeros(B + 8, Ho, Wo, co, device="cuda", dtype=torch.float16)
    out = Fn.Act(big[:B])
    for _ in range(3):
        Fn.conv(x, pk, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    Fn.conv(x, pk, out)
    e1.record()
    torch.cuda.synchronize()
    nblk = B * ((Ho + 15) // 16) * ((Wo + 31) // 32)
    raw = big[B:].reshape(-1).view(torch.int64)[: nblk * 8].view(nblk, 8).cpu().double()
    tot = raw[:, 4]
    print(f"{name}: {nblk} workgroups, kernel {e0.elapsed_time(e1) * 1e3:.1f} us; per workgroup (cycles):")
    for i, n in enumerate(["prologue", "compute", "wait+barrier", "epilogue"]):
        v = raw[:, i]
        print(f"  {n:13s} mean {v.mean():9.0f} ({100 * v.mean() / tot.mean():5.1f} %)  min {v.min():9.0f}  max {v.max():9.0f}")
    print(f"  {'total':13s} mean {tot.mean():9.0f}  min {tot.min():9.0f}  max {tot.max():9.0f}")


if __name__ == "__main__":
    for nm in (sys.argv[1:] or ["wnsa3x3", "wnsa7x7", "rbws_conv2", "conv5x5s2"]):
        run(nm)
