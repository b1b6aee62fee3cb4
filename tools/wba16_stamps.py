"""Per-phase stamps of a -DW16_STAMP=1 build of the wba16 v3 kernel (csrc/wba16.hip).

build: bash tools/build_variant.sh w16stamp "-DW16_STAMP=1" wba16.hip   (-> tools/native/liblic_w16stamp.so)
usage: LIC_LIB=<that .so> python tools/wba16_stamps.py [B H W shift]
Prints wave 0's mean cycles per workgroup in: prologue, and summed over its windows: qkv GEMM, q|k/V^T
stores, barrier 1, next-x store + load issue, attention, barrier 2; and the kernel time (HIP events).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402
from lic_amd.layers.win_attention import WinBasedAttention  # noqa: E402


def main():
    B, H, W, shift = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (32, 64, 64, 4))]
    m = WinBasedAttention(dim=192, num_heads=8, window_size=8, shift_size=shift).cuda()
    x = Fn.Act.from_nchw(torch.randn(B, 192, H, W, device="cuda") * 0.7, torch.float16)
    att = m.attn
    big = torch.zeros(B + 8, H, W, 192, device="cuda", dtype=torch.float16)
    out = Fn.Act(big[:B])
    args = (8, 8, shift, att.relative_position_bias_table, 8, 1, 1 if shift > 0 else 0, float(att.scale))
    pk = att.qkv.packed(torch.float16)
    for _ in range(5):
        Fn.wba16_qkv_attn(x, pk, *args, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        Fn.wba16_qkv_attn(x, pk, *args, out=out)
    e1.record()
    torch.cuda.synchronize()
    nblk = 256
    raw64 = big[B:].reshape(-1).view(torch.int64)[: nblk * 9].view(nblk, 9).cpu()
    raw = raw64.double()
    sub = torch.stack([raw64[:, 7] & 0xFFFFFFFF, raw64[:, 7] >> 32, raw64[:, 8] & 0xFFFFFFFF, raw64[:, 8] >> 32], 1).double()
    names = ["prologue", "gemm", "store", "barrier1", "next_x", "attention", "barrier2"]
    print(f"wba16 v3 {B}x{H}x{W} shift {shift}: kernel {e0.elapsed_time(e1) * 100:.1f} us; wave 0 cycles per workgroup:")
    tot = raw[:, :7].sum(1)
    for i, n in enumerate(names):
        print(f"  {n:10s} {raw[:, i].mean().item():10.0f}  ({100 * raw[:, i].mean().item() / tot.mean().item():5.1f} %)")
    print(f"  total      {tot.mean().item():10.0f}")
    for i, n in enumerate(["attn: S + bias", "attn: mask", "attn: softmax", "attn: PV"]):
        print(f"    {n:16s} {sub[:, i].mean().item():10.0f}")


if __name__ == "__main__":
    main()
