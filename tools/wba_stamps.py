"""Per-phase stamps of a -DW6_STAMP=1 build of the fp32x6 fused qkv + window-attention kernel
(csrc/wba_split.hip, wba_qkv_attn_kernel<false>).

build: bash tools/build_variant.sh w6stamp "-DW6_STAMP=1" wba_split.hip   (-> tools/native/liblic_w6stamp.so)
usage: LIC_LIB=<that .so> python tools/wba_stamps.py [B H W shift]
Prints wave 0's mean cycles per workgroup, summed over its windows: phase A (x split into planes),
the barrier before each group's GEMM, the qkv GEMM (+ its LDS stores), the barrier after it (+ table,
next-x loads), S = K Q^T (incl. the K / Q splits), bias + mask + softmax, PV (incl. the V / P splits and
the output stores), the end-of-window barrier; and the kernel time (HIP events).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402
from lic_amd.layers.win_attention import WinBasedAttention  # noqa: E402


def main():
    B, H, W, shift = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (32, 64, 64, 4))]
    Fn.set_split_mode(Fn.SPLIT_MODES["fp32x6"])
    m = WinBasedAttention(dim=192, num_heads=8, window_size=8, shift_size=shift).cuda()
    x = Fn.Act.from_nchw(torch.randn(B, 192, H, W, device="cuda") * 0.7, torch.float32)
    att = m.attn
    big = torch.zeros(B + 4, H, W, 192, device="cuda", dtype=torch.float32)
    out = Fn.Act(big[:B])
    args = (8, 8, shift, att.relative_position_bias_table, 8, 1, 1 if shift > 0 else 0, float(att.scale))
    pk = att.qkv.packed(torch.float32)
    for _ in range(5):
        Fn.wba_qkv_attn(x, pk, *args, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        Fn.wba_qkv_attn(x, pk, *args, out=out)
    e1.record()
    torch.cuda.synchronize()
    nblk = 256
    raw = big[B:].reshape(-1).view(torch.int64)[: nblk * 8].view(nblk, 8).cpu().double()
    names = ["A split", "barrier0", "gemm", "barrier1", "S", "softmax", "PV", "barrier_end"]
    print(f"wba fp32x6 {B}x{H}x{W} shift {shift}: kernel {e0.elapsed_time(e1) * 100:.1f} us; wave 0 cycles per workgroup:")
    tot = raw.sum(1)
    for i, n in enumerate(names):
        print(f"  {n:12s} {raw[:, i].mean().item():10.0f}  ({100 * raw[:, i].mean().item() / tot.mean().item():5.1f} %)")
    print(f"  total        {tot.mean().item():10.0f}")


if __name__ == "__main__":
    main()
