"""Read the per-block phase stamps of a -DHALO_STAMP=1 build of conv_halo.hip.

usage: LIC_LIB=ab/liblic_stamp.so python tools/halo_stamps.py [shape]
Prints the mean cycles per block in: prologue (first loads), issue, compute,
wait+barrier, epilogue, and the block timeline (s_memrealtime, 100 MHz).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402
from lic_amd.layers import Conv2d  # noqa: E402

SHAPES = {"wnsa3x3": (192, 192, 3, 1, (1, 1, 1, 1), 64), "wnsa7x7": (192, 192, 7, 1, (3, 3, 3, 3), 64),
          "rbws_conv2": (192, 192, 3, 1, (1, 1, 1, 1), 128)}
name = sys.argv[1] if len(sys.argv) > 1 else "wnsa3x3"
ci, co, k, s, pad, H = SHAPES[name]
B = 32
m = Conv2d(ci, co, k, s, 0).cuda()
x = Fn.Act(torch.randn(B, H, H, ci, device="cuda").half())
pk = m.packed(torch.float16, pad)
Ho, Wo = Fn.conv_out_hw(H, H, pk)
big = torch.zeros(B + 4, Ho, Wo, co, device='cuda', dtype=torch.float16)
out = Fn.Act(big[:B])
for _ in range(3):
    Fn.conv(x, pk, out)
torch.cuda.synchronize()
nblk = B * ((Ho + 15) // 16) * ((Wo + 15) // 16)
raw = big[B:].reshape(-1).view(torch.int64)[: nblk * 8].view(nblk, 8).cpu()
names = ["prologue", "issue", "compute", "wait+bar", "epi+rest"]
tot = raw[:, :5].sum(1).double()
for i, n in enumerate(names):
    v = raw[:, i].double()
    print(f"{n:10s} mean {v.mean():10.0f} cyc  ({100 * v.mean() / tot.mean():5.1f}%)  min {v.min():8.0f} max {v.max():8.0f}")
rt0 = raw[:, 5].min()
st, en = (raw[:, 5] - rt0).double() / 100, (raw[:, 6] - rt0).double() / 100  # us
print(f"blocks {nblk}: block duration mean {(en - st).mean():.2f} us, kernel span {en.max():.2f} us")
order = st.argsort()
print("start-time quantiles (us):", [round(float(st[order[int(q * (nblk - 1))]]), 2) for q in (0, .25, .5, .75, 1)])
