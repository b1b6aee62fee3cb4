"""Time lic_win_attn_fwd (MFMA vs VALU kernel) on the bench's attention shapes."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402


def time_it(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    shapes = [(192, 8, 8, 4, 64, 64, 1, False), (192, 8, 8, 2, 64, 64, 1, False), (128, 8, 8, 4, 16, 16, 2, True)]
    for dtype in (torch.float16, torch.float32):
        for C, heads, ws, shift, H, W, mk, sa in shapes:
            qkv = Fn.Act(torch.randn(B, H, W, 3 * C, device="cuda").to(dtype))
            tab = torch.randn((2 * ws - 1) ** 2, heads, device="cuda")
            out = Fn.Act.empty(B, H, W, C, dtype, qkv.t.device)
            res = {}
            for fv in (False, True):
                res[fv] = time_it(lambda: Fn.win_attn(qkv, C, heads, ws, shift, tab, heads, 1, mk, sa, 0.2, out=out,
                                                      force_valu=fv))
            # algorithmic flops: 2 GEMMs of N x N x d per (window, head)
            nwin = B * (H // ws) * (W // ws)
            fl = nwin * heads * 2 * 2 * (ws * ws) ** 2 * (C // heads)
            byt = B * H * W * 4 * C * qkv.t.element_size()
            print(f"{str(dtype):14s} C={C} H={H} ws={ws} mfma {res[False]*1e3:8.1f} us  valu {res[True]*1e3:8.1f} us"
                  f"  mfma {fl / res[False] / 1e9:7.1f} TF/s {byt / res[False] / 1e6:7.1f} GB/s")


if __name__ == "__main__":
    main()
