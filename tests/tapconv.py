"""CPU emulation of the lic_conv2d_fwd tap-form contract (include/lic.h) — used to
test the host-side weight packing / transposed-conv phase decomposition without a GPU."""
import torch

import lic_amd.functional as Fn


def tap_conv(x_nhwc: torch.Tensor, pk: Fn.ConvPack, out: torch.Tensor, *, stride=None, shuffle=False):
    B, H, W, C = x_nhwc.shape
    if pk.phase is None:
        Ho, Wo = Fn.conv_out_hw(H, W, pk)
        mi, mj, oy0, ox0, osy, osx, isy, isx = Ho, Wo, 0, 0, 1, 1, pk.stride, pk.stride
    else:
        ry, rx, s, _, _ = pk.phase
        Ho, Wo = out.shape[1], out.shape[2]
        mi, mj = -(-(Ho - ry) // s), -(-(Wo - rx) // s)
        oy0, ox0, osy, osx, isy, isx = ry, rx, s, s, 1, 1
    w = pk.w.float()
    acc = torch.zeros((B, mi, mj, pk.co), dtype=torch.float64)
    ii = torch.arange(mi)[:, None]
    jj = torch.arange(mj)[None, :]
    xd = x_nhwc.double()
    for t in range(len(pk.dy)):
        iy = ii * isy + pk.dy[t]
        ix = jj * isx + pk.dx[t]
        ok = (iy >= 0) & (iy < H) & (ix >= 0) & (ix < W)
        iyc, ixc = iy.clamp(0, H - 1).expand(mi, mj), ix.clamp(0, W - 1).expand(mi, mj)
        g = xd[:, iyc, ixc, :] * ok[None, :, :, None]
        if pk.groups == 1:
            acc += torch.einsum("bijc,nc->bijn", g, w[:pk.co, t, :C].double())
        else:
            acc += g * w[:pk.co, t, 0].double()
    if pk.bias is not None:
        acc += pk.bias.double()
    acc = acc.float()
    if shuffle:
        Bq, Hq, Wq, Cq = acc.shape
        acc = acc.view(Bq, Hq, Wq, Cq // 4, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(Bq, Hq * 2, Wq * 2, Cq // 4)
        out[...] = acc
        return out
    out[:, oy0::osy, ox0::osx, :][:, :mi, :mj] = acc
    return out
