"""Host-side check (CPU) of the fused 4-phase transposed-conv packing
(functional.pack_conv_transpose2d_fused + out_shuffle=3 contract of include/lic.h)
against F.conv_transpose2d, by emulating the tap-form launch in float64."""
import pytest
import torch
import torch.nn.functional as F

import lic_amd.functional as Fn


def _fused_emulate(x_nhwc, pk, Ho, Wo):
    B, H, W, C = x_nhwc.shape
    mi, mj = Ho // 2, Wo // 2
    acc = torch.zeros((B, mi, mj, pk.co), dtype=torch.float64)
    ii, jj = torch.arange(mi)[:, None], torch.arange(mj)[None, :]
    for t in range(len(pk.dy)):
        iy, ix = ii + pk.dy[t], jj + pk.dx[t]
        ok = (iy >= 0) & (iy < H) & (ix >= 0) & (ix < W)
        g = x_nhwc.double()[:, iy.clamp(0, H - 1).expand(mi, mj), ix.clamp(0, W - 1).expand(mi, mj), :]
        acc += torch.einsum("bijc,nc->bijn", g * ok[None, :, :, None], pk.w[:pk.co, t, :C].double())
    if pk.bias is not None:
        acc += pk.bias.double()
    q = pk.co // 4
    out = torch.zeros((B, Ho, Wo, q), dtype=torch.float64)
    for ph in range(4):
        out[:, ph >> 1::2, ph & 1::2, :] = acc[..., ph * q:(ph + 1) * q]
    return out


@pytest.mark.parametrize("ci,co,k,p,op,prepad,H", [
    (192, 16, 5, 3, 1, (1, 1), 6),    # s_model output layer (ZeroPad2d((1,0,1,0)) + ConvT(5,2,3,1))
    (8, 4, 3, 1, 1, (0, 0), 5),       # plain ConvT 3x3 s2
    (16, 8, 4, 1, 0, (0, 0), 4),      # even kernel
    (8, 3, 5, 2, 1, (0, 0), 3),
])
def test_fused_convT_pack_matches_torch(ci, co, k, p, op, prepad, H):
    torch.manual_seed(ci + co + k)
    w = torch.randn(ci, co, k, k)
    b = torch.randn(co)
    x = torch.randn(2, ci, H, H + 1)
    pk = Fn.pack_conv_transpose2d_fused(w, b, 2, p, torch.float32, prepad)
    assert pk is not None
    xp = F.pad(x, (prepad[1], 0, prepad[0], 0))
    ref = F.conv_transpose2d(xp.double(), w.double(), b.double(), 2, p, op)
    Ho, Wo = ref.shape[2], ref.shape[3]
    if Ho % 2 or Wo % 2:
        pytest.skip("fused form needs an even output map")
    out = _fused_emulate(x.permute(0, 2, 3, 1).contiguous(), pk, Ho, Wo)
    torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, rtol=1e-9, atol=1e-9)
