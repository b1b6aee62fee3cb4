"""CPU checks of the training path's host-side geometry (no GPU): the dgrad weight
packs of lic_amd.autograd, run through the tap-form emulator of lic_conv2d_fwd
(tests/tapconv.py), against torch's own input gradients."""
import pytest
import torch
import torch.nn.functional as F

import lic_amd.autograd as AG
import lic_amd.functional as Fn
from tests.tapconv import tap_conv


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("ci,co,k,s,pad", [
    (8, 16, 3, 1, (1, 1, 1, 1)), (16, 8, 7, 1, (3, 3, 3, 3)), (8, 8, 1, 1, (0, 0, 0, 0)),
    (8, 16, 3, 2, (1, 1, 1, 1)), (8, 16, 5, 2, (1, 1, 2, 2)), (16, 8, 5, 2, (2, 2, 2, 2)),
])
def test_conv_dgrad_packs(ci, co, k, s, pad):
    g = torch.Generator().manual_seed(ci + co + k)
    H, W = 11, 14
    x = torch.randn(2, ci, H, W, generator=g)
    w = torch.randn(co, ci, k, k, generator=g)
    pt, pl, pb, pr = pad
    y = F.conv2d(F.pad(x, (pl, pr, pt, pb)), w, None, s)
    dz = torch.randn(y.shape, generator=g)
    ref = torch.autograd.grad(F.conv2d(F.pad(x.requires_grad_(True), (pl, pr, pt, pb)), w, None, s), x, dz)[0]
    packs = AG.dgrad_packs(w, s, pad, torch.float32, co)
    out = torch.zeros(2, H, W, ci)
    for pk in packs:
        tap_conv(_nhwc(dz), pk, out)
    torch.testing.assert_close(out, _nhwc(ref), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prepad,p", [((1, 1), 3), ((0, 0), 2)])
def test_conv_transpose_dgrad_pack(prepad, p):
    """dL/dx of ZeroPad2d + ConvTranspose2d(k5, s2, p, op1) = strided conv2d of dz with the same
    weight, tap window shifted by s * prepad (the cropped pad rows)."""
    g = torch.Generator().manual_seed(1)
    ci, co, H, W = 8, 16, 6, 7
    x = torch.randn(2, ci, H, W, generator=g, requires_grad=True)
    w = torch.randn(ci, co, 5, 5, generator=g)
    y = F.conv_transpose2d(F.pad(x, (prepad[1], 0, prepad[0], 0)), w, None, 2, p, 1)
    dz = torch.randn(y.shape, generator=g)
    ref = torch.autograd.grad(y, x, dz)[0]
    pk = Fn.pack_conv2d(w, None, 2, (p - 2 * prepad[0], p - 2 * prepad[1], p, p), torch.float32)
    Ho, Wo = Fn.conv_out_hw(y.shape[2], y.shape[3], pk)
    out = torch.zeros(2, Ho, Wo, ci)
    tap_conv(_nhwc(dz), pk, out)
    torch.testing.assert_close(out[:, :H, :W], _nhwc(ref), rtol=1e-4, atol=1e-4)


def test_pad_channels():
    t = torch.randn(2, 3, 4, 3)
    p = AG._pad_channels(t)
    assert p.shape == (2, 3, 4, 4) and torch.equal(p[..., :3], t) and not p[..., 3].any()
    t16 = t.half()
    assert AG._pad_channels(t16).shape[-1] == 8
