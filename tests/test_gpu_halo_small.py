"""GPU parity of the narrow / small-map halo conv configurations (BN 64 / 32,
8x8-pixel tiles) that the slice loop's 16x16 latents and the 16-channel output
ConvTranspose take, against the generic implicit-GEMM kernel and fp32 torch CPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
DTYPES = [torch.float32, torch.float16, torch.bfloat16]


def _close(out, ref, dtype, tol32=1e-4):
    out, ref = out.float().cpu(), ref.float().cpu()
    if dtype != torch.float32:   # 16-bit activations: fp16 2e-2, bf16 4e-2 of the scale
        tol = 2e-2 if dtype == torch.float16 else 4e-2
        assert (out - ref).abs().max().item() <= tol * (ref.abs().max().item() + 1e-6)
    else:
        torch.testing.assert_close(out, ref, rtol=tol32, atol=tol32)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cin,cout,k,s,pad,B,H", [
    (64, 64, 3, 1, (1, 1, 1, 1), 32, 16),     # slice-loop RB 3x3 -> 8x8 tiles, BN 64
    (224, 128, 3, 1, (1, 1, 1, 1), 16, 16),   # cc transform -> 8x8 tiles, BN 64
    (128, 48, 3, 1, (1, 1, 1, 1), 16, 16),    # copad 64, 48 real channels
    (192, 192, 3, 1, (1, 1, 1, 1), 32, 16),   # 8x8 tiles, 3 channel blocks
    (288, 256, 3, 2, (1, 1, 1, 1), 16, 16),   # stride 2 on an 8x8 output
    (64, 64, 7, 1, (3, 3, 3, 3), 16, 16),     # 49 taps (tap groups) on 8x8 tiles
    (96, 96, 3, 1, (1, 1, 1, 1), 16, 50),     # BN 32, ragged 16x16 tiles
    (192, 64, 3, 1, (1, 1, 1, 1), 16, 64),    # BN 64, 16x16 tiles
])
def test_small_halo_matches_generic_and_cpu(dtype, cin, cout, k, s, pad, B, H):
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    torch.manual_seed(30 + cin + cout)
    m = Conv2d(cin, cout, k, s, 0).to(DEV)
    xc = torch.randn(B, cin, H, H)
    x = Fn.Act.from_nchw(xc.to(DEV), dtype)
    pk = m.packed(dtype, pad)
    a = Fn.conv(x, pk)
    b = Fn.conv(x, pk, force_generic=True)
    _close(a.nchw(), b.nchw(), dtype, tol32=1e-5)
    ref = F.conv2d(F.pad(xc, (pad[1], pad[3], pad[0], pad[2])), m.weight.cpu(), m.bias.cpu(), s)
    _close(a.nchw(), ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("B,H", [(8, 32), (16, 64)])
def test_convT_to_16_channels(dtype, B, H):
    """s_model's last layer: ZeroPad2d((1,0,1,0)) + ConvTranspose2d(192, 16, 5, 2, 3, op=1)
    (phases of 16 real / 32 padded output channels)."""
    from lic_amd.layers import ConvTranspose2d
    torch.manual_seed(31)
    m = ConvTranspose2d(192, 16, 5, 2, 3, output_padding=1).to(DEV)
    x = torch.randn(B, 192, H, H)
    import lic_amd.functional as Fn
    out = m.run(Fn.Act.from_nchw(x.to(DEV), dtype), prepad=(1, 1)).nchw()
    ref = F.conv_transpose2d(F.pad(x, (1, 0, 1, 0)), m.weight.cpu(), m.bias.cpu(), 2, 3, 1)
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_small_halo_fused_epilogues(dtype):
    """Residual, gate and GDN epilogues through the 8x8-tile config."""
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    from lic_amd._ffi import EPI_GATE, EPI_GDN_DIV, ACT_GELU
    torch.manual_seed(32)
    B, C, H = 32, 64, 16
    m = Conv2d(C, C, 3, 1, 1).to(DEV)
    xc = torch.randn(B, C, H, H)
    rc, gc, r2c = torch.randn(B, C, H, H), torch.randn(B, C, H, H), torch.randn(B, C, H, H)
    act = lambda t: Fn.Act.from_nchw(t.to(DEV), dtype)
    x, r, g, r2 = act(xc), act(rc), act(gc), act(r2c)
    pk = m.packed(dtype)
    base = F.conv2d(xc.to(dtype).float(), m.weight.cpu(), m.bias.cpu(), 1, 1)
    out = Fn.conv(x, pk, act=ACT_GELU, r1=r)
    _close(out.nchw(), F.gelu(base) + rc.to(dtype).float(), dtype)
    out = Fn.conv(x, pk, epi=EPI_GATE, r1=r, g=g, r2=r2)
    ref = gc.to(dtype).float() * torch.sigmoid(base + rc.to(dtype).float()) + r2c.to(dtype).float()
    _close(out.nchw(), ref, dtype)
    # GDN division needs a positive pre-activation: square the input through the weights
    mp = Conv2d(C, C, 3, 1, 1).to(DEV)
    with torch.no_grad():
        mp.weight.abs_()
        mp.bias.abs_().add_(0.5)
    xa = act(xc.abs())
    out = Fn.conv(xa, mp.packed(dtype), epi=EPI_GDN_DIV, g=g)
    basep = F.conv2d(xc.abs().to(dtype).float(), mp.weight.cpu(), mp.bias.cpu(), 1, 1)
    _close(out.nchw(), gc.to(dtype).float() / torch.sqrt(basep), dtype)
