"""GPU parity of the fused / padded fast paths against the CPU oracle."""
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
DTYPES = [torch.float32, torch.float16, torch.bfloat16]


def _P(module, prefix):
    return {prefix + "." + k: v.detach().float().cpu() for k, v in module.state_dict().items()}


def _close(out, ref, dtype, tol32=1e-4):
    out, ref = out.float().cpu(), ref.float().cpu()
    if dtype != torch.float32:   # 16-bit activations: fp16 2e-2, bf16 4e-2 of the scale
        tol = 2e-2 if dtype == torch.float16 else 4e-2
        assert (out - ref).abs().max().item() <= tol * (ref.abs().max().item() + 1e-6)
    else:
        torch.testing.assert_close(out, ref, rtol=tol32, atol=tol32)


@pytest.mark.parametrize("dtype", DTYPES)
def test_rb3_fused_matches_oracle(dtype):
    """Fused ResidualBottleneck(3) (net_ga.py:89-103, N=3) and the zero-padded output pixels."""
    from lic_amd.model.Block_unet import ResidualBottleneck
    from lic_amd.functional import Act
    torch.manual_seed(20)
    m = ResidualBottleneck(3)
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0, 0.5)
    m = m.to(DEV)
    x = torch.rand(2, 3, 33, 40) * 2 - 1
    xa = Act.from_nchw(x.to(DEV), dtype, pad16=True)
    assert xa.zpad * xa.t.element_size() == 16
    y = m.run(xa)
    assert y.c == 3 and y.ld * y.t.element_size() == 16
    assert y.t[..., 3:].abs().max().item() == 0.0
    _close(y.nchw(), R.residual_bottleneck(x, _P(m, "r"), "r"), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("B,H,W", [(2, 33, 40), (3, 64, 96), (32, 256, 256)])
def test_rb3_chain_equals_three_launches(dtype, B, H, W):
    """The a_model's three ResidualBottleneck(3) blocks (net_ga.py:262-264) in one launch (lic_rb3_chain_fwd)
    equal the three one-block launches bitwise (ragged 32 x 32 tiles included) and the oracle within the
    dtype's bar; the output pixels are zero-padded to 16 bytes."""
    from lic_amd.model.Block_unet import ResidualBottleneck
    from lic_amd.functional import Act
    import lic_amd.functional as Fn
    torch.manual_seed(23 + H)
    ms = [ResidualBottleneck(3) for _ in range(3)]
    for m in ms:
        with torch.no_grad():
            for p in m.parameters():
                p.normal_(0, 0.5)
    ms = [m.to(DEV) for m in ms]
    x = torch.rand(B, 3, H, W) * 2 - 1
    xa = Act.from_nchw(x.to(DEV), dtype, pad16=True)
    ref3 = xa
    for m in ms:
        ref3 = m.run(ref3)
    params = torch.cat([m._rb3_params() for m in ms]).contiguous()
    y = Fn.rb3_chain(xa, params, 3)
    assert torch.equal(y.t, ref3.t)
    assert y.t[..., 3:].abs().max().item() == 0.0
    if B * H * W <= 20000:
        r = x
        for i, m in enumerate(ms):
            r = R.residual_bottleneck(r, _P(m, "r"), "r")
        _close(y.nchw(), r, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_rbws_from_padded_image(dtype):
    """ResidualBlockWithStride(3 -> 192) on the zero-padded 3-channel image runs as Cin=16 B MFMA."""
    from lic_amd.layers import ResidualBlockWithStride
    from lic_amd.functional import Act
    torch.manual_seed(21)
    m = ResidualBlockWithStride(3, 192, 2)
    with torch.no_grad():
        m.gdn.beta.add_(0.2)
    m = m.to(DEV)
    x = torch.rand(2, 3, 64, 48) * 2 - 1
    out = m.run(Act.from_nchw(x.to(DEV), dtype, pad16=True))
    _close(out.nchw(), R.residual_block_with_stride(x, _P(m, "b"), "b"), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_analysis_transform_small(dtype):
    """a_model end to end at 64x64 (both Win_noShift_Attention windows fit) vs the oracle."""
    from lic_amd.model.net_ga import analysisTransformModel, weight_init
    from lic_amd.functional import Act
    torch.manual_seed(22)
    m = analysisTransformModel(3, [192] * 4)
    m.apply(weight_init)
    m = m.to(DEV)
    x = torch.rand(2, 3, 64, 64) * 2 - 1
    out = m.run(Act.from_nchw(x.to(DEV), dtype, pad16=True))
    ref = R.analysis_transform(x, _P(m, "a_model"), "a_model")
    _close(out.nchw(), ref, dtype, tol32=2e-4)
