"""Host-side logic (no GPU): weight packing, tap geometry, transposed-conv phase
decomposition, pixel-shuffle addressing and state_dict compatibility."""
import pytest
import torch
import torch.nn.functional as F

import lic_amd.functional as Fn
from tests.tapconv import tap_conv


@pytest.mark.parametrize("k,s,pad", [(3, 1, (1, 1, 1, 1)), (3, 2, (1, 1, 1, 1)), (5, 2, (1, 1, 2, 2)),
                                     (7, 1, (3, 3, 3, 3)), (1, 1, (0, 0, 0, 0)), (1, 2, (0, 0, 0, 0))])
def test_pack_conv2d_matches_torch(k, s, pad):
    torch.manual_seed(0)
    x = torch.randn(2, 8, 11, 13)
    w = torch.randn(20, 8, k, k)
    b = torch.randn(20)
    pk = Fn.pack_conv2d(w, b, s, pad, torch.float32)
    ref = F.conv2d(F.pad(x, (pad[1], pad[3], pad[0], pad[2])), w, b, s)
    Ho, Wo = Fn.conv_out_hw(11, 13, pk)
    assert (Ho, Wo) == ref.shape[2:]
    out = torch.zeros(2, Ho, Wo, 20)
    tap_conv(x.permute(0, 2, 3, 1).contiguous(), pk, out)
    torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, rtol=1e-4, atol=1e-4)
    assert pk.copad % 32 == 0 and pk.cpad % 16 == 0


@pytest.mark.parametrize("k,s,p,op,prepad", [(5, 2, 3, 1, (1, 1)), (5, 2, 2, 1, (0, 0)), (1, 1, 0, 0, (0, 0)),
                                             (3, 2, 1, 1, (0, 0))])
def test_pack_conv_transpose_phases(k, s, p, op, prepad):
    torch.manual_seed(1)
    x = torch.randn(2, 8, 5, 6)
    w = torch.randn(8, 12, k, k)
    b = torch.randn(12)
    xp = F.pad(x, (prepad[1], 0, prepad[0], 0))
    ref = F.conv_transpose2d(xp, w, b, s, p, op)
    Ho, Wo = Fn.convT_out_hw(5, 6, s, p, op, k, prepad)
    assert (Ho, Wo) == ref.shape[2:]
    packs = Fn.pack_conv_transpose2d(w, b, s, p, op, torch.float32, prepad)
    out = torch.full((2, Ho, Wo, 12), float("nan"))
    for pk in packs:
        tap_conv(x.permute(0, 2, 3, 1).contiguous(), pk, out)
    assert not torch.isnan(out).any(), "phases must cover every output pixel"
    torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, rtol=1e-4, atol=1e-4)


def test_pixel_shuffle_addressing():
    torch.manual_seed(2)
    x = torch.randn(1, 8, 4, 5)
    w = torch.randn(12 * 4, 8, 3, 3)
    pk = Fn.pack_conv2d(w, None, 1, (1, 1, 1, 1), torch.float32)
    ref = F.pixel_shuffle(F.conv2d(x, w, None, 1, 1), 2)
    out = torch.zeros(1, 8, 10, 12)
    tap_conv(x.permute(0, 2, 3, 1).contiguous(), pk, out, shuffle=True)
    torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, rtol=1e-4, atol=1e-4)


def test_depthwise_pack():
    torch.manual_seed(3)
    x = torch.randn(2, 16, 7, 7)
    w = torch.randn(16, 1, 3, 3)
    b = torch.randn(16)
    pk = Fn.pack_conv2d(w, b, 1, (1, 1, 1, 1), torch.float32, groups=16)
    out = torch.zeros(2, 7, 7, 16)
    tap_conv(x.permute(0, 2, 3, 1).contiguous(), pk, out)
    torch.testing.assert_close(out.permute(0, 3, 1, 2), F.conv2d(x, w, b, 1, 1, 1, 16), rtol=1e-4, atol=1e-4)


def test_copad_choice():
    for co in (3, 16, 48, 96, 128, 192, 224, 256, 288, 320, 512, 576, 768):
        cp = Fn._choose_copad(co)
        assert cp >= co and cp % 32 == 0
        assert any(cp % bn == 0 for bn in (192, 128, 96, 64, 32))


def _ref_keys_net_ga():
    """A sample of reference state_dict keys (from the module structure of net_ga.py)."""
    return [
        "a_model.transform.0.branch.0.weight", "a_model.transform.3.conv1.weight", "a_model.transform.3.gdn.beta",
        "a_model.transform.3.gdn.beta_reparam.pedestal", "a_model.transform.3.gdn.beta_reparam.lower_bound.bound",
        "a_model.transform.3.gdn.gamma_reparam.lower_bound.bound", "a_model.transform.3.skip.weight",
        "a_model.transform.4.reparam_offset", "a_model.transform.4.pedestal", "a_model.transform.4.gamma",
        "a_model.transform.6.weight", "a_model.transform.8.conv_a.0.conv1.weight",
        "a_model.transform.8.conv_b.0.attn.relative_position_bias_table",
        "a_model.transform.8.conv_b.0.attn.relative_position_index", "a_model.transform.8.conv_b.0.attn.qkv.weight",
        "a_model.transform.8.conv_b.0.attn.proj.bias", "a_model.transform.8.conv_b.7.weight",
        "a_model.transform.16.conv_b.9.conv2.bias", "s_model.transform.2.weight", "s_model.transform.13.gamma",
        "h_mean_s.2.0.weight", "h_scale_s.6.0.bias", "h_a.8.weight", "syntax_model.WAM.conv_b.0.attn.qkv.weight",
        "syntax_model.Depth_down0.depthwise.weight", "syntax_model.conv.weight", "conv_weights_gen.transform.4.weight",
        "entropy_bottleneck.quantiles", "entropy_bottleneck._matrix0", "entropy_bottleneck._factor3",
        "gaussian_conditional.scale_bound", "atten_mean.0.0.in_conv.weight",
        "atten_mean.3.0.non_local_block.block_2.msa.relative_position_params",
        "atten_mean.1.0.non_local_block.block_1.ln1.weight", "atten_mean.1.0.non_local_block.block_1.mlp.2.weight",
        "atten_scale.2.0.conv_a.1.conv.2.weight", "atten_scale.2.0.conv_b.3.weight", "atten_scale.2.0.out_conv.bias",
        "cc_mean_transforms.3.4.weight", "cc_scale_transforms.0.0.weight", "lrp_transforms.3.0.weight",
        "v_z2_sigma", "z2_sigma", "prediction_model.fc.weight", "prediction_model_syntax.WAM.conv_a.0.conv1.weight",
        "conv_1.weight", "conv_2.bias",
    ]


def test_state_dict_keys_net_ga():
    from lic_amd.model import net_ga
    n = net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False)
    sd = n.state_dict()
    missing = [k for k in _ref_keys_net_ga() if k not in sd]
    assert not missing, missing
    # shapes of a few parameters match the reference constructors
    assert sd["a_model.transform.8.conv_b.0.attn.relative_position_bias_table"].shape == (225, 8)
    assert sd["atten_mean.3.0.non_local_block.block_2.msa.relative_position_params"].shape == (8, 15, 15)
    assert sd["atten_mean.3.0.in_conv.weight"].shape == (128, 336, 1, 1)
    assert sd["lrp_transforms.3.0.weight"].shape == (224, 384, 3, 3)
    assert sd["s_model.transform.12.weight"].shape == (192, 16, 5, 5)
    assert sd["entropy_bottleneck.quantiles"].shape == (192, 1, 3)
    # ignored reference-only buffers are accepted by load_state_dict(strict=True)
    sd2 = dict(sd)
    sd2["y_sampler.sample_filter"] = torch.zeros(1)
    sd2["HAN.head.0.weight"] = torch.zeros(1)
    n.load_state_dict(sd2, strict=True)


def test_state_dict_keys_unet():
    from lic_amd.model import net_unet_ha_hs
    n = net_unet_ha_hs.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False)
    sd = n.state_dict()
    for k in ["h_a.SpatialTransformer1.attn.qkv.weight", "h_a.conv1.conv2.weight", "h_a.middle.1.attn.proj.weight",
              "h_a.down2.weight", "h_s.up1.weight", "h_s.up4.bias", "h_s.conv3.conv3.weight",
              "h_s.SpatialTransformer3.attn.relative_position_bias_table", "entropy_bottleneck.quantiles"]:
        assert k in sd, k
    assert sd["h_s.up1.weight"].shape == (512, 256, 5, 5)
    assert sd["entropy_bottleneck.quantiles"].shape == (512, 1, 3)


def test_gpu_required_message():
    """The product path refuses to run without a GPU instead of falling back to torch."""
    from lic_amd.model import net_ga
    n = net_ga.Net((1, 64, 64, 3), (1, 64, 64, 3), False, False)
    with pytest.raises(RuntimeError):
        n(torch.zeros(1, 3, 64, 64), "test")
