"""HAN post-processing (reference model/han.py, net_ga.py:1096-1100)
on the HIP path against the CPU oracle (oracle/ref_cpu.han_head / net_forward).

Bars: fp32 HAN head within 2e-4 (relative to the output range) with non-zero LAM / CSAM
gammas (default init has both at 0, which makes those blocks identities); full
Net(post_processing=True) fp32: bpp within 1e-5, PSNR within 1e-4 dB."""
import math

import pytest
import torch

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _han(seed=0, gammas=(0.5, 0.7)):
    from lic_amd.model.han import HAN_Head
    torch.manual_seed(seed)
    m = HAN_Head(is_high=False)
    with torch.no_grad():
        m.la.gamma.fill_(gammas[0])
        m.csa.gamma.fill_(gammas[1])
        # keep activations O(1) through 4 groups x 8 blocks of random convs
        for n, p in m.named_parameters():
            if n.endswith("weight") and p.dim() == 4 and "sub_mean" not in n:
                p.mul_(0.5)
    return m


@pytest.mark.parametrize("gammas", [(0.0, 0.0), (0.5, 0.7)])
def test_han_head_fp32_matches_oracle(gammas):
    m = _han(1, gammas)
    P = {"HAN." + k: v.detach().float().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(2)) * 2 - 1
    from lic_amd.functional import Act
    y = m.run(Act.from_nchw(x.to(DEV).contiguous(), torch.float32, pad16=True)).nchw().cpu()
    ref = R.han_head(x, P, "HAN")
    scale = ref.abs().max().item()
    err = (y - ref).abs().max().item()
    print(f"\n[HAN head gammas={gammas}] max |err| {err:.3e} (output range {scale:.3f})")
    assert err <= 2e-4 * max(1.0, scale)


def test_han_glue_kernels_fp16_close():
    m = _han(3).to(DEV)
    P = {"HAN." + k: v.detach().float().cpu().clone() for k, v in m.state_dict().items()}
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(4)) * 2 - 1
    from lic_amd.functional import Act
    y = m.run(Act.from_nchw(x.to(DEV).contiguous(), torch.float16, pad16=True)).nchw().float().cpu()
    ref = R.han_head(x, P, "HAN")
    rel = ((y - ref).abs().max() / ref.abs().max()).item()
    print(f"\n[HAN head fp16] rel err {rel:.3e}")
    assert rel < 3e-2


@pytest.mark.parametrize("arch", ["net_ga", "net_unet_ha_hs"])
def test_net_post_processing_fp32_parity(arch):
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(0)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    net = net_ga.synthetic_syntax_bias_(mod.Net((1, 256, 256, 3), (1, 256, 256, 3), False, True, precision="fp32"))
    with torch.no_grad():
        net.HAN.la.gamma.fill_(0.25)
        net.HAN.csa.gamma.fill_(0.5)
    P = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    net = net.to(DEV)
    x = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(6)) * 2 - 1
    bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
    ref = R.net_forward(x, P, arch=arch, post_processing=True)
    u8 = lambda t: torch.round(torch.clamp((t.float().cpu() + 1) * 127.5, 0, 255)).int()
    d8 = (u8(net.last["x_rec"]) - u8(ref["x_rec"])).abs()
    assert u8(ref["x_rec"]).unique().numel() > 16 and int(d8.max()) <= 1 and (d8 > 0).float().mean() < 1e-4
    print(f"\n[{arch} +HAN fp32] bpp {bpp.item():.8f}/{ref['bpp'].item():.8f} "
          f"psnr {v_psnr.item():.6f}/{ref['v_psnr'].item():.6f}")
    assert abs(bpp.item() - ref["bpp"].item()) <= 1e-5 * max(1.0, abs(ref["bpp"].item()))
    assert abs(v_psnr.item() - ref["v_psnr"].item()) <= 1e-4 or math.isinf(ref["v_psnr"].item())


def test_state_dict_keys_match_reference_names():
    from lic_amd.model import net_ga
    net = net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, True)
    keys = set(net.state_dict())
    for k in ("HAN.sub_mean.weight", "HAN.head.0.weight", "HAN.body.0.body.0.body.3.conv_du.0.weight",
              "HAN.body.0.body.8.weight", "HAN.body.4.bias", "HAN.csa.conv.weight", "HAN.csa.gamma",
              "HAN.la.gamma", "HAN.last_conv.weight", "HAN.last.bias", "conv_weights_gen_HAN.transform.4.weight",
              "add_mean.weight"):
        assert k in keys, k
    net.load_state_dict(net.state_dict(), strict=True)
