"""BASELINE config 1 (source_net plumbing): source_net.Net.forward -> z on the HIP path
against the oracle's restatement (oracle/ref_cpu.py::source_net_forward)."""
import pytest
import torch

from oracle import ref_cpu as R

@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_source_net_z_matches_oracle(precision):
    from lic_amd.model import source_net
    torch.manual_seed(0)
    net = source_net.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision=precision)
    with torch.no_grad():
        for m in net.modules():            # non-trivial GDN parameters
            if hasattr(m, "beta") and isinstance(m.beta, torch.nn.Parameter):
                m.beta.add_(0.1 * torch.rand_like(m.beta))
    P = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    net = net.to("cuda")
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 3, 256, 256, generator=g) * 2 - 1
    z = net(x.to("cuda"), "test").cpu()
    ref = R.source_net_forward(x, P)
    assert z.shape == ref.shape == (1, 192, 4, 4)
    err = (z - ref).abs().max().item()
    scale = ref.abs().max().item()
    tol = 1e-4 if precision == "fp32" else 2e-2
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


def test_source_net_state_dict_keys():
    from lic_amd.model import source_net
    net = source_net.Net((1, 64, 64, 3), (1, 64, 64, 3), False, False)
    keys = set(net.state_dict())
    for k in ("a_model.transform.1.weight", "a_model.transform.2.beta", "a_model.transform.10.bias",
              "h_a.transform.0.weight", "h_a.transform.4.bias"):
        assert k in keys
    sd = dict(net.state_dict())
    sd["s_model.transform.0.weight"] = torch.zeros(1)   # unreachable modules are ignored
    net.load_state_dict(sd, strict=True)
