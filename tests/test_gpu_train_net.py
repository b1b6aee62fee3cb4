"""Training path end to end: the liblic train-mode graph
(lic_amd/train_net.py) against fp32 CPU autograd through the oracle restatement
(oracle/ref_cpu.py) with the same parameters, input and rate noise.

The oracle's LowerBound is torch.max, whose gradient splits ties; the reference's
LowerBound passes the full gradient at the bound (ops/bound_ops.py:25-28).  GDN gammas
are initialised exactly at the bound off the diagonal, so these tests lift every gamma
slightly off it (the rule itself is checked in test_gpu_train.py::test_gdn_grad).

Bar (fp32; MFMA vs oneDNN summation order through ~100 layers): per tensor, max |err| /
max |ref grad| <= 2e-3 for 95 % of the parameter tensors and <= 2e-2 for every one (a
ReLU / LeakyReLU input within ~1e-6 of zero can take the other branch than in oneDNN,
which moves a few entries of small late-layer gradients); forward outputs and the loss
terms 1e-4 relative."""
import math

import pytest
import torch

from oracle import ref_cpu as R
from tests.test_gpu_train import _noise_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lift_gammas(module):
    with torch.no_grad():
        for n, p in module.named_parameters():
            if n.endswith("gamma"):
                p.add_(0.01 + 0.01 * torch.rand(p.shape, generator=torch.Generator().manual_seed(len(n))))


def _params(module, prefix):
    names = {n for n, _ in module.named_parameters()}
    return {(prefix + k if prefix else k): (v.detach().clone().float().requires_grad_(True) if k in names
                                             else v.detach().clone().float())
            for k, v in module.state_dict().items()}


def _grad_close(name, got, ref, tol=2e-3):
    got, ref = got.detach().float().cpu(), ref.detach().float().cpu()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-12, f"{name}: max err {err:.3e} vs scale {scale:.3e}"
    return err / (scale + 1e-30)


def _grads_close(pairs, p95=2e-3, worst=2e-2):
    """Per-tensor relative errors: 95 % of the tensors within p95, every tensor within `worst`.
    (A ReLU / LeakyReLU pre-activation within ~1e-6 of zero can take the other branch on the
    GPU than in oneDNN, which moves a few gradient entries of the small late layers.)"""
    rels = sorted(_grad_close(n, g, r, worst) for n, g, r in pairs)
    assert rels, "no gradients compared"
    q = rels[int(0.95 * (len(rels) - 1))]
    print(f"\n[grads] {len(rels)} tensors: median rel {rels[len(rels) // 2]:.2e}, p95 {q:.2e}, max {rels[-1]:.2e}")
    assert q <= p95, q
    return len(rels)


def test_analysis_transform_train_fp32():
    """a_model (net_ga.py:253-309) forward + backward: z3 and every parameter gradient."""
    from lic_amd.model import net_ga
    from lic_amd import autograd as AG
    from lic_amd import train_net as TN
    torch.manual_seed(0)
    m = net_ga.analysisTransformModel(3, [192] * 4)
    m.apply(net_ga.weight_init)
    _lift_gammas(m)
    P = _params(m, "a_model.")
    x = torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(3)) * 2 - 1
    yr = R.analysis_transform(x, P)
    r = torch.randn(yr.shape, generator=torch.Generator().manual_seed(4))
    (yr * r).sum().backward()
    m = m.to(DEV)
    yg = TN.analysis(m, AG.to_nhwc(x.to(DEV), torch.float32))
    (yg * r.permute(0, 2, 3, 1).to(DEV)).sum().backward()
    torch.cuda.synchronize()
    _grad_close("z3", yg.permute(0, 3, 1, 2), yr, 1e-4)
    pairs = []
    for n, p in m.named_parameters():
        ref = P["a_model." + n].grad
        if ref is None:
            continue
        assert p.grad is not None, n
        pairs.append((n, p.grad, ref))
    assert _grads_close(pairs) > 100


def _rate_ref(y, mu, sc, seed, num_pixels):
    from tests.test_gpu_train import _rate_ref as rr
    bpp, yq = rr(y.permute(0, 2, 3, 1), mu.permute(0, 2, 3, 1), sc.permute(0, 2, 3, 1), seed, num_pixels)
    return bpp, yq.permute(0, 3, 1, 2)


def _net_train_ref(x, P, seed, M=16, ns=4, arch="net_ga"):
    """net_ga.py:981-1115 (net_unet_ha_hs.py:868-1003) in mode 'train' on the oracle, with the
    kernels' noise stream."""
    B, _, H, W = x.shape
    num_pixels = B * H * W
    z3 = R.analysis_transform(x, P)
    if arch == "net_ga":
        z = R.h_a_ga(z3, P)
        med = P["entropy_bottleneck.quantiles"][:, :, 1:2].detach()
        z_hat = R.ste_round(z - med) + med
        latent_scales = R.h_s_ga(z_hat, P, "h_scale_s")
        latent_means = R.h_s_ga(z_hat, P, "h_mean_s")
    else:
        z, middle_x, down_x1, inp = R.unet_ha_new(z3, P)
        latent_scales = R.unet_hs_new(middle_x, down_x1, inp, P)     # two calls, as the reference
        latent_means = R.unet_hs_new(middle_x, down_x1, inp, P)
    syn = R.syntax_model(z3[:, :M], P)
    syn_r = syn + (torch.round(syn) - syn).detach()                     # bypass_round
    cc = lambda t, pfx: R._conv(R.gelu(R._conv(R.gelu(R._conv(t, P, pfx + ".0", 1, 1)), P, pfx + ".2", 1, 1)), P,
                                pfx + ".4", 1, 1)
    y_hats, bpp = [], 0.0
    for i, y in enumerate(z3.chunk(ns, 1)):
        ms = R.swatten(torch.cat([latent_means] + y_hats, 1), P, f"atten_mean.{i}.0")
        mu = cc(ms, f"cc_mean_transforms.{i}")
        ss = R.swatten(torch.cat([latent_scales] + y_hats, 1), P, f"atten_scale.{i}.0")
        sc = cc(ss, f"cc_scale_transforms.{i}")
        b_i, yq = _rate_ref(y, mu, sc, seed * ns + i, num_pixels)
        bpp = bpp + b_i
        lrp = cc(torch.cat([ms, yq], 1), f"lrp_transforms.{i}")
        y_hats.append(yq + 0.5 * torch.tanh(lrp))
    x16 = R.synthesis_transform(torch.cat(y_hats, 1), P)
    cw = R.conv_generator(syn_r, P, "conv_weights_gen", M)
    xt = torch.tanh(R.batch_conv(cw, x16))
    return bpp, ((xt - x) ** 2).mean()


@pytest.mark.parametrize("arch", ["net_ga", "net_unet_ha_hs"])
def test_net_train_step_fp32(arch):
    """Net.forward(x, 'train') -> (bpp, mse), loss = lambda*255^2*mse + bpp (train_net_unet.py:180),
    backward: loss terms and every parameter gradient vs the oracle's autograd (net_ga, and
    net_unet_ha_hs with its U-Net hyper nets, Block_unet.py:774-890)."""
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(0)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    net = net_ga.synthetic_syntax_bias_(mod.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision="fp32"))
    _lift_gammas(net)
    P = _params(net, "")
    x = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(8)) * 2 - 1
    lmbda = 0.0025
    bpp_r, mse_r = _net_train_ref(x, P, seed=5, arch=arch)
    (lmbda * 255 ** 2 * mse_r + bpp_r).backward()
    net = net.to(DEV)
    bpp, mse = net(x.to(DEV), "train", seed=5)
    (lmbda * 255 ** 2 * mse + bpp).backward()
    torch.cuda.synchronize()
    print(f"\n[{arch} train fp32] bpp {bpp.item():.6f} (ref {bpp_r.item():.6f}) mse {mse.item():.6e} "
          f"(ref {mse_r.item():.6e})")
    assert abs(bpp.item() - bpp_r.item()) <= 1e-4 * abs(bpp_r.item())
    assert abs(mse.item() - mse_r.item()) <= 1e-4 * abs(mse_r.item())
    pairs = []
    for n, p in net.named_parameters():
        ref = P[n].grad
        if ref is None or ref.abs().max().item() == 0:
            continue
        assert p.grad is not None, n
        pairs.append((n, p.grad, ref))
    # the decoder is trained too (its gradient is zero when the rounded syntax is 0)
    assert sum(1 for n, _, _ in pairs if n.startswith("s_model.")) > 20
    assert sum(1 for n, _, _ in pairs if n.startswith("conv_weights_gen.")) >= 6
    if arch == "net_unet_ha_hs":
        assert sum(1 for n, _, _ in pairs if n.startswith("h_a.")) > 20
        assert sum(1 for n, _, _ in pairs if n.startswith("h_s.")) > 20
    assert _grads_close(pairs) > 300


def test_eval_net_pre_processing_finetune():
    """eval_net --pre_processing (eval_net.py:160-179): a few encoder finetune steps on the liblic
    training path move only a_model's parameters, the losses stay finite, the test pass runs after."""
    import eval_net
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    net = net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision="fp32").to(DEV)
    x = (eval_net.synthetic_image(3, 256, 256).unsqueeze(0) * 2 - 1).to(DEV)
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    eval_net.finetune_encoder(net, x, 0.0067, 3)
    with torch.no_grad():
        bpp, v_mse, v_psnr = net(x, "test")
    torch.cuda.synchronize()
    assert math.isfinite(bpp.item()) and math.isfinite(v_psnr.item())
    moved = {n for n, p in net.named_parameters() if not torch.equal(p.detach(), before[n])}
    assert moved and all(n.startswith("a_model.") for n in moved), sorted(moved)[:5]


def test_pre_processing_finetune_trajectory():
    """eval_net --pre_processing (eval_net.py:160-179): three online encoder
    finetune steps (Adam(a_model, 1e-5), loss = lambda*mse + bpp in train mode) on the liblic
    training path against the same three steps on the oracle's autograd with the same noise
    streams (seeds 0, 1, 2 = the module's train-call counter).  Bar: the parameter updates of
    every a_model tensor agree (Adam's normalised steps: median |d_gpu - d_ref| <= 1e-3 of the
    3*lr step bound, 99th percentile <= 5e-2 -- an element whose gradient is ~0 may take the
    other sign), only a_model moves, and a fresh train-mode loss after the finetune agrees
    within 1e-4."""
    import eval_net
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    net = net_ga.synthetic_syntax_bias_(net_ga.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False, precision="fp32"))
    _lift_gammas(net)
    P = {k: v.detach().clone().float() for k, v in net.state_dict().items()}
    enc = [k for k, _ in net.named_parameters() if k.startswith("a_model.")]
    for k in enc:
        P[k].requires_grad_(True)
    x = eval_net.synthetic_image(3, 256, 256).unsqueeze(0) * 2 - 1
    lmbda, steps, lr = 0.0067, 3, 1e-5
    opt = torch.optim.Adam([P[k] for k in enc], lr=lr)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [50], 0.5)
    for s in range(steps):
        bpp_r, mse_r = _net_train_ref(x, P, seed=s)
        loss = (lmbda * mse_r + bpp_r).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sch.step()
    net = net.to(DEV)
    before = {k: v.detach().clone() for k, v in net.named_parameters()}
    eval_net.finetune_encoder(net, x.to(DEV), lmbda, steps)
    torch.cuda.synchronize()
    errs, moved = [], []
    for k, p in net.named_parameters():
        d_gpu = (p.detach() - before[k]).float().cpu()
        if not k.startswith("a_model."):
            assert torch.equal(p.detach(), before[k]), k
            continue
        d_ref = (P[k].detach() - before[k].float().cpu())
        errs.append(((d_gpu - d_ref).abs() / (steps * lr)).flatten())
        moved.append(bool(d_gpu.abs().max() > 0))
    e = torch.cat(errs)
    med, p99 = e.median().item(), e.quantile(0.99).item() if e.numel() < 2 ** 24 else e[::4].quantile(0.99).item()
    print(f"\n[pre_processing x{steps}] {e.numel()} encoder weights: update error median {med:.2e}, p99 {p99:.2e} "
          f"(units of {steps}*lr)")
    assert all(moved) and med <= 1e-3 and p99 <= 5e-2
    with torch.no_grad():
        bpp_g, mse_g = net(x.to(DEV), "train", seed=99)
        bpp_r, mse_r = _net_train_ref(x, {k: v.detach() for k, v in P.items()}, seed=99)
    assert abs(bpp_g.item() - bpp_r.item()) <= 1e-4 * abs(bpp_r.item())
    assert abs(mse_g.item() - mse_r.item()) <= 1e-4 * abs(mse_r.item())


def _cos(a, b):
    a, b = a.detach().double().flatten().cpu(), b.detach().double().flatten().cpu()
    return (a @ b / (a.norm() * b.norm() + 1e-300)).item()


@pytest.mark.parametrize("arch,B", [("net_unet_ha_hs", 1), ("net_ga", 1), ("net_unet_ha_hs", 8)])
def test_net_train_step_bf16(arch, B):
    """BASELINE config 5's precision: the train step with bf16 activations (bf16 MFMA operands,
    fp32 accumulation, fp32 parameters) against the fp32 oracle autograd -- at B=1 and at config 5's
    own batch (train_net_unet.py:289 --batch_size 8: the split-K wgrad tiling depends on K = B*H*W).
    bf16 keeps 8 mantissa bits, so the bar is statistical: bpp / mse within 2e-2, and the gradient
    of 90 % of the parameter tensors points the same way as the reference's (cosine >= 0.98;
    median >= 0.995)."""
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(0)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    net = net_ga.synthetic_syntax_bias_(mod.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision="bf16"))
    _lift_gammas(net)
    P = _params(net, "")
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(8)) * 2 - 1
    lmbda = 0.0025
    bpp_r, mse_r = _net_train_ref(x, P, seed=5, arch=arch)
    (lmbda * 255 ** 2 * mse_r + bpp_r).backward()
    net = net.to(DEV)
    bpp, mse = net(x.to(DEV), "train", seed=5)
    (lmbda * 255 ** 2 * mse + bpp).backward()
    torch.cuda.synchronize()
    cos = sorted(_cos(p.grad, P[n].grad) for n, p in net.named_parameters()
                 if P[n].grad is not None and P[n].grad.abs().max() > 0 and p.grad is not None)
    print(f"\n[{arch} train bf16 B={B}] bpp {bpp.item():.5f} (ref {bpp_r.item():.5f}) mse {mse.item():.5e} "
          f"(ref {mse_r.item():.5e}); grad cosine over {len(cos)} tensors: p10 {cos[len(cos) // 10]:.4f} "
          f"median {cos[len(cos) // 2]:.5f} min {cos[0]:.4f}")
    assert abs(bpp.item() - bpp_r.item()) <= 2e-2 * abs(bpp_r.item())
    assert abs(mse.item() - mse_r.item()) <= 2e-2 * abs(mse_r.item())
    assert len(cos) > 300 and cos[len(cos) // 10] >= 0.98 and cos[len(cos) // 2] >= 0.995


def test_train_step_hipgraph_matches_eager():
    """train_net_unet.py --graph: the whole step (forward, backward, clip_grad_norm_, capturable
    Adam) captured once and replayed, with the noise seed on the device (lic_rate_train_* seed_dev),
    gives bit-identical losses and parameters to the same steps run eagerly (same kernels, same
    order), and two eager runs are bit-identical too: every gradient reduction has a fixed order (the
    window-attention table gradient used an LDS atomicAdd until round 2, which Adam's first steps
    amplified -- a near-zero gradient's sign noise becomes a full +-lr update)."""
    import copy
    from lic_amd.model import net_unet_ha_hs, net_ga
    torch.manual_seed(0)
    base = net_ga.synthetic_syntax_bias_(net_unet_ha_hs.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False,
                                                            precision="bf16"))
    x = (torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(9)) * 2 - 1).to(DEV)
    lmbda, steps = 0.0025, 3

    def make():
        net = copy.deepcopy(base).to(DEV)
        params = net.base_params()
        opt = torch.optim.Adam(params, lr=torch.tensor(1e-4, device=DEV), capturable=True)
        return net, params, opt, torch.zeros((1,), dtype=torch.int64, device=DEV)

    def body(net, params, opt, seed_t):
        bpp, mse = net(x, "train", seed_dev=seed_t)
        loss = lmbda * 255 ** 2 * mse + bpp
        loss.backward()
        torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], 1.0)
        opt.step()
        seed_t.add_(1)
        return loss.detach()

    def eager():
        net_a, pa, oa, sa = make()
        losses = []
        for _ in range(steps):
            oa.zero_grad(set_to_none=True)
            losses.append(body(net_a, pa, oa, sa).item())
        return net_a, losses

    net_a, losses_a = eager()
    net_a2, losses_a2 = eager()
    net_b, pb, ob, sb = make()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ob.zero_grad(set_to_none=True)
        first = body(net_b, pb, ob, sb).item()               # eager warm-up = step 1
    torch.cuda.current_stream().wait_stream(side)
    ob.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):   # the warm-up's stream: AccumulateGrad nodes stay on it
        out = body(net_b, pb, ob, sb)
    losses_b = [first]
    for _ in range(steps - 1):
        g.replay()
        losses_b.append(out.item())
    torch.cuda.synchronize()
    print(f"\n[train hipGraph] eager losses {losses_a} / {losses_a2}, graph losses {losses_b}")
    assert int(sb.item()) == steps
    assert losses_a == losses_b == losses_a2
    def dmax(m1, m2):
        return max(((p - q).norm() / (p.norm() + 1e-12)).item() for p, q in zip(m1.parameters(), m2.parameters()))
    d, d_ee = dmax(net_a, net_b), dmax(net_a, net_a2)
    print(f"[train hipGraph] max relative parameter difference graph-eager {d:.2e}, eager-eager {d_ee:.2e}")
    assert d == 0 and d_ee == 0


def test_train_step_frozen_deferred_matches_plain():
    """train_net_unet.py's one-GPU step: the parameters the optimiser does not own (the slice-loop
    modules the reference leaves out of base_params) take no weight gradient, and the backward's
    split-K wgrad reduces run as one batched launch (autograd.WgradDefer).  Neither changes a bit of
    what the optimiser sees: 3 steps of that setup -- eager, and captured + replayed with the
    descriptor table filled after the capture -- give the same losses and parameters as the plain
    eager steps."""
    import contextlib
    import copy
    from lic_amd import autograd as AG
    from lic_amd.model import net_unet_ha_hs, net_ga
    torch.manual_seed(0)
    base = net_ga.synthetic_syntax_bias_(net_unet_ha_hs.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False,
                                                            precision="bf16"))
    x = (torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(9)) * 2 - 1).to(DEV)
    lmbda, steps = 0.0025, 3

    def make(frozen):
        net = copy.deepcopy(base).to(DEV)
        params = net.base_params()
        if frozen:
            ids = {id(p) for p in params}
            for p in net.parameters():
                if id(p) not in ids:
                    p.requires_grad_(False)
        opt = torch.optim.Adam(params, lr=torch.tensor(1e-4, device=DEV), capturable=True)
        return net, params, opt, torch.zeros((1,), dtype=torch.int64, device=DEV)

    def body(net, params, opt, seed_t, defer):
        bpp, mse = net(x, "train", seed_dev=seed_t)
        loss = lmbda * 255 ** 2 * mse + bpp
        with defer if defer is not None else contextlib.nullcontext():
            loss.backward()
        torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], 1.0)
        opt.step()
        seed_t.add_(1)
        return loss.detach()

    def eager(frozen, defer):
        net, p, o, s = make(frozen)
        losses = []
        for _ in range(steps):
            o.zero_grad(set_to_none=True)
            losses.append(body(net, p, o, s, defer).item())
        return net, losses

    net_plain, l_plain = eager(False, None)
    net_fd, l_fd = eager(True, AG.WgradDefer())
    d = AG.WgradDefer()
    net_g, pg, og, sg = make(True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        og.zero_grad(set_to_none=True)
        first = body(net_g, pg, og, sg, d).item()            # eager warm-up = step 1 (sizes the table)
    torch.cuda.current_stream().wait_stream(side)
    og.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        out = body(net_g, pg, og, sg, d)
    d.finalize()
    l_g = [first]
    for _ in range(steps - 1):
        g.replay()
        l_g.append(out.item())
    torch.cuda.synchronize()
    print(f"\n[frozen + deferred] plain {l_plain}, eager {l_fd}, graph {l_g}")
    assert l_plain == l_fd == l_g
    for m in (net_fd, net_g):
        for (n, p), q in zip(net_plain.named_parameters(), m.parameters()):
            assert torch.equal(p, q), n
