"""GPU: lic_pack_taps (one launch per weight pack) writes exactly the bytes of the torch packing it
replaced -- nn.Conv2d packs (padded channels, cin_to, cpad_to, depthwise), the mirrored + transposed
stride-1 dgrad pack, the stride-s dgrad phases and the transposed-conv phases -- in fp32, fp16 and
bf16 (round to nearest even, as torch's cast).  The CPU side of each comparison runs the torch
branch of the same functions on a CPU copy of the weight."""
import pytest
import torch

import lic_amd.autograd as AG
import lic_amd.functional as Fn

pytestmark = pytest.mark.gpu
DEV = "cuda"
DTYPES = [torch.float32, torch.float16, torch.bfloat16]


def _same(gpu_packs, cpu_packs):
    assert len(gpu_packs) == len(cpu_packs)
    for g, c in zip(gpu_packs, cpu_packs):
        assert g.w.dtype == c.w.dtype and g.w.shape == c.w.shape
        assert torch.equal(g.w.cpu(), c.w), (g.w.cpu().float() - c.w.float()).abs().max()
        assert list(g.dy) == list(c.dy) and list(g.dx) == list(c.dx)


def _weight(shape, seed):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(shape, generator=g) * 0.3
    w.view(-1)[::7] *= 1e-3     # small magnitudes: exercises the 16-bit roundings
    return w


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("co,ci,k,kw_", [(192, 192, 3, 3), (48, 128, 3, 3), (192, 3, 3, 3), (128, 320, 1, 1),
                                         (192, 192, 5, 5), (64, 40, 7, 7), (36, 20, 3, 5)])
def test_pack_conv2d(dtype, co, ci, k, kw_):
    w = _weight((co, ci, k, kw_), co + ci + k)
    for kw in (dict(), dict(cin_to=ci + 8), dict(mirror=True)):
        got = Fn.pack_conv2d(w.to(DEV), None, 1, (k // 2, kw_ // 2, k // 2, kw_ // 2), dtype, **kw)
        ref = Fn.pack_conv2d(w, None, 1, (k // 2, kw_ // 2, k // 2, kw_ // 2), dtype, **kw)
        _same([got], [ref])


@pytest.mark.parametrize("dtype", DTYPES)
def test_pack_conv2d_groups_and_cpad_to(dtype):
    w = _weight((64, 1, 3, 3), 3)
    _same([Fn.pack_conv2d(w.to(DEV), None, 1, (1, 1, 1, 1), dtype, groups=64)],
          [Fn.pack_conv2d(w, None, 1, (1, 1, 1, 1), dtype, groups=64)])
    # the depthwise dgrad pack (mirrored taps, read in place)
    _same([Fn.pack_conv2d(w.to(DEV), None, 1, (1, 1, 1, 1), dtype, groups=64, mirror=True)],
          [Fn.pack_conv2d(w, None, 1, (1, 1, 1, 1), dtype, groups=64, mirror=True)])
    w = _weight((32, 3, 3, 3), 4)
    _same([Fn.pack_conv2d(w.to(DEV), None, 2, (0, 0, 1, 1), dtype, cpad_to=8)],
          [Fn.pack_conv2d(w, None, 2, (0, 0, 1, 1), dtype, cpad_to=8)])


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("co,ci,k,s,pad", [(192, 192, 3, 1, (1, 1, 1, 1)), (192, 192, 5, 2, (1, 1, 2, 2)),
                                           (128, 64, 3, 2, (1, 1, 1, 1)), (40, 24, 5, 2, (2, 2, 2, 2)),
                                           (8, 8, 7, 3, (3, 2, 3, 3))])
def test_dgrad_packs(dtype, co, ci, k, s, pad):
    w = _weight((co, ci, k, k), co * 3 + k)
    co_pad = Fn._cpad_for(co, dtype)
    _same(AG.dgrad_packs(w.to(DEV), s, pad, dtype, co_pad), AG.dgrad_packs(w, s, pad, dtype, co_pad))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("ci,co,k,s,p,op,prepad", [(192, 192, 5, 2, 3, 1, (1, 1)), (192, 3, 5, 2, 2, 1, (0, 0)),
                                                   (24, 40, 5, 2, 2, 1, (0, 0)), (16, 8, 3, 2, 1, 1, (1, 0)),
                                                   (192, 192, 1, 1, 0, 0, (0, 0))])
def test_convt_packs(dtype, ci, co, k, s, p, op, prepad):
    w = _weight((ci, co, k, k), ci + co * 5 + k)
    _same(Fn.pack_conv_transpose2d(w.to(DEV), None, s, p, op, dtype, prepad),
          Fn.pack_conv_transpose2d(w, None, s, p, op, dtype, prepad))


def test_pack_taps_rejects_bad_sizes():
    w = torch.zeros(8, 8, 3, 3, device=DEV)
    with pytest.raises(Exception):
        Fn.pack_taps(w, 0, 72, 9, 3, 1, 16, 8, 3, 3, 8, 8, torch.float16)   # no > copad


def test_pack_plan_batch_equals_direct_packs():
    """PackPlan: record a step's packs, change the weights in place (the optimiser step), then one
    lic_pack_taps_batch launch + replay hand back buffers equal to fresh direct packs; a call
    sequence that differs from the recorded one raises."""
    ws = [_weight((192, 192, 3, 3), 11).to(DEV), _weight((128, 64, 5, 5), 12).to(DEV),
          _weight((192, 192, 5, 5), 13).to(DEV), _weight((320, 128, 1, 1), 14).to(DEV)]

    def packs():
        out = [Fn.pack_conv2d(ws[0], None, 1, (1, 1, 1, 1), torch.bfloat16)]
        out += AG.dgrad_packs(ws[0], 1, (1, 1, 1, 1), torch.bfloat16, 192)
        out += AG.dgrad_packs(ws[1], 2, (1, 1, 2, 2), torch.float16, 128)
        out += Fn.pack_conv_transpose2d(ws[2], None, 2, 3, 1, torch.bfloat16, (1, 1))
        out += [Fn.pack_conv2d(ws[3], None, 1, (0, 0, 0, 0), torch.float32)]
        return out

    plan = Fn.PackPlan()
    with plan.record():
        rec = packs()
    plan.finalize()
    for w in ws:
        w.mul_(-1.5).add_(0.01)
    plan.launch_all()
    with plan.replay():
        got = packs()
    ref = packs()
    torch.cuda.synchronize()
    assert len(got) == len(ref) == len(rec)
    for g, r in zip(got, ref):
        assert torch.equal(g.w, r.w)
    with pytest.raises(Exception):
        with plan.replay():
            Fn.pack_conv2d(ws[1], None, 1, (2, 2, 2, 2), torch.bfloat16)    # not the recorded first call
