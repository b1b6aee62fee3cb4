"""Training path, layer level: ``torch.autograd.Function``s whose
forward AND backward run on liblic.

The reference trains with ``loss.backward()`` through ``Net.forward(x, 'train')``
(train_net_unet.py:177-200; the online encoder finetune of eval_net.py:170-179 does
the same through ``a_model``).  Every gradient here is a liblic launch:

* conv dgrad  -> ``lic_conv2d_fwd`` over dz with re-packed weights: stride 1 is the
  transposed, tap-mirrored conv; stride 2 is four transposed-conv phases (sub-pixel
  gather form); a ConvTranspose2d's dgrad is the plain strided conv with its weight.
* conv wgrad  -> ``lic_conv2d_wgrad`` (MFMA implicit GEMM over output pixels).
* bias / beta -> ``lic_channel_sum``; activations / GDN chain rule / LowerBound ->
  ``lic_act_bwd``, ``lic_gdn_bwd_elem`` + ``lic_gdn_bwd_finish``,
  ``lic_lower_bound_sq_bwd``.

Tensors are NHWC ``[B, H, W, C]`` contiguous, fp32 (parity), fp16 or bf16; weights are the
fp32 ``nn.Parameter``s in the reference's layouts (Conv2d ``[co, ci, kh, kw]``,
ConvTranspose2d ``[ci, co, kh, kw]``, GDN ``beta [C]`` / ``gamma [C, C]``), and their
gradients come back fp32 in those layouts.  There is no PyTorch compute fallback.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence, Tuple

import torch

from . import _ffi
from . import functional as Fn
from ._ffi import ACT_NONE, EPI_GDN_DIV, EPI_GDN_RSQRT, EPI_GDN_SQRT, PRO_NONE, PRO_SQUARE, AttnArgs, WgradArgs, check
from .functional import Act, ConvPack, _dp, dtype_id, stream_handle

__all__ = ["conv2d", "conv_transpose2d", "gdn", "activation", "wgrad", "channel_sum", "dgrad_packs", "WgradDefer"]


def _lib():
    return _ffi.load()


def _epc(dtype: torch.dtype) -> int:
    return 16 // torch.empty((), dtype=dtype).element_size()


def _pad_channels(t: torch.Tensor) -> torch.Tensor:
    """NHWC tensor -> contiguous NHWC with C rounded up to 16 bytes (zero channels)."""
    t = t.contiguous()
    epc = _epc(t.dtype)
    C = t.shape[-1]
    cp = -(-C // epc) * epc
    if cp == C:
        return t
    out = torch.zeros(t.shape[:-1] + (cp,), dtype=t.dtype, device=t.device)
    out[..., :C] = t
    return out


def _taps(kh, kw, pt, pl):
    return [ky - pt for ky in range(kh) for kx in range(kw)], [kx - pl for ky in range(kh) for kx in range(kw)]


# --------------------------------------------------------------------------- deferred wgrad reduce
class WgradDefer:
    """The split-K reduces of a backward's weight gradients as ONE launch (lic_wgrad_reduce_batch)
    instead of one per layer (~470 per bf16 training step).  Inside ``with defer:`` the conv /
    transposed-conv backward launch only their wgrad partial sums (lic_conv2d_wgrad_partials) and
    return dw / db that are written by ``flush()`` -- called on exit, before anything reads them
    (train_net_unet.py: after ``loss.backward()``, before the gradient all-reduce / clip / Adam).
    The per-element sums are the per-layer reduce's: bit-identical gradients
    (tests/test_gpu_train.py::test_wgrad_defer_bit_identical).

    Not for a backward whose gradient hooks read .grad during the backward (the eager multi-rank
    GradAllReduce) or whose parameters receive several contributions (the engine would add unreduced
    tensors): the training loop enables it for the one-GPU and captured steps, whose parameters each
    feed one convolution.  Captured steps: the descriptor table is a device buffer sized by an eager
    step; ``finalize()`` after the capture writes the captured call's descriptors into it."""
    def __init__(self):
        self.rows = []        # descriptors of this backward's deferred calls
        self.keep = []        # their workspaces, alive until the reduce is launched
        self.desc = None      # device table [capacity, WORDS] int64
        self.pending = None   # captured rows, written by finalize()

    def __enter__(self):
        global _DEFER
        if _DEFER is not None:
            raise RuntimeError("WgradDefer: already active")
        _DEFER = self
        self.rows, self.keep = [], []
        return self

    def __exit__(self, *exc):
        global _DEFER
        _DEFER = None
        if exc[0] is None:
            self.flush()
        self.rows, self.keep = [], []
        return False

    def add(self, a: WgradArgs, ws: torch.Tensor, nsplit: int) -> None:
        nblk = int(_lib().lic_wgrad_reduce_blocks(ctypes.byref(a)))
        first = self.rows[-1][14] + self.rows[-1][15] if self.rows else 0
        wsb = (a.ws + nsplit * a.ntaps * a.co * a.ci * 4) if a.db else 0
        # (word 15 holds the call's block count while recording; the table's word 15 is 0)
        self.rows.append([a.ws, wsb, a.dw, a.db or 0, a.s_co, a.s_ci, a.s_tap, nsplit, a.ntaps, a.co, a.ci,
                          a.co_out, a.ci_out, a.accumulate, first, nblk])
        self.keep.append(ws)

    def flush(self) -> None:
        if not self.rows:
            return
        n = len(self.rows)
        nblocks = self.rows[-1][14] + self.rows[-1][15]
        if nblocks >= 2 ** 31:
            raise ValueError("WgradDefer: more than 2^31 reduce blocks")
        rows = [r[:15] + [0] for r in self.rows]
        dev = self.keep[0].device
        if torch.cuda.is_current_stream_capturing():
            # no host-to-device copy inside a capture: the table buffer exists (sized by the eager
            # warm-up step) and is filled by finalize() once the capture has ended
            if self.desc is None or self.desc.shape[0] < n:
                raise RuntimeError("WgradDefer: run one eager step with this object before capturing")
            self.pending = rows
        else:
            t = torch.tensor(rows, dtype=torch.int64)
            if self.desc is None or self.desc.shape[0] < n:
                self.desc = torch.zeros((n, _ffi.WGRAD_RED_DESC_WORDS), dtype=torch.int64, device=dev)
            self.desc[:n].copy_(t.to(dev))
        check(_lib().lic_wgrad_reduce_batch(_dp(self.desc), n, int(nblocks), stream_handle()))

    def finalize(self) -> None:
        """After a capture: the captured step's descriptors into the table its reduce launch reads."""
        if self.pending is not None:
            torch.cuda.synchronize()
            self.desc[:len(self.pending)].copy_(torch.tensor(self.pending, dtype=torch.int64).to(self.desc.device))
            torch.cuda.synchronize()
            self.pending = None


_DEFER: Optional[WgradDefer] = None


# --------------------------------------------------------------------------- primitives
def wgrad(x: torch.Tensor, dz: torch.Tensor, dy: Sequence[int], dx: Sequence[int], *, stride: int = 1,
          lattice: Optional[Tuple[int, int]] = None, dw: torch.Tensor, strides: Tuple[int, int, int],
          co_out: int, ci_out: int, prologue: int = PRO_NONE, accumulate: bool = False,
          db: Optional[torch.Tensor] = None, deferrable: bool = False) -> torch.Tensor:
    """dw[n*s_co + c*s_ci + t*s_tap] (+)= sum_pix dz[pix, n] * pro(x[pix*stride + tap_t, c]).
    x, dz: NHWC with 16-byte channel counts; lattice = (mi, mj) output pixels (default dz's map).
    db (fp32 [co_out], optional): the bias gradient sum_pix dz[pix, n] from the same launch.
    deferrable: inside a WgradDefer, dw / db may be written by its flush (nothing reads them before)."""
    if x.dtype != dz.dtype:
        raise ValueError("wgrad: x and dz dtypes differ")
    if dw.dtype != torch.float32 or not dw.is_contiguous():
        raise ValueError("wgrad: dw must be contiguous fp32")
    B, H, W, ci = x.shape
    _, Ho, Wo, co = dz.shape
    mi, mj = lattice if lattice is not None else (Ho, Wo)
    a = WgradArgs()
    a.dtype = dtype_id(x.dtype)
    a.x, a.n, a.h, a.w, a.ci, a.ldx = _dp(x), B, H, W, ci, ci
    a.dz, a.ho, a.wo, a.co, a.ldz = _dp(dz), Ho, Wo, co, co
    a.mi, a.mj, a.oy0, a.ox0, a.osy, a.osx, a.isy, a.isx = mi, mj, 0, 0, 1, 1, stride, stride
    if len(dy) > _ffi.MAX_TAPS:
        raise ValueError("wgrad: too many taps")
    a.ntaps = len(dy)
    for t, (u, v) in enumerate(zip(dy, dx)):
        a.dy[t], a.dx[t] = u, v
    a.prologue = prologue
    a.dw = _dp(dw)
    a.s_co, a.s_ci, a.s_tap = strides
    a.co_out, a.ci_out, a.accumulate = co_out, ci_out, 1 if accumulate else 0
    if db is not None:
        if db.dtype != torch.float32 or not db.is_contiguous() or db.numel() < co_out:
            raise ValueError("wgrad: db must be contiguous fp32 with co_out elements")
        a.db = _dp(db)
    need = int(_lib().lic_conv2d_wgrad_workspace(ctypes.byref(a)))
    if need < 0:
        check(_lib().lic_conv2d_wgrad(ctypes.byref(a), stream_handle()))  # raises with the reason
    ws = torch.empty((max(need, 4) // 4,), dtype=torch.float32, device=x.device)
    a.ws, a.ws_bytes = _dp(ws), need
    if deferrable and _DEFER is not None:
        ns = ctypes.c_int32(0)
        check(_lib().lic_conv2d_wgrad_partials(ctypes.byref(a), ctypes.byref(ns), stream_handle()))
        if ns.value > 0:
            _DEFER.add(a, ws, ns.value)
        return dw
    check(_lib().lic_conv2d_wgrad(ctypes.byref(a), stream_handle()))
    return dw


def channel_sum(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """Per-channel fp32 sum over all pixels of an NHWC tensor (bias gradients)."""
    x = x.contiguous()
    C = x.shape[-1]
    npix = x.numel() // C if C else 0
    if out is None:
        out = torch.empty((C,), dtype=torch.float32, device=x.device)
    ws = torch.empty((int(_lib().lic_channel_sum_workspace(C)) // 4,), dtype=torch.float32, device=x.device)
    check(_lib().lic_channel_sum(dtype_id(x.dtype), _dp(x), C, npix, C, _dp(ws), ws.numel() * 4, _dp(out),
                                 1 if accumulate else 0, stream_handle()))
    return out


def _act_fwd(z: torch.Tensor, act: int, slope: float) -> torch.Tensor:
    C = z.shape[-1]
    y = torch.empty_like(z)
    check(_lib().lic_act_fwd(dtype_id(z.dtype), _dp(z), C, z.numel() // C, C, act, slope, _dp(y), C,
                             stream_handle()))
    return y


def _act_bwd(z: torch.Tensor, dy: torch.Tensor, act: int, slope: float) -> torch.Tensor:
    C = z.shape[-1]
    dy = dy.contiguous()
    dz = torch.empty_like(z)
    check(_lib().lic_act_bwd(dtype_id(z.dtype), _dp(z), C, _dp(dy), C, z.numel() // C, C, act, slope, _dp(dz), C,
                             stream_handle()))
    return dz


def dgrad_packs(weight: torch.Tensor, stride: int, pad: Tuple[int, int, int, int], dtype: torch.dtype,
                co_pad: int):
    """ConvPacks computing dL/dx of conv2d(x, weight, stride, pad) from dz (co_pad channels) with
    lic_conv2d_fwd.  stride 1: one pack (weights transposed, taps mirrored); stride s > 1: one
    pack per output phase (ry, rx) of dx, taps with (r - d) % s == 0 at offset (r - d) // s."""
    co, ci, kh, kw = weight.shape
    pt, pl, pb, pr = pad
    if stride == 1:
        # weights transposed (a view) and taps mirrored (read backwards by the pack launch)
        return [Fn.pack_conv2d(weight.detach().transpose(0, 1), None, 1,
                               (kh - 1 - pt, kw - 1 - pl, kh - 1 - pb, kw - 1 - pr), dtype, cin_to=co_pad,
                               mirror=True)]
    s = stride
    packs = []
    wd = weight.detach()
    for ry in range(s):
        for rx in range(s):
            # the phase's taps: every s-th kernel row / column from (r + pad) mod s, row-major
            ky0, kx0 = (ry + pt) % s, (rx + pl) % s
            kys, kxs = range(ky0, kh, s), range(kx0, kw, s)
            taps = [(ky, kx) for ky in kys for kx in kxs]
            if not taps:
                continue
            cpad = Fn._cpad_for(co_pad, dtype)
            copad = Fn._choose_copad(ci)
            if wd.is_cuda and wd.dtype == torch.float32:
                # one launch per phase (re-packed every step)
                s_co, s_ci, s_y, s_x = wd.stride()
                w = Fn.pack_taps(wd, ky0 * s_y + kx0 * s_x, s_ci, s_co, s * s_y, s * s_x, ci, co, len(kys),
                                 len(kxs), copad, cpad, dtype)
            else:
                w = torch.zeros((copad, len(taps), cpad), dtype=dtype, device=weight.device)
                # one casting copy of the strided phase view (not two launches per tap)
                w[:ci, :, :co].view(ci, len(kys), len(kxs), co).copy_(
                    wd[:, :, ky0::s, kx0::s].permute(1, 2, 3, 0))
            packs.append(ConvPack(w=w, bias=None, ci=co_pad, co=ci,
                                  dy=[(ry - (ky - pt)) // s for ky, kx in taps],
                                  dx=[(rx - (kx - pl)) // s for ky, kx in taps],
                                  kh=kh, kw=kw, stride=s, phase=(ry, rx, s, s, 0)))
    return packs


def _conv_dgrad(dzp: torch.Tensor, weight: torch.Tensor, stride: int, pad, H: int, W: int) -> torch.Tensor:
    B = dzp.shape[0]
    ci = weight.shape[1]
    packs = dgrad_packs(weight, stride, pad, dzp.dtype, dzp.shape[-1])
    if stride == 1:
        return Fn.conv(Act(dzp), packs[0], out_hw=(H, W)).t
    full = len(packs) == stride * stride
    dx = (torch.empty if full else torch.zeros)((B, H, W, ci), dtype=dzp.dtype, device=dzp.device)
    out = Act(dx)
    for pk in packs:
        Fn.conv(Act(dzp), pk, out)
    return dx


# --------------------------------------------------------------------------- Conv2d
# activations whose derivative is a function of the output's sign (slope > 0): the conv applies them in
# its epilogue and the backward reads the saved output -- no separate forward activation launch
_SIGN_ACTS = (_ffi.ACT_RELU, _ffi.ACT_LRELU)


class _Conv2dFn(torch.autograd.Function):
    """y = act(conv(x) + b) [+ residual], or with res_act y = act(conv(x) + b + residual) (the conv's
    RES_ACT epilogue).  The residual add is the conv epilogue's r1 operand (one rounding instead of
    two launches); ReLU / LeakyReLU are epilogue activations whose backward reads the output's sign;
    other activations (GELU) keep the pre-activation z for their backward."""
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, act, slope, residual, res_act):
        co, ci, kh, kw = weight.shape
        if x.shape[-1] != ci:
            raise ValueError(f"conv2d: input has {x.shape[-1]} channels, weight expects {ci}")
        xp = _pad_channels(x)
        pk = Fn.pack_conv2d(weight, bias, stride, pad, x.dtype, cin_to=xp.shape[-1])
        r1 = Act(residual.contiguous()) if residual is not None else None
        if residual is not None and act != ACT_NONE and not res_act:
            raise ValueError("conv2d: an activation before the residual add is not fused (act(conv) + r)")
        if act in _SIGN_ACTS and slope > 0:
            y = Fn.conv(Act(xp), pk, act=act, slope=slope, r1=r1,
                        epi=_ffi.EPI_RES_ACT if r1 is not None else _ffi.EPI_PLAIN).t
            saved, mode = y, 1
        elif act != ACT_NONE:
            z = Fn.conv(Act(xp), pk, r1=r1).t
            y = _act_fwd(z, act, slope)
            saved, mode = z, 2
        else:
            y = Fn.conv(Act(xp), pk, r1=r1).t
            saved, mode = None, 0
        ctx.save_for_backward(xp, weight, saved)
        ctx.geom = (stride, tuple(pad), act, slope, x.shape[1], x.shape[2], bias is not None, mode)
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, weight, z = ctx.saved_tensors
        stride, pad, act, slope, H, W, has_bias, mode = ctx.geom
        co, ci, kh, kw = weight.shape
        # mode 1: z is the output (act' from its sign); 2: the pre-activation
        dz = _act_bwd(z, dy, act, slope) if mode else dy.contiguous()
        dr = dz if ctx.needs_input_grad[7] else None   # the residual sees what the conv output sees
        dzp = _pad_channels(dz)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _conv_dgrad(dzp, weight, stride, pad, H, W)
        want_db = has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            dw = torch.empty((co, ci, kh, kw), dtype=torch.float32, device=dz.device)
            tdy, tdx = _taps(kh, kw, pad[0], pad[1])
            # the bias gradient comes out of the same launch (column sums of the staged dz tiles)
            db = torch.empty((co,), dtype=torch.float32, device=dz.device) if want_db else None
            wgrad(xp, dzp, tdy, tdx, stride=stride, dw=dw, strides=(ci * kh * kw, kh * kw, 1), co_out=co,
                  ci_out=ci, db=db, deferrable=weight.dtype == torch.float32)
            dw = dw.to(weight.dtype)
        if want_db and db is None:
            db = channel_sum(dz)
        return dx, dw, db, None, None, None, None, dr, None


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
           pad=0, act: int = ACT_NONE, slope: float = 0.01, residual: Optional[torch.Tensor] = None,
           res_act: bool = False) -> torch.Tensor:
    """act(F.conv2d(x, weight, bias, stride, padding)) on NHWC; pad = int or (top, left, bottom, right)
    (asymmetric: nn.ZeroPad2d((l, r, t, b)) followed by a padding-0 conv).  residual: + residual after
    the conv (no activation), or with res_act act(conv + residual) -- one launch."""
    if isinstance(pad, int):
        pad = (pad, pad, pad, pad)
    return _Conv2dFn.apply(x, weight, bias, int(stride), tuple(pad), int(act), float(slope), residual,
                           bool(res_act))


# --------------------------------------------------------------------------- ConvTranspose2d
class _ConvT2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, output_padding, prepad, act, slope):
        ci, co, kh, kw = weight.shape
        if x.shape[-1] != ci:
            raise ValueError(f"conv_transpose2d: input has {x.shape[-1]} channels, weight expects {ci}")
        xp = _pad_channels(x)
        B, H, W, _ = x.shape
        Ho, Wo = Fn.convT_out_hw(H, W, stride, padding, output_padding, kh, prepad)
        packs = Fn.pack_conv_transpose2d(weight, bias, stride, padding, output_padding, x.dtype, prepad)
        if xp.shape[-1] != ci:  # padded input channels carry zero weights
            packs = [ConvPack(w=torch.nn.functional.pad(p.w, (0, Fn._cpad_for(xp.shape[-1], x.dtype) - p.cpad)),
                              bias=p.bias, ci=xp.shape[-1], co=p.co, dy=p.dy, dx=p.dx, kh=p.kh, kw=p.kw,
                              stride=p.stride, phase=p.phase) for p in packs]
        z = Fn.conv_transpose(Act(xp), packs, Ho, Wo).t
        y = _act_fwd(z, act, slope) if act != ACT_NONE else z
        ctx.save_for_backward(xp, weight, z if act != ACT_NONE else None)
        ctx.geom = (stride, padding, prepad, act, slope, H, W, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, weight, z = ctx.saved_tensors
        s, p, prepad, act, slope, H, W, has_bias = ctx.geom
        ci, co, kh, kw = weight.shape
        dz = _act_bwd(z, dy, act, slope) if act != ACT_NONE else dy.contiguous()
        dzp = _pad_channels(dz)
        # adjoint = conv2d(dz, weight, stride s, padding p) on the pre-padded grid; the
        # prepad rows/cols are cropped by starting the tap window s*prepad later
        pt, pl = p - s * prepad[0], p - s * prepad[1]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            pk = Fn.pack_conv2d(weight, None, s, (pt, pl, p, p), dz.dtype, cin_to=dzp.shape[-1])
            dx = Fn.conv(Act(dzp), pk, out_hw=(H, W)).t
        if ctx.needs_input_grad[1]:
            # dW[c, n, ky, kx] = sum_i x[i, c] * dz[s*i + ky - pt, n]: a conv2d weight gradient with
            # the roles of input (dz) and output gradient (x) exchanged
            dw = torch.empty((ci, co, kh, kw), dtype=torch.float32, device=dz.device)
            tdy, tdx = _taps(kh, kw, pt, pl)
            wgrad(dzp, xp, tdy, tdx, stride=s, lattice=(H, W), dw=dw, strides=(co * kh * kw, kh * kw, 1),
                  co_out=ci, ci_out=co, deferrable=weight.dtype == torch.float32)
            dw = dw.to(weight.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = channel_sum(dz)
        return dx, dw, db, None, None, None, None, None, None


def conv_transpose2d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
                     padding: int = 0, output_padding: int = 0, prepad: Tuple[int, int] = (0, 0),
                     act: int = ACT_NONE, slope: float = 0.01) -> torch.Tensor:
    """act(ConvTranspose2d(ZeroPad2d(left=prepad[1], top=prepad[0])(x))) on NHWC (net_ga.py:373-397)."""
    return _ConvT2dFn.apply(x, weight, bias, int(stride), int(padding), int(output_padding), tuple(prepad),
                            int(act), float(slope))


# --------------------------------------------------------------------------- GDN / IGDN
class _GDNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, beta, gamma, bounds, inverse, rsqrt):
        bb, gb, ped = bounds
        C = x.shape[-1]
        if C % _epc(x.dtype):
            raise ValueError("gdn: channel count must be a multiple of 16 bytes")
        x = x.contiguous()
        pk = Fn.gdn_prepare(beta, gamma, bb, gb, ped, x.dtype)
        nrm = Fn.conv(Act(x), pk, prologue=PRO_SQUARE).t           # beta' + gamma' x^2
        mode = EPI_GDN_SQRT if inverse else (EPI_GDN_RSQRT if rsqrt else EPI_GDN_DIV)
        y = Fn.gdn(Act(x), pk, mode).t
        ctx.save_for_backward(x, nrm, beta, gamma)
        ctx.cfg = (bb, gb, ped, inverse)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, nrm, beta, gamma = ctx.saved_tensors
        bb, gb, ped, inverse = ctx.cfg
        C = x.shape[-1]
        npix = x.numel() // C
        dy = dy.contiguous()
        dxd = torch.empty_like(x)
        u = torch.empty_like(x)
        dt = dtype_id(x.dtype)
        check(_lib().lic_gdn_bwd_elem(dt, _dp(x), C, _dp(nrm), C, _dp(dy), C, npix, C, 1 if inverse else 0,
                                      _dp(dxd), C, _dp(u), C, stream_handle()))
        dx = dbeta = dgamma = None
        if ctx.needs_input_grad[0]:
            pkt = Fn.gdn_prepare(beta, gamma.detach().t().contiguous(), bb, gb, ped, x.dtype)
            pkt = ConvPack(w=pkt.w, bias=None, ci=C, co=C, dy=[0], dx=[0])
            t = Fn.conv(Act(u), pkt).t                                  # gamma'^T u
            dx = torch.empty_like(x)
            check(_lib().lic_gdn_bwd_finish(dt, _dp(x), C, _dp(t), C, _dp(dxd), C, npix, C, _dp(dx), C, 0,
                                            stream_handle()))
        if ctx.needs_input_grad[1]:
            dbe = channel_sum(u)
            dbeta = torch.empty_like(beta, dtype=torch.float32)
            check(_lib().lic_lower_bound_sq_bwd(_dp(beta.detach().float().contiguous()), _dp(dbe), C, bb,
                                                _dp(dbeta), 0, stream_handle()))
        if ctx.needs_input_grad[2]:
            dge = torch.empty((C, C), dtype=torch.float32, device=x.device)
            wgrad(x, u, [0], [0], dw=dge, strides=(C, 1, 0), co_out=C, ci_out=C, prologue=PRO_SQUARE)
            dgamma = torch.empty((C, C), dtype=torch.float32, device=x.device)
            check(_lib().lic_lower_bound_sq_bwd(_dp(gamma.detach().float().contiguous()), _dp(dge), C * C, gb,
                                                _dp(dgamma), 0, stream_handle()))
        return dx, dbeta, dgamma, None, None, None


def gdn(x: torch.Tensor, beta: torch.Tensor, gamma: torch.Tensor, beta_bound: float, gamma_bound: float,
        pedestal: float, inverse: bool = False, rsqrt: bool = False) -> torch.Tensor:
    """GDN (x / sqrt(n); rsqrt=True: compressai's x * rsqrt(n)) or IGDN (x * sqrt(n)) with
    n = max(beta,bb)^2-ped + (max(gamma,gb)^2-ped) x^2, on NHWC; gradients through LowerBound."""
    return _GDNFn.apply(x, beta, gamma, (float(beta_bound), float(gamma_bound), float(pedestal)), bool(inverse),
                        bool(rsqrt))


# --------------------------------------------------------------------------- activations
class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act, slope):
        x = x.contiguous()
        ctx.save_for_backward(x)
        ctx.cfg = (act, slope)
        return _act_fwd(x, act, slope)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        act, slope = ctx.cfg
        return _act_bwd(x, dy, act, slope), None, None


def activation(x: torch.Tensor, act: int, slope: float = 0.01) -> torch.Tensor:
    return _ActFn.apply(x, int(act), float(slope))


# --------------------------------------------------------------------------- layout / elementwise
def to_nhwc(x_nchw: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Input image NCHW fp32 -> NHWC activation tensor (lic_nchw_to_nhwc); the image is a leaf."""
    return Act.from_nchw(x_nchw.detach().contiguous(), dtype).t


def _npix(t: torch.Tensor) -> int:
    return t.numel() // t.shape[-1]


def _add_raw(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    a, b = a.contiguous(), b.contiguous()
    C = a.shape[-1]
    out = torch.empty_like(a)
    check(_lib().lic_add(dtype_id(a.dtype), _dp(a), C, _dp(b), C, _npix(a), C, _dp(out), C, stream_handle()))
    return out


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return _add_raw(a, b)

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a + b (the residual adds)."""
    return _AddFn.apply(a, b)


class _GateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, b, a, r):
        b, a, r = b.contiguous(), a.contiguous(), r.contiguous()
        C = a.shape[-1]
        y = torch.empty_like(a)
        check(_lib().lic_gate_fwd(dtype_id(a.dtype), _dp(b), C, _dp(a), C, _dp(r), C, _npix(a), C, _dp(y), C,
                                  stream_handle()))
        ctx.save_for_backward(b, a)
        return y

    @staticmethod
    def backward(ctx, g):
        b, a = ctx.saved_tensors
        g = g.contiguous()
        C = a.shape[-1]
        db, da = torch.empty_like(b), torch.empty_like(a)
        check(_lib().lic_gate_bwd(dtype_id(a.dtype), _dp(b), C, _dp(a), C, _dp(g), C, _npix(a), C, _dp(db), C,
                                  _dp(da), C, stream_handle()))
        return db, da, g


def gate(b: torch.Tensor, a: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """a * sigmoid(b) + r (Win_noShift_Attention / AttentionBlock gate, layers/layers.py:105-111)."""
    return _GateFn.apply(b, a, r)


class _HalfTanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r):
        x, r = x.contiguous(), r.contiguous()
        C = x.shape[-1]
        y = torch.empty_like(r)
        check(_lib().lic_half_tanh_fwd(dtype_id(x.dtype), _dp(x), C, _dp(r), C, _npix(x), C, _dp(y), C,
                                       stream_handle()))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = g.contiguous()
        C = x.shape[-1]
        dx = torch.empty_like(x)
        check(_lib().lic_half_tanh_bwd(dtype_id(x.dtype), _dp(x), C, _dp(g), C, _npix(x), C, _dp(dx), C,
                                       stream_handle()))
        return dx, g


def half_tanh_add(x: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """r + 0.5 * tanh(x) (LRP refinement, net_ga.py:1060-1062)."""
    return _HalfTanhFn.apply(x, r)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        B, H, W, C = x.shape
        out = torch.empty((B, 1, 1, C), dtype=x.dtype, device=x.device)
        Fn.avgpool(Act(x), Act(out))
        ctx.shape = (B, H, W, C)
        return out

    @staticmethod
    def backward(ctx, g):
        B, H, W, C = ctx.shape
        g = g.contiguous()
        dx = torch.empty((B, H, W, C), dtype=g.dtype, device=g.device)
        check(_lib().lic_avgpool_bwd(dtype_id(g.dtype), _dp(g), C, B, H * W, C, _dp(dx), C, stream_handle()))
        return dx


def avgpool(x: torch.Tensor) -> torch.Tensor:
    """nn.AdaptiveAvgPool2d(1) on NHWC -> [B, 1, 1, C]."""
    return _AvgPoolFn.apply(x)


class _SteQuantFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, medians):
        return Fn.quantize_median(Act(z.contiguous()), medians).t

    @staticmethod
    def backward(ctx, g):
        return g, None


def ste_quantize(z: torch.Tensor, medians: Optional[torch.Tensor]) -> torch.Tensor:
    """ste_round(z - m) + m (net_ga.py:996-1003): rounded forward, identity gradient."""
    return _SteQuantFn.apply(z, medians)


# --------------------------------------------------------------------------- LayerNorm / attention
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x = x.contiguous()
        w = weight.detach().float().contiguous()
        y = Fn.layernorm(Act(x), w, bias.detach().float().contiguous(), eps).t
        ctx.save_for_backward(x, w)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        C = x.shape[-1]
        npix = _npix(x)
        dx = torch.empty_like(x)
        dwb = torch.empty((2 * C,), dtype=torch.float32, device=x.device)
        nbytes = int(_lib().lic_layernorm_bwd_workspace(npix, C))
        ws = torch.empty((nbytes // 4 + 1,), dtype=torch.float32, device=x.device)
        check(_lib().lic_layernorm_bwd(dtype_id(x.dtype), _dp(x), C, _dp(g), C, npix, C, _dp(w), ctx.eps, _dp(dx),
                                       C, _dp(dwb), 0, _dp(ws), nbytes, stream_handle()))
        return dx, dwb[:C], dwb[C:], None


def layernorm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float) -> torch.Tensor:
    """nn.LayerNorm(C) over the channels of every pixel (net_ga.py:115-127)."""
    return _LayerNormFn.apply(x, weight, bias, float(eps))


def _attn_args(qkv, table, C, heads, ws, shift, tab_sr, tab_sh, mask_kind, scale_after, scale):
    B, H, W, _ = qkv.shape
    a = AttnArgs()
    a.dtype = dtype_id(qkv.dtype)
    a.qkv, a.n, a.h, a.w, a.c, a.ldqkv = _dp(qkv), B, H, W, C, qkv.shape[-1]
    a.out, a.ldo = None, C
    a.heads, a.ws, a.shift = heads, ws, shift
    a.table, a.tab_sr, a.tab_sh = _dp(table), tab_sr, tab_sh
    a.mask_kind, a.scale_after, a.scale = mask_kind, 1 if scale_after else 0, scale
    a.force_valu = 0
    return a


class _WinAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, table, cfg):
        C, heads, ws, shift, tab_sr, tab_sh, mask_kind, scale_after, scale = cfg
        qkv = qkv.contiguous()
        tab = table.detach().float().contiguous()
        out = Fn.win_attn(Act(qkv), C, heads, ws, shift, tab, tab_sr, tab_sh, mask_kind, scale_after, scale).t
        ctx.save_for_backward(qkv, tab)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, g):
        qkv, tab = ctx.saved_tensors
        C = ctx.cfg[0]
        g = g.contiguous()
        a = _attn_args(qkv, tab, *ctx.cfg)
        dqkv = torch.empty_like(qkv)
        dtab = torch.empty_like(tab) if ctx.needs_input_grad[1] else None
        need = int(_lib().lic_win_attn_bwd_workspace(ctypes.byref(a)))
        ws = torch.empty((max(need, 4) // 4,), dtype=torch.float32, device=qkv.device)
        check(_lib().lic_win_attn_bwd(ctypes.byref(a), _dp(g), C, _dp(dqkv), qkv.shape[-1],
                                      _dp(dtab) if dtab is not None else None, 0, _dp(ws), need, stream_handle()))
        return dqkv, dtab, None


def win_attn(qkv: torch.Tensor, table: torch.Tensor, C: int, heads: int, ws: int, shift: int, *, tab_sr: int,
             tab_sh: int, mask_kind: int, scale_after: bool, scale: float) -> torch.Tensor:
    """Window-attention core over a [B, H, W, 3C] qkv tensor (lic_win_attn_fwd / lic_win_attn_bwd):
    WBA (layers/win_attention.py:85-116) or WMSA (model/Block_unet.py:216-252)."""
    return _WinAttnFn.apply(qkv, table, (int(C), int(heads), int(ws), int(shift), int(tab_sr), int(tab_sh),
                                         int(mask_kind), bool(scale_after), float(scale)))


# --------------------------------------------------------------------------- rate / reconstruction
class _RateTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, mu, sc, cfg):
        seed, num_pixels, sb, lb, sdev, smul = cfg
        y, mu, sc = y.contiguous(), mu.contiguous(), sc.contiguous()
        C = y.shape[-1]
        npix = _npix(y)
        nparts = int(_lib().lic_rate_train_parts(npix, C))
        parts = torch.empty((max(nparts, 1),), dtype=torch.float64, device=y.device)
        yhat = torch.empty_like(y)
        check(_lib().lic_rate_train_fwd(dtype_id(y.dtype), _dp(y), C, _dp(mu), C, _dp(sc), C, npix, C, seed,
                                        _dp(sdev) if sdev is not None else None, smul, sb, lb,
                                        _dp(yhat), C, _dp(parts), stream_handle()))
        bpp = torch.empty((), dtype=torch.float32, device=y.device)
        Fn.bpp_finalize(parts, nparts, num_pixels, bpp)
        ctx.save_for_backward(y, mu, sc)
        ctx.cfg = cfg
        return bpp, yhat

    @staticmethod
    def backward(ctx, gb, gy):
        y, mu, sc = ctx.saved_tensors
        seed, num_pixels, sb, lb, sdev, smul = ctx.cfg
        C = y.shape[-1]
        npix = _npix(y)
        if gb is None:
            gb = torch.zeros((), dtype=torch.float32, device=y.device)
        gout = gb.detach().float().reshape(1).contiguous()
        dy, dmu, dsc = torch.empty_like(y), torch.empty_like(mu), torch.empty_like(sc)
        check(_lib().lic_rate_train_bwd(dtype_id(y.dtype), _dp(y), C, _dp(mu), C, _dp(sc), C, npix, C, seed,
                                        _dp(sdev) if sdev is not None else None, smul, sb, lb,
                                        _dp(gout), -1.0 / (math.log(2.0) * num_pixels), _dp(dy), C, _dp(dmu), C,
                                        _dp(dsc), C, stream_handle()))
        if gy is not None:   # ste_round(y - mu) + mu: d/dy = 1, d/dmu = 0
            dy = _add_raw(dy, gy)
        return dy, dmu, dsc, None


def rate_train(y: torch.Tensor, mu: torch.Tensor, scale: torch.Tensor, seed: int, num_pixels: float,
               scale_bound: float = 0.11, likelihood_bound: float = 1e-9, seed_dev: Optional[torch.Tensor] = None,
               seed_mul: int = 0):
    """Training-mode GaussianConditional of one slice (net_ga.py:1049 with noise) -> (bpp contribution
    sum ln L / (-ln 2 * num_pixels) as a 0-d fp32 tensor, ste_round(y - mu) + mu).  With seed_dev (a
    1-element int64 device tensor) the noise seed is seed_dev * seed_mul + seed, read by the kernels,
    so a captured training step draws a fresh stream on every replay."""
    if seed_dev is not None and (seed_dev.dtype != torch.int64 or not seed_dev.is_cuda):
        raise ValueError("rate_train: seed_dev must be an int64 device tensor")
    return _RateTrainFn.apply(y, mu, scale, (int(seed) & (2 ** 64 - 1), float(num_pixels), float(scale_bound),
                                             float(likelihood_bound), seed_dev, int(seed_mul)))


class _ReconMSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x16, cw, img):
        x16, cw, img = x16.contiguous(), cw.contiguous(), img.contiguous()
        B, H, W, C = x16.shape
        nblk = int(_lib().lic_recon_train_blocks(H * W))
        parts = torch.empty((B * nblk,), dtype=torch.float64, device=x16.device)
        check(_lib().lic_recon_train_fwd(dtype_id(x16.dtype), _dp(x16), C, B, H * W, C, _dp(cw), cw.shape[-1],
                                         _dp(img), None, _dp(parts), stream_handle()))
        n = B * 3 * H * W
        mse = torch.empty((), dtype=torch.float32, device=x16.device)
        Fn.bpp_finalize(parts, B * nblk, -n / math.log(2.0), mse)     # = sum / n
        ctx.save_for_backward(x16, cw, img)
        return mse

    @staticmethod
    def backward(ctx, g):
        x16, cw, img = ctx.saved_tensors
        B, H, W, C = x16.shape
        nblk = int(_lib().lic_recon_train_blocks(H * W))
        gout = g.detach().float().reshape(1).contiguous()
        dx16 = torch.empty_like(x16)
        dw = torch.empty((B, 3 * C), dtype=torch.float32, device=x16.device)
        ws = torch.empty((B * nblk * 3 * C,), dtype=torch.float32, device=x16.device)
        check(_lib().lic_recon_train_bwd(dtype_id(x16.dtype), _dp(x16), C, B, H * W, C, _dp(cw), cw.shape[-1],
                                         _dp(img), _dp(gout), 2.0 / (B * 3 * H * W), _dp(dx16), C, _dp(dw), _dp(ws),
                                         ws.numel() * 4, stream_handle()))
        return dx16, dw.view(B, 1, 1, 3 * C).to(cw.dtype), None


def recon_mse(x16: torch.Tensor, cw: torch.Tensor, img: torch.Tensor) -> torch.Tensor:
    """nn.MSELoss()(tanh(batch_conv(cw, x16)), img) (net_ga.py:1089-1092, :1115); x16 NHWC, cw
    [B, 1, 1, 3*C] (row-major (3, C)), img NCHW fp32."""
    return _ReconMSEFn.apply(x16, cw, img)


# --------------------------------------------------------------------------- depthwise conv
class _DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad):
        x = x.contiguous()
        C = x.shape[-1]
        pk = Fn.pack_conv2d(weight, bias, stride, pad, x.dtype, groups=C)
        z = Fn.conv(Act(x), pk).t
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, pad, bias is not None, z.shape[1], z.shape[2])
        return z

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        stride, pad, has_bias, Ho, Wo = ctx.cfg
        B, H, W, C = x.shape
        kh, kw = weight.shape[2], weight.shape[3]
        g = g.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if stride != 1:
                raise NotImplementedError("depthwise conv backward: stride 1 only (Syntax_Model)")
            pt, pl, pb, pr = pad
            pk = Fn.pack_conv2d(weight.detach(), None, 1, (kh - 1 - pt, kw - 1 - pl, kh - 1 - pb, kw - 1 - pr),
                                g.dtype, groups=C, mirror=True)
            dx = Fn.conv(Act(g), pk, out_hw=(H, W)).t
        if ctx.needs_input_grad[1]:
            tdy, tdx = _taps(kh, kw, pad[0], pad[1])
            n = len(tdy)
            ady, adx = (ctypes.c_int8 * n)(*tdy), (ctypes.c_int8 * n)(*tdx)
            need = int(_lib().lic_dwconv_wgrad_workspace(B, Ho, Wo, C, n))
            ws = torch.empty((max(need, 4) // 4,), dtype=torch.float32, device=x.device)
            dw = torch.empty((C, 1, kh, kw), dtype=torch.float32, device=x.device)
            check(_lib().lic_dwconv_wgrad(dtype_id(x.dtype), _dp(x), C, _dp(g), C, B, H, W, Ho, Wo, C, stride, n,
                                          ctypes.cast(ady, ctypes.c_void_p), ctypes.cast(adx, ctypes.c_void_p),
                                          _dp(dw), _dp(ws), need, stream_handle()))
            dw = dw.to(weight.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            db = channel_sum(g)
        return dx, dw, db, None, None


def dwconv2d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pad) -> torch.Tensor:
    """Depthwise nn.Conv2d (groups = C) on NHWC (DepthwiseSeparableConv, UNPINNED restatement)."""
    if isinstance(pad, int):
        pad = (pad,) * 4
    return _DwConvFn.apply(x, weight, bias, int(stride), tuple(pad))
