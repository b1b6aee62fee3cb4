"""Tensor-level wrappers around liblic (NHWC activation views, packed weights).

``Act`` is an NHWC view (tensor [B, H, W, Ctot] contiguous + channel window), so
channel slices and concatenations are free: producers write straight into the
consumer's concat buffer.  All ops enqueue on the current torch stream and never
synchronise.
"""
from __future__ import annotations

import ctypes
import os
import threading
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch

from . import _ffi
from ._ffi import ConvArgs, AttnArgs, RateArgs, check

_DT = {torch.float32: _ffi.LIC_F32, torch.float16: _ffi.LIC_F16, torch.bfloat16: _ffi.LIC_BF16}


def dtype_id(dt: torch.dtype) -> int:
    try:
        return _DT[dt]
    except KeyError:
        raise _ffi.LicError(f"unsupported activation dtype {dt}; use float32, float16 or bfloat16")


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


_AUX_STREAMS = {}


def aux_stream(device, key: str) -> "torch.cuda.Stream":
    """A per-(device, key) side stream for an independent branch of a block (Win_noShift_Attention's /
    SWAtten's conv_a).  Callers fork it from the capture stream only -- one level deep: a stream forked
    from a side stream segfaults in hipGraph capture_end (tools/capture_fork_probe.py)."""
    k = (str(device), key)
    st = _AUX_STREAMS.get(k)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _AUX_STREAMS[k] = st
    return st


def chains_for(B: int) -> int:
    """How many independent image chains the analysis transform runs concurrently (LIC_CHAINS, default 1):
    half-batches on two streams, so one chain's prologue / epilogue-bound phases could overlap the other
    chain's MFMA-bound main loops (images are independent; the arithmetic per image is unchanged).  Measured
    on MI355X at B=32, 256^2 (profiles/r06/chains_ab.txt): fp16 a_model 3.813 -> 3.874 ms, fp32x6 14.097 ->
    14.008 ms -- the half-batch launches lose more than the overlap wins, so it stays an opt-in A/B."""
    n = int(os.environ.get("LIC_CHAINS", "1"))
    return n if (n > 1 and B >= 2 * n) else 1


def fork_enabled() -> bool:
    """conv_a of the 16x16-latent Win_noShift_Attention / the slice loop's mean SWAtten on a side stream
    (LIC_FORK_CONV_A=0: on the current stream, for A/B)."""
    return os.environ.get("LIC_FORK_CONV_A", "1") != "0"


def fork64_enabled() -> bool:
    """conv_a of the 64x64 Win_noShift_Attention blocks (a_model t[8], s_model t[7]) on a side stream too
    (LIC_FORK64=0: off; its launches fill the chip, so only their tails overlap: +0.9 % fp32x6, ±0 fp16)."""
    return fork_enabled() and os.environ.get("LIC_FORK64", "1") != "0"


def _lib():
    return _ffi.load()


def _dp(t: torch.Tensor) -> int:
    """Device pointer of a GPU tensor; host tensors are refused (the kernels would
    dereference a host address)."""
    if not t.is_cuda:
        raise ValueError("liblic: tensor is not on the GPU (move the module / inputs to 'cuda')")
    return t.data_ptr()


class Act:
    """NHWC activation view: channels [c0, c0 + c) of a contiguous [B, H, W, Ctot] tensor.
    ``zpad`` >= c: channels [c0 + c, c0 + zpad) are known to be zero (lets a Cin=3 layer
    run as a zero-padded Cin=8/4 MFMA convolution)."""
    __slots__ = ("t", "c0", "c", "zpad")

    def __init__(self, t: torch.Tensor, c0: int = 0, c: Optional[int] = None, zpad: Optional[int] = None):
        if t.dim() != 4 or not t.is_contiguous():
            raise ValueError("Act expects a contiguous [B, H, W, C] tensor")
        self.t = t
        self.c0 = c0
        self.c = t.shape[3] - c0 if c is None else c
        self.zpad = self.c if zpad is None else zpad

    @property
    def B(self):
        return self.t.shape[0]

    @property
    def H(self):
        return self.t.shape[1]

    @property
    def W(self):
        return self.t.shape[2]

    @property
    def ld(self):
        return self.t.shape[3]

    @property
    def npix(self):
        return self.t.shape[0] * self.t.shape[1] * self.t.shape[2]

    @property
    def ptr(self):
        return _dp(self.t) + self.c0 * self.t.element_size()

    @property
    def dtype(self):
        return self.t.dtype

    def ch(self, a: int, b: int) -> "Act":
        assert 0 <= a <= b <= self.c
        return Act(self.t, self.c0 + a, b - a)

    def batch(self, b0: int, b1: int) -> "Act":
        """Images [b0, b1) of this view (the batch is the outermost dimension: still contiguous)."""
        return Act(self.t[b0:b1], self.c0, self.c, self.zpad)

    def nchw(self) -> torch.Tensor:
        """Logical NCHW tensor (channels_last storage) of this view."""
        v = self.t[..., self.c0:self.c0 + self.c]
        return v.permute(0, 3, 1, 2)

    @staticmethod
    def empty(B, H, W, C, dtype, device) -> "Act":
        return Act(torch.empty((B, H, W, C), dtype=dtype, device=device))

    @staticmethod
    def from_nchw(x: torch.Tensor, dtype: Optional[torch.dtype] = None, pad16: bool = False) -> "Act":
        """NCHW-logical tensor -> NHWC Act (zero copy when already channels_last of the dtype).
        pad16: store pixels padded with zero channels to a 16-byte multiple (Act.zpad)."""
        dtype = dtype or x.dtype
        t = x.permute(0, 2, 3, 1)
        if t.dtype == dtype and t.is_contiguous() and not pad16:
            return Act(t)
        if x.dtype == torch.float32 and x.is_contiguous():
            B, C, H, W = x.shape
            epc = 16 // torch.empty((), dtype=dtype).element_size()
            cp = -(-C // epc) * epc if pad16 else C
            out = Act(torch.empty((B, H, W, cp), dtype=dtype, device=x.device), 0, C, cp)
            check(_lib().lic_nchw_to_nhwc(dtype_id(dtype), _dp(x), B, C, H, W, out.ptr, out.ld, cp,
                                          stream_handle()))
            return out
        return Act(t.to(dtype).contiguous())


# --------------------------------------------------------------------------- packed convolutions
@dataclass
class ConvPack:
    """One conv launch's packed weights and tap geometry."""
    w: torch.Tensor                 # [copad, ntaps, cpad] in activation dtype
    bias: Optional[torch.Tensor]    # fp32 [co]
    ci: int
    co: int
    dy: List[int]
    dx: List[int]
    groups: int = 1
    # lattice (None -> standard conv computed from stride/pad)
    stride: int = 1
    pad: Tuple[int, int, int, int] = (0, 0, 0, 0)  # top, left, bottom, right
    kh: int = 1
    kw: int = 1
    phase: Optional[Tuple[int, int, int, int, int]] = None  # (oy0, ox0, osy, osx, dummy) for convT phases

    @property
    def cpad(self):
        return self.w.shape[2]

    @property
    def copad(self):
        return self.w.shape[0]


def _choose_copad(co: int) -> int:
    best, best_cost = None, None
    for bn in (192, 128, 96, 64, 32):
        nb = -(-co // bn)
        cost = nb * bn * (1 + 0.05 * nb)
        if best_cost is None or cost < best_cost - 1e-9:
            best, best_cost = nb * bn, cost
    return best


def _cpad_for(ci: int, dtype: torch.dtype) -> int:
    bk = 32 if dtype != torch.float32 else 16
    return -(-ci // bk) * bk


def pack_taps(w: torch.Tensor, off: int, so: int, sc: int, sy: int, sx: int, no: int, nc: int, nty: int, ntx: int,
              copad: int, cpad: int, dtype: torch.dtype) -> torch.Tensor:
    """lic_pack_taps: dst[copad][nty*ntx][cpad] (dtype) with dst[o][ty*ntx+tx][c] = w[off + o*so + c*sc +
    ty*sy + tx*sx] (element offsets into w's storage view, signed strides) for o < no, c < nc, zero
    elsewhere -- one launch per pack (the training path re-packs every weight each step)."""
    if w.dtype != torch.float32:
        raise _ffi.LicError("pack_taps: fp32 weights only")
    plan = _PACK_PLAN
    key = (w.data_ptr() + 4 * off, so, sc, sy, sx, no, nc, nty, ntx, copad, cpad, dtype_id(dtype))
    if plan is not None and plan.mode == "replay":
        return plan.take(key)
    dst = torch.empty((copad, nty * ntx, cpad), dtype=dtype, device=w.device)
    check(_lib().lic_pack_taps(dtype_id(dtype), ctypes.c_void_p(key[0]), so, sc, sy, sx, no, nc,
                               nty, ntx, _dp(dst), copad, cpad, stream_handle()))
    if plan is not None and plan.mode == "record":
        plan.items.append((key, dst))
    return dst


class PackPlan:
    """A training step's weight packs as ONE launch (lic_pack_taps_batch).  Weights change only at
    the optimiser step, so every pack of a step can be written at its start.  ``record()`` around
    an eager step notes each pack_taps call (source, strides, sizes) and keeps its output buffer;
    ``finalize()`` uploads the descriptor table; then, per captured / replayed step,
    ``launch_all()`` refreshes every buffer in one launch and ``replay()`` makes pack_taps hand the
    buffers back in call order -- checking each call against the recorded one and raising on any
    difference (a different call sequence cannot silently read another layer's weights)."""

    def __init__(self):
        self.mode = None
        self.items = []
        self.i = 0
        self.desc = None
        self.nblocks = 0

    def __enter__(self):
        global _PACK_PLAN
        if _PACK_PLAN is not None:
            raise _ffi.LicError("PackPlan: another plan is active")
        _PACK_PLAN = self
        return self

    def __exit__(self, *exc):
        global _PACK_PLAN
        _PACK_PLAN = None
        mode, self.mode = self.mode, None
        if mode == "replay" and exc[0] is None and self.i != len(self.items):
            raise _ffi.LicError(f"PackPlan: step used {self.i} of {len(self.items)} recorded packs")
        return False

    def record(self) -> "PackPlan":
        self.mode, self.items = "record", []
        return self

    def replay(self) -> "PackPlan":
        if self.desc is None:
            raise _ffi.LicError("PackPlan: finalize() before replay()")
        self.mode, self.i = "replay", 0
        return self

    def take(self, key) -> torch.Tensor:
        if self.i >= len(self.items) or self.items[self.i][0] != key:
            raise _ffi.LicError(f"PackPlan: pack call {self.i} differs from the recorded step")
        self.i += 1
        return self.items[self.i - 1][1]

    def finalize(self) -> None:
        if not self.items:
            raise _ffi.LicError("PackPlan: nothing recorded")
        per = int(_lib().lic_pack_block_elems())
        rows, first = [], 0
        for key, dst in self.items:
            src, so, sc, sy, sx, no, nc, nty, ntx, copad, cpad, dt = key
            # the batch kernel reads its descriptors with 32-bit offsets and cannot check them itself
            reach = (abs(max(no - 1, 0) * so) + abs(max(nc - 1, 0) * sc) + abs((nty - 1) * sy) +
                     abs((ntx - 1) * sx))
            if max(abs(so), abs(sc), abs(sy), abs(sx), reach) >= 2 ** 31:
                raise _ffi.LicError("PackPlan: source strides / extent do not fit 32-bit offsets")
            rows.append([src, dst.data_ptr(), so, sc, sy, sx, no, nc, nty, ntx, copad, cpad, dt, first, 0, 0])
            first += -(-(copad * nty * ntx * cpad) // per)
        if first >= 2 ** 31:
            raise _ffi.LicError("PackPlan: too many blocks")
        self.desc = torch.tensor(rows, dtype=torch.int64).to(self.items[0][1].device)
        self.nblocks = first

    def launch_all(self) -> None:
        check(_lib().lic_pack_taps_batch(_dp(self.desc), len(self.items), self.nblocks, stream_handle()))


_PACK_PLAN: Optional[PackPlan] = None


def pack_conv2d(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pad, dtype: torch.dtype,
                groups: int = 1, cin_to: Optional[int] = None, cpad_to: Optional[int] = None,
                mirror: bool = False) -> ConvPack:
    """nn.Conv2d weight [co, ci/g, kh, kw] -> packed [copad][kh*kw][cpad]; pad = (top, left, bottom, right).
    cin_to: treat the input as cin_to channels (extra channels known zero; zero weights).
    cpad_to: an explicit packed channel count (>= cin; e.g. one 8-channel fp32 halo chunk).
    mirror: pack weight.flip(2, 3) (the dgrad pack), read in place on the device."""
    co, cig, kh, kw = weight.shape
    pt, pl, pb, pr = pad
    cin = cig if cin_to is None else cin_to
    # channel counts the MFMA kernel cannot take (not a multiple of one 16-byte chunk, or
    # grouped) go to the direct kernel, which wants the weights unpadded
    epc = 8 if dtype != torch.float32 else 4
    cpad = _cpad_for(cin, dtype) if (groups == 1 and cin % epc == 0) else cin
    if dtype == torch.float32 and kh * kw == 1 and groups == 1 and cpad % 32 == 16:
        # fp32 1x1 with an odd number of 16-channel chunks (the slice loop's in_conv, 240 / 336 -> 128):
        # one zero chunk more lets the fp32x6 virtual-tap tiles (two chunks per barrier) take it
        # instead of the register GEMM (40 -> ~12 us in the slice loop); zero on both sides
        cpad += 16
    if cpad_to is not None:
        if cpad_to < cin or groups != 1:
            raise ValueError("pack_conv2d: cpad_to below the channel count or grouped")
        cpad = cpad_to
    copad = _choose_copad(co)
    wd = weight.detach()
    if wd.is_cuda and wd.dtype == torch.float32:
        # one launch (padding zeros, mirror and cast included): the training path re-packs every
        # conv each step, so launches count
        so, sc, sy, sx = wd.stride()
        off = 0
        if mirror:
            off, sy, sx = (kh - 1) * sy + (kw - 1) * sx, -sy, -sx
        w = pack_taps(wd, off, so, sc, sy, sx, co, cig, kh, kw, copad, cpad, dtype)
    else:
        src = (wd.flip(2, 3) if mirror else wd).permute(0, 2, 3, 1).reshape(co, kh * kw, cig)
        w = torch.zeros((copad, kh * kw, cpad), dtype=dtype, device=weight.device)
        w[:co, :, :cig].copy_(src)
    dy = [ky - pt for ky in range(kh) for kx in range(kw)]
    dx = [kx - pl for ky in range(kh) for kx in range(kw)]
    b = bias.detach().float().contiguous() if bias is not None else None
    return ConvPack(w=w, bias=b, ci=cin * groups if cin_to is None else cin, co=co, dy=dy, dx=dx, groups=groups,
                    stride=stride, pad=(pt, pl, pb, pr), kh=kh, kw=kw)


def pack_conv_transpose2d(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, padding: int,
                          output_padding: int, dtype: torch.dtype, prepad: Tuple[int, int] = (0, 0)) -> List[ConvPack]:
    """nn.ConvTranspose2d weight [ci, co, kh, kw] (optionally after ZeroPad2d(top=prepad[0],
    left=prepad[1])) -> one ConvPack per output phase (sub-pixel decomposition, gather form)."""
    ci, co, kh, kw = weight.shape
    s, p = stride, padding
    packs = []
    wt = weight.detach()
    for ry in range(s):
        for rx in range(s):
            # a phase's taps are every s-th row / column of the kernel (ky = (ry + p) mod s, ...)
            ky0, kx0 = (ry + p) % s, (rx + p) % s
            kys, kxs = list(range(ky0, kh, s)), list(range(kx0, kw, s))
            # ascending (dy, dx) = descending (ky, kx): a unit-step grid the split kernels address at
            # compile time (conv_split_wd.hip GEO 1)
            taps = [(ky, kx) for ky in reversed(kys) for kx in reversed(kxs)]
            if not taps:
                continue
            cpad = _cpad_for(ci, dtype)
            copad = _choose_copad(co)
            if wt.is_cuda and wt.dtype == torch.float32:
                # one launch per phase: taps every s-th row / column, read backwards from the last
                s_ci, s_co, s_y, s_x = wt.stride()
                w = pack_taps(wt, kys[-1] * s_y + kxs[-1] * s_x, s_co, s_ci, -s * s_y, -s * s_x, co, ci,
                              len(kys), len(kxs), copad, cpad, dtype)
            else:
                w = torch.zeros((copad, len(taps), cpad), dtype=dtype, device=weight.device)
                # the whole phase as one strided view (not two launches per tap)
                w[:co, :, :ci].view(co, len(kys), len(kxs), ci).copy_(
                    wt[:, :, ky0::s, kx0::s].flip(2, 3).permute(1, 2, 3, 0))
            dy = [(ry + p - ky) // s - prepad[0] for ky, kx in taps]
            dx = [(rx + p - kx) // s - prepad[1] for ky, kx in taps]
            b = bias.detach().float().contiguous() if bias is not None else None
            packs.append(ConvPack(w=w, bias=b, ci=ci, co=co, dy=dy, dx=dx, kh=kh, kw=kw, stride=s,
                                  phase=(ry, rx, s, s, 0)))
    return packs


def pack_conv_transpose2d_fused(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, padding: int,
                                dtype: torch.dtype, prepad: Tuple[int, int] = (0, 0)) -> Optional[ConvPack]:
    """All s*s = 4 phases of a stride-2 nn.ConvTranspose2d as ONE conv over the union tap
    window with 4*co output channels, phase-major (n = (2*ry + rx)*co + c), stored
    sub-pixel by out_shuffle=3.  Taps a phase does not use carry zero weights.  Returns
    None when the union window is not a grid of <= LIC_MAX_TAPS taps."""
    ci, co, kh, kw = weight.shape
    s, p = stride, padding
    if s != 2:
        return None
    ymaps = [{(r + p - ky) // s - prepad[0]: ky for ky in range(kh) if (r + p - ky) % s == 0} for r in range(s)]
    xmaps = [{(r + p - kx) // s - prepad[1]: kx for kx in range(kw) if (r + p - kx) % s == 0} for r in range(s)]
    dys = sorted(set().union(*[m.keys() for m in ymaps]))
    dxs = sorted(set().union(*[m.keys() for m in xmaps]))
    if not dys or not dxs or len(dys) * len(dxs) > 64 or dys != list(range(dys[0], dys[-1] + 1)) \
            or dxs != list(range(dxs[0], dxs[-1] + 1)):
        return None
    cpad = _cpad_for(ci, dtype)
    copad = _choose_copad(4 * co)
    taps = [(dy, dx) for dy in dys for dx in dxs]
    w = torch.zeros((copad, len(taps), cpad), dtype=dtype, device=weight.device)
    wt = weight.detach()
    for ry in range(s):
        for rx in range(s):
            ph = 2 * ry + rx
            for t, (dy, dx) in enumerate(taps):
                ky, kx = ymaps[ry].get(dy), xmaps[rx].get(dx)
                if ky is not None and kx is not None:
                    w[ph * co:(ph + 1) * co, t, :ci] = wt[:, :, ky, kx].t().to(dtype)
    b = bias.detach().float().repeat(4).contiguous() if bias is not None else None
    return ConvPack(w=w, bias=b, ci=ci, co=4 * co, dy=[t[0] for t in taps], dx=[t[1] for t in taps],
                    kh=kh, kw=kw, stride=1)


def conv_out_hw(H, W, pk: ConvPack):
    pt, pl, pb, pr = pk.pad
    return (H + pt + pb - pk.kh) // pk.stride + 1, (W + pl + pr - pk.kw) // pk.stride + 1


def convT_out_hw(H, W, stride, padding, output_padding, k, prepad=(0, 0)):
    Hp, Wp = H + prepad[0], W + prepad[1]
    return (Hp - 1) * stride - 2 * padding + k + output_padding, (Wp - 1) * stride - 2 * padding + k + output_padding


def _ptr(a: Optional[Act]):
    return (a.ptr, a.ld) if a is not None else (None, 0)


# fp32 convolutions on the 16-bit matrix cores (lic_conv_args.mfma_mode, conv_halo_split.hip):
# mode 2 ("fp32x6": three bf16 parts per operand, six products, fp32 grade) while a Net with
# precision='fp32x6' runs, mode 1 ("fp32x3": fp16 parts, three products) for 'fp32x3', 0 otherwise.
# The mode is per host thread: two threads running Nets of different precisions never see each
# other's setting (tests/test_gpu_threads.py).
_SPLIT_TLS = threading.local()
SPLIT_MODES = {"fp32x3": 1, "fp32x6": 2}


def split_mode() -> int:
    """The calling thread's split MFMA mode (0 = exact fp32 products)."""
    return getattr(_SPLIT_TLS, "mode", 0)


def set_split_mode(mode: int) -> None:
    _SPLIT_TLS.mode = int(mode)


class split_f32:
    """Context: fp32 spatial-tile convolutions form their products from 16-bit parts on the
    fp16 / bf16 MFMA (include/lic.h mfma_mode).  `mode`: 0 off, 1 fp32x3, 2 fp32x6 (True = 1).
    Thread-local: it affects only convolutions launched from the thread that entered it."""

    def __init__(self, mode=1):
        self.mode = int(mode)

    def __enter__(self):
        self.prev = split_mode()
        set_split_mode(self.mode)
        return self

    def __exit__(self, *exc):
        set_split_mode(self.prev)
        return False


def _frag_order(parts: Sequence[torch.Tensor]) -> torch.Tensor:
    """[copad][ntaps][cpad] 16-bit parts -> the MFMA-fragment order of csrc/conv_split.h:
    [copad/32][cpad/16][ntaps][part][64 lanes][8], lane = 32 * (channel half) + (co % 32)."""
    co, nt, cp = parts[0].shape
    P = torch.stack(list(parts), 0).view(len(parts), co // 32, 32, nt, cp // 16, 2, 8)
    return P.permute(1, 4, 3, 0, 5, 2, 6).reshape(co // 32, cp // 16, nt, len(parts), 64, 8)


def split_weights_parts(ws: torch.Tensor) -> torch.Tensor:
    """Inverse of the fragment order: the packed split weights as [part][copad][ntaps][cpad]."""
    nt16, nch, nt, npart = ws.shape[:4]
    P = ws.view(nt16, nch, nt, npart, 2, 32, 8).permute(3, 0, 5, 2, 1, 4, 6)
    return P.reshape(npart, nt16 * 32, nt, nch * 16)


def split_weights(pk: ConvPack, mode: int = 1) -> Optional[torch.Tensor]:
    """The 16-bit split pack of an fp32 ConvPack in MFMA-fragment order (csrc/conv_split.h:
    [copad/32][cpad/16][ntaps][part][64][8]), cached on the pack:
    mode 1: fp16 parts W1 = fp16(w) * 2^11, W2 = fp16((w - fp16(w)) * 2^11); None when a weight
            is too large for W1 (|w| >= 31);
    mode 2: bf16 parts w0 = bf16(w), w1 = bf16(w - w0), w2 = bf16(w - w0 - w1) (round to nearest
            even), w = w0 + w1 + w2 exactly."""
    key = "_split%d" % mode
    sw = pk.__dict__.get(key)
    if sw is not None and sw[0] is pk.w and sw[1] == pk.w._version:
        return sw[2]
    w = pk.w
    if w.dtype != torch.float32 or w.shape[2] % 16 or w.shape[0] % 32:
        return None
    if mode == 1 and torch.cuda.is_available() and w.is_cuda and torch.cuda.is_current_stream_capturing():
        # mode 1's range check reads |w|max on the host: not possible inside a capture
        raise _ffi.LicError("split_weights: fp32x3 weight split first needed inside a hipGraph capture; "
                            "run one eager forward before capturing")
    if mode == 2:
        parts, r = [], w
        for _ in range(3):
            q = r.to(torch.bfloat16)
            parts.append(q)
            r = r - q.float()
        out = _frag_order(parts)
    elif float(w.abs().max()) >= 31.0:
        out = None
    else:
        hi = w.half()
        out = _frag_order([(hi.float() * 2048.0).half(), ((w - hi.float()) * 2048.0).half()])
    pk.__dict__[key] = (pk.w, pk.w._version, out)
    return out


_FRAG16 = os.environ.get("LIC_W16_FRAG", "1") != "0"


def frag16_weights(pk: ConvPack) -> Optional[torch.Tensor]:
    """A 16-bit pack's weights in MFMA-fragment order ([copad/32][cpad/16][ntaps][64][8]: one contiguous
    1 KB per A fragment; include/lic.h wgt_split), which the conv16 / conv16s kernels read instead of the
    [copad][ntaps][cpad] rows (32 cache lines per fragment).  Built on a pack's SECOND use with the same
    weights and never inside a hipGraph capture, so the training step -- its packs change every step --
    never pays for the copy and a capture never records it; cached on the pack."""
    w = pk.w
    if not _FRAG16 or w.dtype == torch.float32 or w.shape[0] % 32 or w.shape[2] % 16 or not w.is_cuda:
        return None
    ent = pk.__dict__.get("_frag16")
    if ent is not None and ent[0] is w and ent[1] == w._version:
        if ent[2] is not None or ent[3] < 1 or torch.cuda.is_current_stream_capturing():
            return ent[2]
        out = _frag_order([w]).contiguous()
        pk.__dict__["_frag16"] = (w, w._version, out, ent[3] + 1)
        return out
    pk.__dict__["_frag16"] = (w, w._version, None, 1)
    return None


def stride2_phase_packs(pk: ConvPack) -> Optional[List[ConvPack]]:
    """The input-parity phases of a stride-2 k x k ConvPack (k >= 3, more than 16 input channels):
    four sub-packs holding the taps whose row / column offsets share one parity (5x5: 9, 6, 6 and
    4 taps; 3x3: 4, 2, 2, 1), biased only in the first.  Each phase reads every other input row and column, so the split kernel stages a
    quarter of the stride-2 halo (conv_split_wd.hip, hsy / hsx); the four launches accumulate into
    one output (csrc/conv.hip).  Cached on the pack."""
    if pk.stride != 2 or pk.phase is not None or pk.groups != 1 or min(pk.kh, pk.kw) < 3 or pk.cpad <= 16 or \
            pk.__dict__.get("_s2phase_of") is not None:
        return None
    sub = pk.__dict__.get("_s2phases")
    if sub is not None and sub[0] is pk.w and sub[1] == pk.w._version:
        return sub[2]
    dymin, dxmin = min(pk.dy), min(pk.dx)
    packs = []
    for py in (0, 1):
        for px in (0, 1):
            idx = [t for t in range(len(pk.dy)) if (pk.dy[t] - dymin) % 2 == py and (pk.dx[t] - dxmin) % 2 == px]
            packs.append(ConvPack(w=pk.w[:, idx, :].contiguous(), bias=pk.bias if not packs else None, ci=pk.ci,
                                  co=pk.co, dy=[pk.dy[t] for t in idx], dx=[pk.dx[t] for t in idx],
                                  groups=1, stride=2, pad=pk.pad, kh=pk.kh, kw=pk.kw))
            packs[-1].__dict__["_s2phase_of"] = pk
    pk.__dict__["_s2phases"] = (pk.w, pk.w._version, packs)
    return packs


def kxk_row_packs(pk: ConvPack) -> Optional[List[ConvPack]]:
    """The kernel rows of a stride-1 7x7 ConvPack as 7 one-row sub-packs (7 taps each, biased only in
    the first), for fp32x6 on small maps (the 16x16 latents): each row runs on the weights-direct
    8x8-px tiles with an 8 x 14 halo (a 14 x 14 halo does not fit their registers / LDS), the rows
    accumulated in fp32 through the epilogue's residual operand like the stride-2 phases.  Cached."""
    if pk.stride != 1 or pk.phase is not None or pk.groups != 1 or pk.kh != 7 or pk.kw != 7 or len(pk.dy) != 49:
        return None
    sub = pk.__dict__.get("_rows")
    if sub is not None and sub[0] is pk.w and sub[1] == pk.w._version:
        return sub[2]
    packs = []
    for ky in range(7):
        idx = list(range(7 * ky, 7 * ky + 7))
        packs.append(ConvPack(w=pk.w[:, idx, :].contiguous(), bias=pk.bias if not packs else None, ci=pk.ci,
                              co=pk.co, dy=[pk.dy[t] for t in idx], dx=[pk.dx[t] for t in idx],
                              groups=1, stride=1, pad=pk.pad, kh=pk.kh, kw=pk.kw))
        packs[-1].__dict__["_s2phase_of"] = pk
    pk.__dict__["_rows"] = (pk.w, pk.w._version, packs)
    return packs


def _accumulate_subpacks(x: Act, subs: Sequence[ConvPack], out: Optional[Act], act: int, slope: float,
                         prologue: int, hw) -> Act:
    """One conv as launches of tap subsets into one fp32 output: the first adds the bias, the later
    ones add the running output as the epilogue residual, the activation goes on the last as
    RES_ACT, act(acc + b + r1)."""
    out = conv(x, subs[0], out, prologue=prologue, out_hw=hw)
    for k, ph in enumerate(subs[1:]):
        last = k == len(subs) - 2
        conv(x, ph, out, r1=out, prologue=prologue, out_hw=hw,
             act=act if last else _ffi.ACT_NONE, slope=slope,
             epi=_ffi.EPI_RES_ACT if (last and act != _ffi.ACT_NONE) else _ffi.EPI_PLAIN)
    return out


# fp32x6 stride-2 k x k convs run as input-parity phases from this many input pixels (below, the launch
# takes the exact-fp32 kernel: the hyper analysis' 3x3 s2 convs at 16x16 / 8x8).  Phases from 2048 px
# gained nothing end to end (1044.7 vs 1042.9 images/s, +9 graph nodes) and moved near-tie symbols of
# net_unet_ha_hs (profiles/r04/wd_ab.txt), so the threshold stays; A/B: LIC_S2_PHASE_MIN_PIX
_S2_PHASE_MIN_PIX = int(os.environ.get("LIC_S2_PHASE_MIN_PIX", "16384"))


def conv(x: Act, pk: ConvPack, out: Optional[Act] = None, *, act: int = _ffi.ACT_NONE, slope: float = 0.01,
         epi: int = _ffi.EPI_PLAIN, r1: Optional[Act] = None, g: Optional[Act] = None, r2: Optional[Act] = None,
         y2: Optional[Act] = None, prologue: int = _ffi.PRO_NONE, out_hw=None, shuffle: bool = False,
         force_direct: bool = False, force_generic: bool = False) -> Act:
    """Run one ConvPack launch. For convT phases `out` (full map) must be given."""
    if (split_mode() == 2 and x.dtype == torch.float32 and not (force_direct or force_generic or shuffle) and
            epi == _ffi.EPI_PLAIN and r1 is None and g is None and r2 is None and
            y2 is None and x.B * x.H * x.W >= _S2_PHASE_MIN_PIX):
        phases = stride2_phase_packs(pk)
        if phases is not None and len(phases) > 1:
            # fp32x6 stride-2 k x k conv as its four input-parity phases, accumulated in fp32 through
            # the epilogue's residual operand (the first phase adds the bias); an activation goes on
            # the last phase as RES_ACT, act(acc + b + r1): the same fp32 sum, then the activation
            hw = out_hw if out_hw is not None else conv_out_hw(x.H, x.W, pk)
            return _accumulate_subpacks(x, phases, out, act, slope, prologue, hw)
    if (split_mode() == 2 and x.dtype == torch.float32 and not (force_direct or force_generic or shuffle) and
            epi == _ffi.EPI_PLAIN and r1 is None and g is None and r2 is None and y2 is None and pk.kh == 7):
        hw = out_hw if out_hw is not None else conv_out_hw(x.H, x.W, pk)
        # the weights-direct 16x16-px tiles take 7x7 maps with >= 256 (tile, 64-channel block) pairs;
        # smaller maps (the 16x16 latents) run kernel row by kernel row on its 8x8-px tiles
        t16 = x.B * -(-hw[0] // 16) * -(-hw[1] // 16) * (pk.copad // 64)
        rows = kxk_row_packs(pk) if (t16 < 256 and min(hw) >= 8 and x.B * (hw[0] // 8) * (hw[1] // 8) *
                                     (pk.copad // 64) >= 64 and pk.ci % 16 == 0) else None
        if rows is not None:
            return _accumulate_subpacks(x, rows, out, act, slope, prologue, hw)
    if x.c != pk.ci:
        raise ValueError(f"conv: input has {x.c} channels, weights expect {pk.ci}")
    if pk.w.dtype != x.dtype:
        raise ValueError("conv: packed weight dtype != activation dtype")
    if pk.phase is None:
        Ho, Wo = out_hw if out_hw is not None else conv_out_hw(x.H, x.W, pk)
        mi, mj, oy0, ox0, osy, osx, isy, isx = Ho, Wo, 0, 0, 1, 1, pk.stride, pk.stride
    else:
        if out is None:
            raise ValueError("conv: transposed-conv phase needs the output view")
        ry, rx, s, _, _ = pk.phase
        Ho, Wo = out.H, out.W
        mi, mj = -(-(Ho - ry) // s), -(-(Wo - rx) // s)
        oy0, ox0, osy, osx, isy, isx = ry, rx, s, s, 1, 1
    mode = 0 if not shuffle else (2 if shuffle is True else int(shuffle))
    if out is None:
        if mode:
            out = Act.empty(x.B, Ho * 2, Wo * 2, pk.co // 4, x.dtype, x.t.device)
        else:
            out = Act.empty(x.B, Ho, Wo, pk.co, x.dtype, x.t.device)
    a = ConvArgs()
    a.dtype = dtype_id(x.dtype)
    a.x, a.n, a.h, a.w, a.ci, a.ldx = x.ptr, x.B, x.H, x.W, x.c, x.ld
    a.y, a.ho, a.wo, a.co, a.ldy = out.ptr, out.H, out.W, pk.co, out.ld
    if mode:
        a.ho, a.wo = out.H, out.W
    a.y2, a.ldy2 = _ptr(y2)
    a.mi, a.mj, a.oy0, a.ox0, a.osy, a.osx, a.isy, a.isx = mi, mj, oy0, ox0, osy, osx, isy, isx
    nt = len(pk.dy)
    a.ntaps = nt
    for t in range(nt):
        a.dy[t] = pk.dy[t]
        a.dx[t] = pk.dx[t]
    a.groups = pk.groups
    a.wgt, a.cpad, a.copad = _dp(pk.w), pk.cpad, pk.copad
    a.bias = _dp(pk.bias) if pk.bias is not None else None
    a.prologue, a.act, a.slope, a.epi = prologue, act, slope, epi
    a.r1, a.ldr1 = _ptr(r1)
    a.g, a.ldg = _ptr(g)
    a.r2, a.ldr2 = _ptr(r2)
    a.out_shuffle = mode
    a.force_direct = 1 if force_direct else 0
    a.force_mfma_generic = 1 if force_generic else 0
    if x.dtype != torch.float32 and pk.groups == 1:
        wf = frag16_weights(pk)
        if wf is not None:
            a.wgt_split = _dp(wf)
    smode = split_mode()
    if smode == 1 and prologue == _ffi.PRO_SQUARE:
        smode = 2   # fp32x3's fp16 parts: x^2 leaves fp16's range from |x| >= 256 (GDN) -> bf16 parts
    if smode and x.dtype == torch.float32 and pk.groups == 1:
        ws = split_weights(pk, smode)
        if ws is not None:
            a.mfma_mode, a.wgt_split = smode, _dp(ws)
    check(_lib().lic_conv2d_fwd(ctypes.byref(a), stream_handle()))
    return out


def pack_conv2d_patches(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pad, c: int,
                        dtype: torch.dtype):
    """A k x k conv on a c-channel input (the image, c = 3) as a 1x1 conv over its patch map
    (lic_patches): weights [copad][1][cpad], channel t*c + ch = w[:, ch, ky, kx] with t = ky*kw + kx,
    cpad = k*k*c rounded up to 32.  Returns (pack, dy, dx, stride)."""
    co, cig, kh, kw = weight.shape
    pt, pl = pad[0], pad[1]
    K = kh * kw * c
    cpad = -(-K // 32) * 32
    copad = _choose_copad(co)
    w = torch.zeros((copad, 1, cpad), dtype=dtype, device=weight.device)
    w[:co, 0, :K] = weight.detach()[:, :c].permute(0, 2, 3, 1).reshape(co, K).to(dtype)
    dy = [ky - pt for ky in range(kh) for kx in range(kw)]
    dx = [kx - pl for ky in range(kh) for kx in range(kw)]
    b = bias.detach().float().contiguous() if bias is not None else None
    return ConvPack(w=w, bias=b, ci=cpad, co=co, dy=[0], dx=[0]), dy, dx, stride


def patches(x: Act, dy: Sequence[int], dx: Sequence[int], stride: int, Ho: int, Wo: int, cpad: int) -> Act:
    """lic_patches: the patch map [B, Ho, Wo, cpad] of x for the taps (dy, dx) at `stride`."""
    if x.dtype != torch.float32:
        raise ValueError("patches: fp32 only")
    out = Act.empty(x.B, Ho, Wo, cpad, x.dtype, x.t.device)
    nt = len(dy)
    ady, adx = (ctypes.c_int8 * nt)(*dy), (ctypes.c_int8 * nt)(*dx)
    check(_lib().lic_patches(_ffi.LIC_F32, x.ptr, x.B, x.H, x.W, x.c, x.ld, Ho, Wo, stride, nt, ady, adx,
                             out.ptr, out.ld, cpad, stream_handle()))
    return out


_TAPS3 = ([-1, -1, -1, 0, 0, 0, 1, 1, 1], [-1, 0, 1, -1, 0, 1, -1, 0, 1])


def resunit_fusable(x: Act, p1: ConvPack, p2: ConvPack, p3: ConvPack, out: Optional[Act] = None) -> bool:
    """True when the fused fp32x6 ResidualUnit kernel (lic_resunit_fwd) takes this call: the calling
    thread is in fp32x6 mode, fp32 activations, N = 128, an 8-aligned map, aligned views, the
    three packs are conv1x1 N->N/2, conv3x3 (pad 1) N/2->N/2, conv1x1 N/2->N, and out is not x."""
    N = x.c
    if split_mode() != 2 or x.dtype != torch.float32 or N != 128 or x.H % 8 or x.W % 8:
        return False
    if x.ld % 4 or x.ptr % 16 or (out is not None and (out.ld % 4 or out.ptr % 16 or out.t.data_ptr() == x.t.data_ptr())):
        return False
    geo = ((p1, N, N // 2, 1), (p2, N // 2, N // 2, 9), (p3, N // 2, N, 1))
    for pk, ci, co, nt in geo:
        if (pk.groups != 1 or pk.stride != 1 or pk.phase is not None or pk.ci != ci or pk.co != co or
                pk.copad != co or pk.cpad != ci or len(pk.dy) != nt or pk.bias is None or pk.w.dtype != torch.float32 or
                pk.bias.data_ptr() % 16):
            return False
    return list(p1.dy) == [0] and list(p1.dx) == [0] and list(p3.dy) == [0] and list(p3.dx) == [0] and \
        list(p2.dy) == _TAPS3[0] and list(p2.dx) == _TAPS3[1]


def resunit(x: Act, p1: ConvPack, p2: ConvPack, p3: ConvPack, out: Optional[Act] = None) -> Act:
    """compressai ResidualUnit relu(conv1x1(relu(conv3x3(relu(conv1x1(x))))) + x) in one fp32x6
    launch (csrc/resunit_split.hip); callers check resunit_fusable first."""
    if not resunit_fusable(x, p1, p2, p3, out):
        raise ValueError("resunit: this call is not supported by the fused kernel (see resunit_fusable)")
    ws = [split_weights(pk, 2) for pk in (p1, p2, p3)]
    if any(w is None for w in ws):
        raise ValueError("resunit: no fp32x6 split pack")
    if out is None:
        out = Act.empty(x.B, x.H, x.W, x.c, x.dtype, x.t.device)
    a = _ffi.ResunitArgs()
    a.dtype = dtype_id(x.dtype)
    a.x, a.n, a.h, a.w, a.c, a.ldx = x.ptr, x.B, x.H, x.W, x.c, x.ld
    a.y, a.ldy = out.ptr, out.ld
    a.w1s, a.w2s, a.w3s = _dp(ws[0]), _dp(ws[1]), _dp(ws[2])
    a.b1, a.b2, a.b3 = _dp(p1.bias), _dp(p2.bias), _dp(p3.bias)
    a.mfma_mode = 2
    check(_lib().lic_resunit_fwd(ctypes.byref(a), stream_handle()))
    return out


def conv_transpose(x: Act, packs: Sequence[ConvPack], Ho: int, Wo: int, out: Optional[Act] = None, **kw) -> Act:
    if out is None:
        out = Act.empty(x.B, Ho, Wo, packs[0].co, x.dtype, x.t.device)
    for pk in packs:
        conv(x, pk, out, **kw)
    return out


# --------------------------------------------------------------------------- other ops
def gdn_prepare(beta: torch.Tensor, gamma: torch.Tensor, beta_bound: float, gamma_bound: float, pedestal: float,
                dtype: torch.dtype) -> ConvPack:
    C = beta.shape[0]
    cpad = _cpad_for(C, dtype)
    copad = _choose_copad(C)
    w = torch.empty((copad, 1, cpad), dtype=dtype, device=beta.device)
    b = torch.empty((C,), dtype=torch.float32, device=beta.device)
    check(_lib().lic_gdn_prepare(dtype_id(dtype), _dp(beta.detach().float().contiguous()),
                                 _dp(gamma.detach().float().contiguous()), C, beta_bound, gamma_bound,
                                 pedestal, _dp(w), cpad, copad, _dp(b), stream_handle()))
    return ConvPack(w=w, bias=b, ci=C, co=C, dy=[0], dx=[0])


def gdn(x: Act, pk: ConvPack, mode: int, out: Optional[Act] = None, r1: Optional[Act] = None) -> Act:
    """mode: EPI_GDN_DIV (model/gdn GDN), EPI_GDN_RSQRT (compressai GDN), EPI_GDN_SQRT (IGDN)."""
    return conv(x, pk, out, epi=mode, g=x, r1=r1, prologue=_ffi.PRO_SQUARE)


def win_attn(qkv: Act, C: int, heads: int, ws: int, shift: int, table: torch.Tensor, tab_sr: int, tab_sh: int,
             mask_kind: int, scale_after: bool, scale: float, out: Optional[Act] = None,
             force_valu: bool = False) -> Act:
    if out is None:
        out = Act.empty(qkv.B, qkv.H, qkv.W, C, qkv.dtype, qkv.t.device)
    a = AttnArgs()
    a.dtype = dtype_id(qkv.dtype)
    a.qkv, a.n, a.h, a.w, a.c, a.ldqkv = qkv.ptr, qkv.B, qkv.H, qkv.W, C, qkv.ld
    a.out, a.ldo = out.ptr, out.ld
    a.heads, a.ws, a.shift = heads, ws, shift
    a.table, a.tab_sr, a.tab_sh = _dp(table), tab_sr, tab_sh
    a.mask_kind, a.scale_after, a.scale = mask_kind, 1 if scale_after else 0, scale
    a.force_valu = 1 if force_valu else 0
    a.mfma_mode = 2 if (qkv.dtype == torch.float32 and split_mode() == 2) else 0
    check(_lib().lic_win_attn_fwd(ctypes.byref(a), stream_handle()))
    return out


def wba_qkv_attn_ok(x: Act, C: int, heads: int, ws: int) -> bool:
    """The fused fp32x6 qkv + window-attention launch applies (csrc/wba_split.hip): fp32x6, C = 192,
    8 heads, 8x8 windows, H and W multiples of 8, 16-byte aligned rows -- and a map on which the
    unfused qkv 1x1 runs on the virtual-tap split kernel (>= 64 K pixels, W >= 16,
    csrc/conv_split_wd.hip), whose arithmetic the fused launch reproduces bit for bit: the model's
    numerics do not depend on whether the fusion runs."""
    return (split_mode() == 2 and x.dtype == torch.float32 and C == 192 and heads == 8 and ws == 8 and
            x.c == C and x.H % 8 == 0 and x.W % 8 == 0 and x.W >= 16 and x.B * x.H * x.W >= 65536 and
            x.ld % 4 == 0 and x.ptr % 16 == 0)


def wba_qkv_attn(x: Act, qkv_pk: ConvPack, heads: int, ws: int, shift: int, table: torch.Tensor, tab_sr: int,
                 tab_sh: int, mask_kind: int, scale: float, out: Optional[Act] = None,
                 proj_pk: Optional[ConvPack] = None) -> Act:
    """lic_wba_qkv_attn_fwd: qkv Linear + shifted-window attention of an fp32 map in one launch
    (bit-identical to conv(x, qkv_pk) + win_attn(...) under fp32x6); returns the C-channel attention
    output that the proj Linear consumes -- or, with proj_pk, the whole block x + proj(attention)
    (bit-identical to conv(attention, proj_pk, r1=x))."""
    C = x.c
    ws2 = split_weights(qkv_pk, 2)
    if ws2 is None or qkv_pk.copad != 3 * C or qkv_pk.cpad != C or qkv_pk.bias is None:
        raise _ffi.LicError("wba_qkv_attn: the qkv pack must be an fp32 [3C][1][C] pack with a bias")
    wp = None
    if proj_pk is not None:
        wp = split_weights(proj_pk, 2)
        if wp is None or proj_pk.copad != C or proj_pk.cpad != C or proj_pk.bias is None:
            raise _ffi.LicError("wba_qkv_attn: the proj pack must be an fp32 [C][1][C] pack with a bias")
    if out is None:
        out = Act.empty(x.B, x.H, x.W, C, x.dtype, x.t.device)
    a = _ffi.WbaArgs()
    a.x, a.n, a.h, a.w, a.c, a.ldx = x.ptr, x.B, x.H, x.W, C, x.ld
    a.out, a.ldo = out.ptr, out.ld
    a.heads, a.ws, a.shift, a.mask_kind = heads, ws, shift, mask_kind
    a.scale = scale
    a.table, a.tab_sr, a.tab_sh = _dp(table), tab_sr, tab_sh
    a.qkv_wsplit, a.qkv_bias = _dp(ws2), _dp(qkv_pk.bias)
    if wp is not None:
        a.proj_wsplit, a.proj_bias = _dp(wp), _dp(proj_pk.bias)
    check(_lib().lic_wba_qkv_attn_fwd(ctypes.byref(a), stream_handle()))
    return out


def wba16_qkv_attn_ok(x: Act, C: int, heads: int, ws: int) -> bool:
    """The 16-bit fused qkv + window-attention launch applies (csrc/wba16.hip): fp16 / bf16, C = 192,
    8 heads, 8x8 windows, H and W multiples of 8, 16-byte aligned rows of 8k elements."""
    return (x.dtype in (torch.float16, torch.bfloat16) and C == 192 and heads == 8 and ws == 8 and x.c == C and
            x.H % 8 == 0 and x.W % 8 == 0 and x.ld % 8 == 0 and x.ptr % 16 == 0)


def wba16_qkv_attn(x: Act, qkv_pk: ConvPack, heads: int, ws: int, shift: int, table: torch.Tensor, tab_sr: int,
                   tab_sh: int, mask_kind: int, scale: float, out: Optional[Act] = None) -> Act:
    """lic_wba16_qkv_attn_fwd: qkv Linear + shifted-window attention of a 16-bit map in one launch
    (the arithmetic of conv(x, qkv_pk) + win_attn(...): q, k, v rounded to the 16-bit type after the
    bias); returns the C-channel attention output that the proj Linear consumes."""
    C = x.c
    if (qkv_pk.w.dtype != x.dtype or qkv_pk.copad != 3 * C or qkv_pk.cpad != C or qkv_pk.bias is None or
            len(qkv_pk.dy) != 1 or qkv_pk.co != 3 * C):
        raise _ffi.LicError("wba16_qkv_attn: the qkv pack must be a [3C][1][C] pack of the input's dtype with a bias")
    if out is None:
        out = Act.empty(x.B, x.H, x.W, C, x.dtype, x.t.device)
    a = _ffi.Wba16Args()
    a.dtype = dtype_id(x.dtype)
    a.x, a.n, a.h, a.w, a.c, a.ldx = x.ptr, x.B, x.H, x.W, C, x.ld
    a.out, a.ldo = out.ptr, out.ld
    a.heads, a.ws, a.shift, a.mask_kind = heads, ws, shift, mask_kind
    a.scale = scale
    a.table, a.tab_sr, a.tab_sh = _dp(table), tab_sr, tab_sh
    a.qkv_w, a.qkv_bias = _dp(qkv_pk.w), _dp(qkv_pk.bias)
    check(_lib().lic_wba16_qkv_attn_fwd(ctypes.byref(a), stream_handle()))
    return out


def layernorm(x: Act, weight: torch.Tensor, bias: torch.Tensor, eps: float, out: Optional[Act] = None) -> Act:
    if out is None:
        out = Act.empty(x.B, x.H, x.W, x.c, x.dtype, x.t.device)
    check(_lib().lic_layernorm_fwd(dtype_id(x.dtype), x.ptr, x.npix, x.c, x.ld, _dp(weight), _dp(bias),
                                   eps, out.ptr, out.ld, stream_handle()))
    return out


def rb3(x: Act, params: torch.Tensor, out: Optional[Act] = None) -> Act:
    """Fused ResidualBottleneck(3); the output pixels are zero-padded to 16 bytes (Act.zpad)."""
    if x.c != 3:
        raise ValueError("rb3 expects a 3-channel view")
    if out is None:
        epc = 16 // x.t.element_size()
        out = Act(torch.empty((x.B, x.H, x.W, epc), dtype=x.dtype, device=x.t.device), 0, 3, epc)
    check(_lib().lic_rb3_fwd(dtype_id(x.dtype), x.ptr, x.B, x.H, x.W, x.ld, _dp(params), out.ptr, out.ld,
                             stream_handle()))
    return out


def rb3_chain(x: Act, params: torch.Tensor, nblk: int, out: Optional[Act] = None) -> Act:
    """nblk consecutive fused ResidualBottleneck(3) blocks in one launch (params: nblk x 20 fp32);
    equals nblk rb3() calls.  The output pixels are zero-padded to 16 bytes (Act.zpad)."""
    if x.c != 3:
        raise ValueError("rb3_chain expects a 3-channel view")
    if params.numel() != 20 * nblk or params.dtype != torch.float32 or not params.is_contiguous():
        raise ValueError("rb3_chain: params must be nblk x 20 contiguous fp32")
    if out is None:
        epc = 16 // x.t.element_size()
        out = Act(torch.empty((x.B, x.H, x.W, epc), dtype=x.dtype, device=x.t.device), 0, 3, epc)
    check(_lib().lic_rb3_chain_fwd(dtype_id(x.dtype), x.ptr, x.B, x.H, x.W, x.ld, _dp(params), nblk, out.ptr,
                                   out.ld, stream_handle()))
    return out


def add(a: Act, b: Act, out: Optional[Act] = None) -> Act:
    if out is None:
        out = Act.empty(a.B, a.H, a.W, a.c, a.dtype, a.t.device)
    check(_lib().lic_add(dtype_id(a.dtype), a.ptr, a.ld, b.ptr, b.ld, a.npix, a.c, out.ptr, out.ld, stream_handle()))
    return out


def copy(x: Act, out: Act) -> Act:
    check(_lib().lic_copy(dtype_id(x.dtype), x.ptr, x.ld, x.npix, x.c, dtype_id(out.dtype), out.ptr, out.ld,
                          stream_handle()))
    return out


def avgpool(x: Act, out: Act) -> Act:
    """AdaptiveAvgPool2d(1): out is a [B, 1, 1, C] view."""
    check(_lib().lic_avgpool(dtype_id(x.dtype), x.ptr, x.B, x.H * x.W, x.c, x.ld, out.ptr, out.ld,
                             stream_handle()))
    return out


def quantize_median(z: Act, medians: Optional[torch.Tensor], out: Optional[Act] = None) -> Act:
    if out is None:
        out = Act.empty(z.B, z.H, z.W, z.c, z.dtype, z.t.device)
    check(_lib().lic_quantize_median(dtype_id(z.dtype), z.ptr, z.npix, z.c, z.ld,
                                     _dp(medians) if medians is not None else None,
                                     out.ptr, out.ld, stream_handle()))
    return out


def gauss_rate(y: Act, mu: Act, scale: Act, partials: torch.Tensor, part_off: int, *, yq: Optional[Act] = None,
               yq2: Optional[Act] = None, symbols: Optional[Act] = None, likelihood: Optional[Act] = None,
               scale_bound: float = 0.11, likelihood_bound: float = 1e-9) -> int:
    """Returns the number of partials written at partials[part_off:]."""
    a = RateArgs()
    a.dtype = dtype_id(y.dtype)
    a.npix, a.c = y.npix, y.c
    a.y, a.ldy = y.ptr, y.ld
    a.mu, a.ldmu = mu.ptr, mu.ld
    a.scale, a.ldsc = scale.ptr, scale.ld
    a.yq, a.ldyq = _ptr(yq)
    a.yq2, a.ldyq2 = _ptr(yq2)
    a.symbols, a.ldsym = _ptr(symbols)
    a.likelihood, a.ldlik = _ptr(likelihood)
    n = -(-(y.npix * y.c) // 256)
    if part_off + n > partials.numel():
        raise ValueError("gauss_rate: partials buffer too small")
    a.partials = _dp(partials) + part_off * 8
    a.max_parts = partials.numel() - part_off
    a.scale_bound, a.likelihood_bound = scale_bound, likelihood_bound
    check(_lib().lic_gauss_rate_fwd(ctypes.byref(a), stream_handle()))
    return n


def rate_noise_parts(npix: int, c: int) -> int:
    return int(_lib().lic_rate_train_parts(npix, c))


def rate_noise(y: Act, mu: Act, scale: Act, seed: int, partials: torch.Tensor, part_off: int,
               scale_bound: float = 0.11, likelihood_bound: float = 1e-9) -> int:
    """compressai GaussianConditional.forward in its default (training) mode, as the reference's
    eval runs it (the net is never put in eval(), net_ga.py:1049, eval_net.py:90-96): the
    likelihood of y + U(-1/2, 1/2), with the counter-based noise of lic_rate_train_fwd
    (seed, logical element index of the view).  Writes sum ln L partials at partials[part_off:]
    and returns their count; y_hat / symbols are not touched (gauss_rate writes them)."""
    n = rate_noise_parts(y.npix, y.c)
    if part_off + n > partials.numel():
        raise ValueError("rate_noise: partials buffer too small")
    check(_lib().lic_rate_train_fwd(dtype_id(y.dtype), y.ptr, y.ld, mu.ptr, mu.ld, scale.ptr, scale.ld, y.npix, y.c,
                                    int(seed) & 0xFFFFFFFFFFFFFFFF, None, 0, scale_bound, likelihood_bound, None, 0,
                                    _dp(partials) + part_off * 8, stream_handle()))
    return n


def bpp_finalize(partials: torch.Tensor, nparts: int, num_pixels: float, out: torch.Tensor,
                 sum_out: Optional[torch.Tensor] = None):
    check(_lib().lic_bpp_finalize(_dp(partials), nparts, float(num_pixels), _dp(out),
                                  _dp(sum_out) if sum_out is not None else None, stream_handle()))


def syntax_recon(xtil: Act, wgen: Act, x: torch.Tensor, x_rec: torch.Tensor, parts: torch.Tensor,
                 parts_per_img: int):
    B, _, H, W = x.shape
    check(_lib().lic_syntax_recon_fwd(dtype_id(xtil.dtype), xtil.ptr, B, H, W, xtil.c, xtil.ld, wgen.ptr, wgen.ld,
                                      _dp(x), _dp(x_rec), _dp(parts), parts_per_img,
                                      stream_handle()))


def psnr_finalize(parts: torch.Tensor, B: int, parts_per_img: int, count: float, v_mse: torch.Tensor,
                  v_psnr: torch.Tensor):
    check(_lib().lic_psnr_finalize(_dp(parts), B, parts_per_img, float(count), _dp(v_mse),
                                   _dp(v_psnr), stream_handle()))


def to_nchw_f32(x: Act) -> torch.Tensor:
    out = torch.empty((x.B, x.c, x.H, x.W), dtype=torch.float32, device=x.t.device)
    check(_lib().lic_nhwc_to_nchw(dtype_id(x.dtype), x.ptr, x.B, x.H, x.W, x.c, x.ld, _dp(out),
                                  stream_handle()))
    return out


# --------------------------------------------------------------------------- HAN glue (8(f) rank 3)
def pool_partials(x: Act, nchunk: int, parts: torch.Tensor) -> torch.Tensor:
    """Per-(image, pixel chunk) fp32 channel sums (the first pass of an average pool)."""
    if parts.numel() < x.B * nchunk * x.c or parts.dtype != torch.float32:
        raise ValueError("pool_partials: parts must be fp32 with B * nchunk * C entries")
    check(_lib().lic_pool_partials(dtype_id(x.dtype), x.ptr, x.ld, x.B, x.H * x.W, x.c, nchunk, _dp(parts),
                                   stream_handle()))
    return parts


def ca_apply(r: Act, x: Act, parts: torch.Tensor, nchunk: int, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
             b2: torch.Tensor, out: Optional[Act] = None) -> Act:
    """out = r * sigmoid(W2 relu(W1 mean(r) + b1) + b2) + x (CALayer + RCAB residual)."""
    if out is None:
        out = Act.empty(r.B, r.H, r.W, r.c, r.dtype, r.t.device)
    if parts.numel() < r.B * (nchunk + 1) * r.c:
        raise ValueError("ca_apply: parts must hold B * (nchunk + 1) * C floats")
    cr = w1.shape[0]
    check(_lib().lic_ca_apply_fwd(dtype_id(r.dtype), r.ptr, r.ld, x.ptr, x.ld, r.B, r.H * r.W, r.c, _dp(parts),
                                  nchunk, _dp(w1), _dp(b1), _dp(w2), _dp(b2), cr, out.ptr, out.ld,
                                  stream_handle()))
    return out


def lam(x: Act, ngroups: int, gamma: torch.Tensor, out: Optional[Act] = None) -> Act:
    """LAM_Module over `ngroups` channel windows of x.c // ngroups channels."""
    C = x.c // ngroups
    if out is None:
        out = Act.empty(x.B, x.H, x.W, x.c, x.dtype, x.t.device)
    parts = torch.empty((x.B * int(_lib().lic_lam_parts(ngroups)),), dtype=torch.float64, device=x.t.device)
    check(_lib().lic_lam_fwd(dtype_id(x.dtype), x.ptr, x.ld, x.B, x.H * x.W, ngroups, C, _dp(parts), _dp(gamma),
                             out.ptr, out.ld, stream_handle()))
    return out


def csam(x: Act, params: torch.Tensor, out: Optional[Act] = None) -> Act:
    """CSAM_Module; params = fp32 [w(27), bias, gamma] on the device."""
    if out is None:
        out = Act.empty(x.B, x.H, x.W, x.c, x.dtype, x.t.device)
    check(_lib().lic_csam_fwd(dtype_id(x.dtype), x.ptr, x.ld, x.B, x.H, x.W, x.c, _dp(params), out.ptr, out.ld,
                              stream_handle()))
    return out


def recon(xtil: Act, wgen: Act, mode: int, post: Optional[torch.Tensor] = None, x: Optional[torch.Tensor] = None,
          x_rec: Optional[torch.Tensor] = None, parts: Optional[torch.Tensor] = None, ppi: int = 1,
          y: Optional[Act] = None):
    """Batch-conv reconstruction head (lic_recon_fwd): mode 1 = tanh, 0 = linear; post = 1x1 3->3."""
    B, H, W = xtil.B, xtil.H, xtil.W
    check(_lib().lic_recon_fwd(dtype_id(xtil.dtype), xtil.ptr, B, H, W, xtil.c, xtil.ld, wgen.ptr, wgen.ld, mode,
                               _dp(post) if post is not None else None, _dp(x) if x is not None else None,
                               _dp(x_rec) if x_rec is not None else None, _dp(parts) if parts is not None else None,
                               ppi, y.ptr if y is not None else None, y.ld if y is not None else 0,
                               y.zpad if y is not None else 0, stream_handle()))
