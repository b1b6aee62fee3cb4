"""Entropy coder on the HIP path: CDF tables + Rans64 streams.

The reference never writes a bitstream — it only estimates the rate with compressai's
entropy models (net_ga.py:1049 GaussianConditional, :996-1003 EntropyBottleneck,
bpp at :1104-1107).  This module is the coder those models imply (compressai 1.2.x,
unvendored; see include/lic.h): ``update()``-style CDF tables built on the device
(liblic ``lic_gauss_pmf`` / ``lic_eb_pmf`` + ``lic_pmf_to_cdf``) and one Rans64 string
per (image, channel) stream (``lic_rans_encode`` / ``lic_rans_pack`` /
``lic_rans_decode``).  Only table metadata (centers, lengths: a few hundred integers)
is computed with torch on the host; every per-symbol step runs in liblic.

Per-image string (the element of compressai's ``strings`` lists):
    uint32 C, uint32 words[C] (stream lengths), then the C streams' uint32 words.
"""
from __future__ import annotations

import ctypes
import statistics
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _ffi
from ._ffi import RansArgs, check
from .functional import Act, _dp, _lib, dtype_id, stream_handle

PRECISION = 16


def get_scale_table(min_: float = 0.11, max_: float = 256, levels: int = 64) -> torch.Tensor:
    """compressai.models.utils.get_scale_table (CompressionModel.update's default)."""
    import math
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))


@dataclass
class CoderTables:
    """Device CDF tables in compressai's layout: cdf [T, stride] int32, sizes [T]
    (= pmf length + 2), offsets [T] (symbol value of entry 0)."""
    cdf: torch.Tensor
    sizes: torch.Tensor
    offsets: torch.Tensor
    status: torch.Tensor

    @property
    def ncdf(self):
        return self.cdf.shape[0]

    @property
    def stride(self):
        return self.cdf.shape[1]

    def check(self):
        bad = int((self.status != 0).sum())
        if bad:
            raise _ffi.LicError(f"{bad} CDF tables could not be quantized (degenerate pmf)")
        return self


def _pmf_to_cdf(pmf: torch.Tensor, nsym: torch.Tensor, sizes, offsets) -> CoderTables:
    T, stride = pmf.shape
    dev = pmf.device
    cdf = torch.zeros((T, stride + 1), dtype=torch.int32, device=dev)
    status = torch.empty((T,), dtype=torch.int32, device=dev)
    check(_lib().lic_pmf_to_cdf(_dp(pmf), _dp(nsym), T, stride, PRECISION, _dp(cdf), stride + 1, _dp(status),
                                stream_handle()))
    return CoderTables(cdf, sizes.to(dev, torch.int32).contiguous(), offsets.to(dev, torch.int32).contiguous(),
                       status)


def gauss_tables(scale_table: torch.Tensor, tail_mass: float = 1e-9) -> CoderTables:
    """GaussianConditional.update(): tables for every entry of the scale table."""
    dev = scale_table.device
    st = scale_table.detach().float().cpu()
    multiplier = -statistics.NormalDist().inv_cdf(tail_mass / 2)
    center = torch.ceil(st * multiplier).int()
    length = 2 * center + 1
    stride = int(length.max()) + 1
    pmf = torch.zeros((len(st), stride), dtype=torch.float32, device=dev)
    st_d = st.to(dev).contiguous()
    center_d = center.to(dev).contiguous()
    check(_lib().lic_gauss_pmf(_dp(st_d), _dp(center_d), len(st), stride, _dp(pmf), stream_handle()))
    nsym = (length + 1).to(dev).contiguous()
    return _pmf_to_cdf(pmf, nsym, length + 2, -center)


_EB_ORDER = ([f"_matrix{i}" for i in range(5)] + [f"_bias{i}" for i in range(5)] +
             [f"_factor{i}" for i in range(4)])


def eb_tables(eb) -> Tuple[CoderTables, torch.Tensor]:
    """EntropyBottleneck.update() for the default filters (3, 3, 3, 3): (tables, medians [C] fp32)."""
    if tuple(eb.filters) != (3, 3, 3, 3):
        raise _ffi.LicError("lic_eb_pmf supports EntropyBottleneck filters (3, 3, 3, 3) only")
    q = eb.quantiles.detach().float()
    dev = q.device
    qc = q.cpu()
    medians = qc[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - qc[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(qc[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    length = maxima + minima + 1
    C = q.shape[0]
    params = torch.cat([getattr(eb, n).detach().float().reshape(C, -1) for n in _EB_ORDER], 1).contiguous()
    assert params.shape[1] == _ffi.LIC_EB_PARAMS
    stride = int(length.max()) + 1
    pmf = torch.zeros((C, stride), dtype=torch.float32, device=dev)
    ps, ln = pmf_start.to(dev).contiguous(), length.to(dev, torch.int32).contiguous()
    check(_lib().lic_eb_pmf(_dp(params.to(dev)), _dp(ps), _dp(ln), C, stride, _dp(pmf), stream_handle()))
    nsym = (length + 1).to(dev, torch.int32).contiguous()
    return _pmf_to_cdf(pmf, nsym, length + 2, -minima), medians.to(dev).contiguous()


def gauss_indexes(scales: Act, scale_table: torch.Tensor, bound: float, out: Act):
    """GaussianConditional.build_indexes on the device (out: int32 Act)."""
    check(_lib().lic_gauss_indexes(dtype_id(scales.dtype), scales.ptr, scales.npix, scales.c, scales.ld,
                                   _dp(scale_table), scale_table.numel(), float(bound), out.ptr, out.ld,
                                   stream_handle()))


def quantize_symbols(z: Act, medians: Optional[torch.Tensor], out: Act):
    check(_lib().lic_quantize_symbols(dtype_id(z.dtype), z.ptr, z.npix, z.c, z.ld,
                                      _dp(medians) if medians is not None else None, out.ptr, out.ld,
                                      stream_handle()))


def _args(tab: CoderTables, n, hw, c, ctot, c0) -> RansArgs:
    a = RansArgs()
    a.n, a.hw, a.c, a.ctot, a.c0 = n, hw, c, ctot, c0
    a.cdfs, a.cdf_stride = _dp(tab.cdf), tab.stride
    a.cdf_sizes, a.offsets, a.ncdf = _dp(tab.sizes), _dp(tab.offsets), tab.ncdf
    return a


def encode_streams(sym: Act, idx: Optional[Act], tab: CoderTables) -> Tuple[torch.Tensor, torch.Tensor]:
    """All (image, channel) streams of an int32 symbol view -> (words [cap*nstreams] int32
    device buffer, offsets_w [nstreams+1] int32 device); stream s = b*C + ch."""
    B, H, W, C = sym.B, sym.H, sym.W, sym.c
    hw, ns = H * W, B * C
    dev = sym.t.device
    cap = int(_lib().lic_rans_cap(hw))
    scratch = torch.empty((ns, cap), dtype=torch.int32, device=dev)
    lengths = torch.empty((ns,), dtype=torch.int32, device=dev)
    a = _args(tab, B, hw, C, C, 0)
    a.symbols, a.ldsym = sym.ptr, sym.ld
    if idx is not None:
        a.indexes, a.ldidx = idx.ptr, idx.ld
    a.scratch, a.cap, a.lengths = _dp(scratch), cap, _dp(lengths)
    check(_lib().lic_rans_encode(ctypes.byref(a), stream_handle()))
    offsets = torch.empty((ns + 1,), dtype=torch.int32, device=dev)
    words = torch.empty((ns * cap,), dtype=torch.int32, device=dev)
    # a failed stream reports -1; pack only after checking (the scan needs lengths >= 0)
    if int(lengths.min()) < 0:
        raise _ffi.LicError("rans encode: a stream overflowed or used an invalid table index")
    check(_lib().lic_rans_pack(_dp(scratch), cap, _dp(lengths), ns, _dp(offsets), _dp(words), stream_handle()))
    return words, offsets


def decode_streams(words: torch.Tensor, offsets: torch.Tensor, tab: CoderTables, B: int, hw: int, ctot: int,
                   c0: int, c: int, idx: Optional[Act] = None, yq: Optional[Act] = None,
                   mu: Optional[Act] = None, mu_ch: Optional[torch.Tensor] = None,
                   symbols: Optional[Act] = None, status: Optional[torch.Tensor] = None):
    """Decode the streams of channels [c0, c0+c) of every image; writes symbols and/or
    yq = symbol + mean (per-element ``mu`` or per-channel ``mu_ch``)."""
    a = _args(tab, B, hw, c, ctot, c0)
    a.words, a.offsets_w = _dp(words), _dp(offsets)
    if idx is not None:
        a.indexes, a.ldidx = idx.ptr, idx.ld
    dt = yq.dtype if yq is not None else (mu.dtype if mu is not None else torch.float32)
    a.dtype = dtype_id(dt)
    if symbols is not None:
        a.out_symbols, a.ldosym = symbols.ptr, symbols.ld
    if mu is not None:
        a.mu, a.ldmu = mu.ptr, mu.ld
    if mu_ch is not None:
        a.mu_ch = _dp(mu_ch)
    if yq is not None:
        a.yq, a.ldyq = yq.ptr, yq.ld
    if status is not None:
        if status.numel() < B * c:
            raise ValueError("decode_streams: status needs B*c entries")
        a.status = _dp(status)
    check(_lib().lic_rans_decode(ctypes.byref(a), stream_handle()))


# ------------------------------------------------------------------ per-image strings
def to_strings(words: torch.Tensor, offsets: torch.Tensor, B: int, C: int) -> List[bytes]:
    """Device streams -> one bytes string per image (header + words)."""
    off = offsets.cpu().numpy().astype(np.int64)
    total = int(off[-1])
    w = words[:total].cpu().numpy().view(np.uint32)
    out = []
    for b in range(B):
        lo, hi = off[b * C], off[(b + 1) * C]
        lens = np.diff(off[b * C:(b + 1) * C + 1]).astype(np.uint32)
        out.append(np.uint32(C).tobytes() + lens.tobytes() + w[lo:hi].tobytes())
    return out


def from_strings(strings: Sequence[bytes], C: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Inverse of to_strings: (words int32 device, offsets_w int32 device [B*C+1])."""
    ws, lens = [], []
    for s in strings:
        a = np.frombuffer(s, dtype=np.uint32)
        if len(a) < 1 or int(a[0]) != C or len(a) < 1 + C:
            raise ValueError("bitstream header does not match the latent's channel count")
        ln = a[1:1 + C].astype(np.int64)
        body = a[1 + C:]
        if int(ln.sum()) != len(body):
            raise ValueError("bitstream truncated or corrupt (stream lengths do not add up)")
        lens.append(ln)
        ws.append(body)
    ln = np.concatenate(lens) if lens else np.zeros(0, np.int64)
    off = np.zeros(len(ln) + 1, dtype=np.int64)
    np.cumsum(ln, out=off[1:])
    if off[-1] >= 2 ** 31:
        raise ValueError("bitstream too large")
    words = torch.from_numpy(np.concatenate(ws).view(np.int32).copy() if ws else np.zeros(0, np.int32))
    return words.to(device), torch.from_numpy(off.astype(np.int32)).to(device)
