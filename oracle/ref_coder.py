"""TEST INFRASTRUCTURE ONLY — CPU oracle of the entropy coder.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, as the checker of the HIP coder (csrc/rans.hip).

The reference has no coder (it estimates the rate only: net_ga.py:1049, :1104-1107);
its entropy models are compressai's (unvendored, unpinned >= 1.1).
This module restates compressai 1.2.x:
  * get_scale_table / GaussianConditional.update   (entropy_models.py) -> gauss_tables
  * EntropyBottleneck.update / _logits_cumulative   (entropy_models.py) -> eb_tables
  * pmf_to_quantized_cdf, encode/decode_with_indexes -> oracle/rans_ref.c (ctypes)
in fp32 torch CPU ops, as compressai computes them.  Parity with compressai itself
is UNPINNED (no fixtures exist); tests pin this restatement by known answers and
round trips, and the HIP coder bit-exactly against it.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Dict, List, Tuple

import numpy as np
import scipy.stats
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "librans_ref.so")
PRECISION = 16
TAIL_MASS = 1e-9
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "librans_ref.so"], check=True, capture_output=True)
        L = ctypes.CDLL(LIB)
        P, I = ctypes.c_void_p, ctypes.c_int
        L.ref_pmf_to_quantized_cdf.argtypes = [P, I, I, P]
        L.ref_rans_encode.argtypes = [P, P, I, P, I, P, P, I, P, I, P]
        L.ref_rans_decode.argtypes = [P, I, P, I, P, I, P, P, I, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def pmf_to_quantized_cdf(pmf: List[float], precision: int = PRECISION) -> np.ndarray:
    """compressai ops.cpp pmf_to_quantized_cdf (input: pmf entries + tail mass)."""
    p = np.ascontiguousarray(np.asarray(pmf, dtype=np.float32))
    cdf = np.zeros(len(p) + 1, dtype=np.uint32)
    if lib().ref_pmf_to_quantized_cdf(_p(p), len(p), precision, _p(cdf)) != 0:
        raise ValueError("pmf_to_quantized_cdf: no frequency to steal")
    return cdf.astype(np.int32)


def get_scale_table(min_: float = 0.11, max_: float = 256, levels: int = 64) -> torch.Tensor:
    """compressai.models.utils get_scale_table."""
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))


def _standardized_cumulative(x: torch.Tensor) -> torch.Tensor:
    half = float(0.5)
    const = float(-(2 ** -0.5))
    return half * torch.erfc(const * x)


def gauss_pmfs(scale_table: torch.Tensor, tail_mass: float = TAIL_MASS):
    """GaussianConditional.update(): (pmf [T, max_length], tail [T, 1], pmf_length [T], pmf_center [T])."""
    multiplier = -scipy.stats.norm.ppf(tail_mass / 2)
    pmf_center = torch.ceil(scale_table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = torch.max(pmf_length).item()
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None])
    samples_scale = scale_table.unsqueeze(1)
    samples = samples.float()
    upper = _standardized_cumulative((0.5 - samples) / samples_scale)
    lower = _standardized_cumulative((-0.5 - samples) / samples_scale)
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    return pmf, tail, pmf_length, pmf_center


def tables_from_pmf(pmf: torch.Tensor, tail: torch.Tensor, pmf_length: torch.Tensor, offsets: torch.Tensor):
    """_pmf_to_quantized_cdf + the (cdf [T, max_length+2], cdf_sizes, offsets) triple."""
    T = pmf.shape[0]
    max_length = int(pmf_length.max())
    cdf = np.zeros((T, max_length + 2), dtype=np.int32)
    for i in range(T):
        prob = torch.cat((pmf[i, : int(pmf_length[i])], tail[i]), dim=0)
        c = pmf_to_quantized_cdf(prob.tolist())
        cdf[i, : len(c)] = c
    return cdf, (pmf_length + 2).numpy().astype(np.int32), offsets.numpy().astype(np.int32)


def gauss_tables(scale_table: torch.Tensor = None):
    st = get_scale_table() if scale_table is None else scale_table
    pmf, tail, length, center = gauss_pmfs(st)
    return tables_from_pmf(pmf, tail, length, -center)


def eb_logits_cumulative(P: Dict[str, torch.Tensor], prefix: str, inputs: torch.Tensor, nfilters: int = 4):
    """EntropyBottleneck._logits_cumulative (inputs [C, 1, N])."""
    logits = inputs
    for i in range(nfilters + 1):
        matrix = torch.nn.functional.softplus(P[f"{prefix}_matrix{i:d}"])
        logits = torch.matmul(matrix, logits)
        logits = logits + P[f"{prefix}_bias{i:d}"]
        if i < nfilters:
            factor = torch.tanh(P[f"{prefix}_factor{i:d}"])
            logits = logits + factor * torch.tanh(logits)
    return logits


def eb_pmfs(P: Dict[str, torch.Tensor], prefix: str = "entropy_bottleneck."):
    """EntropyBottleneck.update(): (pmf [C, max_length], tail [C, 1], pmf_length, offsets, medians)."""
    q = P[prefix + "quantiles"]
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = pmf_length.max().item()
    samples = torch.arange(max_length)
    samples = samples[None, :] + pmf_start[:, None, None]
    half = float(0.5)
    lower = eb_logits_cumulative(P, prefix, samples - half)
    upper = eb_logits_cumulative(P, prefix, samples + half)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    pmf = pmf[:, 0, :]
    tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    return pmf, tail, pmf_length, -minima, medians


def eb_tables(P, prefix="entropy_bottleneck."):
    pmf, tail, length, offsets, medians = eb_pmfs(P, prefix)
    cdf, sizes, offs = tables_from_pmf(pmf, tail, length, offsets)
    return cdf, sizes, offs, medians


def build_indexes(scales: torch.Tensor, scale_table: torch.Tensor, bound: float = 0.11) -> torch.Tensor:
    """GaussianConditional.build_indexes (after lower_bound_scale)."""
    scales = torch.max(scales, torch.tensor([bound], dtype=torch.float32))
    indexes = scales.new_full(scales.size(), len(scale_table) - 1).int()
    for s in scale_table[:-1]:
        indexes -= (scales <= s).int()
    return indexes


def encode(symbols: np.ndarray, indexes: np.ndarray, cdf: np.ndarray, sizes: np.ndarray,
           offsets: np.ndarray) -> np.ndarray:
    """encode_with_indexes + flush of ONE symbol list -> uint32 words."""
    s = np.ascontiguousarray(symbols, dtype=np.int32).ravel()
    ix = np.ascontiguousarray(indexes, dtype=np.int32).ravel()
    cdf = np.ascontiguousarray(cdf, dtype=np.int32)
    cap = (len(s) * 52 + 31) // 32 + 4
    out = np.zeros(cap, dtype=np.uint32)
    first = ctypes.c_int(0)
    n = lib().ref_rans_encode(_p(s), _p(ix), len(s), _p(cdf), cdf.shape[1], _p(np.ascontiguousarray(sizes)),
                              _p(np.ascontiguousarray(offsets)), cdf.shape[0], _p(out), cap, ctypes.byref(first))
    if n < 0:
        raise ValueError("rans encode failed")
    return out[first.value:first.value + n].copy()


def decode(words: np.ndarray, indexes: np.ndarray, cdf: np.ndarray, sizes: np.ndarray,
           offsets: np.ndarray) -> np.ndarray:
    w = np.ascontiguousarray(words, dtype=np.uint32)
    ix = np.ascontiguousarray(indexes, dtype=np.int32).ravel()
    cdf = np.ascontiguousarray(cdf, dtype=np.int32)
    out = np.zeros(len(ix), dtype=np.int32)
    if lib().ref_rans_decode(_p(w), len(w), _p(ix), len(ix), _p(cdf), cdf.shape[1],
                             _p(np.ascontiguousarray(sizes)), _p(np.ascontiguousarray(offsets)), cdf.shape[0],
                             _p(out)) != 0:
        raise ValueError("rans decode failed")
    return out


def encode_latent(symbols: np.ndarray, indexes, cdf, sizes, offsets) -> Tuple[np.ndarray, np.ndarray]:
    """lic stream layout: symbols/indexes [B, H, W, C] (NHWC); one string per (b, c),
    raster order -> (words concatenated, offsets_w [B*C+1])."""
    B, H, W, C = symbols.shape
    if indexes is None:
        indexes = np.broadcast_to(np.arange(C, dtype=np.int32), symbols.shape)
    parts, offs = [], [0]
    for b in range(B):
        for c in range(C):
            w = encode(symbols[b, :, :, c], indexes[b, :, :, c], cdf, sizes, offsets)
            parts.append(w)
            offs.append(offs[-1] + len(w))
    return np.concatenate(parts) if parts else np.zeros(0, np.uint32), np.asarray(offs, dtype=np.uint32)
