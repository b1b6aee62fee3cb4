#!/usr/bin/env python3
"""Entropy-coder throughput: Net.compress / Net.decompress of a
batch of 256x256 images on one GPU, and the coder kernels alone (lic_rans_encode +
pack, lic_rans_decode of all slices) timed with HIP events, next to the C oracle
(oracle/rans_ref.c, one host thread) encoding the same symbols.

Prints one JSON line.  usage: python tools/coder_bench.py [--batch 32] [--precision fp16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from lic_amd import entropy_coder as EC
    from lic_amd.functional import Act
    from lic_amd.model import net_ga
    dev = "cuda"
    torch.manual_seed(0)
    B, S = args.batch, args.size
    net = net_ga.Net((B, S, S, 3), (B, S, S, 3), False, False, precision=args.precision).to(dev)
    x = (torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(1)) * 2 - 1).to(dev)
    net.update()
    enc = net.compress(x)
    dec = net.decompress(enc["strings"], enc["shape"], enc["syntax"])
    assert torch.equal(dec["symbols"].cpu(), enc["symbols"].cpu())
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.iters

    t_comp = timed(lambda: net.compress(x))
    t_dec = timed(lambda: net.decompress(enc["strings"], enc["shape"], enc["syntax"]))
    nbytes = sum(len(s) for lst in enc["strings"] for s in lst)

    # coder kernels alone on the y symbols of this batch
    cs = net._coder_state()
    SYM = enc["symbols"]
    hh, ww = SYM.shape[1], SYM.shape[2]
    sc = torch.rand(B, hh, ww, 192, device=dev) * 4 + 0.05
    IDX = torch.empty(B, hh, ww, 192, dtype=torch.int32, device=dev)
    EC.gauss_indexes(Act(sc), cs["scale_table"], 0.11, Act(IDX))
    st = torch.cuda.current_stream()

    def ev_time(fn, n=args.iters):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / n

    words, offs = EC.encode_streams(Act(SYM), Act(IDX), cs["gauss"])
    t_enc_k = ev_time(lambda: EC.encode_streams(Act(SYM), Act(IDX), cs["gauss"]))
    out = torch.empty_like(SYM)
    t_dec_k = ev_time(lambda: EC.decode_streams(words, offs, cs["gauss"], B, hh * ww, 192, 0, 192, idx=Act(IDX),
                                                symbols=Act(out)))
    assert torch.equal(out, SYM)
    nsym = SYM.numel()
    # C oracle, one thread, on a bounded sample of the same streams
    from oracle import ref_coder as C
    sym_np, idx_np = SYM.cpu().numpy(), IDX.cpu().numpy()
    cdf = cs["gauss"].cdf.cpu().numpy()
    sizes, offsets = cs["gauss"].sizes.cpu().numpy(), cs["gauss"].offsets.cpu().numpy()
    nb = max(1, min(B, 4))
    t0 = time.perf_counter()
    C.encode_latent(sym_np[:nb], idx_np[:nb], cdf, sizes, offsets)
    t_cpu = time.perf_counter() - t0
    cpu_sym_s = nb * hh * ww * 192 / t_cpu
    print(json.dumps({
        "workload": f"net_ga {args.precision}, batch {B} x {S}x{S}",
        "compress_ms": round(t_comp * 1e3, 3), "decompress_ms": round(t_dec * 1e3, 3),
        "compress_images_per_s": round(B / t_comp, 1), "decompress_images_per_s": round(B / t_dec, 1),
        "coded_bytes": nbytes, "coded_bpp_incl_headers": round(8 * nbytes / (B * S * S), 4),
        "y_symbols": nsym, "encode_kernels_ms": round(t_enc_k * 1e3, 3), "decode_kernel_ms": round(t_dec_k * 1e3, 3),
        "encode_Msym_per_s": round(nsym / t_enc_k / 1e6, 1), "decode_Msym_per_s": round(nsym / t_dec_k / 1e6, 1),
        "cpu_oracle_encode_Msym_per_s": round(cpu_sym_s / 1e6, 2),
        "cpu_oracle_sample": f"{nb} images' y streams, oracle/rans_ref.c, 1 thread"}), flush=True)


if __name__ == "__main__":
    main()
