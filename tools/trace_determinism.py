#!/usr/bin/env python3
"""Per-launch determinism trace: wraps the liblic op wrappers of lic_amd.functional so
that every launch appends an integer checksum of its output view, runs the same
forward several times and reports, per run, the first launch whose output differs
from run 0 (with its op name, shapes and the kernel-choice inputs).
usage: python tools/trace_determinism.py [--runs 8] [--batch 32] [--precision fp16] [--what forward|a_model]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TRACE = []
PRE = [None]   # optional hook run before every wrapped launch (LDS poisoning)


def _h(a):
    if a is None:
        return None
    t = a.t[..., a.c0:a.c0 + a.c] if hasattr(a, "c0") else a
    if t.dtype == torch.float16:
        v = t.view(torch.int16)
    elif t.dtype == torch.float32:
        v = t.view(torch.int32)
    else:
        v = t
    return v.to(torch.int64).sum()


def install():
    from lic_amd import functional as Fn
    orig_conv = Fn.conv
    lib = Fn._lib()

    class _Proxy:   # PRE hook before every liblic launch
        def __getattr__(self, name):
            f = getattr(lib, name)
            if not name.startswith("lic_") or name.endswith(("_workspace", "_parts")) or name == "lic_last_error":
                return f

            def call(*a):
                if PRE[0]:
                    PRE[0]()
                return f(*a)
            return call
    proxy = _Proxy()
    Fn._lib = lambda: proxy

    def conv(x, pk, out=None, **kw):
        y = orig_conv(x, pk, out, **kw)
        desc = dict(op="conv", x=[x.B, x.H, x.W, x.c, x.ld], co=pk.co, copad=pk.copad, cpad=pk.cpad, taps=len(pk.dy),
                    stride=pk.stride, phase=pk.phase is not None, epi=kw.get("epi", 0), act=kw.get("act", 0),
                    out=[y.H, y.W, y.c, y.ld], shuffle=kw.get("shuffle", False))
        TRACE.append((desc, _h(y), _h(kw.get("y2"))))
        return y
    Fn.conv = conv
    for name in ("win_attn", "layernorm", "rb3", "avgpool", "quantize_median", "add", "copy"):
        orig = getattr(Fn, name)

        def wrap(*a, _orig=orig, _name=name, **kw):
            y = _orig(*a, **kw)
            x = a[0]
            TRACE.append((dict(op=_name, x=[x.B, x.H, x.W, x.c, x.ld]), _h(y), None))
            return y
        setattr(Fn, name, wrap)
    orig_rate = Fn.gauss_rate

    def gauss_rate(y, mu, scale, partials, part_off, **kw):
        n = orig_rate(y, mu, scale, partials, part_off, **kw)
        TRACE.append((dict(op="gauss_rate", x=[y.B, y.H, y.W, y.c]), _h(kw.get("yq")), _h(kw.get("symbols"))))
        return n
    Fn.gauss_rate = gauss_rate


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--what", default="forward", choices=["forward", "a_model", "a_model_layers"])
    ap.add_argument("--poison-random", action="store_true")
    ap.add_argument("--multi-stream", action="store_true", help="keep the side streams (default: single stream)")
    ap.add_argument("--lds-poison", action="store_true", help="fill every CU's LDS with a new pattern before each run")
    ap.add_argument("--lds-poison-each", action="store_true",
                    help="fill every CU's LDS with the run's pattern before every launch (finds kernels that read "
                         "LDS they did not write: the first differing launch is the culprit)")
    args = ap.parse_args()
    if args.what != "a_model_layers":
        install()
    from lic_amd.functional import Act
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B = args.batch
    net = net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision=args.precision).to("cuda")
    if not args.multi_stream:
        net.__dict__["_lic_single_stream"] = True
    x = (torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1)) * 2 - 1).to("cuda")

    layers = []
    if args.what == "a_model_layers":
        # capture every transform step's output view (no extra kernels between launches)
        for i, m in enumerate(net.a_model.transform):
            if not hasattr(m, "run"):
                continue
            def wrap(*a, _orig=m.run, _i=i, **kw):
                y = _orig(*a, **kw)
                layers.append((_i, type(m).__name__, y))
                return y
            m.run = wrap
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from determinism_probe import poison

    from lds_poison import poison_lds
    nrun = [0]

    if args.lds_poison_each:
        PRE[0] = lambda: poison_lds(nrun[0])

    def once():
        nrun[0] += 0 if args.lds_poison else 1
        if args.poison_random:
            poison(random=True)
        if args.lds_poison:
            nrun[0] += 1
            poison_lds(nrun[0])
        if args.what == "a_model_layers":
            layers.clear()
            net.a_model.run(Act.from_nchw(x, net.dtype, pad16=True))
            torch.cuda.synchronize()
            out = [(dict(op=f"t[{i}] {n}", x=[y.B, y.H, y.W, y.c]), y.t[..., y.c0:y.c0 + y.c].clone(), None)
                   for i, n, y in layers]
            layers.clear()
            return out
        TRACE.clear()
        if args.what == "forward":
            net(x, "test")
        else:
            net.a_model.run(Act.from_nchw(x, net.dtype, pad16=True))
        torch.cuda.synchronize()
        return [(d, None if h is None else int(h), None if h2 is None else int(h2)) for d, h, h2 in TRACE]

    ref = once()
    runs = []
    for r in range(args.runs):
        tr = once()
        first = None
        ndiff = 0
        for k, (a, b) in enumerate(zip(ref, tr)):
            same = torch.equal(a[1], b[1]) if torch.is_tensor(a[1]) else a[1:] == b[1:]
            if not same:
                ndiff += 1
                if first is None:
                    first = dict(index=k, **a[0])
        runs.append({"n_launches": len(tr), "n_diff": ndiff, "first": first})
    print(json.dumps({"what": args.what, "batch": B, "precision": args.precision, "runs": runs}), flush=True)


if __name__ == "__main__":
    main()
