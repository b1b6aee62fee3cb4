"""Per-op GPU time of one Net.forward (eager, each op synchronised and timed with
HIP events), aggregated by calling module and op shape.

usage: python tools/layer_profile.py [--arch net_ga] [--batch 32] [--size 256] [--top 40]
Timings are serialised (no stream overlap), so their sum exceeds the graph-replay
step time; use them to rank ops, not to predict the step.  A wrapped op that calls
another (GDN.run -> conv) is charged its self time only (the r03 and r04t logs counted
the nested conv twice).
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lic_amd.functional as Fn  # noqa: E402

REC = collections.defaultdict(lambda: [0, 0.0, 0.0])   # calls, ms, FLOP


def _label(name, args):
    site = "?"
    fr = sys._getframe(2)
    for _ in range(8):
        if fr is None:
            break
        slf = fr.f_locals.get("self")
        if slf is not None and isinstance(slf, torch.nn.Module):
            site = f"{type(slf).__name__}.{fr.f_code.co_name}"
            break
        fr = fr.f_back
    shape = ""
    x = args[0] if args else None
    if isinstance(x, Fn.Act):
        shape = f"{x.H}x{x.W}x{x.c}"
    if name in ("conv", "conv_transpose") and len(args) > 1:
        pk = args[1][0] if isinstance(args[1], (list, tuple)) else args[1]
        shape += f" {pk.ci}->{pk.co} k{pk.kh}s{pk.stride}"
    return f"{name:14s} {site:40s} {shape}"


_NEST = []   # child time of the wrapped ops in flight (Fn.gdn calls Fn.conv: count that time once)


def wrap(name):
    fn = getattr(Fn, name)

    def w(*args, **kw):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        _NEST.append(0.0)
        e0.record()
        try:
            out = fn(*args, **kw)
        finally:
            child = _NEST.pop()
        e1.record()
        e1.synchronize()
        dt = e0.elapsed_time(e1)
        if _NEST:
            _NEST[-1] += dt
        r = REC[_label(name, args)]
        r[0] += 1
        r[1] += max(0.0, dt - child)   # self time: nested wrapped ops keep their own rows
        if name == "conv" and isinstance(out, Fn.Act) and len(args) > 1:
            pk = args[1]
            mi, mj = kw.get("out_hw") or (out.H, out.W)
            if kw.get("shuffle") is True:
                mi, mj = out.H // 2, out.W // 2
            if pk.phase is not None:   # a transposed-conv phase computes every s-th output pixel only
                ry, rx, s = pk.phase[0], pk.phase[1], pk.phase[2]
                mi, mj = -(-(out.H - ry) // s), -(-(out.W - rx) // s)
            r[2] += 2.0 * out.B * mi * mj * pk.co * pk.ci * len(pk.dy) / max(1, pk.groups)
        return out
    setattr(Fn, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="net_ga")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--post-processing", action="store_true")
    ap.add_argument("--precision", default="fp16", choices=["fp16", "fp32", "bf16", "fp32x3", "fp32x6"])
    ap.add_argument("--what", default="forward", choices=["forward", "a_model"])
    args = ap.parse_args()
    import bench
    net = bench.build_net(args.arch, args.precision, args.size, args.batch, "cpu",
                          post_processing=args.post_processing).to("cuda")
    if args.what == "a_model":
        xin = Fn.Act.from_nchw(torch.rand(args.batch, 3, args.size, args.size, device="cuda") * 2 - 1, net.dtype,
                               pad16=True)
        def run():
            with Fn.split_f32(Fn.SPLIT_MODES.get(args.precision, 0)):
                return net.a_model.run(xin)
    else:
        run = None
    x = torch.rand(args.batch, 3, args.size, args.size, device="cuda") * 2 - 1
    with torch.no_grad():
        print("warm-up forward", flush=True)
        run() if run else net(x, "test")
        torch.cuda.synchronize()
        print("profiled forward", flush=True)
        for n in ("conv", "conv_transpose", "gdn", "win_attn", "layernorm", "rb3", "add", "copy", "avgpool",
                  "quantize_median", "gauss_rate", "syntax_recon", "bpp_finalize", "psnr_finalize",
                  "recon", "pool_partials", "ca_apply", "lam", "csam"):
            wrap(n)
        run() if run else net(x, "test")
        torch.cuda.synchronize()
    peak = {"fp16": 2516.6, "bf16": 2516.6, "fp32": 157.3, "fp32x3": 2516.6 / 3, "fp32x6": 2516.6 / 6}[args.precision]
    tot = sum(v[1] for v in REC.values())
    fl = sum(v[2] for v in REC.values())
    print(f"# {args.what} {args.arch} {args.precision} B={args.batch} {args.size}^2: serialised op time {tot:.3f} ms "
          f"over {sum(v[0] for v in REC.values())} ops; conv {fl / 1e9:.1f} GFLOP -> "
          f"{fl / tot / 1e9:.1f} TFLOP/s ({100 * fl / tot / 1e9 / peak:.1f} % of {peak})")
    for k, (n, t, f) in sorted(REC.items(), key=lambda kv: -kv[1][1])[:args.top]:
        tf = f"{f / t / 1e9:7.1f} TF/s {100 * f / t / 1e9 / peak:5.1f}%" if f else " " * 20
        print(f"{t:8.3f} ms {100 * t / tot:5.1f}% x{n:<4d} {tf}  {k}")


if __name__ == "__main__":
    main()
