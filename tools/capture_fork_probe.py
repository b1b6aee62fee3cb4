"""hipGraph capture of nested stream fork / join patterns (the LIC_CONCURRENT_RU side streams).

Finding (r05l): the nested pattern segfaults in capture_end with plain torch kernels and every
capture_error_mode; flat and sibling forks capture and replay bit-exactly.  The nested side streams
were removed from the model; tests/test_gpu_capture.py keeps the one-level forks the slice loop uses.

Round 4 saw `bench.py` segfault inside torch.cuda.graphs.capture_end with LIC_CONCURRENT_RU=1: the
slice loop forks its scale branch to a stream (net_ga._slice_loop) and, inside it, SWAtten forks its
conv_a chain to a per-instance stream; Win_noShift_Attention (16x16 latents) does the same on the main
stream.  This probe captures the same topologies with plain torch kernels and with liblic convolutions,
one case per child process (the parent never touches the GPU), and reports each case's exit status:
a segfault in capture_end shows as -11.

usage: python tools/capture_fork_probe.py [pattern:lic:mode ...]
       python tools/capture_fork_probe.py --one PATTERN LIC MODE      (one case, in this process)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def conv_op(x):
    import torch
    """One liblic launch (1x1 conv on the 16x16 latent shape) when the library is there, else a torch op."""
    import lic_amd.functional as Fn
    from lic_amd.layers import Conv2d
    if "m" not in conv_op.__dict__:   # (created by the eager pass, before any capture)
        conv_op.m = Conv2d(128, 128, 1, 1, 0).cuda()
    m = conv_op.m
    return Fn.conv(Fn.Act(x), m.packed(x.dtype)).t


def fork(parent, child, body):
    import torch
    child.wait_stream(parent)
    with torch.cuda.stream(child):
        out = body()
    return out


def pattern(name, op, x, s1, s2):
    import torch
    main = torch.cuda.current_stream()
    if name == "flat":            # main -> s1, join
        a = fork(main, s1, lambda: op(x))
        main.wait_stream(s1)
        return op(a)
    if name == "nested":          # main -> s1 -> s2, joins s2 -> s1 -> main (slice loop + SWAtten)
        def on_s1():
            b = fork(s1, s2, lambda: op(op(x)))
            c = op(x)
            s1.wait_stream(s2)
            return op(b + c)
        a = fork(main, s1, on_s1)
        d = op(x)
        main.wait_stream(s1)
        return a + d
    if name == "nested_repeat":   # the nested pattern 4x with the same two streams (4 slices)
        y = x
        for _ in range(4):
            def on_s1(y=y):
                b = fork(s1, s2, lambda: op(op(y)))
                c = op(y)
                s1.wait_stream(s2)
                return op(b + c)
            a = fork(main, s1, on_s1)
            d = op(y)
            main.wait_stream(s1)
            y = a + d
        return y
    if name == "sibling":         # main -> s1 and main -> s2 in the same region (WNSA + SWAtten)
        a = fork(main, s1, lambda: op(x))
        b = fork(main, s2, lambda: op(x))
        c = op(x)
        main.wait_stream(s1)
        main.wait_stream(s2)
        return a + b + c
    raise ValueError(name)


def run(name, use_lic, mode="global"):
    import torch
    torch.manual_seed(0)
    x = torch.randn(32, 16, 16, 128, device="cuda", dtype=torch.float32)
    op = conv_op if use_lic else (lambda t: torch.relu(t * 1.01 + 0.5))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    eager = pattern(name, op, x, s1, s2)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    print(f"begin {name} lic={use_lic} capture_error_mode={mode}", flush=True)
    with torch.cuda.graph(g, stream=cap, capture_error_mode=mode):
        out = pattern(name, op, x, s1, s2)
    print(f"  capture_end ok", flush=True)
    g.replay()
    torch.cuda.synchronize()
    same = torch.equal(out, eager)
    print(f"  replay == eager: {same}", flush=True)
    return same


if __name__ == "__main__":
    if sys.argv[1:2] == ["--one"]:
        sys.exit(0 if run(sys.argv[2], sys.argv[3] == "1", sys.argv[4]) else 1)
    # cases "pattern:lic:mode"; the probe stops at the first case that does not exit 0 or 1 (a segfault or
    # abort: nothing more runs on the GPU after it)
    cases = sys.argv[1:] or ["flat:0:global", "sibling:0:global", "sibling:1:global", "nested:0:relaxed",
                             "nested:0:thread_local", "nested:0:global"]
    rows = []
    for c in cases:
        n, use_lic, mode = c.split(":")
        try:
            rc = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--one", n, use_lic, mode],
                                timeout=90).returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
        rows.append((c, rc))
        print(f"== {c:28s} exit {rc}", flush=True)
        if rc not in (0, 1):
            break
    print("summary:", " ".join(f"{c}={rc}" for c, rc in rows))
    sys.exit(0 if all(rc == 0 for _, rc in rows) else 1)
