#!/usr/bin/env python3
"""Diagnostic: do workgroups keep their static LDS contents while other kernels share
the CU?  tools/native/lds_probe.hip fills / re-checks its LDS while noise kernels run
on a second stream (liblic conv / attention launches); prints mismatch counts."""
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HERE = os.path.join(ROOT, "tools", "native")
SO = os.path.join(HERE, "liblds_probe.so")
SIZES = {0: 21008, 1: 21504, 2: 42016, 3: 8192, 4: 65536}


def build():
    src = os.path.join(HERE, "lds_probe.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-shared", "-fPIC", src, "-o", SO],
                   check=True)


def main():
    if "--build" in sys.argv:
        build()
        return
    lib = ctypes.CDLL(SO)
    lib.lds_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p]
    from lic_amd.functional import Act
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    B = 32
    net = net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision="fp16").to("cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    wn = net.a_model.transform[8]
    wba = wn.conv_b[0]
    y64 = Act((torch.randn(B, 64, 64, 192, device="cuda", generator=g) * 0.5).half())
    noises = {"none": lambda: None,
              "qkv_conv1x1": lambda: wba.attn.qkv.run(y64),
              "conv3x3_halo": lambda: wn.conv_b[4].run(y64),
              "wba_full": lambda: wba.run(y64),
              "probe_self": None}
    side = torch.cuda.Stream()
    err = torch.zeros(3, dtype=torch.int32, device="cuda")
    rep = {}
    for sel, size in SIZES.items():
        for nname, nf in noises.items():
            err.zero_()
            err[1] = 0x7FFFFFFF
            for r in range(6):
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(4):
                        if nf is None:
                            lib.lds_probe(sel, ctypes.c_void_p(err.data_ptr() + 0), 99, 20, 2048,
                                          ctypes.c_void_p(side.cuda_stream))
                        else:
                            nf()
                st = torch.cuda.current_stream().cuda_stream
                for k in range(4):
                    if lib.lds_probe(sel, ctypes.c_void_p(err.data_ptr()), 1000 * r + k, 50, 4096,
                                     ctypes.c_void_p(st)) != 0:
                        raise RuntimeError("launch")
                torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            e = err.cpu().tolist()
            rep[f"{size}/{nname}"] = {"mismatch_dwords": e[0], "min_off": e[1] if e[0] else None,
                                      "max_off": e[2] if e[0] else None}
            print(f"{size}/{nname}", rep[f"{size}/{nname}"], flush=True)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
