"""Diagnostic helper: poison_lds(seed) fills every CU's LDS with a seed-dependent
pattern on the current stream (tools/native/lds_poison.hip, built on first use into
tools/native/liblds_poison.so).  A kernel that reads LDS it never wrote then gives
results that change with the seed."""
import ctypes
import os
import subprocess

import torch

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
SO = os.path.join(HERE, "liblds_poison.so")
_lib = None


def build():
    src = os.path.join(HERE, "lds_poison.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-shared", "-fPIC", src, "-o", SO],
                       check=True)


def poison_lds(seed: int, blocks: int = 256 * 8):
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        _lib = ctypes.CDLL(SO)
        _lib.lds_poison.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream
    if _lib.lds_poison(seed & 0xFFFFFFFF, blocks, ctypes.c_void_p(st)) != 0:
        raise RuntimeError("lds_poison launch failed")
