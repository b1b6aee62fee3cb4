"""Code-generation guard for liblic.so (CPU, no GPU needed).

gfx950: a packed-FP32 VALU op (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32 / v_pk_mov_b32)
could read a source VGPR after an LDS read issued later had already overwritten it when
the SIMD was shared with other kernels' waves: the MFMA window attention of the slice
loop then used a neighbouring relative-position bias entry in a few windows, and the
B=32 fp16 forward / entropy coder were not bit-reproducible (round-1 open issue,
tools/attn_interference.py).  csrc/Makefile builds every kernel without packed-FP32 ops;
this test keeps it that way.
"""
import os
import shutil
import subprocess
import tempfile

import pytest

from lic_amd import _ffi

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PACKED = ("v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_pk_mov_b32")


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not available")
def test_no_packed_fp32_valu_ops_in_device_code():
    assert _ffi.LIB_PATH.exists(), "liblic.so not built"
    d = tempfile.mkdtemp()
    try:
        so = os.path.join(d, "liblic.so")
        shutil.copy(_ffi.LIB_PATH, so)
        subprocess.run([OBJDUMP, "--offloading", so], cwd=d, check=True, capture_output=True)
        cos = [f for f in os.listdir(d) if "gfx950" in f]
        assert cos, "no gfx950 code objects in liblic.so"
        found = {}
        for f in cos:
            asm = subprocess.run([OBJDUMP, "-d", os.path.join(d, f)], check=True, capture_output=True,
                                 text=True).stdout
            for op in PACKED:
                n = asm.count(op + " ")
                if n:
                    found[op] = found.get(op, 0) + n
        assert not found, f"packed-FP32 VALU ops in liblic.so device code: {found}"
    finally:
        shutil.rmtree(d, ignore_errors=True)
