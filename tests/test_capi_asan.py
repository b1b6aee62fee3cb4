"""The C ABI's host side under AddressSanitizer (race / memory-error row): a
host-only ASan build of liblic (csrc/Makefile `asan`) driven by tests/native/capi_asan.c
-- every host helper, the argument validation of the launch entry points, and
lic_last_error from 8 threads.  CPU only; any ASan report fails the test."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "learning-driven-image-compression-algorithm_amd", "csrc")
CLANG = "/opt/rocm/llvm/bin/clang"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang not available")
def test_capi_host_side_under_asan(tmp_path):
    subprocess.run(["make", "-C", CSRC, "-j8", "asan"], check=True, capture_output=True)
    so_dir = os.path.join(CSRC, "build_asan")
    exe = str(tmp_path / "capi_asan")
    subprocess.run([CLANG, "-fsanitize=address", "-fno-omit-frame-pointer", "-g", "-O1",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "capi_asan.c"),
                    "-L", so_dir, "-llic_asan", "-Wl,-rpath," + so_dir, "-lpthread", "-o", exe],
                   check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "CAPI_OK" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "AddressSanitizer" not in r.stderr
