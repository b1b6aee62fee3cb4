"""The C-ABI library loads (no GPU needed) and exports every symbol include/lic.h declares."""
import pathlib
import re

import lic_amd
from lic_amd import _ffi

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _declared():
    txt = (ROOT / "include" / "lic.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|const char\*)\s+(lic_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_expected_entry_points():
    decl = _declared()
    assert set(decl) == set(_ffi.EXPORTED_SYMBOLS), (set(decl) ^ set(_ffi.EXPORTED_SYMBOLS))


def test_library_exports_all_declared_symbols():
    assert _ffi.LIB_PATH.exists(), "liblic.so not built (run __graft_entry__.build())"
    present = _ffi.symbols_present()
    missing = [s for s in _declared() if s not in present]
    assert not missing, missing


def test_library_loads_and_reports_version():
    lib = lic_amd.load_library()
    assert b"gfx950" in lib.lic_version()


def test_abi_version_and_struct_sizes():
    """The loader's ABI gate: the library reports the header's LIC_ABI_VERSION and the sizes
    of every args struct it was built with, equal to the ctypes layouts."""
    import ctypes
    lib = lic_amd.load_library()
    hdr = (ROOT / "include" / "lic.h").read_text()
    assert int(re.search(r"#define LIC_ABI_VERSION (\d+)", hdr).group(1)) == _ffi.ABI_VERSION
    assert lib.lic_abi_version() == _ffi.ABI_VERSION
    for k, st in enumerate((_ffi.ConvArgs, _ffi.AttnArgs, _ffi.RateArgs, _ffi.RansArgs, _ffi.WgradArgs)):
        assert lib.lic_args_size(k) == ctypes.sizeof(st), st.__name__
    assert lib.lic_args_size(99) == -1


def test_ctypes_struct_layout_matches_header():
    import ctypes
    # the largest args struct: sizes must agree with the C compiler's layout
    a = _ffi.ConvArgs()
    assert ctypes.sizeof(a) % 8 == 0
    names = [f[0] for f in _ffi.ConvArgs._fields_]
    hdr = (ROOT / "include" / "lic.h").read_text()
    body = hdr[hdr.index("typedef struct lic_conv_args"):hdr.index("} lic_conv_args;")]
    for n in names:
        assert re.search(r"\b%s\b" % n, body), n


def test_ctypes_struct_offsets_match_c_compiler(tmp_path):
    """Every args struct of include/lic.h: sizeof and each field's offsetof from gcc
    equal the ctypes layout (the ABI the Python host passes by pointer)."""
    import ctypes
    import shutil
    import subprocess
    import pytest
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"lic_conv_args": _ffi.ConvArgs, "lic_attn_args": _ffi.AttnArgs,
               "lic_rate_args": _ffi.RateArgs, "lic_rans_args": _ffi.RansArgs, "lic_wgrad_args": _ffi.WgradArgs,
               "lic_resunit_args": _ffi.ResunitArgs, "lic_wba_args": _ffi.WbaArgs, "lic_wba16_args": _ffi.Wba16Args}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "lic.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


def test_library_built_from_this_tree():
    """Build provenance: the library's lic_source_hash equals the hash of this tree's csrc/ and
    include/lic.h (csrc/Makefile SRC_HASH), and lic_version carries it."""
    lib = lic_amd.load_library()
    tree = _ffi.source_hash()
    assert tree is not None and len(tree) == 16
    assert lib.lic_source_hash().decode() == tree
    assert f"src {tree}".encode() in lib.lic_version()


def test_loader_refuses_a_library_from_other_sources(monkeypatch):
    """_ffi.load raises LicError when the tree's sources differ from the ones the .so was built from."""
    import pytest
    monkeypatch.setattr(_ffi, "_lib", None)
    monkeypatch.setattr(_ffi, "_load_error", None)
    monkeypatch.setattr(_ffi, "source_hash", lambda: "0000000000000000")
    with pytest.raises(_ffi.LicError, match="built from other sources"):
        _ffi.load()
