# Local wrapper around gpurun: rebuild liblic.so and refuse to push unless the library's baked
# source hash (lic_source_hash) equals the tree's (_ffi.source_hash) -- a stale .so is refused on the
# box by _ffi.load and would waste the metered run (r05b, r05p).
# usage: bash tools/push.sh TIMEOUT 'command run on the box'
set -e -o pipefail
cd "$(dirname "$0")/.."
timeout_s=$1; shift
make -s -C learning-driven-image-compression-algorithm_amd/csrc -j8 >/dev/null
python3 - <<'EOF'
import ctypes, importlib.util, sys
spec = importlib.util.spec_from_file_location("lic_ffi", "learning-driven-image-compression-algorithm_amd/_ffi.py")
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
lib = ctypes.CDLL(str(m.LIB_PATH)); lib.lic_source_hash.restype = ctypes.c_char_p
built, tree = lib.lic_source_hash().decode(), m.source_hash()
if built != tree:
    sys.exit(f"push.sh: liblic.so hash {built} != tree {tree} after make; not pushing")
print(f"push.sh: liblic.so matches the tree ({tree})")
EOF
exec /usr/local/graft/bin/gpurun --timeout "$timeout_s" -- "$@"
