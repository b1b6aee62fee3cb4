# VGPR / SGPR / spill / LDS figures of every kernel in one built object (csrc/build/NAME.o)
# usage: bash tools/kernel_resources.sh wba16 [name-filter]
set -e
B=learning-driven-image-compression-algorithm_amd/csrc/build
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
cp "$B/$1.o" "$tmp/k.o"
(cd "$tmp" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o >/dev/null)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$tmp"/k.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 |
  grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_spill_count|\.vgpr_spill_count|\.private_segment_fixed_size" |
  paste - - - - - | sed 's/  */ /g' | grep -E "${2:-.}" || true
rm -rf "$tmp"
