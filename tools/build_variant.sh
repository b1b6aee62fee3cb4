#!/bin/bash
# tools/build_variant.sh NAME "DEFINES" file.hip... : liblic with some objects rebuilt with
# extra defines -> tools/native/liblic_NAME.so (diagnostic A/B builds; select with LIC_LIB=; OUT=dir: elsewhere --
# tools/native/*.so does not travel to the GPU box)
set -e
name=$1; defs=$2; shift 2
C=learning-driven-image-compression-algorithm_amd/csrc
out=/tmp/lic_var_$name; mkdir -p $out
objs=""
for o in $C/build/*.o; do
  b=$(basename $o .o)
  hit=0
  for f in "$@"; do [ "$(basename $f .hip)" = "$b" ] && hit=1; done
  if [ $hit = 1 ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-variable -Xclang -target-feature -Xclang -packed-fp32-ops $defs -c $C/$b.hip -o $out/$b.o
    objs="$objs $out/$b.o"
  else objs="$objs $o"; fi
done
dest=${OUT:-tools/native}; mkdir -p $dest
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $dest/liblic_$name.so
