#!/bin/bash
# Builds an ablation copy of libslamgpu.so: tools/build_abl.sh <name> [extra hipcc flags...]
# (sources may be patched first by the caller into tools/abl/src_<name>/).
set -e
name=$1; shift
src=${SRC:-slam_framework_amd/csrc}
obj=/tmp/abl_$name; mkdir -p $obj
for f in $src/*.hip $src/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 "$@" -c $f -o $obj/$(basename $f).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/abl/libslamgpu_$name.so $obj/*.o -lz
echo tools/abl/libslamgpu_$name.so
