#!/bin/bash
# Builds an ablation copy of libslamgpu.so: tools/build_abl.sh <name> [extra hipcc flags...]
# (sources may be patched first by the caller into a copy and passed as SRC=<dir>). Every object
# is rebuilt from scratch; any failed compile fails the build.
set -e
name=$1; shift
src=${SRC:-slam_framework_amd/csrc}
obj=/tmp/abl_$name; rm -rf $obj; mkdir -p $obj ${ABL_DIR:-ab}
pids=()
for f in $src/*.hip $src/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 "$@" -c $f -o $obj/$(basename $f).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ${ABL_DIR:-ab}/libslamgpu_$name.so $obj/*.o -lz
echo ${ABL_DIR:-ab}/libslamgpu_$name.so
