#!/bin/bash
# One library variant for an A/B: the csrc files SRCS (comma-separated) compiled with extra FLAGS,
# linked with the in-tree objects of every other source (slam_framework_amd/build, last build).
#   tools/build_variant.sh OUT.so SRC.hip[,SRC2.cpp ...] [-DNAME=VALUE ...]
set -e
OUT=$1; SRCS=$2; shift 2
B=slam_framework_amd/build
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable"
T=$(mktemp -d)
objs=$(ls $B/*.o)
for src in ${SRCS//,/ }; do
  /opt/rocm/bin/hipcc $F "$@" -c $src -o $T/$(basename $src).o
  objs=$(echo "$objs" | grep -v "/$(basename $src).o$")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $objs $T/*.o -lz
rm -rf $T
