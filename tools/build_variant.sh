#!/bin/bash
# One library variant for an A/B: SRC (a csrc file) compiled with extra FLAGS, linked with the
# in-tree objects of every other source (slam_framework_amd/build, from the last build).
#   tools/build_variant.sh OUT.so SRC.hip [-DNAME=VALUE ...]
set -e
OUT=$1; SRC=$2; shift 2
B=slam_framework_amd/build
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable"
/opt/rocm/bin/hipcc $F "$@" -c $SRC -o /tmp/variant_$$.o
objs=$(ls $B/*.o | grep -v "/$(basename $SRC).o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $objs /tmp/variant_$$.o -lz
rm -f /tmp/variant_$$.o
