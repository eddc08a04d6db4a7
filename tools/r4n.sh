set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_octprof.so) timeout -k 10 200 python tools/lat_loop.py > $O/octprof.log 2>&1 || exit 1
exit 0
