set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_egprof.so) timeout -k 10 200 python tools/eg_prof.py 1000 > $O/egprof1000.log 2>&1 || exit 1
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_egprof.so) timeout -k 10 200 python tools/eg_prof.py 400 > $O/egprof400.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/eg_trace -o run -- python3 tools/eg_prof.py 1000 > $O/eg_trace.log 2>&1
exit 0
