set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 120 tools/clock_probe > $O/clock_probe.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_match_gpu.py tests/test_capi_cpp.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
timeout -k 10 500 python tools/lat_ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_lat1.so tools/abl/libslamgpu_lat3.so tools/abl/libslamgpu_base.so tools/abl/libslamgpu_lat1.so tools/abl/libslamgpu_lat3.so > $O/lat_ab.log 2>&1 || exit 1
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_poseprof.so) timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from slam_framework_amd import slamgpu as G, synthetic as S
p = S.c4_problem(7)
for _ in range(3):
    r = G.Optimizer.PoseOptimization(p[0], p[1].copy(), S.KITTI_CAM, p[3])
print('done')
" > $O/poseprof_host.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/lat_trace -o run -- python3 tools/lat_loop.py > $O/lat_trace.log 2>&1
exit 0
