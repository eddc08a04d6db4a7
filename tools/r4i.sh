set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_undistort_gpu.py tests/test_match_gpu.py tests/test_golden.py tests/test_capi_cpp.py tests/test_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
L=tools/abl/libslamgpu_r3end.so
timeout -k 10 500 python tools/lat_ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_lat1.so tools/abl/libslamgpu_lat2.so $L:SLAMGPU_PYR_FUSED=1 tools/abl/libslamgpu_base.so tools/abl/libslamgpu_lat1.so tools/abl/libslamgpu_lat2.so $L:SLAMGPU_PYR_FUSED=1 > $O/lat_ab.log 2>&1
timeout -k 10 300 python tools/eg_ab.py tools/abl/libslamgpu_egB.so tools/abl/libslamgpu_egM.so tools/abl/libslamgpu_egB.so tools/abl/libslamgpu_egM.so > $O/eg_ab.log 2>&1
timeout -k 10 700 python -u -m pytest tests/test_ba_gpu.py tests/test_gba_gpu.py tests/test_eg_gpu.py tests/test_pose_gpu.py -x -q --timeout 300 --timeout-method thread > $O/ba_tests.log 2>&1 || exit 1
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_poseprof.so) timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from slam_framework_amd import slamgpu as G, synthetic as S
p = S.c4_problem(7)
for _ in range(3):
    r = G.Optimizer.PoseOptimization(p[0], p[1].copy(), S.KITTI_CAM, p[3])
print('done')
" > $O/poseprof_host.log 2>&1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/lat_trace -o run -- python3 tools/lat_loop.py > $O/lat_trace.log 2>&1
timeout -k 10 400 python tools/pose_lat_ab.py tools/abl/libslamgpu_cur.so tools/abl/libslamgpu_pa.so tools/abl/libslamgpu_cur.so tools/abl/libslamgpu_pa.so > $O/pose_ab.log 2>&1
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_pa.so) timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pose_tests_pa.log 2>&1
exit 0
