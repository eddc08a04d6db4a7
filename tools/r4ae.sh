set -o pipefail
O=gpurun_out/r4af; mkdir -p $O
A=tools/abl/libslamgpu_
timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pose_tests.log 2>&1 || exit 1
timeout -k 10 500 python tools/pose_lat_ab.py ${A}pswap.so ${A}pfused.so ${A}pswap.so ${A}pfused.so > $O/pose_ab.log 2>&1 || exit 1
SLAMGPU_LIB=$(realpath ${A}pprof.so) timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from slam_framework_amd import slamgpu as G, synthetic as S
p = S.c4_problem(7)
for _ in range(3):
    r = G.Optimizer.PoseOptimization(p[0], p[1].copy(), S.KITTI_CAM, p[3])
print('done')
" > $O/poseprof_host.log 2>&1 || exit 1
exit 0
