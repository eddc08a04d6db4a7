set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_gba_gpu.py tests/test_eg_gpu.py tests/test_pose_gpu.py -x -v --timeout 300 --timeout-method thread > $O/ba_tests.log 2>&1 &&
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_poseprof.so) timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from slam_framework_amd import slamgpu as G, synthetic as S
p = S.c4_problem(7)
for _ in range(3):
    r = G.Optimizer.PoseOptimization(p[0], p[1].copy(), S.KITTI_CAM, p[3])
print('done')
" > $O/poseprof_host.log 2>&1
