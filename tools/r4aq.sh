set -o pipefail
O=gpurun_out/r4aq; mkdir -p $O
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_pprof2.so) timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from slam_framework_amd import slamgpu as G, synthetic as S
p = S.c4_problem(7)
for _ in range(3):
    r = G.Optimizer.PoseOptimization(p[0], p[1].copy(), S.KITTI_CAM, p[3])
print('done')
" > $O/poseprof_host.log 2>&1 || exit 1
exit 0
