"""The single-frame drop-in loop alone (for a rocprofv3 kernel trace): 20 calls."""
import sys
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402
Ls, Rs = S.layered_sequence(1000, 4)
c = G.Context(S.KITTI_COLS, S.KITTI_ROWS, 2000, 1.2, 8, 20, 7, max_frames=1, device=0)
for i in range(20):
    c.frame_stereo(Ls[i % 4], Rs[i % 4], S.KITTI_CAM)
    c.keypoints(0)
    c.keypoints(1)
    c.stereo(0)
print("ok")
