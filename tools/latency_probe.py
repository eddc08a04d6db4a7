"""Single-frame drop-in latency breakdown: wall time of slamgpu_frame_stereo and of the
downloads, and the per-kernel device time of one frame (the library's HIP-event timer)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S

Ls, Rs = S.sequence(1000, 4)
c = G.Context(S.KITTI_COLS, S.KITTI_ROWS, 2000, 1.2, 8, 20, 7, max_frames=1)
for _ in range(5):
    c.frame_stereo(Ls[0], Rs[0], S.KITTI_CAM)
w = {"frame_stereo": [], "kps": [], "stereo": []}
for i in range(30):
    t0 = time.perf_counter()
    c.frame_stereo(Ls[i % 4], Rs[i % 4], S.KITTI_CAM)
    t1 = time.perf_counter()
    c.keypoints(0)
    c.keypoints(1)
    t2 = time.perf_counter()
    c.stereo(0)
    t3 = time.perf_counter()
    w["frame_stereo"].append(t1 - t0)
    w["kps"].append(t2 - t1)
    w["stereo"].append(t3 - t2)
print({k: round(1e3 * float(np.median(v)), 3) for k, v in w.items()})
names = ["pyr_down", "fast_cells", "octree", "octree_global", "orient_desc",
         "stereo_rows", "stereo_match", "stereo_median", "grid_build", "frame_pack"]
c.timing_start("*", 4096)
for i in range(10):
    c.frame_stereo(Ls[i % 4], Rs[i % 4], S.KITTI_CAM)
c.timing_stop()
tot = 0
for n in names:
    ms, k = c.timing_read(n)
    tot += ms / 10
    print(f"{n:14s} {ms / 10 * 1e3:8.1f} us/frame  launches/frame {k / 10:.1f}")
print(f"sum of kernel times {tot * 1e3:.1f} us/frame")
