"""Per-phase device time of the map-scale global BA (the bench's global_ba_1500kf_loop: a closed
loop of 1500 keyframes, S in block-profile storage). Run with SLAMGPU_BA_PROFILE=1: the runtime
prints work-group 0's per-phase wall time (linearise, barriers, S assembly, build, factor, ...)."""
import sys
import time

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S

n_kf = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
PM = S.map_problem(40 + n_kf, n_kf)
for _ in range(2):
    t0 = time.perf_counter()
    r = G.Optimizer.BundleAdjustment(PM["kf_Tcw"], PM["kf_mode"], PM["points"],
                                     PM["point_obs_start"], PM["obs"], S.KITTI_CAM,
                                     PM["inv_sigma2"], n_iterations=10)
    print(f"{n_kf} keyframes: wall {1e3 * (time.perf_counter() - t0):.1f} ms, lm {r[2]}",
          flush=True)
