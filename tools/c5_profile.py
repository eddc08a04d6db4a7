"""Per-phase device wall time of the single-problem LocalBA on SURVEY 8(d) C5 (SLAMGPU_BA_PROFILE
must be set; work-group 0's clock) at several grid sizes (SLAMGPU_BA_WGS is read per process, so
run once per size)."""
import sys
import time
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S
P = S.c5_problem(11)
for _ in range(4):
    t0 = time.perf_counter()
    r = G.Optimizer.LocalBundleAdjustment(P["kf_Tcw"], P["kf_mode"], P["points"], P["point_obs_start"], P["obs"], S.KITTI_CAM, P["inv_sigma2"])
    print(f"wall {1e3 * (time.perf_counter() - t0):.3f} ms lm {r[3]}", flush=True)
