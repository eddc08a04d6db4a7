"""Timing probe of the host LocalBA stop flag: call duration and LM iterations vs raise delay."""
import ctypes
import sys
import threading
import time

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S

P = S.c5_problem(11)


def run(stop):
    return G.Optimizer.LocalBundleAdjustment(P["kf_Tcw"], P["kf_mode"], P["points"],
                                             P["point_obs_start"], P["obs"], S.KITTI_CAM,
                                             P["inv_sigma2"], stop_flag=stop)


for _ in range(2):
    t0 = time.perf_counter()
    r = run(ctypes.c_bool(False))
    print("full", r[3], f"{(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
for delay in (0.0005, 0.001, 0.002, 0.004, 0.008):
    flag = ctypes.c_bool(False)
    t_set = []
    t = threading.Timer(delay, lambda: (setattr(flag, "value", True), t_set.append(time.perf_counter())))
    t0 = time.perf_counter()
    t.start()
    r = run(flag)
    t1 = time.perf_counter()
    t.join()
    print(f"delay {delay * 1e3:.1f} ms: its {r[3]}, call {(t1 - t0) * 1e3:.2f} ms, "
          f"flag set at {(t_set[0] - t0) * 1e3 if t_set else -1:.2f} ms", flush=True)
