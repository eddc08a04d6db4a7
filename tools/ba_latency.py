"""Wall-clock latency of the single-problem drop-in calls (slamgpu_local_bundle_adjustment on
SURVEY 8(d) C5 and larger windows, slamgpu_global_bundle_adjustment), host buffers in and out,
as the LocalMapper / LoopCloser would call them.
Usage: python tools/ba_latency.py [reps] [--ba-only] [--oracle]"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
CAM = S.KITTI_CAM
out = {}


def timeit(fn):
    fn()  # warm-up (allocations, code objects)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        t.append(1e3 * (time.perf_counter() - t0))
    return float(np.median(t)), float(np.min(t)), r


for name, P in [("C5", S.c5_problem(11)),
                ("local48", S.ba_problem(12, n_local=48, n_fixed=6, n_points=5000, spacing=0.6))]:
    med, mn, r = timeit(lambda: G.Optimizer.LocalBundleAdjustment(
        P["kf_Tcw"], P["kf_mode"], P["points"], P["point_obs_start"], P["obs"], CAM,
        P["inv_sigma2"]))
    out[name] = {"median_ms": round(med, 3), "min_ms": round(mn, 3), "lm_iterations": r[3],
                 "keyframes": int(len(P["kf_mode"])), "points": int(len(P["points"])),
                 "observations": int(len(P["obs"]))}
    print(name, out[name], flush=True)
for nkf, npt in [(30, 4000), (100, 12000)]:
    P = S.ba_problem(34, n_local=nkf, n_fixed=0, n_points=npt, first_local_fixed=True, spacing=0.8)
    med, mn, r = timeit(lambda: G.Optimizer.BundleAdjustment(
        P["kf_Tcw"], P["kf_mode"], P["points"], P["point_obs_start"], P["obs"], CAM,
        P["inv_sigma2"], n_iterations=10))
    key = f"gba{nkf}"
    out[key] = {"median_ms": round(med, 3), "min_ms": round(mn, 3), "lm_iterations": r[2],
                "keyframes": nkf, "points": npt, "observations": int(len(P["obs"]))}
    print(key, out[key], flush=True)
if "--ba-only" in sys.argv:
    print(json.dumps(out))
    sys.exit(0)
# OptimizeSim3: one loop candidate (SIM3 matches of a keyframe pair), and a batch of 8
isig = S.level_inv_sigma2()
for n in (300, 1000):
    m, S0, _, _, _ = S.sim3_problem(40 + n, n, outlier_frac=0.2)
    med, mn, r = timeit(lambda: G.Optimizer.OptimizeSim3(m, S0, CAM, CAM, isig, isig, 10.0, False))
    key = f"sim3_{n}"
    out[key] = {"median_ms": round(med, 3), "min_ms": round(mn, 3), "n_inliers": r[0],
                "matches": int(len(m))}
    print(key, out[key], flush=True)
# OptimizeEssentialGraph: loop closures over n keyframes (covisibility 3, an older loop edge)
for n in (100, 400, 1000):
    Scw, fixed, E, _, _ = S.essential_graph_problem(60 + n, n, fix_scale=True,
                                                    old_loop=(n // 2, n // 5))
    med, mn, r = timeit(lambda: G.Optimizer.OptimizeEssentialGraph(Scw, fixed, E, True, 20))
    key = f"essential_graph_{n}"
    out[key] = {"median_ms": round(med, 3), "min_ms": round(mn, 3), "lm_iterations": r[3],
                "keyframes": n, "edges": int(len(E))}
    print(key, out[key], flush=True)
if "--oracle" in sys.argv:  # the CPU restatement beside it (one thread)
    sys.path.insert(0, "tests")
    import oracle_lib as O
    for n in (300, 1000):
        m, S0, _, _, _ = S.sim3_problem(40 + n, n, outlier_frac=0.2)
        t0 = time.perf_counter()
        O.optimize_sim3(CAM, CAM, isig, isig, m, S0, 10.0, False)
        out[f"sim3_{n}"]["oracle_1thread_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
    for n in (100, 400, 1000):
        Scw, fixed, E, _, _ = S.essential_graph_problem(60 + n, n, fix_scale=True,
                                                        old_loop=(n // 2, n // 5))
        t0 = time.perf_counter()
        O.optimize_essential_graph(Scw, fixed, E, True, 20)
        out[f"essential_graph_{n}"]["oracle_1thread_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
print(json.dumps(out))
