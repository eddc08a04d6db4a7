"""A/B of the single-frame drop-in latency (bench.py drop_in.single_frame: slamgpu_frame_stereo +
the downloads the stereo Frame ctor keeps, one frame per call from host memory) across builds and
environment settings: python tools/lat_ab.py LIB[:NAME=VALUE,...] ...
Each variant runs in its own process (SLAMGPU_LIB + the settings) under a time limit and prints
the median / p90 over 60 calls."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, time
import numpy as np
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S
Ls, Rs = S.layered_sequence(1000, 16)
c = G.Context(S.KITTI_COLS, S.KITTI_ROWS, 2000, 1.2, 8, 20, 7, max_frames=1, device=0)
ms = []
for i in range(63):
    f = i % len(Ls)
    t0 = time.perf_counter()
    c.frame_stereo(Ls[f], Rs[f], S.KITTI_CAM)
    c.keypoints(0)
    c.keypoints(1)
    c.stereo(0)
    ms.append(1e3 * (time.perf_counter() - t0))
ms = np.array(ms[3:])
print(f"median {np.median(ms):.3f} ms p90 {np.percentile(ms, 90):.3f} ms min {ms.min():.3f} ms")
'''

for spec in sys.argv[1:]:
    lib, _, envs = spec.partition(":")
    env = dict(os.environ, SLAMGPU_LIB=os.path.abspath(lib))
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=", 1)
        env[k] = v
    p = subprocess.run(["timeout", "-k", "10", "150", sys.executable, "-c", CHILD], cwd=ROOT,
                       env=env, capture_output=True, text=True)
    if p.returncode != 0:
        print(spec, "FAILED rc", p.returncode, p.stderr[-1500:], flush=True)
        sys.exit(1)
    print(f"{spec:60s} {p.stdout.strip()}", flush=True)
