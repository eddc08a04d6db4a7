"""A/B timing of OptimizeEssentialGraph (optimizer.cpp:718-960) across library builds:
  python tools/eg_ab.py tools/abl/libslamgpu_a.so tools/abl/libslamgpu_b.so ...
Each build runs in its own process (SLAMGPU_LIB) under a time limit: 100 / 400 / 1000 keyframe
loops (bench.py's 400-keyframe problem), median wall ms of 5 calls and the LM iteration count,
plus the Sim3 of every vertex hashed so that builds that must agree bit for bit can be compared."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import hashlib, sys, time
import numpy as np
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S
out = []
for n, seed in ((100, 160), (400, 460), (1000, 1060)):
    Scw, fx, E, _, _ = S.essential_graph_problem(seed, n, fix_scale=True, old_loop=(n // 2, n // 5))
    r = G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
        ts.append(1e3 * (time.perf_counter() - t0))
    h = hashlib.sha1(np.ascontiguousarray(r[0]).tobytes()).hexdigest()[:10]
    out.append(f"{n}kf {sorted(ts)[2]:.2f} ms lm {r[3]} sim3 {h}")
print(" | ".join(out))
'''

for lib in sys.argv[1:]:
    env = dict(os.environ, SLAMGPU_LIB=os.path.abspath(lib))
    p = subprocess.run(["timeout", "-k", "10", "200", sys.executable, "-c", CHILD], cwd=ROOT,
                       env=env, capture_output=True, text=True)
    if p.returncode != 0:
        print(lib, "FAILED rc", p.returncode, p.stderr[-1500:], flush=True)
        sys.exit(1)
    print(f"{os.path.basename(lib):26s} {p.stdout.strip()}", flush=True)
