"""OptimizeEssentialGraph on bench.py's 400-keyframe loop (and 1000 with an argument), 5 timed
calls after one warm-up; for `rocprofv3 --kernel-trace --stats -- python3 tools/eg_time.py`."""
import sys
import time

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
seed = {100: 160, 400: 460, 1000: 1060}.get(n, 460)
Scw, fx, E, _, _ = S.essential_graph_problem(seed, n, fix_scale=True, old_loop=(n // 2, n // 5))
r = G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    r = G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
    ts.append(1e3 * (time.perf_counter() - t0))
print(f"{n} keyframes: median {sorted(ts)[2]:.2f} ms, LM iterations {r[3]}")
