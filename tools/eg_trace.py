"""OptimizeEssentialGraph (optimizer.cpp:718-960) at the given keyframe counts (default 400), 5
calls each after a warm-up, for a rocprofv3 kernel trace: which launches a call spends its time in.
  rocprofv3 --kernel-trace --stats -d gpurun_out/x -o eg -- python3 tools/eg_trace.py 100"""
import sys
import time

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [400]
for n in sizes:
    seed = n + 60
    Scw, fx, E, _, _ = S.essential_graph_problem(seed, n, fix_scale=True, old_loop=(n // 2, n // 5))
    G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
    t0 = time.perf_counter()
    for _ in range(5):
        r = G.Optimizer.OptimizeEssentialGraph(Scw, fx, E, True, 20)
    print(f"{n} keyframes: {1e3 * (time.perf_counter() - t0) / 5:.2f} ms per call, lm {r[3]}")
