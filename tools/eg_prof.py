"""One OptimizeEssentialGraph call of n keyframes (for rocprofv3 kernel stats)."""
import sys
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
Scw, fixed, E, _, _ = S.essential_graph_problem(60 + n, n, fix_scale=True, old_loop=(n // 2, n // 5))
for _ in range(2):
    r = G.Optimizer.OptimizeEssentialGraph(Scw, fixed, E, True, 20)
print("lm", r[3])
