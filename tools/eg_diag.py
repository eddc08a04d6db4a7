"""Diagnostic: device vs oracle OptimizeEssentialGraph on one case (chi2, iterations)."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import oracle_lib as O
from slam_framework_amd import slamgpu as G, synthetic as S

for seed, n, fix, noise, old in [(5, 120, False, 0.002, (90, 30)), (2, 60, False, None, None)]:
    Scw, fixed, E, _, _ = S.essential_graph_problem(seed, n, fix_scale=fix, meas_noise=noise,
                                                    old_loop=old)
    chi = lambda Sv: sum(O.sim3_edge_eval(Sv[e["i"]], Sv[e["j"]], e["Sji"])[0] for e in E)
    print("case", seed, "chi0", chi(Scw))
    for iters in (20, 200):
        S_o, _, it_o = O.optimize_essential_graph(Scw, fixed, E, fix_scale=fix, n_iterations=iters)
        S_g, _, _, it_g = G.Optimizer.OptimizeEssentialGraph(Scw, fixed, E, fix, iters)
        print(f"  iters {iters}: oracle chi {chi(S_o):.12g} it {it_o} | gpu chi {chi(S_g):.12g} it {it_g} | max dS {np.abs(S_o - S_g).max():.3g}", flush=True)
