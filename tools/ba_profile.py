"""Per-phase cycle split of one configs[4] local BA (instrumented build: SLAMGPU_BA_PROFILE).
SLAMGPU_LIB=tools/abl/libslamgpu_baprof.so python tools/ba_profile.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

P = S.ba_problem(1)
nk, npn, no = len(P["kf_mode"]), len(P["points"]), len(P["obs"])
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
d_desc = t(np.array([(0, nk, 0, npn)], np.int32))
d_kf, d_pts = t(P["kf_Tcw"]), t(P["points"])
d_er = torch.zeros(no, dtype=torch.uint8, device=dev)
d_st = torch.zeros(2 + 16, dtype=torch.int32, device=dev)
d_ws = torch.empty(G.local_ba_workspace_bytes(nk, npn, no), dtype=torch.uint8, device=dev)
G.local_bundle_adjustment_device(S.KITTI_CAM, P["inv_sigma2"], d_desc, 1, d_kf, t(P["kf_mode"]),
                                 d_pts, t(P["point_obs_start"]), t(P["obs"]), d_er, d_st, d_ws,
                                 nk, npn, no)
torch.cuda.synchronize()
st = d_st.cpu().numpy()
prof = st[2:].view(np.float64)
names = ["structure", "linearise", "schur_points", "assemble_S", "factor_solve", "update+errors",
         "sum", "other"]
tot = prof.sum()
print(f"LM iterations {st[0]}; total {tot:.3g} cycles")
for n, v in zip(names, prof):
    print(f"  {n:14s} {v:12.4g} cycles {100 * v / tot:5.1f}%")
