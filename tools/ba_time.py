"""Times slamgpu_local_bundle_adjustment_device on B copies of a configs[4] problem
(20 local keyframes + 6 fixed, 3000 map points)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
P = S.ba_problem(1)
nk, npn, no = len(P["kf_mode"]), len(P["points"]), len(P["obs"])
desc = np.array([(i * nk, nk, i * npn, npn) for i in range(B)], np.int32)
start = np.concatenate([P["point_obs_start"][:-1] + i * no for i in range(B)] + [[B * no]]).astype(np.int32)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(s)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
d_desc, d_mode, d_start = t(desc), t(np.tile(P["kf_mode"], B)), t(start)
d_obs = t(np.tile(P["obs"], B))
kf0, pts0 = t(np.tile(P["kf_Tcw"], (B, 1, 1))), t(np.tile(P["points"], (B, 1)))
d_kf, d_pts = kf0.clone(), pts0.clone()
d_er = torch.zeros(B * no, dtype=torch.uint8, device=dev)
d_st = torch.zeros(B, dtype=torch.int32, device=dev)
d_ws = torch.empty(G.local_ba_workspace_bytes(B * nk, B * npn, B * no), dtype=torch.uint8, device=dev)
ms = []
for r in range(reps + 1):
    d_kf.copy_(kf0)
    d_pts.copy_(pts0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    G.local_bundle_adjustment_device(S.KITTI_CAM, P["inv_sigma2"], d_desc, B, d_kf, d_mode, d_pts,
                                     d_start, d_obs, d_er, d_st, d_ws, B * nk, B * npn, B * no,
                                     stream=s.cuda_stream)
    b.record(s)
    b.synchronize()
    if r:
        ms.append(a.elapsed_time(b))
print(f"B={B} local BA problems ({nk} KF, {npn} pts, {no} obs): {np.median(ms):.3f} ms/launch "
      f"-> {B / np.median(ms) * 1e3:.1f} problems/s; LM iterations {d_st.cpu().numpy()[:4]}")
