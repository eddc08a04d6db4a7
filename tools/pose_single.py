"""20 single-frame PoseOptimization device calls on bench.py's configs[3] problem (the library
from SLAMGPU_LIB), for `rocprofv3 --pmc ... -- python3 tools/pose_single.py` A/Bs."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
p = S.c4_problem(7)
edges, T0, isig = p[0], p[1], p[3]
d_e = torch.from_numpy(edges.view(np.uint8).copy()).to(dev)
d_s = torch.tensor([0, len(edges)], dtype=torch.int32, device=dev)
d_T0 = torch.from_numpy(T0[None].copy()).to(dev)
d_T = d_T0.clone()
d_o = torch.zeros(len(edges), dtype=torch.uint8, device=dev)
d_r = torch.zeros(1, dtype=torch.int32, device=dev)
d_it = torch.zeros(1, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(20):
    d_T.copy_(d_T0)
    G.pose_optimization_device(S.KITTI_CAM, isig, d_e, d_s, 1, d_T, d_o, d_r, d_it, st)
torch.cuda.synchronize()
print("inliers", int(d_r.item()), "LM iterations", int(d_it.item()))
