"""Times slamgpu_pose_optimization_device on a batch of synthetic 2000-edge frames (configs[3])."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
edges, start, poses, isig, _ = S.pose_batch(500, 64)
# tile 64 distinct problems to B frames
k = (B + 63) // 64
E = np.concatenate([edges] * k)
st = np.concatenate([start[:-1] + i * start[-1] for i in range(k)] + [[k * start[-1]]]).astype(np.int32)
st = st[:B + 1]
P = np.concatenate([poses] * k)[:B]
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(s)
d_e = torch.from_numpy(E.view(np.uint8).copy()).to(dev)
d_s = torch.from_numpy(st).to(dev)
d_T0 = torch.from_numpy(P.copy()).to(dev)
d_T = d_T0.clone()
d_o = torch.zeros(len(E), dtype=torch.uint8, device=dev)
d_r = torch.zeros(B, dtype=torch.int32, device=dev)
d_it = torch.zeros(B, dtype=torch.int32, device=dev)
for _ in range(2):
    d_T.copy_(d_T0)
    G.pose_optimization_device(S.KITTI_CAM, isig, d_e, d_s, B, d_T, d_o, d_r, d_it, s.cuda_stream)
torch.cuda.synchronize()
ms = []
for _ in range(reps):
    d_T.copy_(d_T0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    G.pose_optimization_device(S.KITTI_CAM, isig, d_e, d_s, B, d_T, d_o, d_r, d_it, s.cuda_stream)
    b.record(s)
    b.synchronize()
    ms.append(a.elapsed_time(b))
its = d_it.cpu().numpy()
print(f"B={B} frames x 2000 edges: {np.median(ms):.3f} ms/launch -> {B / np.median(ms) * 1e3:.0f} "
      f"frames/s; LM iterations/frame mean {its.mean():.1f}")
