"""A/B of Optimizer::PoseOptimization builds (optimizer.cpp:209-411) on bench.py's configs[3]
problems: the single-frame device call (median of 20, HIP events) and a 2048-frame batch, per
library build (SLAMGPU_LIB), each in its own process under a time limit.
  python tools/pose_lat_ab.py tools/abl/libslamgpu_a.so tools/abl/libslamgpu_b.so ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G, synthetic as S
dev = torch.device("cuda", 0)
st_ = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(st_)
B, distinct = 2048, 64
probs = [S.c4_problem(7 + i) for i in range(distinct)]
edges = np.concatenate([p[0] for p in probs])
start = np.zeros(distinct + 1, np.int64)
start[1:] = np.cumsum([len(p[0]) for p in probs])
poses = np.stack([p[1] for p in probs])
isig = probs[0][3]
k = B // distinct
E = np.concatenate([edges] * k)
st = np.concatenate([start[:-1] + i * start[-1] for i in range(k)] + [[k * start[-1]]])
d_e = torch.from_numpy(E.view(np.uint8).copy()).to(dev)
d_s = torch.from_numpy(st.astype(np.int32)).to(dev)
d_T0 = torch.from_numpy(np.concatenate([poses] * k)).to(dev)
d_T = d_T0.clone()
d_o = torch.zeros(len(E), dtype=torch.uint8, device=dev)
d_r = torch.zeros(B, dtype=torch.int32, device=dev)
d_it = torch.zeros(B, dtype=torch.int32, device=dev)
def run(n):
    d_T.copy_(d_T0)
    G.pose_optimization_device(S.KITTI_CAM, isig, d_e, d_s, n, d_T, d_o, d_r, d_it, st_.cuda_stream)
def ev_ms(fn, reps):
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st_); fn(); b.record(st_); b.synchronize()
        out.append(a.elapsed_time(b))
    return sorted(out)[len(out) // 2]
run(B); torch.cuda.synchronize()
msB = ev_ms(lambda: run(B), 5)
itsB = float(d_it.cpu().numpy().mean())
run(1); torch.cuda.synchronize()
ms1 = ev_ms(lambda: run(1), 21)
its1 = int(d_it[0].item())
T1 = d_T[0].cpu().numpy()
print(f"single {ms1:.4f} ms ({its1} LM it) | batch {msB:.3f} ms {B / msB * 1e3:.0f} f/s ({itsB:.2f} LM it/frame) | T0 {T1[0, 3]:.6f} {T1[1, 3]:.6f} {T1[2, 3]:.6f}")
'''

for lib in sys.argv[1:]:
    env = dict(os.environ, SLAMGPU_LIB=os.path.abspath(lib))
    p = subprocess.run(["timeout", "-k", "10", "200", sys.executable, "-c", CHILD], cwd=ROOT,
                       env=env, capture_output=True, text=True)
    if p.returncode != 0:
        print(lib, "FAILED rc", p.returncode, p.stderr[-1500:], flush=True)
        sys.exit(1)
    print(f"{os.path.basename(lib):26s} {p.stdout.strip()}", flush=True)
