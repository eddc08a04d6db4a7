"""Dev check: repeat the bench's batched step and print matches per step (state carry-over)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
cols, rows, cam = S.KITTI_COLS, S.KITTI_ROWS, S.KITTI_CAM
Ls, Rs = S.sequence(1000, 16)
pitch = 1280
hl = np.zeros((B, rows, pitch), np.uint8); hr = np.zeros((B, rows, pitch), np.uint8)
for f in range(B):
    hl[f, :, :cols] = Ls[f % 16]; hr[f, :, :cols] = Rs[f % 16]
d_l = torch.from_numpy(hl).to(dev); d_r = torch.from_numpy(hr).to(dev)
poses = np.zeros(B, G.F2F_POSE_DTYPE)
for f in range(B):
    poses["Rcw"][f] = S.rotation(f % 16).astype(np.float32).reshape(-1)
poses["baseline"] = np.float32(cam[4]) / np.float32(cam[0]); poses["th"] = 7.0; poses["check_ori"] = 1
d_poses = torch.from_numpy(poses.view(np.uint8).copy()).to(dev)
ctx = G.Context(cols, rows, 2000, 1.2, 8, 20, 7, max_frames=B)
kc = ctx.kp_cap
d_q = torch.empty(B * kc * G.F2F_QUERY_DTYPE.itemsize, dtype=torch.uint8, device=dev)
d_qs = torch.empty(B, dtype=torch.int32, device=dev); d_qc = torch.empty(B, dtype=torch.int32, device=dev)
d_mp = torch.empty(B * kc, dtype=torch.int32, device=dev); d_blk = torch.empty(B * kc, dtype=torch.uint8, device=dev)
d_nm = torch.empty(B, dtype=torch.int32, device=dev)
for it in range(6):
    st = torch.cuda.current_stream().cuda_stream
    ctx.frontend_device(int(d_l.data_ptr()), int(d_r.data_ptr()), rows * pitch, pitch, B, cam, st)
    ctx.make_vo_queries_device(d_poses, 1, d_q, d_qs, d_qc, B, st)
    d_mp.fill_(-1); d_blk.zero_()
    ctx.search_by_projection_frame_device(d_q, B * kc, d_qs, d_qc, kc, d_poses, d_mp, d_blk, kc, d_nm, B, st)
    torch.cuda.synchronize(); ctx.sync()
    nk = [ctx.keypoints(i)[0].shape[0] for i in range(4)]
    print(it, "kps", nk, "q", d_qc.cpu().numpy()[:6].tolist(), "m", d_nm.cpu().numpy()[:6].tolist(),
          "ur0", float(np.nansum(ctx.stereo(0)[0] >= 0)), flush=True)
