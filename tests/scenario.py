"""Matcher scenarios built from oracle front-end results (test infrastructure).

`vo_queries` mirrors Tracker::UpdateLastFrame's visual-odometry points (tracker.cpp:695-753):
every last-frame keypoint with stereo depth becomes a map point at UnprojectStereo(i)
(frame.cpp:594-607), with the keypoint's descriptor. Poses come from synthetic.rotation().
"""
import numpy as np

from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S


def unproject(kps, depth, Rcw, cam, tcw=None):
    """Frame::UnprojectStereo: Rwc Xc + Ow (Ow = -Rcw^T tcw)."""
    fx, fy, cx, cy, _ = [np.float32(v) for v in cam]
    z = depth.astype(np.float32)
    x = (kps["x"] - cx) * z * (np.float32(1) / fx)
    y = (kps["y"] - cy) * z * (np.float32(1) / fy)
    Xc = np.stack([x, y, z], 1).astype(np.float64)
    R = np.asarray(Rcw, np.float64)
    Xw = Xc @ R  # Rwc @ Xc, Rwc = Rcw^T
    if tcw is not None:
        Xw -= R.T @ np.asarray(tcw, np.float64)
    return Xw.astype(np.float32)


def vo_queries(kps_last, desc_last, depth_last, t_last, rng=None, blocks_frac=1.0, cam=S.KITTI_CAM,
               layered=False):
    """Queries in last-frame keypoint order; returns (queries, last_mp, last_outlier, mp_xyz,
    mp_desc, mp_nobs) for both the oracle and the HIP path. layered: the last frame's pose is
    synthetic.layered_pose(t_last) (rotation + forward motion), else rotation(t_last)."""
    n = len(kps_last)
    has = depth_last > 0
    idx = np.nonzero(has)[0]
    if layered:
        R, t = S.layered_pose(t_last)
        xyz = unproject(kps_last[idx], depth_last[idx], R, cam, t)
    else:
        xyz = unproject(kps_last[idx], depth_last[idx], S.rotation(t_last), cam)
    rng = rng or np.random.default_rng(0)
    blocks = (rng.random(len(idx)) < blocks_frac).astype(np.int32)
    q = np.zeros(len(idx), G.F2F_QUERY_DTYPE)
    q["xyz"] = xyz
    q["last_angle"] = kps_last["angle"][idx]
    q["last_octave"] = kps_last["octave"][idx]
    q["mp_id"] = np.arange(len(idx), dtype=np.int32)
    q["blocks"] = blocks
    q["desc"] = desc_last[idx]
    last_mp = np.full(n, -1, np.int32)
    last_mp[idx] = np.arange(len(idx), dtype=np.int32)
    last_outlier = np.zeros(n, np.uint8)
    return q, last_mp, last_outlier, xyz, desc_last[idx].copy(), blocks.astype(np.int32)


def pose(t, th=7.0, mono=0, check_ori=1, cam=S.KITTI_CAM, layered=False, t_last=None):
    """F2F pose of frame t (layered: synthetic.layered_pose, with tlc_z = z of frame t's centre
    in frame t_last's camera, t_last defaulting to t - 1)."""
    p = np.zeros(1, G.F2F_POSE_DTYPE)
    if layered:
        R, tc = S.layered_pose(t)
        p["Rcw"] = R.astype(np.float32).reshape(-1)
        p["tcw"] = tc.astype(np.float32)
        tl = t - 1 if t_last is None else t_last
        p["tlc_z"] = np.float32((S.rotation(tl) @ (S.camera_center(t) - S.camera_center(tl)))[2])
        p["th"] = th
        p["baseline"] = np.float32(cam[4]) / np.float32(cam[0])
        p["mono"] = mono
        p["check_ori"] = check_ori
        return p
    p["Rcw"] = S.rotation(t).astype(np.float32).reshape(-1)
    p["tcw"] = 0.0
    p["tlc_z"] = 0.0
    p["baseline"] = np.float32(cam[4]) / np.float32(cam[0])
    p["th"] = th
    p["mono"] = mono
    p["check_ori"] = check_ori
    return p
