"""Matcher scenarios built from oracle front-end results (test infrastructure).

`vo_queries` mirrors Tracker::UpdateLastFrame's visual-odometry points (tracker.cpp:695-753):
every last-frame keypoint with stereo depth becomes a map point at UnprojectStereo(i)
(frame.cpp:594-607), with the keypoint's descriptor. Poses come from synthetic.rotation().
"""
import numpy as np

from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S


def unproject(kps, depth, Rcw, cam):
    fx, fy, cx, cy, _ = [np.float32(v) for v in cam]
    z = depth.astype(np.float32)
    x = (kps["x"] - cx) * z * (np.float32(1) / fx)
    y = (kps["y"] - cy) * z * (np.float32(1) / fy)
    Xc = np.stack([x, y, z], 1).astype(np.float64)
    return (Xc @ np.asarray(Rcw, np.float64)).astype(np.float32)  # Rwc @ Xc, Rwc = Rcw^T


def vo_queries(kps_last, desc_last, depth_last, t_last, rng=None, blocks_frac=1.0, cam=S.KITTI_CAM):
    """Queries in last-frame keypoint order; returns (queries, last_mp, last_outlier, mp_xyz,
    mp_desc, mp_nobs) for both the oracle and the HIP path."""
    n = len(kps_last)
    has = depth_last > 0
    idx = np.nonzero(has)[0]
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


def pose(t, th=7.0, mono=0, check_ori=1, cam=S.KITTI_CAM):
    p = np.zeros(1, G.F2F_POSE_DTYPE)
    p["Rcw"] = S.rotation(t).astype(np.float32).reshape(-1)
    p["tcw"] = 0.0
    p["tlc_z"] = 0.0
    p["baseline"] = np.float32(cam[4]) / np.float32(cam[0])
    p["th"] = th
    p["mono"] = mono
    p["check_ori"] = check_ori
    return p
