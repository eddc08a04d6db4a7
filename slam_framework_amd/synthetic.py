"""Seeded synthetic stereo input: no KITTI data exists on any box.

A scene is 600-1200 axis-aligned rectangles (side U[4, 80] px, intensity U[0, 255]) painted
over a U[60, 200] background, plus N(0, 3) noise, clamped to u8. The right view renders the
same rectangles shifted left by a per-rectangle disparity U[2, 90] px, painted far-to-near
(small disparity first), with fresh noise. Frame t of a sequence is seen by a camera rotated
by about (3 px, -1 px) of image motion and 0.5 degree of roll per frame, so that
frame-to-frame matching has real correspondences. Frame t is rendered through the homography of a
pure camera rotation (`rotation(t)`), so the pose of frame t is Tcw = [rotation(t) | 0].

numpy's PCG64 stream is platform independent, so every box regenerates identical bytes.
"""
from __future__ import annotations

import numpy as np

KITTI_COLS = 1241
KITTI_ROWS = 376


def _scene(rng: np.random.Generator, cols: int, rows: int):
    n = int(rng.integers(600, 1201))
    w = rng.integers(4, 81, size=n)
    h = rng.integers(4, 81, size=n)
    x = rng.integers(-40, cols, size=n)
    y = rng.integers(-40, rows, size=n)
    val = rng.integers(0, 256, size=n)
    disp = rng.uniform(2.0, 90.0, size=n)
    bg = int(rng.integers(60, 201))
    return bg, x, y, w, h, val, disp


KITTI_CAM = (718.856, 718.856, 607.1928, 185.2157, 386.1448)  # fx, fy, cx, cy, bf


def rotation(t: int) -> np.ndarray:
    """Camera rotation Rcw of sequence frame t (pure rotation about the left camera centre):
    per frame -1 px / +3 px of image motion at the principal point and 0.5 deg of roll."""
    fx = KITTI_CAM[0]
    w = np.array([-1.0 / fx, 3.0 / fx, np.deg2rad(0.5)]) * t
    th = float(np.linalg.norm(w))
    if th == 0.0:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def _homography(t: int) -> np.ndarray:
    fx, fy, cx, cy, _ = KITTI_CAM
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    return K @ rotation(t) @ np.linalg.inv(K)


def _render(cols, rows, bg, x, y, w, h, val, shift, order, rng, H=None):
    img = np.full((rows, cols), float(bg), dtype=np.float32)
    for i in order:
        cxr, cyr = x[i] + 0.5 * w[i], y[i] + 0.5 * h[i]
        if H is not None:  # move the rectangle centre by the frame's rotation homography
            p = H @ np.array([cxr, cyr, 1.0])
            cxr, cyr = p[0] / p[2], p[1] / p[2]
        px, py = cxr - shift[i] - 0.5 * w[i], cyr - 0.5 * h[i]
        x0, y0 = int(round(px)), int(round(py))
        x1, y1 = max(0, x0), max(0, y0)
        x2, y2 = min(cols, x0 + int(w[i])), min(rows, y0 + int(h[i]))
        if x1 < x2 and y1 < y2:
            img[y1:y2, x1:x2] = val[i]
    img += rng.normal(0.0, 3.0, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def stereo_pair(seed: int, cols: int = KITTI_COLS, rows: int = KITTI_ROWS, t: int = 0):
    """Left/right u8 images (rows x cols) of the scene `seed` at sequence frame `t`."""
    rng = np.random.Generator(np.random.PCG64(seed))
    bg, x, y, w, h, val, disp = _scene(rng, cols, rows)
    noise = np.random.Generator(np.random.PCG64([seed, t, 17]))
    H = _homography(t) if t else None
    zero = np.zeros_like(disp)
    order = np.argsort(disp, kind="stable")  # far (small disparity) first
    left = _render(cols, rows, bg, x, y, w, h, val, zero, order, noise, H)
    right = _render(cols, rows, bg, x, y, w, h, val, disp, order, noise, H)
    return left, right


def image(seed: int, cols: int = KITTI_COLS, rows: int = KITTI_ROWS):
    return stereo_pair(seed, cols, rows)[0]


def stereo_batch(seeds, cols: int = KITTI_COLS, rows: int = KITTI_ROWS, t0: int = 0):
    """Stack of stereo pairs: returns (left[B, rows, cols], right[B, rows, cols]) u8."""
    L = np.empty((len(seeds), rows, cols), np.uint8)
    R = np.empty_like(L)
    for i, s in enumerate(seeds):
        L[i], R[i] = stereo_pair(int(s), cols, rows, t0)
    return L, R


def sequence(seed: int, n: int, cols: int = KITTI_COLS, rows: int = KITTI_ROWS):
    """n consecutive stereo frames of one moving scene: (left[n], right[n])."""
    L = np.empty((n, rows, cols), np.uint8)
    R = np.empty_like(L)
    for t in range(n):
        L[t], R[t] = stereo_pair(seed, cols, rows, t)
    return L, R


def _rodrigues(w: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(w))
    if th == 0.0:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def level_inv_sigma2(scale_factor: float = 1.2, nlevels: int = 8) -> np.ndarray:
    """Frame::mvInvLevelSigma2 as ORBextractor builds it (orb_extractor.cpp:357-369, f32)."""
    s2 = np.ones(nlevels, np.float32)
    sc = np.float32(1.0)
    sf = float(np.float32(scale_factor))  # float ctor argument kept in a double member
    for i in range(1, nlevels):
        sc = np.float32(float(sc) * sf)
        s2[i] = np.float32(sc * sc)
    return (np.float32(1.0) / s2).astype(np.float32)


def pose_problem(seed: int, n: int = 2000, stereo_frac: float = 0.6, outlier_frac: float = 0.1,
                 noise_px: float = 0.7, rot_err: float = 0.02, trans_err: float = 0.1,
                 cam=KITTI_CAM, cols: int = KITTI_COLS, rows: int = KITTI_ROWS, nlevels: int = 8,
                 scale_factor: float = 1.2):
    """One PoseOptimization input (configs[3]): n map point / keypoint correspondences of a
    KITTI-like stereo frame.

    True pose: a random rotation (about 10 degrees) and translation (about 5 m). Each point is a
    pixel drawn uniformly over the image at depth U[2, 60] m, seen at octave ~ Geometric(0.45)
    capped at nlevels-1 with N(0, noise_px * scale^octave) pixel noise; a stereo_frac fraction
    has a right coordinate ur = u - bf / z (same noise), the rest ur = -1 (monocular).
    outlier_frac of the observations are replaced by uniform pixels (gross mismatches). The
    initial pose is the true one perturbed by rot_err rad and trans_err m, as a constant-velocity
    prediction would be. Returns (edges[POSE_EDGE_DTYPE order], Tcw_init f32 4x4, Tcw_true f64
    4x4, inv_sigma2 f32[nlevels], is_outlier bool[n])."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    Rt = _rodrigues(rng.normal(0, 0.1, 3))
    tt = rng.normal(0, 3.0, 3)
    u = rng.uniform(0, cols, n)
    v = rng.uniform(0, rows, n)
    z = rng.uniform(2.0, 60.0, n)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Xc - tt) @ Rt  # Rt^T (Xc - t)
    octave = np.minimum(rng.geometric(0.45, n) - 1, nlevels - 1).astype(np.int32)
    sig = noise_px * np.power(scale_factor, octave)
    uo = u + rng.normal(0, 1, n) * sig
    vo = v + rng.normal(0, 1, n) * sig
    stereo = rng.uniform(0, 1, n) < stereo_frac
    uro = np.where(stereo, u - bf / z + rng.normal(0, 1, n) * sig, -1.0)
    bad = rng.uniform(0, 1, n) < outlier_frac
    uo = np.where(bad, rng.uniform(0, cols, n), uo)
    vo = np.where(bad, rng.uniform(0, rows, n), vo)
    uro = np.where(bad & stereo, np.maximum(uo - rng.uniform(0, 90, n), 0.0), uro)
    from .slamgpu import POSE_EDGE_DTYPE
    edges = np.zeros(n, POSE_EDGE_DTYPE)
    edges["xw"] = Xw.astype(np.float32)
    edges["u"] = uo.astype(np.float32)
    edges["v"] = vo.astype(np.float32)
    edges["ur"] = uro.astype(np.float32)
    edges["octave"] = octave
    T_true = np.eye(4)
    T_true[:3, :3], T_true[:3, 3] = Rt, tt
    T0 = np.eye(4)
    T0[:3, :3] = _rodrigues(rng.normal(0, rot_err / np.sqrt(3), 3)) @ Rt
    T0[:3, 3] = tt + rng.normal(0, trans_err / np.sqrt(3), 3)
    return edges, T0.astype(np.float32), T_true, level_inv_sigma2(scale_factor, nlevels), bad


def pose_batch(seed: int, n_frames: int, n: int = 2000, **kw):
    """n_frames independent pose problems packed as the device call takes them: edges of frame f
    at [start[f], start[f+1]), poses (n_frames, 4, 4) f32."""
    probs = [pose_problem(seed + f, n, **kw) for f in range(n_frames)]
    edges = np.concatenate([p[0] for p in probs])
    start = np.zeros(n_frames + 1, np.int32)
    start[1:] = np.cumsum([len(p[0]) for p in probs])
    poses = np.stack([p[1] for p in probs])
    return edges, start, poses, probs[0][3], probs
