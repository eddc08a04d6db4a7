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


# ---- the bench's KITTI-like sequence ---------------------------------------------------------
# 200-320 fronto-parallel surfaces (side 30-220 x 20-160 px at frame 0, one disparity each,
# U[3, 50] px), each carrying 4-12 small patches (3-24 px) at its own depth, over a U[60, 200]
# background, N(0, 3) noise per view. Corners mostly lie INSIDE a surface (patch corners), so
# the right view sees them unchanged, as on KITTI's textured road and facades: ~45-50 % of the
# left keypoints get stereo depth (the rectangles scene above: ~17 %), ~950 frame-to-frame
# queries and ~700 matches per frame. The camera moves forward FORWARD_M per frame and turns as
# rotation(t) (about 3 px / -1 px of image motion and 0.5 deg of roll), so near surfaces grow
# and move faster than far ones (parallax), as in SURVEY.md section 8(d)'s motion model.
FORWARD_M = 0.3


def camera_center(t: int) -> np.ndarray:
    return np.array([0.0, 0.0, FORWARD_M * t])


def layered_pose(t: int):
    """(Rcw, tcw) of frame t of layered_sequence: Rcw = rotation(t), tcw = -Rcw C(t)."""
    R = rotation(t)
    return R, -R @ camera_center(t)


def _layered_scene(rng: np.random.Generator, cols: int, rows: int):
    items = []  # (x, y, w, h, val, disparity, surface, patch index)
    ns = int(rng.integers(200, 321))
    for i in range(ns):
        w, h = int(rng.integers(30, 220)), int(rng.integers(20, 160))
        x, y = int(rng.integers(-60, cols)), int(rng.integers(-40, rows))
        d = float(rng.uniform(3.0, 50.0))
        items.append((x, y, w, h, int(rng.integers(0, 256)), d, i, 0))
        for j in range(int(rng.integers(4, 13))):
            pw = int(rng.integers(3, max(4, min(24, w // 2))))
            ph = int(rng.integers(3, max(4, min(24, h // 2))))
            px = x + int(rng.integers(0, max(1, w - pw)))
            py = y + int(rng.integers(0, max(1, h - ph)))
            items.append((px, py, pw, ph, int(rng.integers(0, 256)), d, i, j + 1))
    return int(rng.integers(60, 201)), items


def layered_pair(seed: int, t: int = 0, cols: int = KITTI_COLS, rows: int = KITTI_ROWS):
    """Left/right u8 images of frame t of the layered scene `seed` (pose layered_pose(t))."""
    rng = np.random.Generator(np.random.PCG64([seed, 23]))
    bg, items = _layered_scene(rng, cols, rows)
    fx, fy, cx0, cy0, bf = KITTI_CAM
    R, C = rotation(t), camera_center(t)
    draw = []
    for (x, y, w, h, val, d, surf, j) in items:
        z0 = bf / d
        cx, cy = x + 0.5 * w, y + 0.5 * h
        Xw = np.array([(cx - cx0) * z0 / fx, (cy - cy0) * z0 / fy, z0])
        Xc = R @ (Xw - C)
        if Xc[2] < 1.0:
            continue
        sc = z0 / Xc[2]
        u, v = fx * Xc[0] / Xc[2] + cx0, fy * Xc[1] / Xc[2] + cy0
        draw.append((bf / Xc[2], surf, j, u, v, w * sc, h * sc, val))
    draw.sort(key=lambda e: (e[0], e[1], e[2]))  # far to near; a surface before its patches
    noise = np.random.Generator(np.random.PCG64([seed, t, 29]))
    out = []
    for right in (False, True):
        img = np.full((rows, cols), float(bg), dtype=np.float32)
        for (disp, _, _, u, v, w, h, val) in draw:
            x0 = int(round(u - (disp if right else 0.0) - 0.5 * w))
            y0 = int(round(v - 0.5 * h))
            x1, y1 = max(0, x0), max(0, y0)
            x2, y2 = min(cols, x0 + max(1, int(round(w)))), min(rows, y0 + max(1, int(round(h))))
            if x1 < x2 and y1 < y2:
                img[y1:y2, x1:x2] = val
        img += noise.normal(0.0, 3.0, size=img.shape).astype(np.float32)
        out.append(np.clip(np.rint(img), 0, 255).astype(np.uint8))
    return out[0], out[1]


def layered_sequence(seed: int, n: int, cols: int = KITTI_COLS, rows: int = KITTI_ROWS):
    """n consecutive stereo frames of the layered scene: (left[n], right[n])."""
    L = np.empty((n, rows, cols), np.uint8)
    R = np.empty_like(L)
    for t in range(n):
        L[t], R[t] = layered_pair(seed, t, cols, rows)
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


def sim3_problem(seed: int, n: int = 300, outlier_frac: float = 0.1, noise_px: float = 0.7,
                 scale: float = 1.3, rot_err: float = 0.03, trans_err: float = 0.2,
                 scale_err: float = 0.05, fix_scale: bool = False, cam1=KITTI_CAM, cam2=KITTI_CAM,
                 cols: int = KITTI_COLS, rows: int = KITTI_ROWS, nlevels: int = 8,
                 scale_factor: float = 1.2):
    """One OptimizeSim3 input (optimizer.cpp:962-1152): n matched map points between a loop
    keyframe pair. The true S12 maps camera-2 coordinates into camera 1: X1c = s R X2c + t
    (scale 1 when fix_scale, as the stereo loop closer uses it). Points are drawn in camera 2's
    view at depth U[3, 40] m; each is observed by keyframe 1 at project(K1, X1c) and keyframe 2
    at project(K2, X2c) with N(0, noise_px * 1.2^octave) pixel noise; outlier_frac of the pairs
    get a uniform keyframe-1 pixel. The initial S12 (the RANSAC Sim3Solver's) is the truth
    perturbed by rot_err rad, trans_err m and exp(N(0, scale_err)). Returns (matches
    [SIM3_MATCH_DTYPE], S12_init f64[8] (qx, qy, qz, qw, t, s), S12_true, inv_sigma2, bad)."""
    rng = np.random.default_rng(seed)
    s_true = 1.0 if fix_scale else float(scale)
    R = _rodrigues(rng.normal(0, 0.15, 3))
    t = rng.normal(0, 1.5, 3)
    fx2, fy2, cx2, cy2 = cam2[:4]
    fx1, fy1, cx1, cy1 = cam1[:4]
    u2 = rng.uniform(0, cols, n)
    v2 = rng.uniform(0, rows, n)
    z2 = rng.uniform(3.0, 40.0, n)
    X2 = np.stack([(u2 - cx2) / fx2 * z2, (v2 - cy2) / fy2 * z2, z2], 1)
    X1 = s_true * X2 @ R.T + t
    keep = X1[:, 2] > 0.5
    X1, X2, u2, v2 = X1[keep], X2[keep], u2[keep], v2[keep]
    n = len(X1)
    o1 = np.minimum(rng.geometric(0.45, n) - 1, nlevels - 1).astype(np.int32)
    o2 = np.minimum(rng.geometric(0.45, n) - 1, nlevels - 1).astype(np.int32)
    u1 = X1[:, 0] / X1[:, 2] * fx1 + cx1 + rng.normal(0, 1, n) * noise_px * scale_factor ** o1
    v1 = X1[:, 1] / X1[:, 2] * fy1 + cy1 + rng.normal(0, 1, n) * noise_px * scale_factor ** o1
    u2o = u2 + rng.normal(0, 1, n) * noise_px * scale_factor ** o2
    v2o = v2 + rng.normal(0, 1, n) * noise_px * scale_factor ** o2
    bad = rng.uniform(0, 1, n) < outlier_frac
    u1 = np.where(bad, rng.uniform(0, cols, n), u1)
    v1 = np.where(bad, rng.uniform(0, rows, n), v1)
    from .slamgpu import SIM3_MATCH_DTYPE
    m = np.zeros(n, SIM3_MATCH_DTYPE)
    m["x1c"] = X1.astype(np.float32)
    m["x2c"] = X2.astype(np.float32)
    m["u1"], m["v1"] = u1.astype(np.float32), v1.astype(np.float32)
    m["u2"], m["v2"] = u2o.astype(np.float32), v2o.astype(np.float32)
    m["octave1"], m["octave2"] = o1, o2

    def pack(Rm, tv, sv):
        q = _quat_from_R(Rm)
        return np.array([q[0], q[1], q[2], q[3], tv[0], tv[1], tv[2], sv], np.float64)

    S_true = pack(R, t, s_true)
    R0 = _rodrigues(rng.normal(0, rot_err / np.sqrt(3), 3)) @ R
    t0 = t + rng.normal(0, trans_err / np.sqrt(3), 3)
    s0 = s_true if fix_scale else s_true * float(np.exp(rng.normal(0, scale_err)))
    return m, pack(R0, t0, s0), S_true, level_inv_sigma2(scale_factor, nlevels), bad


def _sim3_pack(R, t, s):
    q = _quat_from_R(R)
    return np.array([q[0], q[1], q[2], q[3], t[0], t[1], t[2], s], np.float64)


def _sim3_mat(S8):
    x, y, z, w = S8[:4]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    M = np.eye(4)
    M[:3, :3] = S8[7] * R
    M[:3, 3] = S8[4:7]
    return M


def _sim3_from_mat(M):
    s = float(np.cbrt(np.linalg.det(M[:3, :3])))
    return _sim3_pack(M[:3, :3] / s, M[:3, 3], s)


def essential_graph_problem(seed: int, n_kf: int = 60, fix_scale: bool = True,
                            drift_rot: float = 0.004, drift_trans: float = 0.02,
                            drift_scale: float = 0.01, meas_noise=None,
                            covis: int = 3, neighbourhood: int = 4, loop_kf: int = 1,
                            old_loop=None):
    """One OptimizeEssentialGraph input (optimizer.cpp:718-960) for a loop closure: n_kf
    keyframes on a circle (truth), their drifted estimates (rotation / translation / scale random
    walks; scale kept at 1 when fix_scale, the stereo case), and the graph the reference builds:
      1. loop connections (:784-812): each keyframe of the current keyframe's neighbourhood
         (the last `neighbourhood` ones) to the loop keyframe's (loop_kf - 1 .. loop_kf + 2),
         measured from the corrected poses vScw;
      2. per keyframe in id order (:815-909): the spanning-tree edge to its parent (the previous
         keyframe), loop edges to older keyframes (old_loop = (a, b), a > b), covisibility edges
         to the `covis` previous keyframes that are not its parent and not already a loop
         connection, measured from the non-corrected poses.
    The current keyframe's neighbourhood is corrected to the truth (what ComputeSim3 + the loop
    correction give, corrected_sim3); non_corrected keeps their drifted poses. meas_noise None:
    measurements Sjw * Swi from those estimates, as the reference forms them; a float: the true
    relative Sim3s perturbed by that much (0: a consistent graph whose optimum is the truth).
    Returns (Scw_init [n][8], fixed [n] u8, edges [SIM3_EDGE_DTYPE], Scw_true [n][8],
    Scw_drift [n][8])."""
    rng = np.random.default_rng(seed)
    from .slamgpu import SIM3_EDGE_DTYPE
    n = n_kf
    radius = 30.0
    truth, drift = [], []
    D = np.eye(4)
    for k in range(n):
        a = 2 * np.pi * k / n
        Rwc = _rodrigues(np.array([0.0, -a, 0.0]))
        twc = np.array([radius * np.sin(a), 0.0, radius * (1 - np.cos(a))])
        Tcw = np.eye(4)
        Tcw[:3, :3] = Rwc.T
        Tcw[:3, 3] = -Rwc.T @ twc
        truth.append(Tcw)
        if k == 0:
            D = Tcw.copy()
        else:
            rel = truth[k] @ np.linalg.inv(truth[k - 1])  # T_k,k-1
            N = np.eye(4)
            N[:3, :3] = _rodrigues(rng.normal(0, drift_rot, 3))
            N[:3, 3] = rng.normal(0, drift_trans, 3)
            sc = 1.0 if fix_scale else float(np.exp(rng.normal(0, drift_scale)))
            D = N @ rel @ D
            if not fix_scale:
                D = np.diag([sc, sc, sc, 1.0]) @ D
        drift.append(D.copy())
    S_true = np.stack([_sim3_from_mat(T) for T in truth])
    S_drift = np.stack([_sim3_from_mat(T) for T in drift])
    cur = n - 1
    hood = list(range(n - neighbourhood, n))
    S_cw = S_drift.copy()
    for k in hood:
        S_cw[k] = S_true[k]  # corrected_sim3
    S_cw[loop_kf] = S_true[loop_kf]
    S_drift[loop_kf] = S_true[loop_kf]
    fixed = np.zeros(n, np.uint8)
    fixed[loop_kf] = 1
    noncorr = {k: S_drift[k] for k in hood}

    def meas(j, i, Sj, Si):
        if meas_noise is None:  # the reference: Sji = Sjw * Swi from the estimates
            return _sim3_from_mat(_sim3_mat(Sj) @ np.linalg.inv(_sim3_mat(Si)))
        M = truth[j] @ np.linalg.inv(truth[i])
        if meas_noise > 0:
            N = np.eye(4)
            N[:3, :3] = _rodrigues(rng.normal(0, meas_noise, 3))
            N[:3, 3] = rng.normal(0, 10 * meas_noise, 3)
            M = N @ M
        return _sim3_from_mat(M)

    edges = []
    inserted = set()
    loop_hood = [k for k in range(loop_kf - 1, loop_kf + 3) if 0 <= k < n]
    for i in hood:
        for j in loop_hood:
            edges.append((i, j, meas(j, i, S_cw[j], S_cw[i])))
            inserted.add((min(i, j), max(i, j)))
    for i in range(n):
        Si = noncorr.get(i, S_cw[i])
        if i > 0:
            p = i - 1
            edges.append((i, p, meas(p, i, noncorr.get(p, S_cw[p]), Si)))
        loops = [old_loop[1]] if old_loop is not None and i == old_loop[0] else []
        for l in loops:
            edges.append((i, l, meas(l, i, noncorr.get(l, S_cw[l]), Si)))
        for j in range(max(0, i - covis), i - 1):
            if j in loops or (min(i, j), max(i, j)) in inserted:
                continue
            edges.append((i, j, meas(j, i, noncorr.get(j, S_cw[j]), Si)))
    E = np.zeros(len(edges), SIM3_EDGE_DTYPE)
    for k, (i, j, M) in enumerate(edges):
        E[k]["i"], E[k]["j"], E[k]["Sji"] = i, j, M
    return S_cw, fixed, E, S_true, S_drift


def _quat_from_R(R: np.ndarray) -> np.ndarray:
    """(x, y, z, w) of a rotation matrix, w >= 0."""
    w = np.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.copysign(np.sqrt(max(0.0, 1.0 + R[0, 0] - R[1, 1] - R[2, 2])) / 2, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] + R[1, 1] - R[2, 2])) / 2, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] - R[1, 1] + R[2, 2])) / 2, R[1, 0] - R[0, 1])
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q)


def c4_problem(seed: int = 7, n: int = 2000, cam=KITTI_CAM, nlevels: int = 8,
               scale_factor: float = 1.2):
    """SURVEY.md section 8(d) C4, the PoseOptimization bench workload: n world points uniform in
    x in [-15, 15], y in [-3, 3], z in [5, 40] m (camera frame of the true pose), KITTI
    intrinsics, 60% stereo observations (ur = u - bf / z), octave U{0..7} with N(0, sigma_l^2)
    pixel noise (sigma_l = 1.2^l), 10% gross outliers (+-30 px), initial pose perturbed by
    2 degrees / 0.3 m. Same return tuple as pose_problem."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    Rt = _rodrigues(rng.normal(0, 0.1, 3))
    tt = rng.normal(0, 3.0, 3)
    Xc = np.stack([rng.uniform(-15, 15, n), rng.uniform(-3, 3, n), rng.uniform(5, 40, n)], 1)
    Xw = (Xc - tt) @ Rt
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    octave = rng.integers(0, nlevels, n).astype(np.int32)
    sig = np.power(scale_factor, octave)
    uo, vo = u + rng.normal(0, 1, n) * sig, v + rng.normal(0, 1, n) * sig
    stereo = rng.uniform(0, 1, n) < 0.6
    uro = np.where(stereo, u - bf / Xc[:, 2] + rng.normal(0, 1, n) * sig, -1.0)
    bad = rng.uniform(0, 1, n) < 0.1
    uo = np.where(bad, uo + rng.choice([-30.0, 30.0], n), uo)
    vo = np.where(bad, vo + rng.choice([-30.0, 30.0], n), vo)
    uro = np.where(bad & stereo, uro + rng.choice([-30.0, 30.0], n), uro)
    from .slamgpu import POSE_EDGE_DTYPE
    edges = np.zeros(n, POSE_EDGE_DTYPE)
    edges["xw"] = Xw.astype(np.float32)
    edges["u"], edges["v"], edges["ur"] = uo, vo, uro
    edges["octave"] = octave
    T_true = np.eye(4)
    T_true[:3, :3], T_true[:3, 3] = Rt, tt
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    tdir = rng.normal(size=3)
    tdir /= np.linalg.norm(tdir)
    T0 = np.eye(4)
    T0[:3, :3] = _rodrigues(np.deg2rad(2.0) * axis) @ Rt
    T0[:3, 3] = tt + 0.3 * tdir
    return edges, T0.astype(np.float32), T_true, level_inv_sigma2(scale_factor, nlevels), bad


def c5_problem(seed: int = 11, **kw):
    """SURVEY.md section 8(d) C5, the LocalBundleAdjustment bench workload: 20 free + 5 fixed
    keyframes on a forward trajectory with 1 m spacing (the oldest, keyframe 0, among the fixed),
    3000 points each seen by 2-6 keyframes (about 12k edges), the C4 noise model."""
    args = dict(n_local=20, n_fixed=5, n_points=3000, max_obs=6, spacing=1.0)
    args.update(kw)
    return ba_problem(seed, **args)


def pose_batch(seed: int, n_frames: int, n: int = 2000, **kw):
    """n_frames independent pose problems packed as the device call takes them: edges of frame f
    at [start[f], start[f+1]), poses (n_frames, 4, 4) f32."""
    probs = [pose_problem(seed + f, n, **kw) for f in range(n_frames)]
    edges = np.concatenate([p[0] for p in probs])
    start = np.zeros(n_frames + 1, np.int32)
    start[1:] = np.cumsum([len(p[0]) for p in probs])
    poses = np.stack([p[1] for p in probs])
    return edges, start, poses, probs[0][3], probs


def ba_problem(seed: int, n_local: int = 20, n_fixed: int = 6, n_points: int = 3000,
               max_obs: int = 6, stereo_frac: float = 0.6, outlier_frac: float = 0.05,
               noise_px: float = 0.7, rot_err: float = 0.003, trans_err: float = 0.03,
               point_err: float = 0.05, first_local_fixed: bool = False, spacing: float = 1.2,
               cam=KITTI_CAM,
               cols: int = KITTI_COLS, rows: int = KITTI_ROWS, nlevels: int = 8,
               scale_factor: float = 1.2):
    """One LocalBundleAdjustment input (configs[4]: 20 keyframes x 3000 map points).

    A KITTI-like drive: keyframe k sits `spacing` m further along z with a slow yaw. The n_fixed
    oldest keyframes are fixed cameras (kf_mode 2), the n_local newest the local window
    (kf_mode 0; the first one 1 = local but fixed, like keyframe id 0, if first_local_fixed).
    Each map point lies ahead of the window and is observed by 2..max_obs keyframes that see it
    inside the image at depth (1, 60) m, with at least one local keyframe among them, in random
    order (the reference iterates a std::map keyed by KeyFrame*); observations carry
    octave-scaled pixel noise, stereo_frac of them a right coordinate, outlier_frac are gross
    mismatches. The local poses and the points start perturbed (rot_err rad, trans_err m,
    point_err m). Returns a dict of the arrays the device call takes plus the ground truth."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    n_kf = n_fixed + n_local
    Rs, cs = [], []
    for k in range(n_kf):
        yaw = 0.01 * k
        R_wc = _rodrigues(np.array([0.0, yaw, 0.0]))
        c = np.array([3.0 * np.sin(0.01 * k), 0.0, spacing * k])
        Rs.append(R_wc.T)  # Rcw
        cs.append(c)
    T_true = np.zeros((n_kf, 4, 4))
    for k in range(n_kf):
        T_true[k, :3, :3] = Rs[k]
        T_true[k, :3, 3] = -Rs[k] @ cs[k]
        T_true[k, 3, 3] = 1.0
    mode = np.full(n_kf, 2, np.uint8)
    mode[n_fixed:] = 0
    if first_local_fixed:
        mode[n_fixed] = 1
    local = np.nonzero(mode != 2)[0]
    pts, obs_lists = [], []
    z0, z1 = cs[n_fixed][2] + 2.0, cs[-1][2] + 45.0
    while len(pts) < n_points:
        X = np.array([rng.uniform(-25, 25), rng.uniform(-4, 3), rng.uniform(z0, z1)])
        seen = []
        for k in range(n_kf):
            Xc = T_true[k, :3, :3] @ X + T_true[k, :3, 3]
            if not (1.0 < Xc[2] < 60.0):
                continue
            u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
            if 0 <= u < cols and 0 <= v < rows:
                seen.append(k)
        if len(seen) < 2 or not any(mode[k] == 0 for k in seen):
            continue
        m = int(rng.integers(2, max_obs + 1))
        if len(seen) > m:
            loc = [k for k in seen if mode[k] == 0]
            first = int(rng.choice(loc))
            rest = [k for k in seen if k != first]
            seen = [first] + list(rng.choice(rest, m - 1, replace=False))
        rng.shuffle(seen)
        pts.append(X)
        obs_lists.append(seen)
    from .slamgpu import BA_OBS_DTYPE
    n_obs = sum(len(o) for o in obs_lists)
    obs = np.zeros(n_obs, BA_OBS_DTYPE)
    start = np.zeros(n_points + 1, np.int32)
    i = 0
    for p, (X, ks) in enumerate(zip(pts, obs_lists)):
        start[p] = i
        for k in ks:
            Xc = T_true[k, :3, :3] @ X + T_true[k, :3, 3]
            u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
            octv = min(int(rng.geometric(0.45)) - 1, nlevels - 1)
            sig = noise_px * scale_factor ** octv
            uo, vo = u + rng.normal(0, sig), v + rng.normal(0, sig)
            stereo = rng.uniform() < stereo_frac
            uro = u - bf / Xc[2] + rng.normal(0, sig) if stereo else -1.0
            if rng.uniform() < outlier_frac:
                uo, vo = rng.uniform(0, cols), rng.uniform(0, rows)
                if stereo:
                    uro = max(uo - rng.uniform(0, 90), 0.0)
            obs[i] = (k, uo, vo, uro, octv)
            i += 1
    start[n_points] = i
    kf = T_true.copy()
    for k in np.nonzero(mode == 0)[0]:
        kf[k, :3, :3] = _rodrigues(rng.normal(0, rot_err / np.sqrt(3), 3)) @ kf[k, :3, :3]
        kf[k, :3, 3] += rng.normal(0, trans_err / np.sqrt(3), 3)
    P = np.array(pts) + rng.normal(0, point_err / np.sqrt(3), (n_points, 3))
    return {"kf_Tcw": kf.astype(np.float32), "kf_mode": mode, "points": P.astype(np.float32),
            "point_obs_start": start, "obs": obs,
            "inv_sigma2": level_inv_sigma2(scale_factor, nlevels),
            "kf_true": T_true, "points_true": np.array(pts)}


def map_problem(seed: int, n_kf: int = 1500, points_per_kf: int = 40, max_obs: int = 6,
                spacing: float = 1.0, stereo_frac: float = 0.6, outlier_frac: float = 0.02,
                noise_px: float = 0.7, rot_err: float = 0.002, trans_err: float = 0.05,
                point_err: float = 0.05, cam=KITTI_CAM, cols: int = KITTI_COLS,
                rows: int = KITTI_ROWS, nlevels: int = 8, scale_factor: float = 1.2):
    """A map-scale global BundleAdjustment input (optimizer.cpp:18-207 over every keyframe): a
    closed loop of n_kf keyframes `spacing` m apart on a circle (a KITTI-00-like drive that comes
    back to its start), keyframe 0 fixed (kf_mode 1, Id() == 0), the others free. Each keyframe
    spawns points_per_kf points 4-40 m ahead of it; a point is observed by up to max_obs of the
    keyframes within +-12 of its spawner that see it in the image (vectorised: no per-keyframe
    Python loop), so the keyframes at the end of the loop co-observe points with those at its
    start -- the reduced camera system is a band plus the rows a loop closure reaches back from.
    Same noise model as ba_problem; returns its dict."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    Rr = n_kf * spacing / (2 * np.pi)
    ang = 2 * np.pi * np.arange(n_kf) / n_kf
    C = np.stack([Rr * np.sin(ang), np.zeros(n_kf), Rr * (1 - np.cos(ang))], 1)  # centres
    T_true = np.zeros((n_kf, 4, 4))
    for k in range(n_kf):
        R_wc = _rodrigues(np.array([0.0, -ang[k], 0.0]))  # heading along the tangent
        T_true[k, :3, :3] = R_wc.T
        T_true[k, :3, 3] = -R_wc.T @ C[k]
        T_true[k, 3, 3] = 1.0
    mode = np.zeros(n_kf, np.uint8)
    mode[0] = 1
    n_pts = n_kf * points_per_kf
    home = np.repeat(np.arange(n_kf), points_per_kf)
    Xc0 = np.stack([rng.uniform(-12, 12, n_pts), rng.uniform(-3, 2, n_pts),
                    rng.uniform(4, 40, n_pts)], 1)
    Rwc = np.transpose(T_true[home, :3, :3], (0, 2, 1))
    X = np.einsum("nij,nj->ni", Rwc, Xc0) + C[home]
    offs = np.arange(-12, 13)
    cand = (home[:, None] + offs[None, :]) % n_kf                  # [n_pts, 25]
    Rc, tc = T_true[cand, :3, :3], T_true[cand, :3, 3]
    Xc = np.einsum("npij,nj->npi", Rc, X) + tc
    with np.errstate(divide="ignore", invalid="ignore"):
        u = fx * Xc[..., 0] / Xc[..., 2] + cx
        v = fy * Xc[..., 1] / Xc[..., 2] + cy
    vis = (Xc[..., 2] > 1.0) & (Xc[..., 2] < 60.0) & (u >= 0) & (u < cols) & (v >= 0) & (v < rows)
    vis[:, 12] = True  # the spawner sees it (4-40 m straight ahead)
    # up to max_obs observers per point: random order among the visible candidates
    keys = np.where(vis, rng.random(vis.shape), 2.0)
    order = np.argsort(keys, 1)[:, :max_obs]
    nvis = np.minimum(vis.sum(1), max_obs)
    keep = nvis >= 2
    order, nvis = order[keep], nvis[keep]
    X, cand, Xc, u, v = X[keep], cand[keep], Xc[keep], u[keep], v[keep]
    n_pts = len(X)
    from .slamgpu import BA_OBS_DTYPE
    start = np.zeros(n_pts + 1, np.int32)
    start[1:] = np.cumsum(nvis)
    n_obs = int(start[-1])
    rowi = np.repeat(np.arange(n_pts), nvis)
    coli = order[np.arange(max_obs)[None, :] < nvis[:, None]]
    kk, uu, vv, zz = cand[rowi, coli], u[rowi, coli], v[rowi, coli], Xc[rowi, coli, 2]
    octv = np.minimum(rng.geometric(0.45, n_obs) - 1, nlevels - 1)
    sig = noise_px * scale_factor ** octv
    uo, vo = uu + rng.normal(0, 1, n_obs) * sig, vv + rng.normal(0, 1, n_obs) * sig
    stereo = rng.random(n_obs) < stereo_frac
    uro = np.where(stereo, uu - bf / zz + rng.normal(0, 1, n_obs) * sig, -1.0)
    out = rng.random(n_obs) < outlier_frac
    uo[out], vo[out] = rng.uniform(0, cols, out.sum()), rng.uniform(0, rows, out.sum())
    uro[out & stereo] = np.maximum(uo[out & stereo] - rng.uniform(0, 90, (out & stereo).sum()), 0)
    obs = np.zeros(n_obs, BA_OBS_DTYPE)
    obs["keyframe"], obs["u"], obs["v"], obs["ur"], obs["octave"] = kk, uo, vo, uro, octv
    kf = T_true.copy()
    for k in range(1, n_kf):
        kf[k, :3, :3] = _rodrigues(rng.normal(0, rot_err / np.sqrt(3), 3)) @ kf[k, :3, :3]
        kf[k, :3, 3] += rng.normal(0, trans_err / np.sqrt(3), 3)
    P = X + rng.normal(0, point_err / np.sqrt(3), (n_pts, 3))
    return {"kf_Tcw": kf.astype(np.float32), "kf_mode": mode, "points": P.astype(np.float32),
            "point_obs_start": start, "obs": obs,
            "inv_sigma2": level_inv_sigma2(scale_factor, nlevels),
            "kf_true": T_true, "points_true": X}


# ---- DBoW2 vocabularies: ORBvoc.txt is not in the reference ------
def vocabulary(seed: int, k: int = 10, L: int = 6, pool=None, scoring: int = 0,
               weighting: int = 0, stop_frac: float = 0.02):
    """A DBoW2 vocabulary as the arrays TemplatedVocabulary::loadFromTextFile builds
    (TemplatedVocabulary.h:1335-1421): a complete k-ary tree of depth L in breadth-first node order
    (parent < child, node 0 = root), the depth-L leaves flagged as words (ORBvoc.txt's shape is
    k = 10, L = 6, L1_NORM / TF_IDF). Level-1 and level-2 centres are drawn from `pool` (real ORB
    descriptors) when it is large enough, so that similar descriptors descend alike; otherwise,
    and deeper, a child flips each bit of its parent's descriptor with probability 1/2 (levels
    1-2), 1/8 (level 3) or 1/16. Word weights are idf-like U(0.1, 8), stop_frac of them 0
    (stopped words); internal nodes weigh 0."""
    rng = np.random.default_rng(seed)
    sizes = [k ** l for l in range(L + 1)]
    n = sum(sizes)
    parent = np.zeros(n, np.int32)
    leaf = np.zeros(n, np.uint8)
    desc = np.zeros((n, 32), np.uint8)
    weight = np.zeros(n, np.float64)
    prev, start = 0, 1
    for lvl in range(1, L + 1):
        cnt = sizes[lvl]
        par = prev + np.arange(cnt) // k
        parent[start:start + cnt] = par
        if pool is not None and lvl <= 2 and len(pool) >= cnt:
            d = np.asarray(pool, np.uint8).reshape(-1, 32)[rng.choice(len(pool), cnt,
                                                                      replace=False)]
        else:
            m = rng.integers(0, 256, (cnt, 32), dtype=np.uint8)
            for _ in range(0 if lvl <= 2 else (2 if lvl == 3 else 3)):
                m &= rng.integers(0, 256, (cnt, 32), dtype=np.uint8)
            d = desc[par] ^ m
        desc[start:start + cnt] = d
        prev, start = start, start + cnt
    leaf[prev:] = 1
    w = rng.uniform(0.1, 8.0, sizes[L])
    w[rng.random(sizes[L]) < stop_frac] = 0.0
    weight[prev:] = w
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=parent, leaf=leaf,
                desc=desc, weight=weight)


def random_tree_vocabulary(seed: int, n_nodes: int = 300, scoring: int = 0, weighting: int = 0,
                           unflagged_frac: float = 0.1, stop_frac: float = 0.1):
    """An unbalanced vocabulary tree (every node's parent a uniformly chosen earlier node):
    leaves at mixed depths, childless nodes without the leaf flag (word id 0 with their own
    weight, the Node() default), stopped words. L = the tree's depth."""
    rng = np.random.default_rng(seed)
    parent = np.zeros(n_nodes, np.int32)
    depth = np.zeros(n_nodes, np.int32)
    for i in range(1, n_nodes):
        parent[i] = rng.integers(0, i)
        depth[i] = depth[parent[i]] + 1
    has_child = np.zeros(n_nodes, bool)
    has_child[parent[1:]] = True
    leaf = (~has_child).astype(np.uint8)
    leaf[0] = 0
    leaf[(rng.random(n_nodes) < unflagged_frac)] = 0
    desc = rng.integers(0, 256, (n_nodes, 32), dtype=np.uint8)
    weight = rng.uniform(0.1, 5.0, n_nodes)
    weight[rng.random(n_nodes) < stop_frac] = 0.0
    weight[0] = 0.0
    return dict(k=min(20, int(np.bincount(parent[1:]).max())), L=int(depth.max()), scoring=scoring,
                weighting=weighting, parent=parent, leaf=leaf, desc=desc, weight=weight)


def vocabulary_text(V, trailing_newline: bool = True) -> str:
    """V in the text format loadFromTextFile reads (saveToTextFile's layout, :1426-1446)."""
    lines = [f"{V['k']} {V['L']}  {V['scoring']} {V['weighting']}"]
    for i in range(1, len(V["parent"])):
        lines.append(f"{int(V['parent'][i])} {int(V['leaf'][i])} "
                     + " ".join(str(int(b)) for b in V["desc"][i])
                     + f"  {repr(float(V['weight'][i]))}")
    return "\n".join(lines) + ("\n" if trailing_newline else "")
