"""Keyframe scenes for the SearchForTriangulation / Fuse parity tests: two keyframes built from
the oracle's ORB features of consecutive synthetic frames (no KITTI on any box), their stereo
right coordinates, DBoW2 FeatureVectors on an ORBvoc-shaped vocabulary, and map points
unprojected from the first keyframe's stereo depths."""
import numpy as np

from slam_framework_amd import synthetic as S

CAM = S.KITTI_CAM


def levels_arrays(scale_factor=1.2, nlevels=8):
    sc = np.ones(nlevels, np.float32)
    for i in range(1, nlevels):
        sc[i] = np.float32(float(sc[i - 1]) * float(np.float32(scale_factor)))
    s2 = (sc * sc).astype(np.float32)
    return sc, s2, (np.float32(1.0) / s2).astype(np.float32), \
        np.float32(np.log(np.float64(np.float32(scale_factor))))


def pose(t, trans=(0.0, 0.0, 0.0)):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = S.rotation(t).astype(np.float32)
    T[:3, 3] = np.asarray(trans, np.float32)
    return T


def center(T):
    R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
    return (-R.T @ t).astype(np.float32)


def fundamental(T1, T2, cam=CAM):
    """LocalMapper::ComputeF12: F12 = K^-T [t12]x R12 K^-1 (float64 here, stored f32)."""
    fx, fy, cx, cy, _ = cam
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    R1, t1 = T1[:3, :3].astype(np.float64), T1[:3, 3].astype(np.float64)
    R2, t2 = T2[:3, :3].astype(np.float64), T2[:3, 3].astype(np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    Ki = np.linalg.inv(K)
    return (Ki.T @ tx @ R12 @ Ki).astype(np.float32)


def keyframes(oracle, seed=4100, vocab_seed=41, mp_frac=0.3):
    """Frames 0 and 1 of a sequence as keyframes: kps, desc, ur (stereo right coordinate or -1),
    depth, FeatureVector (levelsup 4) and a has-map-point mask."""
    t = oracle.tables()
    L, R = S.sequence(seed, 2)
    kfs = []
    for i in range(2):
        kl, dl, pl = oracle.extract(t, L[i], True)
        kr, dr, pr = oracle.extract(t, R[i], True)
        ur, depth, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
        kfs.append(dict(kps=kl, desc=dl, ur=ur, depth=depth))
    V = S.vocabulary(vocab_seed, k=10, L=6, pool=kfs[0]["desc"])
    ov = oracle.OracleVocab(V)
    rng = np.random.default_rng(seed)
    for k in kfs:
        k["fv"] = oracle.bow_transform(ov, k["desc"], 4)[2:]
        k["mp"] = (rng.random(len(k["desc"])) < mp_frac).astype(np.uint8)
    return kfs, V


def fuse_points(kf, T, n_extra=40, seed=7):
    """Map points unprojected from keyframe `kf`'s stereo depths at pose T (FUSE_POINT records),
    plus points behind the camera, outside the image, facing away, skipped ones."""
    from slam_framework_amd.kfmatch import FUSE_POINT_DTYPE
    fx, fy, cx, cy, _ = CAM
    sc = levels_arrays()[0]
    rng = np.random.default_rng(seed)
    idx = np.nonzero(kf["depth"] > 0)[0]
    R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
    Ow = center(T).astype(np.float64)
    pts = np.zeros(len(idx) + n_extra, FUSE_POINT_DTYPE)
    for j, i in enumerate(idx):
        z = float(kf["depth"][i])
        kp = kf["kps"][i]
        Xc = np.array([(kp["x"] - cx) * z / fx, (kp["y"] - cy) * z / fy, z])
        Xw = R.T @ (Xc - t)
        d = float(np.linalg.norm(Xw - Ow))
        pts[j]["xyz"] = Xw
        pts[j]["normal"] = (Xw - Ow) / d
        pts[j]["max_dist"] = d * sc[kp["octave"]]
        pts[j]["min_dist"] = d * sc[kp["octave"]] / sc[-1]
        pts[j]["desc"] = kf["desc"][i]
    base = len(idx)
    for e in range(n_extra):
        p = pts[rng.integers(0, base)].copy()
        kind = e % 4
        if kind == 0:
            p["xyz"] = -p["xyz"]  # behind the camera
        elif kind == 1:
            p["xyz"][0] += 200.0  # outside the image
        elif kind == 2:
            p["normal"] = -p["normal"]  # viewed from behind (> 60 deg)
        else:
            p["max_dist"] *= 0.5  # outside the scale-invariance range
        pts[base + e] = p
    pts["skip"] = (rng.random(len(pts)) < 0.1).astype(np.int32)
    return pts
