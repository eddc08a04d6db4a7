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
