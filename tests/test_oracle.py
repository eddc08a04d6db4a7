"""CPU tests of the oracle (the parity checker) against everything that can pin it here:
host glibc for sinf/cosf, SURVEY.md section 8's derived tables, brute-force definitions of the
OpenCV primitives, and structural invariants of DistributeOctTree and the matchers."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from slam_framework_amd import synthetic as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---- ctor tables (orb_extractor.cpp:351-411) vs SURVEY.md section 8 ----------------------
def test_tables_match_survey(oracle):
    t = oracle.tables()
    assert list(t.features_per_level)[:8] == [434, 362, 302, 251, 209, 175, 145, 122]
    assert list(t.umax) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    pyr = oracle.OraclePyramid(t, 1241, 376)
    sizes = [(pyr.p.w[l], pyr.p.h[l]) for l in range(8)]
    assert sizes == [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151),
                     (416, 126), (346, 105)]
    assert abs(t.scale[7] - 3.583181) < 1e-5


def test_cell_grid_matches_survey(oracle):
    """ComputeKeyPointsOctTree cell grid (:712-733): cols x rows, wCell x hCell per level."""
    import math
    want = [(40, 11, 31, 32), (33, 9, 31, 32), (27, 7, 31, 33), (22, 6, 32, 31), (18, 4, 32, 38),
            (15, 3, 32, 40), (12, 3, 32, 32), (10, 2, 32, 37)]
    sizes = [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151),
             (416, 126), (346, 105)]
    for (w, h), exp in zip(sizes, want):
        width = np.float32(w - 19 + 3 - 16)
        height = np.float32(h - 19 + 3 - 16)
        nc, nr = int(width / np.float32(30)), int(height / np.float32(30))
        assert (nc, nr, math.ceil(width / nc), math.ceil(height / nr)) == exp


# ---- glibc sinf/cosf port --------------------------------------------------------------------
def test_sincosf_matches_glibc_sampled(oracle):
    libm = C.CDLL("libm.so.6")
    libm.sinf.argtypes = libm.cosf.argtypes = [C.c_float]
    libm.sinf.restype = libm.cosf.restype = C.c_float
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(0, 2 * np.pi, 20000).astype(np.float32),
                         np.float32([0.0, 1e-30, 0.7853981, 0.7853982, 3.1415927, 6.2831855])])
    L = oracle.lib()
    for x in xs:
        assert L.oc_sinf(float(x)) == libm.sinf(float(x))
        assert L.oc_cosf(float(x)) == libm.cosf(float(x))


def test_sincosf_exhaustive_range():
    """Every float in [0, 2pi) bit-exact against host glibc (oracle/check_sincosf.c)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "check_sincosf"], check=True)
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    out = subprocess.run([os.path.join(ROOT, "oracle", "check_sincosf")], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
    assert '"sin_mismatch": 0, "cos_mismatch": 0' in out.stdout


# ---- fastAtan2 --------------------------------------------------------------------------------
def test_fast_atan2(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(1)
    for _ in range(5000):
        y, x = rng.integers(-200000, 200000, 2).astype(np.float32)
        a = L.oc_fast_atan2(float(y), float(x))
        ref = np.degrees(np.arctan2(y, x)) % 360.0
        d = abs(a - ref)
        assert 0.0 <= a < 360.0 + 1e-3
        assert min(d, 360 - d) < 0.02
    assert L.oc_fast_atan2(0.0, 0.0) == 0.0


# ---- FAST-9/16 against a brute-force definition ---------------------------------------------
RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
        (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def brute_fast(img, th, nonmax):
    h, w = img.shape
    I = img.astype(np.int32)
    s = np.full((h, w), -1000, np.int32)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            d = np.array([I[y, x] - I[y + dy, x + dx] for dx, dy in RING])
            dd = np.concatenate([d, d])
            sd = max(dd[k:k + 9].min() for k in range(16))
            sb = max((-dd[k:k + 9]).min() for k in range(16))
            s[y, x] = max(sd, sb)
    corner = s > th
    score = np.where(corner, s - 1, 0)
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if not corner[y, x]:
                continue
            if nonmax:
                nb = score[y - 1:y + 2, x - 1:x + 2].copy()
                nb[1, 1] = -1
                if not (score[y, x] > nb).all():
                    continue
            out.append((x, y, score[y, x] if nonmax else 0))  # cv::FAST stores no score w/o NMS
    return out


@pytest.mark.parametrize("seed,th,nonmax", [(0, 20, 1), (1, 7, 1), (2, 20, 0), (3, 40, 1)])
def test_fast_matches_bruteforce(oracle, seed, th, nonmax):
    rng = np.random.default_rng(seed)
    img = S.image(100 + seed, 64, 64)[:40, :48].copy()
    img[rng.random(img.shape) < 0.05] = 255
    out = np.zeros(4096, oracle.KP_DTYPE)
    n = oracle.lib().oc_fast16(oracle.ptr(img), img.shape[1], img.shape[0], img.shape[1], th,
                               nonmax, oracle.ptr(out), 4096)
    got = [(int(k["x"]), int(k["y"]), int(k["response"])) for k in out[:n]]
    assert got == brute_fast(img, th, nonmax)
    assert n > 0


# ---- resize / blur against independent numpy restatements -----------------------------------
def np_resize(src, dw, dh):
    sh, sw = src.shape
    sx_scale, sy_scale = 1.0 / (dw / sw), 1.0 / (dh / sh)
    out = np.zeros((dh, dw), np.uint8)
    xs, a0, a1 = [], [], []
    for dx in range(dw):
        fx = np.float32((dx + 0.5) * sx_scale - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx >= sw - 1:
            fx, sx = np.float32(0), sw - 1
        xs.append(sx)
        a0.append(int(np.rint(np.float32(1 - fx) * 2048)))
        a1.append(int(np.rint(fx * np.float32(2048))))
    I = src.astype(np.int64)
    for dy in range(dh):
        fy = np.float32((dy + 0.5) * sy_scale - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        b0, b1 = int(np.rint(np.float32(1 - fy) * 2048)), int(np.rint(fy * np.float32(2048)))
        y0, y1 = min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1)
        for dx in range(dw):
            sx = xs[dx]
            if sx + 1 < sw:
                r0 = I[y0, sx] * a0[dx] + I[y0, sx + 1] * a1[dx]
                r1 = I[y1, sx] * a0[dx] + I[y1, sx + 1] * a1[dx]
            else:
                r0, r1 = I[y0, sx] * 2048, I[y1, sx] * 2048
            out[dy, dx] = (((b0 * (r0 >> 4)) >> 16) + ((b1 * (r1 >> 4)) >> 16) + 2) >> 2
    return out


def test_resize_matches_numpy(oracle):
    src = S.image(7, 120, 90)
    for dw, dh in [(100, 75), (83, 63)]:
        dst = np.zeros((dh, dw), np.uint8)
        oracle.lib().oc_resize_linear_u8(oracle.ptr(src), 120, 90, 120, oracle.ptr(dst), dw, dh, dw)
        np.testing.assert_array_equal(dst, np_resize(src, dw, dh))


def test_blur_matches_numpy(oracle):
    src = S.image(8, 70, 50)
    h, w = src.shape
    k = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)
    pad = np.pad(src.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == REFLECT_101
    H = sum(k[i] * pad[:, i:i + w] for i in range(7))
    V = sum(k[i] * H[i:i + h, :] for i in range(7))
    xvec = w - w % 4
    out = np.where(np.arange(w)[None, :] < xvec,
                   np.rint((V.astype(np.float32) * np.float32(1 / 65536))).astype(np.int64),
                   (V + 32768) >> 16)
    want = np.clip(out, 0, 255).astype(np.uint8)
    got = np.zeros_like(src)
    oracle.lib().oc_gaussian_blur7_u8(oracle.ptr(src), w, h, w, oracle.ptr(got), w)
    np.testing.assert_array_equal(got, want)


# ---- DistributeOctTree invariants ---------------------------------------------------------------
def test_octree_invariants(oracle):
    t = oracle.tables()
    img = S.image(1234)
    _, _, pyr = oracle.extract(t, img, with_pyramid=True)
    for l in range(8):
        cand = oracle.level_candidates(t, pyr, l)
        N = t.features_per_level[l]
        out = oracle.distribute_octree(t, pyr, l, cand)
        assert len(out) <= max(N + 2, 0) or len(out) <= len(cand)
        keys = set(oracle.pack_keys(cand).tolist())
        got = oracle.pack_keys(out).tolist()
        assert len(set(got)) == len(got) and set(got) <= keys
        # with a budget above the candidate count every candidate survives, in some order
        w, h = pyr.p.w[l], pyr.p.h[l]
        big = np.zeros(len(cand) + 1, oracle.KP_DTYPE)
        n = oracle.lib().oc_distribute_octree(oracle.ptr(cand), len(cand), 16, w - 16, 16, h - 16,
                                              len(cand) + 10, oracle.ptr(big), len(big))
        assert sorted(oracle.pack_keys(big[:n]).tolist()) == sorted(keys)


def test_descriptor_distance(oracle):
    rng = np.random.default_rng(3)
    for _ in range(200):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        want = int(np.unpackbits(a ^ b).sum())
        assert oracle.lib().oc_descriptor_distance(oracle.ptr(a), oracle.ptr(b)) == want


def test_stereo_geometry(oracle):
    t = oracle.tables()
    L, R = S.stereo_pair(77)
    kl, dl, pl = oracle.extract(t, L, True)
    kr, dr, pr = oracle.extract(t, R, True)
    ur, depth, sad = oracle.stereo(t, kl, dl, kr, dr, pl, pr, S.KITTI_CAM[0], S.KITTI_CAM[4])
    m = depth > 0
    assert m.sum() > 100
    assert np.all(ur[m] <= kl["x"][m])
    np.testing.assert_allclose(depth[m], S.KITTI_CAM[4] / (kl["x"][m] - ur[m]), rtol=1e-5)
    assert np.all(ur[~m] == -1) and np.all(sad[m] >= 0)


_FAST_PROBE = r'''
import hashlib, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import oracle_lib as O
from slam_framework_amd import synthetic as S
import scenario
if sys.argv[1] == "fast":
    O.use_fast()
t = O.tables()
L, R = S.sequence(4100, 2)
h = hashlib.sha256()
prev = None
for f in range(2):
    kl, dl, pl = O.extract(t, L[f], True)
    kr, dr, pr = O.extract(t, R[f], True)
    ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, S.KITTI_CAM[0], S.KITTI_CAM[4])
    for a in (kl, dl, kr, dr, ur, depth):
        h.update(np.ascontiguousarray(a).tobytes())
    if prev is not None:
        q, lmp, lout, xyz, md, nobs = scenario.vo_queries(prev[0], prev[1], prev[2], f - 1)
        p = scenario.pose(f)
        mp = np.full(len(kl), -1, np.int32)
        O.search_frame(t, O.grid_geom(S.KITTI_COLS, S.KITTI_ROWS), kl, dl, ur, mp, prev[0], lmp,
                       lout, xyz, md, nobs, p["Rcw"][0].reshape(3, 3), p["tcw"][0], 0.0,
                       float(p["baseline"][0]), S.KITTI_CAM, 7.0, 0, 1)
        h.update(mp.tobytes())
    prev = (kl, dl, depth)
P = S.c5_problem(11)
kf, pts, er, its = O.local_ba(S.KITTI_CAM, P)
h.update(kf.tobytes() + pts.tobytes() + er.tobytes())
e, T0, _, isig, _ = S.pose_problem(77, 2000)
r, T, out, _ = O.pose_optimization(S.KITTI_CAM, isig, e, T0)
h.update(T.tobytes() + out.tobytes())
print(h.hexdigest())
'''


def test_fast_build_is_the_same_oracle(oracle):
    """The CPU baseline's -O3 x86-64-v3 build (liborb_oracle_fast.so) produces the test oracle's
    (-O2) results byte for byte: extraction, stereo, frame-to-frame search, local BA, pose."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = [subprocess.run([sys.executable, "-c", _FAST_PROBE, m], cwd=root, capture_output=True,
                          text=True, check=True).stdout.strip() for m in ("ref", "fast")]
    assert out[0] == out[1] and len(out[0]) == 64
