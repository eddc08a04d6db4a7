"""Pins oracle/kfmatch_oracle.c against an independent pure-Python restatement of
OrbMatcher::SearchForTriangulation (src/orb_features/orb_matcher.cpp:634-802, with
CheckDistEpipolarLine :114-131) and of Fuse's candidate search (:804-928, with
MapPoint::PredictScale map_point.cpp:366-381 and KeyFrame::GetFeaturesInArea keyframe.cpp:
442-476), and the glibc logf port (oracle/check_logf.c, every positive float). Parity against
the reference binary is unpinned."""
import ctypes as C
import math
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

import kf_scenario as KS
import test_bow_oracle as TB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f32 = np.float32


def fmaf(a, b, c):
    """Single-rounding float fma (the exact rational rounded once through double: the double
    rounding this adds is far below anything these tests can reach)."""
    return f32(float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))))


def gemm_row(R, r, x, c):
    dot = f32(f32(f32(R[3 * r] * x[0]) + f32(R[3 * r + 1] * x[1])) + f32(R[3 * r + 2] * x[2]))
    return f32(float(dot) + float(c))


def py_triangulation(k1, k2, C1w, T2w, cam4, scale, sigma2, F, only_stereo, check_ori):
    fx, fy, cx, cy = (f32(c) for c in cam4)
    c2 = [gemm_row(T2w, r, C1w, T2w[9 + r]) for r in range(3)]
    invz = f32(f32(1.0) / c2[2])
    ex, ey = fmaf(f32(fx * c2[0]), invz, cx), fmaf(f32(fy * c2[1]), invz, cy)
    fv1, fv2 = TB.fv_dict(*k1["fv"]), TB.fv_dict(*k2["fv"])
    m12 = [-1] * len(k1["desc"])
    hist = [[] for _ in range(30)]
    nm = 0
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if k1["mp"][i1]:
                continue
            st1 = k1["ur"][i1] >= 0
            if only_stereo and not st1:
                continue
            p1 = k1["kps"][i1]
            best, bi = 50, -1
            for i2 in fv2[node]:
                if k2["mp"][i2]:
                    continue
                st2 = k2["ur"][i2] >= 0
                if only_stereo and not st2:
                    continue
                d = TB.hamming(k1["desc"][i1], k2["desc"][i2])
                if d > 50 or d > best:
                    continue
                p2 = k2["kps"][i2]
                if not st1 and not st2:
                    dx, dy = f32(ex - p2["x"]), f32(ey - p2["y"])
                    if fmaf(dx, dx, f32(dy * dy)) < f32(f32(100) * scale[p2["octave"]]):
                        continue
                a = f32(fmaf(p1["x"], F[0], f32(p1["y"] * F[3])) + F[6])
                b = f32(fmaf(p1["x"], F[1], f32(p1["y"] * F[4])) + F[7])
                c = f32(fmaf(p1["x"], F[2], f32(p1["y"] * F[5])) + F[8])
                num = f32(fmaf(a, p2["x"], f32(b * p2["y"])) + c)
                den = fmaf(a, a, f32(b * b))
                if den == 0:
                    continue
                if float(f32(f32(num * num) / den)) < 3.84 * float(sigma2[p2["octave"]]):
                    best, bi = d, i2
            if bi >= 0:
                m12[i1] = bi
                nm += 1
                if check_ori:
                    rot = f32(k1["kps"][i1]["angle"] - k2["kps"][bi]["angle"])
                    if rot < 0.0:
                        rot = f32(rot + f32(360.0))
                    b = TB.roundf(f32(rot * f32(f32(1.0) / f32(30))))
                    hist[0 if b == 30 else b].append(i1)
    if check_ori:
        keep = TB.three_maxima([len(h) for h in hist])
        for b in range(30):
            if b not in keep:
                for i in hist[b]:
                    m12[i] = -1
                    nm -= 1
    return nm, np.array(m12, np.int32)


def _tri_inputs(oracle):
    kfs, _ = KS.keyframes(oracle)
    T1, T2 = KS.pose(0), KS.pose(1, (-0.4, 0.02, 0.1))
    T2w = np.concatenate([T2[:3, :3].reshape(-1), T2[:3, 3]]).astype(np.float32)
    return kfs, KS.center(T1), T2w, KS.fundamental(T1, T2).reshape(-1)


@pytest.fixture(scope="module")
def tri(oracle):
    return _tri_inputs(oracle)


@pytest.mark.parametrize("only_stereo", [False, True])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_triangulation_matches_python(oracle, tri, only_stereo, check_ori):
    kfs, C1w, T2w, F = tri
    sc, s2, _, _ = KS.levels_arrays()
    cam4 = KS.CAM[:4]
    # a third of the features keeps the pure-Python walk to seconds
    sub = [dict(k) for k in kfs]
    for k in sub:
        nodes, start, feats = k["fv"]
        keep = feats % 3 == 0
        cnt = np.add.reduceat(keep.astype(np.int64), start[:-1]) if len(nodes) else np.zeros(0)
        st = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
        k["fv"] = (nodes, st, feats[keep])
    nm_o, m_o = oracle.search_for_triangulation(sub[0], sub[1], C1w, T2w, cam4, sc, s2, F,
                                                only_stereo, check_ori)
    nm_p, m_p = py_triangulation(sub[0], sub[1], C1w, T2w, cam4, sc, s2, F, only_stereo,
                                 check_ori)
    assert nm_o == nm_p
    np.testing.assert_array_equal(m_o, m_p)
    assert nm_o > 10


def py_features_in_area(kps, grid, x, y, r):
    out = []
    cw, ch = f32(grid.cell_w), f32(grid.cell_h)
    x, y, r = f32(x), f32(y), f32(r)
    x0 = max(0, math.floor(f32(f32(f32(x - f32(grid.min_x)) - r) / cw)))
    x1 = min(63, math.ceil(f32(f32(f32(x - f32(grid.min_x)) + r) / cw)))
    y0 = max(0, math.floor(f32(f32(f32(y - f32(grid.min_y)) - r) / ch)))
    y1 = min(47, math.ceil(f32(f32(f32(y - f32(grid.min_y)) + r) / ch)))
    if x1 < 0 or x0 >= 64 or y1 < 0 or y0 >= 48:
        return out
    cells = {}
    for j, kp in enumerate(kps):
        px = TB.roundf(f32(f32(kp["x"] - f32(grid.min_x)) / cw))
        py = TB.roundf(f32(f32(kp["y"] - f32(grid.min_y)) / ch))
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((px, py), []).append(j)
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for j in cells.get((ix, iy), []):
                if abs(f32(kps[j]["x"] - x)) < r and abs(f32(kps[j]["y"] - y)) < r:
                    out.append(j)
    return out


def py_fuse(oracle, kf, grid, T, cam, lv_arrays, pts, th):
    fx, fy, cx, cy, bf = (f32(c) for c in cam)
    sc, _, isig, lsf = lv_arrays
    R, t = T[:3, :3].reshape(-1), T[:3, 3]
    Ow = KS.center(T)
    logf = oracle._kf_lib().oc_logf  # pinned separately against glibc (check_logf)
    bi, bd = [], []
    for P in pts:
        bi.append(-1)
        bd.append(256)
        if P["skip"]:
            continue
        xc, yc, zc = (gemm_row(R, r, P["xyz"], t[r]) for r in range(3))
        if zc < 0:
            continue
        invz = f32(f32(1) / zc)
        u, v = fmaf(fx, f32(xc * invz), cx), fmaf(fy, f32(yc * invz), cy)
        if not (grid.min_x <= u < grid.max_x and grid.min_y <= v < grid.max_y):
            continue
        urp = fmaf(-bf, invz, u)
        po = (P["xyz"] - Ow).astype(np.float32)
        d3 = f32(math.sqrt(sum(float(p) * float(p) for p in po)))
        if d3 < f32(f32(0.8) * P["min_dist"]) or d3 > f32(f32(1.2) * P["max_dist"]):
            continue
        if sum(float(a) * float(b) for a, b in zip(po, P["normal"])) < 0.5 * float(d3):
            continue
        lvl = math.ceil(f32(f32(logf(float(f32(P["max_dist"] / d3)))) / lsf))
        lvl = min(max(lvl, 0), len(sc) - 1)
        r = f32(f32(th) * sc[lvl])
        best, idx = 256, -1
        for j in py_features_in_area(kf["kps"], grid, u, v, r):
            kp = kf["kps"][j]
            o = int(kp["octave"])
            if o < lvl - 1 or o > lvl:
                continue
            ex, ey = f32(u - kp["x"]), f32(v - kp["y"])
            if kf["ur"][j] >= 0:
                er = f32(urp - kf["ur"][j])
                e2 = fmaf(er, er, fmaf(ex, ex, f32(ey * ey)))
                if float(f32(e2 * isig[o])) > 7.8:
                    continue
            elif float(f32(fmaf(ex, ex, f32(ey * ey)) * isig[o])) > 5.99:
                continue
            d = TB.hamming(P["desc"], kf["desc"][j])
            if d < best:
                best, idx = d, j
        bd[-1] = best
        if best <= 50:
            bi[-1] = idx
    return np.array(bi, np.int32), np.array(bd, np.int32)


def test_fuse_matches_python(oracle):
    kfs, _ = KS.keyframes(oracle)
    T0, T1 = KS.pose(0), KS.pose(1)
    pts = KS.fuse_points(kfs[0], T0)[::3]
    grid = oracle.grid_geom(1241, 376)
    lva = KS.levels_arrays()
    Rcw = T1[:3, :3].reshape(-1)
    nf, bi, bd = oracle.fuse(kfs[1]["kps"], kfs[1]["desc"], kfs[1]["ur"], grid, Rcw, T1[:3, 3],
                             KS.center(T1), KS.CAM, lva[0], lva[2], lva[3], pts, 3.0)
    pbi, pbd = py_fuse(oracle, kfs[1], grid, T1, KS.CAM, lva, pts, 3.0)
    np.testing.assert_array_equal(bi, pbi)
    np.testing.assert_array_equal(bd, pbd)
    assert nf == int((bi >= 0).sum()) and nf > 30


def test_logf_matches_glibc_sampled(oracle):
    libm = C.CDLL("libm.so.6")
    libm.logf.argtypes = [C.c_float]
    libm.logf.restype = C.c_float
    L = oracle._kf_lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0.2, 8.0, 20000).astype(np.float32),
                         np.float32([1.0, 1.2, 2.0, 1e-40, 3e38, 0.999999, 1.0000001])])
    for x in xs:
        assert L.oc_logf(float(x)) == libm.logf(float(x))


def test_logf_exhaustive():
    """Every positive float bit-exact against host glibc logf (oracle/check_logf.c)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "check_logf"], check=True)
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    out = subprocess.run([os.path.join(ROOT, "oracle", "check_logf")], env=env,
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout
    assert '"logf_mismatch": 0' in out.stdout
