"""The LocalMapper's keyframe-rate matchers on the device: ctypes binding of
include/slamgpu_kfmatch.h with reference-shaped names.

  search_for_triangulation   OrbMatcher::SearchForTriangulation (orb_matcher.cpp:634-802)
  fuse                       OrbMatcher::Fuse(pKF, vpMapPoints, th) (orb_matcher.cpp:804-954),
                             the candidate search; fuse_apply is the reference's sequential
                             Replace / AddObservation walk over its result
libslamgpu.so is the only compute path (no CPU fallback); errors raise SlamGpuError.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import slamgpu as G

MAX_FEATURES = 4096
TH_LOW = 50

FUSE_POINT_DTYPE = np.dtype([("xyz", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_dist", "<f4"),
                             ("max_dist", "<f4"), ("skip", "<i4"), ("pad", "<i4", (3,)),
                             ("desc", "u1", (32,))])
TRI_PAIR_DTYPE = np.dtype([("kf1", "<i4"), ("kf2", "<i4"), ("F12", "<f4", (9,)),
                           ("only_stereo", "<i4")])
# slamgpu_kf with device addresses (the *_device calls)
KF_DTYPE = np.dtype([("kps", "<u8"), ("desc", "<u8"), ("u_right", "<u8"), ("has_mp", "<u8"),
                     ("nodes", "<u8"), ("node_start", "<u8"), ("node_feats", "<u8"),
                     ("n", "<i4"), ("n_nodes", "<i4"), ("Rcw", "<f4", (9,)), ("tcw", "<f4", (3,)),
                     ("Ow", "<f4", (3,)), ("pad", "<f4")])
assert FUSE_POINT_DTYPE.itemsize == 80 and TRI_PAIR_DTYPE.itemsize == 48
assert KF_DTYPE.itemsize == 128


class Levels(C.Structure):
    """slamgpu_levels: a KeyFrame's per-level tables."""
    _fields_ = [("nlevels", C.c_int32), ("log_scale_factor", C.c_float),
                ("scale", C.c_float * 32), ("sigma2", C.c_float * 32),
                ("inv_sigma2", C.c_float * 32)]


class KfGrid(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("min_x", "max_x", "min_y", "max_y", "cell_w", "cell_h")]


class Kf(C.Structure):
    """slamgpu_kf (host pointers in the synchronous calls)."""
    _fields_ = [(n, C.c_void_p) for n in ("kps", "desc", "u_right", "has_mp", "nodes",
                                          "node_start", "node_feats")] + [
        ("n", C.c_int32), ("n_nodes", C.c_int32), ("Rcw", C.c_float * 9), ("tcw", C.c_float * 3),
        ("Ow", C.c_float * 3), ("pad", C.c_float)]


def levels(scale_factor=1.2, nlevels=8):
    """The extractor's tables as KeyFrame copies them (orb_extractor.cpp:357-369, f32; log via
    the float std::log of Frame)."""
    lv = Levels()
    lv.nlevels = nlevels
    sf = np.float32(scale_factor)
    lv.log_scale_factor = float(np.float32(np.log(np.float64(sf))))
    sc = np.float32(1.0)
    for i in range(nlevels):
        if i:
            sc = np.float32(float(sc) * float(np.float32(scale_factor)))
        lv.scale[i] = float(sc)
        s2 = np.float32(sc * sc)
        lv.sigma2[i] = float(s2)
        lv.inv_sigma2[i] = float(np.float32(1.0) / s2)
    return lv


def kf_grid(cols, rows):
    """KeyFrame::min_x_ .. max_y_ and the 64 x 48 cell sizes of an undistorted cols x rows
    image (Frame::ComputeImageBounds k1 == 0, frame.cpp:223-224)."""
    return KfGrid(0.0, float(int(cols)), 0.0, float(int(rows)),
                  float(np.float32(cols) / np.float32(64)), float(np.float32(rows) / np.float32(48)))


_bound = False


def lib():
    global _bound
    L = G.lib()
    if not _bound:
        vp, ip = C.c_void_p, C.c_int
        L.slamgpu_kfmatch_last_error.argtypes = []
        L.slamgpu_kfmatch_last_error.restype = C.c_char_p
        L.slamgpu_search_for_triangulation.argtypes = [
            C.POINTER(Kf), C.POINTER(Kf), vp, C.POINTER(G.Camera), C.POINTER(Levels), ip, ip, vp,
            C.POINTER(ip)]
        L.slamgpu_search_for_triangulation_device.argtypes = [
            vp, vp, ip, C.POINTER(G.Camera), C.POINTER(Levels), ip, vp, C.c_int64, vp, vp]
        L.slamgpu_fuse.argtypes = [C.POINTER(Kf), vp, ip, C.c_float, C.POINTER(G.Camera),
                                   C.POINTER(Levels), C.POINTER(KfGrid), vp, vp, C.POINTER(ip)]
        L.slamgpu_fuse_device.argtypes = [vp, vp, vp, ip, C.c_float, C.POINTER(G.Camera),
                                          C.POINTER(Levels), C.POINTER(KfGrid), vp, vp, vp]
        _bound = True
    return L


def _check(rc):
    if rc != 0:
        raise G.SlamGpuError(f"slamgpu error {rc}: {lib().slamgpu_kfmatch_last_error().decode()}")


_p = G._ptr


def _cam(cam):
    return G.Camera(*[float(np.float32(c)) for c in cam])


def host_kf(kps, desc, u_right, Tcw, has_mp=None, feature_vec=None):
    """A slamgpu_kf over host arrays (kept alive in the returned tuple). Tcw: 4x4 f32 pose;
    Ow = -R^T t as the caller's KeyFrame holds it (pass Ow explicitly via .Ow to override)."""
    k = np.ascontiguousarray(kps)
    if len(k) and k.dtype != G.KP_DTYPE:
        k = k.view(G.KP_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    ur = np.ascontiguousarray(u_right, np.float32)
    mp = None if has_mp is None else np.ascontiguousarray(has_mp, np.uint8)
    keep = [k, d, ur, mp]
    s = Kf()
    s.kps, s.desc, s.u_right, s.has_mp = _p(k), _p(d), _p(ur), _p(mp)
    s.n = len(d)
    if feature_vec is not None:
        nodes, start, feats = (np.ascontiguousarray(a, t) for a, t in zip(
            feature_vec.arrays(), (np.uint32, np.int32, np.uint32)))
        keep += [nodes, start, feats]
        s.nodes, s.node_start, s.node_feats = _p(nodes), _p(start), _p(feats)
        s.n_nodes = len(nodes)
    T = np.asarray(Tcw, np.float32)
    R, t = T[:3, :3], T[:3, 3]
    s.Rcw[:] = [float(x) for x in R.reshape(-1)]
    s.tcw[:] = [float(x) for x in t]
    s.Ow[:] = [float(x) for x in camera_center(T)]
    return s, keep


def camera_center(Tcw):
    """KeyFrame::SetPose's Ow = -Rcw^T tcw in float cv::Mat arithmetic (OpenCV gemm: float dot
    products added in double, as matcher_oracle.c restates Rcw * X + tcw)."""
    T = np.asarray(Tcw, np.float32)
    Rt = T[:3, :3].T
    t = T[:3, 3]
    out = np.zeros(3, np.float32)
    for r in range(3):
        dot = np.float32(np.float32(Rt[r, 0] * t[0]) + np.float32(Rt[r, 1] * t[1]))
        dot = np.float32(dot + np.float32(Rt[r, 2] * t[2]))
        out[r] = np.float32(-dot)
    return out


def search_for_triangulation(kf1, kf2, F12, cam, lv, only_stereo=False, check_ori=True):
    """kf1 / kf2: (Kf, keep) from host_kf (with has_mp and feature_vec). Returns (nmatches,
    match12) with match12[i] = vMatches12[i]."""
    s1, s2 = kf1[0], kf2[0]
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    m = np.full(max(s1.n, 1), -1, np.int32)
    nm = C.c_int()
    _check(lib().slamgpu_search_for_triangulation(C.byref(s1), C.byref(s2), _p(F),
                                                  C.byref(_cam(cam)), C.byref(lv),
                                                  int(bool(only_stereo)), int(bool(check_ori)),
                                                  _p(m), C.byref(nm)))
    return nm.value, m[:s1.n]


def search_for_triangulation_device(d_kfs, d_pairs, n_pairs, cam, lv, check_ori, d_match,
                                    match_stride, d_nmatches, stream=None):
    from .bow import _dev
    _check(lib().slamgpu_search_for_triangulation_device(
        _dev(d_kfs), _dev(d_pairs), n_pairs, C.byref(_cam(cam)), C.byref(lv),
        int(bool(check_ori)), _dev(d_match), match_stride, _dev(d_nmatches),
        C.c_void_p(stream or 0)))


def fuse(kf, points, th, cam, lv, grid):
    """kf: (Kf, keep) from host_kf; points: FUSE_POINT_DTYPE. Returns (nfused, best_idx,
    best_dist)."""
    pts = np.ascontiguousarray(points).view(FUSE_POINT_DTYPE)
    n = len(pts)
    bi, bd = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.int32)
    nf = C.c_int()
    _check(lib().slamgpu_fuse(C.byref(kf[0]), _p(pts), n, float(th), C.byref(_cam(cam)),
                              C.byref(lv), C.byref(grid), _p(bi), _p(bd), C.byref(nf)))
    return nf.value, bi[:n], bd[:n]


def fuse_device(d_kfs, d_pts, d_point_kf, n_pts, th, cam, lv, grid, d_best_idx, d_best_dist,
                stream=None):
    from .bow import _dev
    _check(lib().slamgpu_fuse_device(_dev(d_kfs), _dev(d_pts), _dev(d_point_kf), n_pts, float(th),
                                     C.byref(_cam(cam)), C.byref(lv), C.byref(grid),
                                     _dev(d_best_idx), _dev(d_best_dist), C.c_void_p(stream or 0)))


def fuse_apply(best_idx, kf_map_points, mp_ids, mp_nobs, mp_bad, mp_in_kf):
    """The reference's walk over Fuse's result (orb_matcher.cpp:821-951) on an id-based map:
    kf_map_points[j] = map point id of keypoint j (-1 none), mp_ids[i] = id of offered point i,
    mp_nobs / mp_bad / mp_in_kf indexed by id (mutated). Replace(a -> b) moves a's keyframe slot
    to b and marks a bad. Returns nFused."""
    nfused = 0
    for i, mid in enumerate(mp_ids):
        if mid < 0 or mp_bad[mid] or mp_in_kf[mid] or best_idx[i] < 0:
            continue
        j = int(best_idx[i])
        cur = int(kf_map_points[j])
        if cur >= 0:
            if not mp_bad[cur]:
                keep, drop = (cur, mid) if mp_nobs[cur] > mp_nobs[mid] else (mid, cur)
                mp_bad[drop] = True
                mp_nobs[keep] += mp_nobs[drop]
                kf_map_points[kf_map_points == drop] = keep
                mp_in_kf[keep] = True
        else:
            mp_nobs[mid] += 1
            mp_in_kf[mid] = True
            kf_map_points[j] = mid
        nfused += 1
    return nfused
