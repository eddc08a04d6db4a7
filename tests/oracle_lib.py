"""ctypes binding of oracle/liborb_oracle.so -- the CPU restatement used as the parity checker.

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liborb_oracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28

MAX_LEVELS = 32


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


class OrbTables(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("nlevels", C.c_int), ("ini_th_fast", C.c_int),
                ("min_th_fast", C.c_int), ("scale_factor", C.c_double),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("features_per_level", C.c_int * MAX_LEVELS), ("umax", C.c_int * 16)]


class Pyramid(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("w", C.c_int * MAX_LEVELS), ("h", C.c_int * MAX_LEVELS),
                ("step", C.c_size_t * MAX_LEVELS), ("data", C.POINTER(C.c_uint8) * MAX_LEVELS)]


class GridGeom(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float), ("cell_w", C.c_float), ("cell_h", C.c_float)]


class FrameView(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("u_right", C.c_void_p),
                ("n", C.c_int), ("map_point", C.c_void_p)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liborb_oracle.so", "liborb_oracle_fast.so"],
                   check=True)


def use_fast() -> None:
    """Load the -O3 x86-64-v3 build (oracle/Makefile liborb_oracle_fast.so) instead: the CPU
    baseline's library. Must run before the first lib() call of the process."""
    global LIB_PATH
    assert _lib is None, "oracle library already loaded"
    LIB_PATH = os.path.join(ORACLE_DIR, "liborb_oracle_fast.so")


def use_lib(path: str) -> None:
    """Load the oracle build at `path` (e.g. bench.py's -march=native build for the CPU
    baseline). Must run before the first lib() call of the process."""
    global LIB_PATH
    assert _lib is None, "oracle library already loaded"
    LIB_PATH = path


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, ip, fp = C.c_void_p, C.c_int, C.c_float
        L.oc_orb_init.argtypes = [C.POINTER(OrbTables), C.POINTER(OrbParams)]
        L.oc_cv_round.argtypes = [fp]
        L.oc_fast_atan2.argtypes = [fp, fp]
        L.oc_fast_atan2.restype = fp
        L.oc_sinf.argtypes = [fp]
        L.oc_sinf.restype = fp
        L.oc_cosf.argtypes = [fp]
        L.oc_cosf.restype = fp
        L.oc_resize_linear_u8.argtypes = [vp, ip, ip, C.c_size_t, vp, ip, ip, C.c_size_t]
        L.oc_gaussian_blur7_u8.argtypes = [vp, ip, ip, C.c_size_t, vp, C.c_size_t]
        L.oc_fast16.argtypes = [vp, ip, ip, C.c_size_t, ip, ip, vp, ip]
        L.oc_pyramid_alloc.argtypes = [C.POINTER(Pyramid), C.POINTER(OrbTables), ip, ip]
        L.oc_pyramid_free.argtypes = [C.POINTER(Pyramid)]
        L.oc_compute_pyramid.argtypes = [C.POINTER(OrbTables), vp, C.c_size_t, C.POINTER(Pyramid)]
        L.oc_level_candidates.argtypes = [C.POINTER(OrbTables), C.POINTER(Pyramid), ip, vp, ip]
        L.oc_distribute_octree.argtypes = [vp, ip, ip, ip, ip, ip, ip, vp, ip]
        L.oc_ic_angle.argtypes = [vp, C.c_size_t, fp, fp, vp]
        L.oc_ic_angle.restype = fp
        L.oc_orb_descriptor.argtypes = [vp, vp, C.c_size_t, vp]
        L.oc_orb_extract.argtypes = [C.POINTER(OrbTables), vp, ip, ip, C.c_size_t, vp, vp, ip,
                                     C.POINTER(Pyramid)]
        L.oc_descriptor_distance.argtypes = [vp, vp]
        L.oc_stereo_match.argtypes = [C.POINTER(OrbTables), vp, vp, ip, vp, vp, ip,
                                      C.POINTER(Pyramid), C.POINTER(Pyramid), fp, fp, vp, vp, vp]
        L.oc_grid_geom_init.argtypes = [C.POINTER(GridGeom), ip, ip]
        L.oc_grid_geom_init_dist.argtypes = [C.POINTER(GridGeom), ip, ip, vp, vp, ip]
        L.oc_undistort_points.argtypes = [vp, vp, ip, vp, vp, ip]
        L.oc_undistort_keypoints.argtypes = [vp, vp, ip, vp, vp, ip]
        L.oc_features_in_area.argtypes = [C.POINTER(GridGeom), vp, ip, fp, fp, fp, ip, ip, vp, ip]
        L.oc_search_by_projection_frame.argtypes = [
            C.POINTER(GridGeom), C.POINTER(OrbTables), C.POINTER(FrameView), vp, vp, vp, ip,
            vp, vp, vp, vp, vp, fp, fp, fp, fp, fp, fp, fp, fp, ip, ip]
        L.oc_search_by_projection_mps.argtypes = [
            C.POINTER(GridGeom), C.POINTER(OrbTables), C.POINTER(FrameView), ip, vp, vp, vp, vp,
            vp, vp, vp, vp, vp, fp, ip]
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def tables(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7) -> OrbTables:
    p = OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th)
    t = OrbTables()
    lib().oc_orb_init(C.byref(t), C.byref(p))
    return t


class OraclePyramid:
    """Owns an oc_pyramid; .level(l) returns a numpy view copy."""

    def __init__(self, t: OrbTables, cols: int, rows: int):
        self.p = Pyramid()
        if lib().oc_pyramid_alloc(C.byref(self.p), C.byref(t), cols, rows) != 0:
            raise MemoryError("oc_pyramid_alloc")

    def level(self, l: int) -> np.ndarray:
        w, h, s = self.p.w[l], self.p.h[l], self.p.step[l]
        buf = np.ctypeslib.as_array(self.p.data[l], shape=(h * s,))
        return buf.reshape(h, s)[:, :w].copy()

    def __del__(self):
        try:
            lib().oc_pyramid_free(C.byref(self.p))
        except Exception:
            pass


def extract(t: OrbTables, img: np.ndarray, with_pyramid=False):
    """ORBextractor::Compute on a 2-D u8 image -> (kps[N] KP_DTYPE, desc[N,32] u8[, pyramid])."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    rows, cols = img.shape
    cap = t.nfeatures + 64 * t.nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    pyr = OraclePyramid(t, cols, rows)
    n = lib().oc_orb_extract(C.byref(t), ptr(img), rows, cols, cols, ptr(kps), ptr(desc), cap,
                             C.byref(pyr.p))
    if n < 0:
        cap = -n
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = lib().oc_orb_extract(C.byref(t), ptr(img), rows, cols, cols, ptr(kps), ptr(desc),
                                 cap, C.byref(pyr.p))
    if with_pyramid:
        return kps[:n].copy(), desc[:n].copy(), pyr
    return kps[:n].copy(), desc[:n].copy()


def stereo(t, kl, dl, kr, dr, pyr_l, pyr_r, fx, bf):
    nl = len(kl)
    ur = np.zeros(nl, np.float32)
    depth = np.zeros(nl, np.float32)
    sad = np.zeros(nl, np.int32)
    kl = np.ascontiguousarray(kl)
    kr = np.ascontiguousarray(kr)
    dl = np.ascontiguousarray(dl)
    dr = np.ascontiguousarray(dr)
    lib().oc_stereo_match(C.byref(t), ptr(kl), ptr(dl), nl, ptr(kr), ptr(dr), len(kr),
                          C.byref(pyr_l.p), C.byref(pyr_r.p), fx, bf, ptr(ur), ptr(depth),
                          ptr(sad))
    return ur, depth, sad


def grid_geom(cols, rows, cam=None, dist=None) -> GridGeom:
    """Frame image bounds + grid cell size; with cam (fx, fy, cx, cy, ...) and DistCoef `dist`,
    the undistorted bounds of Frame::ComputeImageBounds."""
    g = GridGeom()
    if dist is None:
        lib().oc_grid_geom_init(C.byref(g), cols, rows)
    else:
        k = np.ascontiguousarray(cam[:4], np.float32)
        d = np.ascontiguousarray(dist, np.float32)
        lib().oc_grid_geom_init_dist(C.byref(g), cols, rows, ptr(k), ptr(d), d.size)
    return g


def undistort_points(cam, dist, xy):
    """cv::undistortPoints(xy, ., K, DistCoef, noArray(), K) restated (oc_undistort_points)."""
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    out = np.zeros_like(xy)
    k = np.ascontiguousarray(cam[:4], np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    lib().oc_undistort_points(ptr(k), ptr(d), d.size, ptr(xy), ptr(out), len(xy))
    return out


def undistort_keypoints(cam, dist, kps):
    """Frame::UndistortKeyPoints restated (oc_undistort_keypoints)."""
    kps = np.ascontiguousarray(kps)
    out = np.zeros_like(kps)
    k = np.ascontiguousarray(cam[:4], np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    lib().oc_undistort_keypoints(ptr(k), ptr(d), d.size, ptr(kps), ptr(out), len(kps))
    return out


def pack_keys(kps) -> np.ndarray:
    """oc_keypoint candidates (octree coords) -> packed keys as the HIP path stores them."""
    x = kps["x"].astype(np.int64)
    y = kps["y"].astype(np.int64)
    s = kps["response"].astype(np.int64)
    return (x | (y << 12) | (s << 23)).astype(np.uint32)


def level_candidates(t, pyr, level):
    cap = 1 << 17
    out = np.zeros(cap, KP_DTYPE)
    n = lib().oc_level_candidates(C.byref(t), C.byref(pyr.p), level, ptr(out), cap)
    return out[:n].copy()


def distribute_octree(t, pyr, level, cands):
    w, h = pyr.p.w[level], pyr.p.h[level]
    cands = np.ascontiguousarray(cands)
    out = np.zeros(len(cands) + 1, KP_DTYPE)
    n = lib().oc_distribute_octree(ptr(cands), len(cands), 16, w - 16, 16, h - 16,
                                   t.features_per_level[level], ptr(out), len(out))
    return out[:n].copy()


def _frame_view(kps, desc, ur, mp):
    fv = FrameView()
    fv.kps = kps.ctypes.data
    fv.desc = desc.ctypes.data
    fv.u_right = ur.ctypes.data
    fv.n = len(kps)
    fv.map_point = mp.ctypes.data
    return fv


def search_frame(t, g, cur_kps, cur_desc, cur_ur, cur_mp, last_kps, last_mp, last_outlier,
                 mp_xyz, mp_desc, mp_nobs, Rcw, tcw, tlc_z, baseline, cam, th, mono, check_ori):
    """OrbMatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono); cur_mp is in/out."""
    arrs = [np.ascontiguousarray(a) for a in (cur_kps, cur_desc, cur_ur)]
    fv = _frame_view(arrs[0], arrs[1], arrs[2], cur_mp)
    last_kps = np.ascontiguousarray(last_kps)
    mp_xyz = np.ascontiguousarray(mp_xyz, np.float32)
    mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
    mp_nobs = np.ascontiguousarray(mp_nobs, np.int32)
    R = np.ascontiguousarray(Rcw, np.float32).reshape(-1)
    tt = np.ascontiguousarray(tcw, np.float32).reshape(-1)
    fx, fy, cx, cy, bf = cam
    return lib().oc_search_by_projection_frame(
        C.byref(g), C.byref(t), C.byref(fv), ptr(last_kps), ptr(last_mp), ptr(last_outlier),
        len(last_kps), ptr(mp_xyz), ptr(mp_desc), ptr(mp_nobs), ptr(R), ptr(tt), tlc_z, baseline,
        fx, fy, cx, cy, bf, th, mono, check_ori)


def search_mps(t, g, cur_kps, cur_desc, cur_ur, cur_mp, q, mp_nobs, nnratio, th):
    """OrbMatcher::SearchByProjection(F, vpMapPoints, th) with map point id == query index."""
    arrs = [np.ascontiguousarray(a) for a in (cur_kps, cur_desc, cur_ur)]
    fv = _frame_view(arrs[0], arrs[1], arrs[2], cur_mp)
    cols = {k: np.ascontiguousarray(q[k]) for k in q.dtype.names}
    in_view = cols["in_view"].astype(np.uint8)
    is_bad = cols["is_bad"].astype(np.uint8)
    level = cols["level"].astype(np.int32)
    desc = np.ascontiguousarray(q["desc"], np.uint8)
    mp_nobs = np.ascontiguousarray(mp_nobs, np.int32)
    return lib().oc_search_by_projection_mps(
        C.byref(g), C.byref(t), C.byref(fv), len(q), ptr(in_view), ptr(is_bad), ptr(level),
        ptr(cols["view_cos"]), ptr(cols["proj_x"]), ptr(cols["proj_y"]), ptr(cols["proj_xr"]),
        ptr(desc), ptr(mp_nobs), nnratio, th)


# ---- PoseOptimization (oracle/pose_oracle.c) ------------------------------------------------
POSE_EDGE_DTYPE = np.dtype([("xw", "<f4", (3,)), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                            ("octave", "<i4")])


def _pose_lib():
    L = lib()
    if not getattr(L, "_pose_bound", False):
        vp, ip = C.c_void_p, C.c_int
        L.oc_pose_optimization.argtypes = [vp, vp, vp, ip, vp, vp, C.POINTER(ip)]
        L.oc_se3_exp.argtypes = [vp, vp, vp]
        L.oc_se3_exp.restype = None
        L.oc_pose_edge_eval.argtypes = [vp, vp, vp, vp, C.c_float, vp, vp]
        L.oc_pose_edge_eval.restype = C.c_double
        L._pose_bound = True
    return L


def pose_optimization(cam, inv_sigma2, edges, Tcw):
    """Optimizer::PoseOptimization restated: returns (n_inliers, Tcw', outlier, lm_iterations)."""
    cam = np.asarray(cam, np.float32)
    isig = np.ascontiguousarray(inv_sigma2, np.float32)
    e = np.ascontiguousarray(edges).view(POSE_EDGE_DTYPE)
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32).reshape(4, 4)).copy()
    outl = np.zeros(max(len(e), 1), np.uint8)
    it = C.c_int()
    r = _pose_lib().oc_pose_optimization(ptr(cam), ptr(isig), ptr(e), len(e), ptr(T), ptr(outl),
                                         C.byref(it))
    return r, T, outl[:len(e)].astype(bool), it.value


def se3_exp(u):
    u = np.ascontiguousarray(u, np.float64)
    R, t = np.zeros(9), np.zeros(3)
    _pose_lib().oc_se3_exp(ptr(u), ptr(R), ptr(t))
    return R.reshape(3, 3), t


def pose_edge_eval(cam, R, t, edge, inv_sigma2):
    """(chi2, error[3], Jacobian[3, 6]) of one edge at pose (R, t)."""
    cam = np.asarray(cam, np.float32)
    R = np.ascontiguousarray(R, np.float64)
    t = np.ascontiguousarray(t, np.float64)
    e1 = np.ascontiguousarray(np.asarray(edge).reshape(1)).view(POSE_EDGE_DTYPE)
    err, J = np.zeros(3), np.zeros(18)
    c = _pose_lib().oc_pose_edge_eval(ptr(cam), ptr(R), ptr(t), ptr(e1), float(inv_sigma2),
                                      ptr(err), ptr(J))
    return c, err, J.reshape(3, 6)


# ---- LocalBundleAdjustment (oracle/ba_oracle.c) -------------------------------------------
BA_OBS_DTYPE = np.dtype([("keyframe", "<i4"), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                         ("octave", "<i4")])


def _ba_lib():
    L = lib()
    if not getattr(L, "_ba_bound", False):
        vp, ip = C.c_void_p, C.c_int
        L.oc_local_bundle_adjustment.argtypes = [vp, vp, vp, vp, ip, vp, ip, vp, vp, vp,
                                                 C.POINTER(ip)]
        L.oc_local_bundle_adjustment_stop.argtypes = [vp, vp, vp, vp, ip, vp, ip, vp, vp, ip,
                                                      vp, C.POINTER(ip)]
        L.oc_global_bundle_adjustment_stop.argtypes = [vp, vp, vp, vp, ip, vp, ip, vp, vp, ip,
                                                       ip, ip, C.POINTER(ip)]
        L.oc_ba_edge_eval.argtypes = [vp, vp, vp, vp, vp, C.c_float, vp, vp, vp]
        L.oc_ba_linearize.argtypes = [vp, vp, vp, vp, ip, vp, ip, vp, vp, vp, vp, vp, vp, vp, vp]
        L.oc_ba_linearize.restype = C.c_double
        L.oc_ba_edge_eval.restype = C.c_double
        L._ba_bound = True
    return L


def local_ba(cam, prob, stop_after=-1):
    """Optimizer::LocalBundleAdjustment restated on a synthetic.ba_problem dict, with the
    reference's stop_flag raised after `stop_after` polls of it (< 0: never). Returns
    (kf_Tcw', points', erase, lm_iterations)."""
    cam = np.asarray(cam, np.float32)
    kf = np.ascontiguousarray(prob["kf_Tcw"], np.float32).copy()
    pts = np.ascontiguousarray(prob["points"], np.float32).copy()
    mode = np.ascontiguousarray(prob["kf_mode"], np.uint8)
    start = np.ascontiguousarray(prob["point_obs_start"], np.int32)
    obs = np.ascontiguousarray(prob["obs"]).view(BA_OBS_DTYPE)
    isig = np.ascontiguousarray(prob["inv_sigma2"], np.float32)
    erase = np.zeros(max(len(obs), 1), np.uint8)
    it = C.c_int()
    r = _ba_lib().oc_local_bundle_adjustment_stop(ptr(cam), ptr(isig), ptr(kf), ptr(mode),
                                                  len(mode), ptr(pts), len(pts), ptr(start),
                                                  ptr(obs), stop_after, ptr(erase), C.byref(it))
    assert r == 0
    return kf, pts, erase[:len(obs)].astype(bool), it.value


def global_ba(cam, prob, n_iterations=10, robust=True, stop_after=-1):
    """Optimizer::BundleAdjustment restated on a synthetic problem dict (kf_mode 1 = the fixed
    keyframe id 0, 0 = optimised). Returns (kf_Tcw', points', lm_iterations)."""
    cam = np.asarray(cam, np.float32)
    kf = np.ascontiguousarray(prob["kf_Tcw"], np.float32).copy()
    pts = np.ascontiguousarray(prob["points"], np.float32).copy()
    mode = np.ascontiguousarray(prob["kf_mode"], np.uint8)
    start = np.ascontiguousarray(prob["point_obs_start"], np.int32)
    obs = np.ascontiguousarray(prob["obs"]).view(BA_OBS_DTYPE)
    isig = np.ascontiguousarray(prob["inv_sigma2"], np.float32)
    it = C.c_int()
    r = _ba_lib().oc_global_bundle_adjustment_stop(ptr(cam), ptr(isig), ptr(kf), ptr(mode),
                                                   len(mode), ptr(pts), len(pts), ptr(start),
                                                   ptr(obs), n_iterations, int(robust),
                                                   stop_after, C.byref(it))
    assert r == 0
    return kf, pts, it.value


def ba_edge_eval(cam, R, t, X, ob, inv_sigma2):
    """(chi2, error[3], Jl[3, 3], Jp[3, 6]) of one binary edge."""
    cam = np.asarray(cam, np.float32)
    R, t, X = (np.ascontiguousarray(a, np.float64) for a in (R, t, X))
    o1 = np.ascontiguousarray(np.asarray(ob).reshape(1)).view(BA_OBS_DTYPE)
    err, Jl, Jp = np.zeros(3), np.zeros(9), np.zeros(18)
    c = _ba_lib().oc_ba_edge_eval(ptr(cam), ptr(R), ptr(t), ptr(X), ptr(o1), float(inv_sigma2),
                                  ptr(err), ptr(Jl), ptr(Jp))
    return c, err, Jl.reshape(3, 3), Jp.reshape(3, 6)


def ba_linearize(cam, prob):
    """computeActiveErrors + buildSystem of LocalBundleAdjustment's first optimize() at the input
    estimates (slamgpu_ba_linear layout). Returns a dict of arrays + the robust chi2."""
    cam = np.asarray(cam, np.float32)
    kf = np.ascontiguousarray(prob["kf_Tcw"], np.float32)
    pts = np.ascontiguousarray(prob["points"], np.float32)
    mode = np.ascontiguousarray(prob["kf_mode"], np.uint8)
    start = np.ascontiguousarray(prob["point_obs_start"], np.int32)
    obs = np.ascontiguousarray(prob["obs"]).view(BA_OBS_DTYPE)
    isig = np.ascontiguousarray(prob["inv_sigma2"], np.float32)
    no, npn, nk = len(obs), len(pts), len(mode)
    out = {"chi2": np.zeros(max(no, 1)), "hpl": np.zeros((max(no, 1), 18)),
           "hll": np.zeros((max(npn, 1), 6)), "bl": np.zeros((max(npn, 1), 3)),
           "hpp": np.zeros((max(nk, 1), 21)), "bp": np.zeros((max(nk, 1), 6))}
    chi = _ba_lib().oc_ba_linearize(ptr(cam), ptr(isig), ptr(kf), ptr(mode), nk, ptr(pts), npn,
                                    ptr(start), ptr(obs), *[ptr(out[k]) for k in
                                                            ("chi2", "hpl", "hll", "bl", "hpp",
                                                             "bp")])
    out["chi"] = chi
    return out


# ---- DBoW2 transform, SearchByBoW, ComputeDistinctiveDescriptors, cvtColor (bow_oracle.c) ------
class VocabArrays(C.Structure):
    _fields_ = [("k", C.c_int), ("L", C.c_int), ("scoring", C.c_int), ("weighting", C.c_int),
                ("n_nodes", C.c_int), ("parent", C.c_void_p), ("leaf_flag", C.c_void_p),
                ("desc", C.c_void_p), ("weight", C.c_void_p)]


def _bow_lib():
    L = lib()
    if not getattr(L, "_bow_bound", False):
        vp, ip = C.c_void_p, C.c_int
        L.oc_vocab_build.argtypes = [C.POINTER(VocabArrays)]
        L.oc_vocab_build.restype = vp
        L.oc_vocab_free.argtypes = [vp]
        L.oc_vocab_free.restype = None
        L.oc_vocab_transform_one.argtypes = [vp, vp, ip, vp, vp, vp, vp]
        L.oc_vocab_transform_one.restype = None
        L.oc_bow_transform.argtypes = [vp, vp, ip, ip, vp, vp, C.POINTER(ip), vp, vp, vp,
                                       C.POINTER(ip)]
        L.oc_search_by_bow.argtypes = [vp, vp, vp, ip, vp, vp, vp, ip, vp, vp, vp, ip, vp, vp, vp,
                                       ip, ip, C.c_float, ip, vp]
        L.oc_distinctive_descriptors.argtypes = [vp, vp, ip, vp]
        L.oc_distinctive_descriptors.restype = None
        L.oc_cvt_gray.argtypes = [vp, C.c_size_t, ip, ip, ip, ip, vp, C.c_size_t]
        L.oc_cvt_gray.restype = None
        L._bow_bound = True
    return L


class OracleVocab:
    """oc_vocab built from a vocabulary dict (synthetic.vocabulary layout)."""

    def __init__(self, V):
        self.keep = [np.ascontiguousarray(V["parent"], np.int32),
                     np.ascontiguousarray(V["leaf"], np.uint8),
                     np.ascontiguousarray(V["desc"], np.uint8).reshape(-1, 32),
                     np.ascontiguousarray(V["weight"], np.float64)]
        a = VocabArrays(int(V["k"]), int(V["L"]), int(V["scoring"]), int(V["weighting"]),
                        len(self.keep[0]), *[x.ctypes.data for x in self.keep])
        self.h = _bow_lib().oc_vocab_build(C.byref(a))
        if not self.h:
            raise ValueError("oc_vocab_build rejected the arrays")

    def __del__(self):
        try:
            _bow_lib().oc_vocab_free(self.h)
        except Exception:
            pass


def transform_one(ov, d, levelsup=4):
    """(word, weight, nid, leaf) of one descriptor."""
    d = np.ascontiguousarray(d, np.uint8)
    w, n, f = (np.zeros(1, np.uint32) for _ in range(3))
    wt = np.zeros(1)
    _bow_lib().oc_vocab_transform_one(ov.h, ptr(d), levelsup, ptr(w), ptr(wt), ptr(n), ptr(f))
    return int(w[0]), float(wt[0]), int(n[0]), int(f[0])


def bow_transform(ov, desc, levelsup=4):
    """transform(features, BowVector, FeatureVector, levelsup) ->
    (words, values, nodes, node_start, node_feats)."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(d)
    m = max(n, 1)
    words, vals = np.zeros(m, np.uint32), np.zeros(m)
    nodes, feats = np.zeros(m, np.uint32), np.zeros(m, np.uint32)
    start = np.zeros(m + 1, np.int32)
    nw, nn = C.c_int(), C.c_int()
    _bow_lib().oc_bow_transform(ov.h, ptr(d), n, levelsup, ptr(words), ptr(vals), C.byref(nw),
                                ptr(nodes), ptr(start), ptr(feats), C.byref(nn))
    nw, nn = nw.value, nn.value
    return (words[:nw].copy(), vals[:nw].copy(), nodes[:nn].copy(), start[:nn + 1].copy(),
            feats[:start[nn]].copy())


def search_by_bow(a_desc, a_kps, a_valid, a_fv, b_desc, b_kps, b_valid, b_fv, strict_lt, nnratio,
                  check_ori):
    """a_fv / b_fv = (nodes, node_start, node_feats); b_valid None = every B feature.
    Returns (nmatches, match_a)."""
    def arrs(desc, kps, valid, fv):
        return (np.ascontiguousarray(desc, np.uint8).reshape(-1, 32),
                np.ascontiguousarray(kps).view(KP_DTYPE) if len(kps) else np.zeros(1, KP_DTYPE),
                None if valid is None else np.ascontiguousarray(valid, np.uint8),
                np.ascontiguousarray(fv[0], np.uint32), np.ascontiguousarray(fv[1], np.int32),
                np.ascontiguousarray(fv[2], np.uint32))
    A = arrs(a_desc, a_kps, a_valid, a_fv)
    B = arrs(b_desc, b_kps, b_valid, b_fv)
    na = len(A[0])
    match = np.zeros(max(na, 1), np.int32)
    p = lambda x: None if x is None else ptr(x)  # noqa: E731
    nm = _bow_lib().oc_search_by_bow(p(A[0]), p(A[1]), p(A[2]), na, p(A[3]), p(A[4]), p(A[5]),
                                     len(A[3]), p(B[0]), p(B[1]), p(B[2]), len(B[0]), p(B[3]),
                                     p(B[4]), p(B[5]), len(B[3]), int(bool(strict_lt)),
                                     float(nnratio), int(bool(check_ori)), ptr(match))
    return nm, match[:na]


def distinctive(desc, start):
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    st = np.ascontiguousarray(start, np.int32)
    best = np.zeros(max(len(st) - 1, 1), np.int32)
    _bow_lib().oc_distinctive_descriptors(ptr(d), ptr(st), len(st) - 1, ptr(best))
    return best[:len(st) - 1]


def cvt_gray(img, rgb=True):
    a = np.ascontiguousarray(img, np.uint8)
    rows, cols, cn = a.shape
    out = np.zeros((rows, cols), np.uint8)
    _bow_lib().oc_cvt_gray(ptr(a), a.strides[0], cn, int(bool(rgb)), cols, rows, ptr(out), cols)
    return out


# ---- SearchForTriangulation, Fuse (kfmatch_oracle.c) -------------------------------------------
def _kf_lib():
    L = lib()
    if not getattr(L, "_kf_bound", False):
        vp, ip, fp = C.c_void_p, C.c_int, C.c_float
        L.oc_search_for_triangulation.argtypes = [vp, vp, vp, vp, ip, vp, vp, vp, ip,
                                                  vp, vp, vp, vp, vp, vp, vp, ip,
                                                  vp, vp, fp, fp, fp, fp, vp, vp, vp, ip, ip, vp]
        L.oc_fuse.argtypes = [vp, vp, vp, ip, C.POINTER(GridGeom), vp, vp, vp, fp, fp, fp, fp, fp,
                              vp, vp, ip, fp, vp, ip, fp, vp, vp]
        L.oc_predict_scale.argtypes = [fp, fp, fp, ip]
        L.oc_logf.argtypes = [fp]
        L.oc_logf.restype = fp
        L._kf_bound = True
    return L


def search_for_triangulation(kf1, kf2, C1w, T2w, cam4, scale, sigma2, F12, only_stereo,
                             check_ori):
    """kf = dict(kps, desc, ur, mp (u8), fv=(nodes, start, feats)). T2w = R (row-major) + t.
    Returns (nmatches, match12)."""
    def arrs(k):
        return (np.ascontiguousarray(k["kps"]).view(KP_DTYPE) if len(k["kps"]) else
                np.zeros(1, KP_DTYPE),
                np.ascontiguousarray(k["desc"], np.uint8).reshape(-1, 32),
                np.ascontiguousarray(k["ur"], np.float32), np.ascontiguousarray(k["mp"], np.uint8),
                np.ascontiguousarray(k["fv"][0], np.uint32),
                np.ascontiguousarray(k["fv"][1], np.int32),
                np.ascontiguousarray(k["fv"][2], np.uint32))
    A, B = arrs(kf1), arrs(kf2)
    n1 = len(A[1])
    m = np.zeros(max(n1, 1), np.int32)
    f = lambda a: np.ascontiguousarray(a, np.float32).reshape(-1)  # noqa: E731
    keep = [f(C1w), f(T2w), f(scale), f(sigma2), f(F12)]
    nm = _kf_lib().oc_search_for_triangulation(
        ptr(A[0]), ptr(A[1]), ptr(A[2]), ptr(A[3]), n1, ptr(A[4]), ptr(A[5]), ptr(A[6]), len(A[4]),
        ptr(B[0]), ptr(B[1]), ptr(B[2]), ptr(B[3]), ptr(B[4]), ptr(B[5]), ptr(B[6]), len(B[4]),
        ptr(keep[0]), ptr(keep[1]), *[float(np.float32(c)) for c in cam4], ptr(keep[2]),
        ptr(keep[3]), ptr(keep[4]), int(bool(only_stereo)), int(bool(check_ori)), ptr(m))
    return nm, m[:n1]


def fuse(kps, desc, ur, grid, Rcw, tcw, Ow, cam, scale, inv_sigma2, log_scale_factor, points, th):
    """Fuse's candidate search; grid = GridGeom; points = FUSE_POINT records (80 B).
    Returns (nfused, best_idx, best_dist)."""
    k = np.ascontiguousarray(kps).view(KP_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    u = np.ascontiguousarray(ur, np.float32)
    f = lambda a: np.ascontiguousarray(a, np.float32).reshape(-1)  # noqa: E731
    keep = [f(Rcw), f(tcw), f(Ow), f(scale), f(inv_sigma2)]
    pts = np.ascontiguousarray(points)
    n = len(pts)
    bi, bd = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.int32)
    nf = _kf_lib().oc_fuse(ptr(k), ptr(d), ptr(u), len(d), C.byref(grid), ptr(keep[0]),
                           ptr(keep[1]), ptr(keep[2]), *[float(np.float32(c)) for c in cam],
                           ptr(keep[3]), ptr(keep[4]), len(keep[3]), float(log_scale_factor),
                           ptr(pts), n, float(th), ptr(bi), ptr(bd))
    return nf, bi[:n], bd[:n]


# ---- OptimizeSim3 (oracle/sim3_oracle.c) ----------------------------------------------------
def _sim3_lib():
    L = lib()
    if not getattr(L, "_sim3_bound", False):
        vp, ip = C.c_void_p, C.c_int
        L.oc_optimize_sim3.argtypes = [vp, vp, vp, vp, ip, vp, ip, C.c_float, ip, vp, vp,
                                       C.POINTER(ip)]
        for name, n in [("oc_sim3_exp", 2), ("oc_sim3_log", 2), ("oc_sim3_mul", 3),
                        ("oc_sim3_inverse", 2), ("oc_sim3_map", 3)]:
            getattr(L, name).argtypes = [vp] * n
            getattr(L, name).restype = None
        L.oc_sim3_pair_eval.argtypes = [vp, vp, vp, vp, ip, vp, vp]
        L.oc_sim3_pair_eval.restype = None
        L._sim3_bound = True
    return L


def optimize_sim3(K1, K2, isig1, isig2, matches, S12, th2=10.0, fix_scale=False):
    """Optimizer::OptimizeSim3 restated: returns (n_in, S12', inlier, lm_iterations)."""
    from slam_framework_amd.slamgpu import SIM3_MATCH_DTYPE
    K1 = np.ascontiguousarray(K1[:4], np.float32)
    K2 = np.ascontiguousarray(K2[:4], np.float32)
    i1 = np.ascontiguousarray(isig1, np.float32)
    i2 = np.ascontiguousarray(isig2, np.float32)
    m = np.ascontiguousarray(matches).view(SIM3_MATCH_DTYPE)
    S = np.ascontiguousarray(S12, np.float64).copy()
    inl = np.zeros(max(len(m), 1), np.uint8)
    it = C.c_int()
    r = _sim3_lib().oc_optimize_sim3(ptr(K1), ptr(K2), ptr(i1), ptr(i2), len(i1), ptr(m), len(m),
                                     float(th2), int(bool(fix_scale)), ptr(S), ptr(inl),
                                     C.byref(it))
    return r, S, inl[:len(m)].astype(bool), it.value


def _s8(a):
    return np.ascontiguousarray(a, np.float64)


def sim3_exp(u):
    o = np.zeros(8)
    _sim3_lib().oc_sim3_exp(ptr(_s8(u)), ptr(o))
    return o


def sim3_log(S):
    o = np.zeros(7)
    _sim3_lib().oc_sim3_log(ptr(_s8(S)), ptr(o))
    return o


def sim3_mul(a, b):
    o = np.zeros(8)
    _sim3_lib().oc_sim3_mul(ptr(_s8(a)), ptr(_s8(b)), ptr(o))
    return o


def sim3_inverse(a):
    o = np.zeros(8)
    _sim3_lib().oc_sim3_inverse(ptr(_s8(a)), ptr(o))
    return o


def sim3_map(a, x):
    o = np.zeros(3)
    _sim3_lib().oc_sim3_map(ptr(_s8(a)), ptr(_s8(x)), ptr(o))
    return o


def sim3_pair_eval(K1, K2, match, S12, fix_scale=False):
    """(e[4] = e12, e21; J[2 edges][2][7]) of one correspondence at S12 (numeric Jacobians)."""
    from slam_framework_amd.slamgpu import SIM3_MATCH_DTYPE
    K1 = np.ascontiguousarray(K1[:4], np.float32)
    K2 = np.ascontiguousarray(K2[:4], np.float32)
    m = np.ascontiguousarray(np.asarray(match).reshape(1)).view(SIM3_MATCH_DTYPE)
    e, J = np.zeros(4), np.zeros(28)
    _sim3_lib().oc_sim3_pair_eval(ptr(K1), ptr(K2), ptr(m), ptr(_s8(S12)), int(bool(fix_scale)),
                                  ptr(e), ptr(J))
    return e, J.reshape(2, 2, 7)


# ---- OptimizeEssentialGraph (oracle/eg_oracle.c) --------------------------------------------
def _eg_lib():
    L = _sim3_lib()
    if not getattr(L, "_eg_bound", False):
        vp, ip = C.c_void_p, C.c_int
        L.oc_optimize_essential_graph.argtypes = [ip, vp, vp, vp, ip, ip, ip, vp, C.POINTER(ip)]
        L.oc_correct_points_sim3.argtypes = [vp, vp, vp, vp, ip]
        L.oc_correct_points_sim3.restype = None
        L.oc_sim3_edge_eval.argtypes = [vp, vp, vp, ip, vp, vp, vp]
        L.oc_sim3_edge_eval.restype = C.c_double
        L._eg_bound = True
    return L


def optimize_essential_graph(Scw, fixed, edges, fix_scale=True, n_iterations=20):
    """OptimizeEssentialGraph restated: returns (Scw' [n][8], Tcw' [n][4][4] f32, lm_iterations)."""
    from slam_framework_amd.slamgpu import SIM3_EDGE_DTYPE
    S = np.ascontiguousarray(Scw, np.float64).copy()
    fx = np.ascontiguousarray(fixed, np.uint8)
    E = np.ascontiguousarray(edges).view(SIM3_EDGE_DTYPE)
    T = np.zeros((max(len(S), 1), 4, 4), np.float32)
    it = C.c_int()
    _eg_lib().oc_optimize_essential_graph(len(S), ptr(S), ptr(fx), ptr(E), len(E),
                                          int(bool(fix_scale)), int(n_iterations), ptr(T),
                                          C.byref(it))
    return S, T[:len(S)], it.value


def correct_points_sim3(Scw_before, Scw_after, ref, points):
    P = np.ascontiguousarray(points, np.float32).copy()
    _eg_lib().oc_correct_points_sim3(ptr(_s8(Scw_before)), ptr(_s8(Scw_after)),
                                     ptr(np.ascontiguousarray(ref, np.int32)), ptr(P), len(P))
    return P


def sim3_edge_eval(Si, Sj, Sji, fix_scale=False):
    e, Ji, Jj = np.zeros(7), np.zeros(49), np.zeros(49)
    c = _eg_lib().oc_sim3_edge_eval(ptr(_s8(Si)), ptr(_s8(Sj)), ptr(_s8(Sji)),
                                    int(bool(fix_scale)), ptr(e), ptr(Ji), ptr(Jj))
    return c, e, Ji.reshape(7, 7), Jj.reshape(7, 7)
