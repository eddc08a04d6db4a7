"""GPU parity of the LocalMapper's keyframe-rate matchers against
the oracle (oracle/kfmatch_oracle.c, pinned by tests/test_kfmatch_oracle.py), through the C ABI
(include/slamgpu_kfmatch.h): bit-exact match arrays and counts of
OrbMatcher::SearchForTriangulation (orb_matcher.cpp:634-802) and bit-exact best keypoint /
distance per map point of OrbMatcher::Fuse's candidate search (:804-928), on keyframes built
from real ORB features of synthetic frames (kf_scenario.py), single and batched calls."""
import numpy as np
import pytest

import kf_scenario as KS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(gpu_lib):
    from slam_framework_amd import kfmatch
    return kfmatch


@pytest.fixture(scope="module")
def scene(oracle):
    kfs, _ = KS.keyframes(oracle)
    return kfs


def _fv(B, k):
    from slam_framework_amd.bow import FeatureVector
    return FeatureVector(*k["fv"])


POSES = [(KS.pose(0), KS.pose(1, (-0.4, 0.02, 0.1))), (KS.pose(0), KS.pose(1, (0.0, 0.0, 0.8))),
         (KS.pose(1, (0.3, -0.1, 0.0)), KS.pose(0))]


@pytest.mark.parametrize("poses", range(len(POSES)))
@pytest.mark.parametrize("only_stereo", [False, True])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_triangulation(oracle, K, scene, poses, only_stereo, check_ori):
    T1, T2 = POSES[poses]
    k1, k2 = scene
    F = KS.fundamental(T1, T2)
    lv = K.levels()
    sc, s2, _, _ = KS.levels_arrays()
    T2w = np.concatenate([T2[:3, :3].reshape(-1), T2[:3, 3]]).astype(np.float32)
    a = K.host_kf(k1["kps"], k1["desc"], k1["ur"], T1, k1["mp"], _fv(None, k1))
    b = K.host_kf(k2["kps"], k2["desc"], k2["ur"], T2, k2["mp"], _fv(None, k2))
    nm_o, m_o = oracle.search_for_triangulation(k1, k2, np.array(a[0].Ow, np.float32), T2w,
                                                KS.CAM[:4], sc, s2, F, only_stereo, check_ori)
    nm_g, m_g = K.search_for_triangulation(a, b, F, KS.CAM, lv, only_stereo, check_ori)
    assert nm_g == nm_o
    np.testing.assert_array_equal(m_g, m_o)
    assert nm_o > 20


def test_search_for_triangulation_reference_surface(oracle, K, scene):
    """OrbMatcher.SearchForTriangulation: vMatchedPairs in ascending pKF1 order."""
    import types
    from slam_framework_amd.slamgpu import OrbMatcher
    T1, T2 = POSES[0]
    k1, k2 = scene
    mk = lambda k, T: types.SimpleNamespace(  # noqa: E731
        keypoints=k["kps"], descriptors=k["desc"], u_right=k["ur"],
        map_points=np.where(k["mp"] > 0, 7, -1), feature_vec=_fv(None, k), Tcw=T)
    F = KS.fundamental(T1, T2)
    nm, pairs = OrbMatcher(0.6, True).SearchForTriangulation(mk(k1, T1), mk(k2, T2), F, KS.CAM,
                                                             K.levels())
    a = K.host_kf(k1["kps"], k1["desc"], k1["ur"], T1, k1["mp"], _fv(None, k1))
    b = K.host_kf(k2["kps"], k2["desc"], k2["ur"], T2, k2["mp"], _fv(None, k2))
    _, m = K.search_for_triangulation(a, b, F, KS.CAM, K.levels())
    assert nm == len(pairs) == int((m >= 0).sum())
    np.testing.assert_array_equal(pairs[:, 1], m[pairs[:, 0]])
    assert (np.diff(pairs[:, 0]) > 0).all()


@pytest.mark.parametrize("th", [1.0, 3.0, 5.0])
def test_fuse(oracle, K, scene, th):
    k0, k1 = scene
    T0, T1 = KS.pose(0), KS.pose(1)
    pts = KS.fuse_points(k0, T0)
    lv = K.levels()
    lva = KS.levels_arrays()
    grid_o = oracle.grid_geom(1241, 376)
    kf = K.host_kf(k1["kps"], k1["desc"], k1["ur"], T1)
    nf_o, bi_o, bd_o = oracle.fuse(k1["kps"], k1["desc"], k1["ur"], grid_o,
                                   T1[:3, :3].reshape(-1), T1[:3, 3], np.array(kf[0].Ow, np.float32),
                                   KS.CAM, lva[0], lva[2], float(lv.log_scale_factor), pts, th)
    nf_g, bi_g, bd_g = K.fuse(kf, pts, th, KS.CAM, lv, K.kf_grid(1241, 376))
    assert nf_g == nf_o
    np.testing.assert_array_equal(bi_g, bi_o)
    np.testing.assert_array_equal(bd_g, bd_o)
    assert nf_o > 100


def test_fuse_apply_counts(K, scene):
    """fuse_apply: nFused = #(best_idx >= 0) for distinct, unskipped points; Replace keeps the
    point with more observations."""
    best = np.array([3, -1, 3, 5], np.int32)
    kf_mp = np.full(10, -1)
    kf_mp[5] = 9
    nobs = np.array([2, 1, 4, 1, 0, 0, 0, 0, 0, 3])
    bad = np.zeros(10, bool)
    in_kf = np.zeros(10, bool)
    in_kf[9] = True
    n = K.fuse_apply(best, kf_mp, [0, 1, 2, 3], nobs, bad, in_kf)
    assert n == 3
    assert kf_mp[3] == 2 and bad[0]       # 2 (4 obs) replaced 0 (3 obs after AddObservation)
    assert kf_mp[5] == 9 and bad[3]       # 9 (3 obs) kept over 3 (1 obs)


def test_batched_device_calls(oracle, K, scene, torch_dev=None):
    import torch
    dev = torch.device("cuda", 0)
    k0, k1 = scene
    Ts = [KS.pose(0), KS.pose(1, (-0.4, 0.02, 0.1)), KS.pose(1)]
    frames = [k0, k1, k1]
    keep = []

    def dev_arr(a):
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
        keep.append(t)
        return int(t.data_ptr())

    kfs = np.zeros(3, K.KF_DTYPE)
    for i, (k, T) in enumerate(zip(frames, Ts)):
        h = K.host_kf(k["kps"], k["desc"], k["ur"], T, k["mp"], _fv(None, k))[0]
        kfs[i]["kps"], kfs[i]["desc"] = dev_arr(k["kps"]), dev_arr(k["desc"])
        kfs[i]["u_right"], kfs[i]["has_mp"] = dev_arr(k["ur"]), dev_arr(k["mp"])
        kfs[i]["nodes"] = dev_arr(k["fv"][0].astype(np.uint32))
        kfs[i]["node_start"] = dev_arr(k["fv"][1].astype(np.int32))
        kfs[i]["node_feats"] = dev_arr(k["fv"][2].astype(np.uint32))
        kfs[i]["n"], kfs[i]["n_nodes"] = len(k["desc"]), len(k["fv"][0])
        kfs[i]["Rcw"], kfs[i]["tcw"], kfs[i]["Ow"] = list(h.Rcw), list(h.tcw), list(h.Ow)
    d_kfs = torch.from_numpy(kfs.view(np.uint8).copy()).to(dev)
    pairs = np.zeros(3, K.TRI_PAIR_DTYPE)
    for p, (a, b, st) in enumerate([(0, 1, 0), (1, 0, 1), (0, 2, 0)]):
        pairs[p] = (a, b, KS.fundamental(Ts[a], Ts[b]).reshape(-1), st)
    d_pairs = torch.from_numpy(pairs.view(np.uint8).copy()).to(dev)
    cap = 2100
    d_m = torch.full((3, cap), -9, dtype=torch.int32, device=dev)
    d_nm = torch.zeros(3, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lv = K.levels()
    K.search_for_triangulation_device(d_kfs, d_pairs, 3, KS.CAM, lv, True, d_m, cap, d_nm, st)
    # Fuse: the same points into keyframes 1 and 2 (batched by d_point_kf)
    pts = KS.fuse_points(k0, Ts[0])
    allp = np.concatenate([pts, pts])
    pkf = np.concatenate([np.full(len(pts), 1), np.full(len(pts), 2)]).astype(np.int32)
    d_pts = torch.from_numpy(allp.view(np.uint8).copy()).to(dev)
    d_pkf = torch.from_numpy(pkf).to(dev)
    d_bi = torch.zeros(len(allp), dtype=torch.int32, device=dev)
    d_bd = torch.zeros(len(allp), dtype=torch.int32, device=dev)
    K.fuse_device(d_kfs, d_pts, d_pkf, len(allp), 3.0, KS.CAM, lv, K.kf_grid(1241, 376), d_bi,
                  d_bd, st)
    torch.cuda.synchronize()
    sc, s2, _, _ = KS.levels_arrays()
    m, nm = d_m.cpu().numpy(), d_nm.cpu().numpy()
    for p, (a, b, stereo) in enumerate([(0, 1, 0), (1, 0, 1), (0, 2, 0)]):
        T2w = np.concatenate([Ts[b][:3, :3].reshape(-1), Ts[b][:3, 3]]).astype(np.float32)
        nm_o, m_o = oracle.search_for_triangulation(frames[a], frames[b], kfs[a]["Ow"], T2w,
                                                    KS.CAM[:4], sc, s2,
                                                    pairs[p]["F12"], stereo, True)
        assert nm[p] == nm_o
        np.testing.assert_array_equal(m[p, :len(frames[a]["desc"])], m_o)
    bi, bd = d_bi.cpu().numpy(), d_bd.cpu().numpy()
    grid_o = oracle.grid_geom(1241, 376)
    lva = KS.levels_arrays()
    for q, ki in enumerate((1, 2)):
        _, bi_o, bd_o = oracle.fuse(frames[ki]["kps"], frames[ki]["desc"], frames[ki]["ur"],
                                    grid_o, Ts[ki][:3, :3].reshape(-1), Ts[ki][:3, 3],
                                    kfs[ki]["Ow"], KS.CAM, lva[0], lva[2],
                                    float(lv.log_scale_factor), pts, 3.0)
        np.testing.assert_array_equal(bi[q * len(pts):(q + 1) * len(pts)], bi_o)
        np.testing.assert_array_equal(bd[q * len(pts):(q + 1) * len(pts)], bd_o)


def test_errors_are_loud(K, scene):
    from slam_framework_amd.slamgpu import SlamGpuError
    k1 = scene[0]
    kps = k1["kps"].copy()
    kps["octave"][0] = 40
    a = K.host_kf(kps, k1["desc"], k1["ur"], KS.pose(0), k1["mp"], _fv(None, k1))
    with pytest.raises(SlamGpuError):
        K.search_for_triangulation(a, a, np.eye(3), KS.CAM, K.levels())
    lv = K.levels()
    lv.nlevels = 0
    b = K.host_kf(k1["kps"], k1["desc"], k1["ur"], KS.pose(0))
    with pytest.raises(SlamGpuError):
        K.fuse(b, KS.fuse_points(k1, KS.pose(0))[:4], 3.0, KS.CAM, lv, K.kf_grid(1241, 376))


def test_device_malformed_keyframe_flags_pair(K, scene):
    """Batched SearchForTriangulation with a FeatureVector entry naming a feature >= n, and with a
    keypoint octave outside [0, nlevels): the pair reports -1 and nothing outside its match row
    (or the LDS bin table) is written; a well-formed pair of the same launch is unaffected."""
    import torch
    dev = torch.device("cuda", 0)
    k0, k1 = scene
    T0, T1 = KS.pose(0), KS.pose(1, (-0.4, 0.02, 0.1))
    keep = []

    def dev_arr(a):
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
        keep.append(t)
        return int(t.data_ptr())

    bad_feats = k0["fv"][2].astype(np.uint32).copy()
    bad_feats[len(bad_feats) // 2] = 60000            # feature index far past n
    bad_kps = k1["kps"].copy()
    bad_kps["octave"][:] = 31                         # >= nlevels (8)
    variants = [(k0, k0["fv"][2], k0["kps"]), (k0, bad_feats, k0["kps"]), (k1, k1["fv"][2], bad_kps),
                (k1, k1["fv"][2], k1["kps"])]
    kfs = np.zeros(len(variants), K.KF_DTYPE)
    for i, (k, feats, kps) in enumerate(variants):
        T = T0 if k is k0 else T1
        h = K.host_kf(k["kps"], k["desc"], k["ur"], T, k["mp"], _fv(None, k))[0]
        kfs[i]["kps"], kfs[i]["desc"] = dev_arr(kps), dev_arr(k["desc"])
        kfs[i]["u_right"], kfs[i]["has_mp"] = dev_arr(k["ur"]), dev_arr(k["mp"])
        kfs[i]["nodes"] = dev_arr(k["fv"][0].astype(np.uint32))
        kfs[i]["node_start"] = dev_arr(k["fv"][1].astype(np.int32))
        kfs[i]["node_feats"] = dev_arr(feats.astype(np.uint32))
        kfs[i]["n"], kfs[i]["n_nodes"] = len(k["desc"]), len(k["fv"][0])
        kfs[i]["Rcw"], kfs[i]["tcw"], kfs[i]["Ow"] = list(h.Rcw), list(h.tcw), list(h.Ow)
    d_kfs = torch.from_numpy(kfs.view(np.uint8).copy()).to(dev)
    plist = [(0, 3), (1, 3), (0, 2)]                  # good, bad FeatureVector in kf1, bad octaves in kf2
    pairs = np.zeros(len(plist), K.TRI_PAIR_DTYPE)
    for p, (a, b) in enumerate(plist):
        pairs[p] = (a, b, KS.fundamental(T0, T1).reshape(-1), 0)
    d_pairs = torch.from_numpy(pairs.view(np.uint8).copy()).to(dev)
    cap = 2100
    guard = 64
    d_m = torch.full((len(plist) * cap + guard,), -9, dtype=torch.int32, device=dev)
    d_nm = torch.zeros(len(plist), dtype=torch.int32, device=dev)
    K.search_for_triangulation_device(d_kfs, d_pairs, len(plist), KS.CAM, K.levels(), True, d_m,
                                      cap, d_nm, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    nm, m = d_nm.cpu().numpy(), d_m.cpu().numpy()
    assert nm[0] > 20 and nm[1] == -1 and nm[2] == -1
    assert (m[len(plist) * cap:] == -9).all(), "wrote past the last match row"
