"""Parity of the HIP stereo matcher and projection matchers against the oracle.

Stereo: Frame::ComputeStereoMatches (src/data/frame.cpp:406-577).
Frame-to-frame: OrbMatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
(src/orb_features/orb_matcher.cpp:1312-1453). Local map: SearchByProjection(Frame&,
vector<MapPoint*>, th) (:13-103). Inputs are synthetic sequences (no KITTI on any box); the
oracle is the CPU restatement in oracle/ (parity vs the unbuildable reference is unpinned)."""
import numpy as np
import pytest

import scenario
from slam_framework_amd import synthetic as S

pytestmark = pytest.mark.gpu
CAM = S.KITTI_CAM


@pytest.fixture(scope="module")
def seq(oracle):
    """Oracle front-end results of 3 frames of one synthetic sequence."""
    t = oracle.tables()
    L, R = S.sequence(2000, 3)
    frames = []
    for i in range(3):
        kl, dl, pl = oracle.extract(t, L[i], True)
        kr, dr, pr = oracle.extract(t, R[i], True)
        ur, depth, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
        frames.append(dict(kl=kl, dl=dl, kr=kr, dr=dr, ur=ur, depth=depth))
    return t, L, R, frames


@pytest.fixture(scope="module")
def ctx(gpu_lib):
    return gpu_lib.Context(S.KITTI_COLS, S.KITTI_ROWS)


def _eq_kps(a, b):
    assert len(a) == len(b)
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("i", [0, 1, 2])
def test_stereo_matches_oracle(seq, ctx, i):
    t, L, R, fr = seq
    ctx.frame_stereo(L[i], R[i], CAM)
    kl, dl = ctx.keypoints(0)
    kr, dr = ctx.keypoints(1)
    _eq_kps(kl, fr[i]["kl"])
    _eq_kps(kr, fr[i]["kr"])
    np.testing.assert_array_equal(dl, fr[i]["dl"])
    np.testing.assert_array_equal(dr, fr[i]["dr"])
    ur, depth = ctx.stereo(0)
    assert ur.tobytes() == fr[i]["ur"].tobytes(), np.nonzero(ur != fr[i]["ur"])[0][:10]
    assert depth.tobytes() == fr[i]["depth"].tobytes()
    assert (depth > 0).sum() > 100


def test_frame_graph_recapture_and_eager(seq, gpu_lib, oracle):
    """slamgpu_frame_stereo replays one captured HIP graph per (camera, distortion): a camera
    change re-captures it (depth follows the new bf), and the eager launch chain (taken while
    kernel timing is on) gives the same bytes."""
    t, L, R, fr = seq
    c = gpu_lib.Context(S.KITTI_COLS, S.KITTI_ROWS)
    cam2 = tuple(CAM[:4]) + (CAM[4] * 1.25,)
    kl, dl, pl = oracle.extract(t, L[1], True)
    kr, dr, pr = oracle.extract(t, R[1], True)
    ur2, depth2, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, cam2[0], cam2[4])
    for cam, ref_ur, ref_depth in ((CAM, fr[1]["ur"], fr[1]["depth"]), (cam2, ur2, depth2),
                                   (CAM, fr[1]["ur"], fr[1]["depth"])):
        for eager in (False, True):
            if eager:
                c.timing_start("*", 256)
            c.frame_stereo(L[1], R[1], cam)
            if eager:
                c.timing_stop()
            _eq_kps(c.keypoints(0)[0], fr[1]["kl"])
            ur, depth = c.stereo(0)
            assert ur.tobytes() == ref_ur.tobytes()
            assert depth.tobytes() == ref_depth.tobytes()


@pytest.mark.parametrize("blocks_frac,check_ori,th", [(1.0, 1, 7.0), (0.0, 1, 7.0), (0.5, 0, 14.0),
                                                      (0.5, 1, 7.0)])
def test_f2f_matches_oracle(seq, ctx, oracle, blocks_frac, check_ori, th):
    t, L, R, fr = seq
    g = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
    for cur in (1, 2):
        last = fr[cur - 1]
        q, last_mp, last_out, xyz, mdesc, nobs = scenario.vo_queries(
            last["kl"], last["dl"], last["depth"], cur - 1, np.random.default_rng(cur), blocks_frac)
        p = scenario.pose(cur, th=th, check_ori=check_ori)
        n = len(fr[cur]["kl"])
        mp_o = np.full(n, -1, np.int32)
        nm_o = oracle.search_frame(t, g, fr[cur]["kl"], fr[cur]["dl"], fr[cur]["ur"], mp_o,
                                   last["kl"], last_mp, last_out, xyz, mdesc, nobs,
                                   p["Rcw"][0].reshape(3, 3), p["tcw"][0], 0.0,
                                   float(p["baseline"][0]), CAM, th, 0, check_ori)
        ctx.frame_stereo(L[cur], R[cur], CAM)
        mp_g = np.full(n, -1, np.int32)
        blk = np.zeros(n, np.uint8)
        nm_g = ctx.search_by_projection_frame(0, q, p, mp_g, blk)
        assert nm_g == nm_o
        np.testing.assert_array_equal(mp_g, mp_o)
        assert nm_o > 20, "scenario should produce real frame-to-frame matches"


def test_f2f_claim_fallback(seq, ctx, oracle):
    """Many identical blocking queries compete for the same keypoints: later queries exhaust
    their kept top-K candidates and must rescan with the live claims."""
    t, L, R, fr = seq
    g = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
    last = fr[0]
    q, last_mp, last_out, xyz, mdesc, nobs = scenario.vo_queries(
        last["kl"], last["dl"], last["depth"], 0, np.random.default_rng(5), 1.0)
    rep = 12
    sel = np.arange(min(40, len(q)))
    q2 = np.repeat(q[sel], rep)
    q2["mp_id"] = np.arange(len(q2))
    # oracle view: one last-frame keypoint per query, in query order
    lk = np.repeat(last["kl"][np.nonzero(last_mp >= 0)[0][sel]], rep)
    lmp = np.arange(len(q2), dtype=np.int32)
    lout = np.zeros(len(q2), np.uint8)
    p = scenario.pose(1, th=14.0, check_ori=0)
    n = len(fr[1]["kl"])
    mp_o = np.full(n, -1, np.int32)
    nm_o = oracle.search_frame(t, g, fr[1]["kl"], fr[1]["dl"], fr[1]["ur"], mp_o, lk, lmp, lout,
                               q2["xyz"], q2["desc"], np.ones(len(q2), np.int32),
                               p["Rcw"][0].reshape(3, 3), p["tcw"][0], 0.0,
                               float(p["baseline"][0]), CAM, 14.0, 0, 0)
    ctx.frame_stereo(L[1], R[1], CAM)
    mp_g = np.full(n, -1, np.int32)
    nm_g = ctx.search_by_projection_frame(0, q2, p, mp_g, np.zeros(n, np.uint8))
    assert nm_g == nm_o
    np.testing.assert_array_equal(mp_g, mp_o)


@pytest.mark.parametrize("th,nnratio", [(1, 0.8), (3, 0.8), (5, 0.6)])
def test_mps_matches_oracle(seq, ctx, oracle, th, nnratio):
    t, L, R, fr = seq
    g = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
    rng = np.random.default_rng(th)
    cur = fr[1]
    src = fr[0]
    # local map points: last-frame keypoints projected with the true rotation + small noise
    m = len(src["kl"])
    from slam_framework_amd import slamgpu as G
    q = np.zeros(m, G.MPS_QUERY_DTYPE)
    H = S._homography(1)
    uv = np.stack([src["kl"]["x"], src["kl"]["y"], np.ones(m, np.float32)], 1) @ H.T
    q["proj_x"] = (uv[:, 0] / uv[:, 2] + rng.normal(0, 0.7, m)).astype(np.float32)
    q["proj_y"] = (uv[:, 1] / uv[:, 2] + rng.normal(0, 0.7, m)).astype(np.float32)
    d = np.where(src["depth"] > 0, CAM[4] / np.maximum(src["depth"], 1e-3), 30.0)
    q["proj_xr"] = (q["proj_x"] - d).astype(np.float32)
    q["view_cos"] = rng.choice(np.array([0.9, 0.998, 0.999], np.float32), m)
    q["level"] = src["kl"]["octave"]
    q["in_view"] = rng.random(m) < 0.9
    q["is_bad"] = rng.random(m) < 0.05
    q["mp_id"] = np.arange(m)
    q["blocks"] = rng.random(m) < 0.8
    q["desc"] = src["dl"]
    n = len(cur["kl"])
    # pre-existing matches in the current frame (ids >= m), some with observations
    extra = 64
    nobs = np.concatenate([q["blocks"].astype(np.int32), rng.integers(0, 2, extra).astype(np.int32)])
    mp0 = np.full(n, -1, np.int32)
    pre = rng.choice(n, extra, replace=False)
    mp0[pre] = m + np.arange(extra)
    mp_o = mp0.copy()
    nm_o = oracle.search_mps(t, g, cur["kl"], cur["dl"], cur["ur"], mp_o, q, nobs, nnratio, th)
    ctx.frame_stereo(L[1], R[1], CAM)
    mp_g = mp0.copy()
    blk = np.zeros(n, np.uint8)
    blk[pre] = nobs[m:] > 0
    nm_g = ctx.search_by_projection_mps(0, q, nnratio, th, mp_g, blk)
    assert nm_g == nm_o
    np.testing.assert_array_equal(mp_g, mp_o)
    assert nm_o > 50
