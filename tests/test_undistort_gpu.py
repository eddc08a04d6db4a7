"""Device Frame::UndistortKeyPoints (frame.cpp:614-641) and the frame matchers on undistorted
keypoints with a distorted camera's image bounds (ComputeImageBounds :644-675, grid :234-248),
bit-compared with the oracle. Parity of the oracle vs OpenCV is unpinned (tests/test_undistort.py
pins it against a numpy statement of cvUndistortPoints)."""
import numpy as np
import pytest

import scenario
from slam_framework_amd import synthetic as S
from test_undistort import DISTS

pytestmark = pytest.mark.gpu
CAM = S.KITTI_CAM


@pytest.fixture(scope="module")
def seq(oracle):
    t = oracle.tables()
    L, R = S.sequence(2100, 2)
    frames = []
    for i in range(2):
        kl, dl, pl = oracle.extract(t, L[i], True)
        kr, dr, pr = oracle.extract(t, R[i], True)
        ur, depth, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
        frames.append(dict(kl=kl, dl=dl, ur=ur, depth=depth))
    return t, L, R, frames


@pytest.mark.parametrize("di", range(len(DISTS)))
def test_frame_undistorted_keypoints(seq, oracle, gpu_lib, di):
    t, L, R, fr = seq
    ctx = gpu_lib.Context(S.KITTI_COLS, S.KITTI_ROWS)
    ctx.set_distortion(DISTS[di])
    ctx.frame_stereo(L[0], R[0], CAM)
    un = ctx.undistorted_keypoints(0)
    ref = oracle.undistort_keypoints(CAM, DISTS[di], fr[0]["kl"])
    assert un.tobytes() == ref.tobytes()
    kl, _ = ctx.keypoints(0)  # the distorted keypoints stay as extracted
    assert kl.tobytes() == fr[0]["kl"].tobytes()
    ctx.set_distortion(None)
    ctx.frame_stereo(L[0], R[0], CAM)
    assert ctx.undistorted_keypoints(0).tobytes() == fr[0]["kl"].tobytes()


def test_undistort_device_batched(seq, oracle, gpu_lib):
    import torch
    t, L, R, fr = seq
    sets = [fr[0]["kl"], fr[1]["kl"], fr[0]["kl"][:7], fr[1]["kl"][:0]]
    cap = max(len(s) for s in sets)
    buf = np.zeros((len(sets), cap), oracle.KP_DTYPE)
    for i, s in enumerate(sets):
        buf[i, :len(s)] = s
    cnt = np.array([len(s) for s in sets], np.int32)
    d_in = torch.from_numpy(buf.view(np.uint8)).cuda()
    d_cnt = torch.from_numpy(cnt).cuda()
    d_out = torch.zeros_like(d_in)
    gpu_lib.undistort_keypoints_device(CAM, DISTS[1], d_in, cap, d_cnt, 1, d_out, cap, len(sets),
                                       cap)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().view(oracle.KP_DTYPE).reshape(len(sets), cap)
    for i, s in enumerate(sets):
        ref = oracle.undistort_keypoints(CAM, DISTS[1], s)
        assert out[i, :len(s)].tobytes() == ref.tobytes()


@pytest.mark.parametrize("di", [0, 2])
def test_f2f_search_on_undistorted(seq, oracle, gpu_lib, di):
    """SearchByProjection(Frame, Frame) reads undistorted keypoints through the grid built on
    the undistorted image bounds."""
    t, L, R, fr = seq
    dist = DISTS[di]
    g = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS, CAM, dist)
    last, cur = fr[0], fr[1]
    last_un = oracle.undistort_keypoints(CAM, dist, last["kl"])
    cur_un = oracle.undistort_keypoints(CAM, dist, cur["kl"])
    q, last_mp, last_out, xyz, mdesc, nobs = scenario.vo_queries(
        last_un, last["dl"], last["depth"], 0, np.random.default_rng(7), 0.5)
    p = scenario.pose(1, th=7.0, check_ori=1)
    n = len(cur["kl"])
    mp_o = np.full(n, -1, np.int32)
    nm_o = oracle.search_frame(t, g, cur_un, cur["dl"], cur["ur"], mp_o, last_un, last_mp,
                               last_out, xyz, mdesc, nobs, p["Rcw"][0].reshape(3, 3), p["tcw"][0],
                               0.0, float(p["baseline"][0]), CAM, 7.0, 0, 1)
    ctx = gpu_lib.Context(S.KITTI_COLS, S.KITTI_ROWS)
    ctx.set_distortion(dist)
    ctx.frame_stereo(L[1], R[1], CAM)
    mp_g = np.full(n, -1, np.int32)
    nm_g = ctx.search_by_projection_frame(0, q, p, mp_g, np.zeros(n, np.uint8))
    assert nm_g == nm_o
    np.testing.assert_array_equal(mp_g, mp_o)
    assert nm_o > (10 if di == 0 else 0)
