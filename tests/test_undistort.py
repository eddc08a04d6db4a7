"""Frame::UndistortKeyPoints / ComputeImageBounds (src/data/frame.cpp:614-675): the oracle's
cv::undistortPoints restatement (OpenCV 3.3.1 cvUndistortPoints) pinned against an independent
numpy statement of the same published iteration, the host C-ABI entry point of libslamgpu.so
(pure host code, no device needed) against the oracle, and size-independent properties.
Parity against OpenCV itself is unpinned (OpenCV is not in the image)."""
import numpy as np
import pytest

from slam_framework_amd import synthetic as S

CAM = S.KITTI_CAM
# k1 k2 p1 p2 [k3]: a mild 4-coefficient set, a 5-coefficient set, strong barrel, k1 == 0
DISTS = [np.array([-0.05, 0.01, 1e-4, -2e-4], np.float32),
         np.array([0.02, -0.03, -5e-4, 3e-4, 0.004], np.float32),
         np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32)]


def np_undistort(cam, dist, xy):
    """cvUndistortPoints for R = I, P = K, in float64, operation by operation."""
    k = np.zeros(14)
    k[:len(dist)] = dist.astype(np.float64)
    fx, fy, cx, cy = (np.float64(np.float32(v)) for v in cam[:4])
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (xy[:, 0].astype(np.float64) - cx) * ifx
    y = (xy[:, 1].astype(np.float64) - cy) * ify
    x0, y0 = x.copy(), y.copy()
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    xx = fx * x + 0.0 * y + cx
    yy = 0.0 * x + fy * y + cy
    ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
    return np.stack([(xx * ww).astype(np.float32), (yy * ww).astype(np.float32)], 1)


def distort(cam, dist, xy):
    """Forward Brown-Conrady model (cv::projectPoints' distortion), float64."""
    k = np.zeros(5)
    k[:len(dist)] = dist
    fx, fy, cx, cy = cam[:4]
    x = (xy[:, 0] - cx) / fx
    y = (xy[:, 1] - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k[0] * r2 + k[1] * r2 * r2 + k[4] * r2 ** 3
    xd = x * rad + 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
    yd = y * rad + k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


def points(seed, n=4000):
    rng = np.random.default_rng(seed)
    xy = np.stack([rng.uniform(0, S.KITTI_COLS, n), rng.uniform(0, S.KITTI_ROWS, n)], 1)
    xy[:4] = [[0, 0], [S.KITTI_COLS, 0], [0, S.KITTI_ROWS], [S.KITTI_COLS, S.KITTI_ROWS]]
    return xy.astype(np.float32)


@pytest.mark.parametrize("di", range(len(DISTS)))
def test_oracle_matches_numpy_restatement(oracle, di):
    xy = points(di)
    a = oracle.undistort_points(CAM, DISTS[di], xy)
    b = np_undistort(CAM, DISTS[di], xy)
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("di", range(len(DISTS)))
def test_host_abi_matches_oracle(oracle, gpu_lib, di):
    xy = points(10 + di)
    a = oracle.undistort_points(CAM, DISTS[di], xy)
    b = gpu_lib.undistort_points(CAM, DISTS[di], xy)
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("di", [0, 1])
def test_undistort_inverts_distortion(oracle, di):
    """Five fixed-point iterations invert mild distortion to well under a pixel."""
    xy = points(20 + di).astype(np.float64)
    und = oracle.undistort_points(CAM, DISTS[di], xy.astype(np.float32)).astype(np.float64)
    back = distort(CAM, DISTS[di].astype(np.float64), und)
    assert np.abs(back - xy).max() < 0.05


def test_keypoints_k1_zero_is_identity(oracle):
    kps = np.zeros(50, oracle.KP_DTYPE)
    rng = np.random.default_rng(3)
    kps["x"] = rng.uniform(0, 1241, 50)
    kps["y"] = rng.uniform(0, 376, 50)
    kps["angle"] = rng.uniform(0, 360, 50)
    kps["octave"] = rng.integers(0, 8, 50)
    out = oracle.undistort_keypoints(CAM, np.array([0.0, 0.3, 0.01, 0.02], np.float32), kps)
    assert out.tobytes() == kps.tobytes()  # frame.cpp:616-619 tests k1 only
    out = oracle.undistort_keypoints(CAM, DISTS[0], kps)
    for f in ("size", "angle", "response", "octave", "class_id"):
        np.testing.assert_array_equal(out[f], kps[f])
    assert (out["x"] != kps["x"]).any()


def test_image_bounds(oracle):
    g0 = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
    assert (g0.min_x, g0.max_x, g0.min_y, g0.max_y) == (0.0, 1241.0, 0.0, 376.0)
    g = oracle.grid_geom(S.KITTI_COLS, S.KITTI_ROWS, CAM, DISTS[2])
    c = np_undistort(CAM, DISTS[2], points(0)[:4])
    assert g.min_x == min(c[0, 0], c[2, 0]) and g.max_x == max(c[1, 0], c[3, 0])
    assert g.min_y == min(c[0, 1], c[1, 1]) and g.max_y == max(c[2, 1], c[3, 1])
    assert g.cell_w == np.float32(np.float32(g.max_x - g.min_x) / np.float32(64))
