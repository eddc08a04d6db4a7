"""The C ABI from a C++ caller (tests/capi_check.cpp, built by g++ against include/*.h and linked
to libslamgpu.so -- no Python or ctypes between caller and library): ORBextractor::Compute on the
committed 320x240 golden fixture (bit-exact), PoseOptimization on a C4-style problem and
LocalBundleAdjustment on a small graph (oracle tolerance of tests/test_pose_gpu.py /
tests/test_ba_gpu.py)."""
import os
import subprocess

import numpy as np
import pytest

from slam_framework_amd import build as B
from slam_framework_amd import slamgpu as G
from slam_framework_amd import synthetic as S

HERE = os.path.dirname(os.path.abspath(__file__))
CAM = S.KITTI_CAM
EPS32 = np.finfo(np.float32).eps


def test_capi_check_builds_and_links():
    """CPU leg: the C++ caller compiles against the public headers alone and links the library."""
    exe = B.build_capi_check()
    out = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libslamgpu.so" in out and "not found" not in out.split("libslamgpu.so")[1].split("\n")[0]


def _write_inputs(d, img, nfeat, pose, lba):
    with open(os.path.join(d, "image.hdr"), "w") as f:
        f.write(f"{img.shape[1]} {img.shape[0]} {nfeat}\n")
    img.tofile(os.path.join(d, "image.u8"))
    cam = np.asarray(CAM, np.float32)
    edges, T0, isig = pose
    with open(os.path.join(d, "pose.bin"), "wb") as f:
        f.write(cam.tobytes() + np.int32(len(isig)).tobytes() + isig.astype(np.float32).tobytes())
        f.write(np.int32(len(edges)).tobytes() + np.ascontiguousarray(edges).tobytes())
        f.write(np.asarray(T0, np.float32).reshape(16).tobytes())
    P = lba
    nk = len(P["kf_mode"])
    mode = np.zeros((nk + 3) & ~3, np.uint8)
    mode[:nk] = P["kf_mode"]
    with open(os.path.join(d, "lba.bin"), "wb") as f:
        isg = np.asarray(P["inv_sigma2"], np.float32)
        f.write(cam.tobytes() + np.int32(len(isg)).tobytes() + isg.tobytes())
        f.write(np.int32(nk).tobytes() + np.asarray(P["kf_Tcw"], np.float32).tobytes())
        f.write(mode.tobytes() + np.int32(len(P["points"])).tobytes())
        f.write(np.asarray(P["points"], np.float32).tobytes())
        f.write(np.asarray(P["point_obs_start"], np.int32).tobytes())
        f.write(np.ascontiguousarray(P["obs"]).tobytes())


@pytest.mark.gpu
def test_cpp_caller_matches_golden_and_oracle(oracle, gpu_lib, tmp_path):
    z = np.load(os.path.join(HERE, "golden", "orb_small_320x240.npz"))
    edges, T0, _, isig, _ = S.pose_problem(77, 2000)
    P = S.ba_problem(78, n_local=6, n_fixed=2, n_points=400)
    _write_inputs(str(tmp_path), z["image"], 500, (edges, T0, isig), P)
    exe = B.build_capi_check()
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # ORBextractor::Compute: the committed golden keypoints and descriptors, byte for byte
    kps = np.fromfile(os.path.join(tmp_path, "extract.kps"), np.uint8)
    desc = np.fromfile(os.path.join(tmp_path, "extract.desc"), np.uint8)
    assert kps.tobytes() == z["keypoints"].tobytes()
    assert desc.tobytes() == z["descriptors"].tobytes()
    # the adapters' OpenCV-free ORBextractor (include/slamgpu_adapters.hpp): the same outputs, and
    # GetImagePyramid's level 1 = the oracle's resize of the image
    assert np.fromfile(os.path.join(tmp_path, "core.kps"), np.uint8).tobytes() == kps.tobytes()
    assert np.fromfile(os.path.join(tmp_path, "core.desc"), np.uint8).tobytes() == desc.tobytes()
    t = oracle.tables(nfeatures=500)
    _, _, pyr = oracle.extract(t, z["image"], True)
    assert np.fromfile(os.path.join(tmp_path, "core.pyr1"), np.uint8).tobytes() == \
        np.ascontiguousarray(pyr.level(1)).tobytes()
    # PoseOptimization: the oracle's inlier count and outliers, pose within the tolerance
    out = np.fromfile(os.path.join(tmp_path, "pose.out"), np.uint8)
    n_inl = int(out[:4].view(np.int32)[0])
    T = out[4:68].view(np.float32).reshape(4, 4)
    outl = out[68:68 + len(edges)].astype(bool)
    r_o, T_o, out_o, _ = oracle.pose_optimization(CAM, isig, edges, T0)
    assert n_inl == r_o and np.array_equal(outl, out_o)
    tol = 1e-5 * np.abs(T_o.astype(np.float64) - T0).max() + 4 * EPS32 * np.maximum(np.abs(T_o), 1)
    assert (np.abs(T.astype(np.float64) - T_o) <= tol).all()
    # LocalBundleAdjustment: the oracle's erase list, poses within the tolerance
    lo = np.fromfile(os.path.join(tmp_path, "lba.out"), np.uint8)
    nk, npt, no = len(P["kf_mode"]), len(P["points"]), len(P["obs"])
    its = int(lo[:4].view(np.int32)[0])
    kf = lo[4:4 + 64 * nk].view(np.float32).reshape(nk, 4, 4)
    er = lo[4 + 64 * nk + 12 * npt:4 + 64 * nk + 12 * npt + no].astype(bool)
    kf_o, _, er_o, its_o = oracle.local_ba(CAM, P)
    assert its > 0 and np.array_equal(er, er_o)
    tol = 1e-5 * np.abs(kf_o.astype(np.float64) - P["kf_Tcw"]).max() + 4 * EPS32 * np.maximum(
        np.abs(kf_o), 1)
    assert (np.abs(kf.astype(np.float64) - kf_o) <= tol).all()
