"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py from the oracle).

CPU leg: the oracle still reproduces its committed outputs. GPU leg: the HIP path reproduces the
same bytes through the C ABI. Both pin drift only -- parity vs the (unbuildable) reference binary
is unpinned."""
import json
import os

import numpy as np
import pytest

from golden import make_golden as MG

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _small():
    z = np.load(os.path.join(HERE, "orb_small_320x240.npz"))
    return z["image"], z["keypoints"], z["descriptors"]


def test_oracle_reproduces_small_fixture(oracle):
    img, k, d = _small()
    img2, k2, d2 = MG.small_case()
    np.testing.assert_array_equal(img2, img)
    assert k2.view(np.uint8).reshape(len(k2), 28).tobytes() == k.tobytes()
    np.testing.assert_array_equal(d2, d)


def test_oracle_reproduces_kitti_hashes(oracle):
    js = json.load(open(os.path.join(HERE, "kitti_synthetic_hashes.json")))
    for seed, want in js["cases"].items():
        assert MG.kitti_case(int(seed)) == want


@pytest.mark.gpu
def test_gpu_reproduces_small_fixture(gpu_lib):
    img, k, d = _small()
    ctx = gpu_lib.Context(320, 240, nfeatures=500)
    kg, dg = ctx.extract(img)
    assert kg.view(np.uint8).reshape(len(kg), 28).tobytes() == k.tobytes()
    np.testing.assert_array_equal(dg, d)


@pytest.mark.gpu
def test_gpu_reproduces_kitti_hashes(gpu_lib):
    from slam_framework_amd import synthetic as S
    js = json.load(open(os.path.join(HERE, "kitti_synthetic_hashes.json")))
    ctx = gpu_lib.Context(S.KITTI_COLS, S.KITTI_ROWS)
    for seed, want in js["cases"].items():
        L, R = S.stereo_pair(int(seed))
        ctx.frame_stereo(L, R, S.KITTI_CAM)
        kl, dl = ctx.keypoints(0)
        kr, dr = ctx.keypoints(1)
        ur, depth = ctx.stereo(0)
        got = dict(n_left=len(kl), n_right=len(kr), n_stereo=int((depth > 0).sum()),
                   image_left=MG.sha(L), image_right=MG.sha(R), kps_left=MG.sha(kl),
                   desc_left=MG.sha(dl), kps_right=MG.sha(kr), desc_right=MG.sha(dr),
                   u_right=MG.sha(ur), depth=MG.sha(depth))
        assert got == want
