"""Edge cases of the extractor path against the oracle, bit-exact (ORBextractor::Compute,
orb_extractor.cpp:985-1049):

  - flat images: no FAST corner anywhere, so every cell takes the minThFAST fallback (:753-757)
    and every level's DistributeOctTree gets no candidates;
  - low-texture images: most cells find nothing at iniThFAST and fall back;
  - an image that is a view into a wider buffer with an odd row pitch (the unaligned tile path),
    and odd image sizes;
  - other ORBextractor parameters (nfeatures, scaleFactor, nlevels, thresholds);
  - an empty image returns nothing (:990-991), an image too small for the pyramid is rejected.
"""
import numpy as np
import pytest

from slam_framework_amd import synthetic as S

pytestmark = pytest.mark.gpu


def check(oracle, G, img, params=(2000, 1.2, 8, 20, 7)):
    t = oracle.tables(*params)
    kps_o, desc_o = oracle.extract(t, img)
    kps_g, desc_g = G.ORBextractor(*params).Compute(img)
    assert kps_g.tobytes() == kps_o.tobytes(), f"{len(kps_g)} vs {len(kps_o)} keypoints"
    assert np.array_equal(desc_g, desc_o)
    return len(kps_o)


@pytest.mark.parametrize("shape,value", [((240, 320), 0), ((376, 1241), 128), ((479, 641), 255)])
def test_flat_image(oracle, gpu_lib, shape, value):
    img = np.full(shape, value, np.uint8)
    assert check(oracle, gpu_lib, img) == 0


def test_low_texture_image_uses_fallback(oracle, gpu_lib):
    rng = np.random.default_rng(5)
    y, x = np.mgrid[0:376, 0:1241]
    img = (96 + 40 * np.sin(x / 90.0) * np.cos(y / 70.0) + rng.normal(0, 2.5, (376, 1241)))
    img = np.clip(img, 0, 255).astype(np.uint8)
    n = check(oracle, gpu_lib, img)
    assert n > 0  # the smooth field has few corners at th = 20: most come from the th = 7 pass


@pytest.mark.parametrize("cols,rows", [(641, 479), (1241, 376), (333, 201)])
def test_odd_pitch_view(oracle, gpu_lib, cols, rows):
    L, _ = S.stereo_pair(77, cols, rows)
    pitch = cols + 1
    while pitch % 4 != 1:
        pitch += 1
    buf = np.zeros((rows, pitch), np.uint8)  # row pitch = 1 mod 4
    buf[:, 1:cols + 1] = L
    view = buf[:, 1:cols + 1]  # odd base offset too
    assert view.strides[0] % 4 == 1
    check(oracle, gpu_lib, view)


@pytest.mark.parametrize("params", [(1000, 1.2, 8, 20, 7), (500, 1.5, 4, 30, 10),
                                    (1500, 1.3, 6, 12, 5)])
def test_other_extractor_parameters(oracle, gpu_lib, params):
    L, _ = S.stereo_pair(2024, S.KITTI_COLS, S.KITTI_ROWS)
    assert check(oracle, gpu_lib, L, params) > 0


def test_too_small_image_is_rejected(gpu_lib):
    # 160x120 at 8 levels: level 7 is 45x33, below the FAST cell grid's minimum -- the
    # reference divides by a zero cell count there (orb_extractor.cpp:712-733)
    with pytest.raises(gpu_lib.SlamGpuError, match="too small"):
        gpu_lib.ORBextractor(2000, 1.2, 8, 20, 7).Compute(np.zeros((120, 160), np.uint8))


def test_empty_image(gpu_lib):
    assert gpu_lib.ORBextractor(2000, 1.2, 8, 20, 7).Compute(np.zeros((0, 0), np.uint8)) is None
