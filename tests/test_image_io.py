"""The ingest step before the hot path (include/slamgpu_io.h):
LoadKittiImages (examples/main_stereo.cpp:16-49) and the 8-bit PNG reader behind
cv::imread(path, CV_LOAD_IMAGE_UNCHANGED) (:105-106). CPU only (host code in libslamgpu.so).

The committed fixtures (tests/golden/png/, made by tests/golden/make_png.py) decode byte for byte
to their pixels in cv::imread's channel order: every row filter, Adam7, split IDAT, an ancillary
chunk, gray / RGB / RGBA / gray+alpha / 4-bit palette with tRNS / 1-bit gray, and a file Pillow
encoded. KITTI itself is absent from the image; its sequence layout is built in a temp dir."""
import glob
import os

import numpy as np
import pytest

from slam_framework_amd import slamgpu as G

HERE = os.path.dirname(os.path.abspath(__file__))
PNG = os.path.join(HERE, "golden", "png")


@pytest.fixture(scope="module")
def lib():
    from slam_framework_amd import build
    build.build()
    return G.lib()


@pytest.mark.parametrize("name", sorted(os.path.basename(p)[:-4]
                                        for p in glob.glob(os.path.join(PNG, "*.png"))))
def test_png_fixture_decodes_exactly(lib, name):
    exp = np.load(os.path.join(PNG, "expected.npz"))[name]
    data = open(os.path.join(PNG, name + ".png"), "rb").read()
    got = G.png_decode(data)
    assert got.shape == exp.shape and got.dtype == np.uint8
    assert got.tobytes() == exp.tobytes()
    assert G.imread_png(os.path.join(PNG, name + ".png")).tobytes() == exp.tobytes()


def test_png_rejects_bad_files(lib):
    good = open(os.path.join(PNG, "rgb8.png"), "rb").read()
    bad_crc = bytearray(good)
    bad_crc[40] ^= 0xFF                                  # inside IHDR/first chunks: CRC fails
    sixteen = bytearray(good)
    sixteen[24] = 16                                     # IHDR bit depth 16 (CRC then fails too)
    for data in (b"not a png at all" * 4, bytes(bad_crc), good[:60], bytes(sixteen)):
        with pytest.raises(G.SlamGpuError):
            G.png_decode(data)
    with pytest.raises(G.SlamGpuError):
        G.imread_png(os.path.join(PNG, "missing.png"))


def test_png_small_output_buffer(lib):
    import ctypes as C
    data = np.frombuffer(open(os.path.join(PNG, "rgb8.png"), "rb").read(), np.uint8)
    out = np.zeros(100, np.uint8)
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    rc = lib.slamgpu_png_decode(G._ptr(data), data.size, G._ptr(out), 183, out.size,
                                C.byref(w), C.byref(h), C.byref(c))
    assert rc == -3 and (w.value, h.value, c.value) == (61, 17, 3)   # SLAMGPU_ECAP, sizes known


def test_kitti_load_images(lib, tmp_path):
    seq = tmp_path / "00"
    seq.mkdir()
    times = [0.0, 0.103736, 0.207472, 1.2e3]
    (seq / "times.txt").write_text("".join(f"{t:e}\n" for t in times) + "\n")
    left, right, ts = G.kitti_load_images(str(seq))
    assert np.array_equal(ts, np.array(times))
    assert left[2] == f"{seq}/image_2/000002.png" and right[3] == f"{seq}/image_3/000003.png"
    assert len(left) == len(right) == 4
    with pytest.raises(G.SlamGpuError):
        G.kitti_load_images(str(tmp_path / "missing"))
    # a decoded KITTI-like pair through the listing: image_2/000000.png from the Pillow fixture
    (seq / "image_2").mkdir()
    data = open(os.path.join(PNG, "pil_rgb8.png"), "rb").read()
    (seq / "image_2" / "000000.png").write_bytes(data)
    img = G.imread_png(left[0])
    assert img.shape == (48, 124, 3)
    assert img.tobytes() == np.load(os.path.join(PNG, "expected.npz"))["pil_rgb8"].tobytes()
