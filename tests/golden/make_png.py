"""Generates the committed PNG fixtures of tests/test_image_io.py (tests/golden/png/): small
files covering what include/slamgpu_io.h's decoder must handle -- every row filter, Adam7
interlacing, gray / RGB / RGBA / gray+alpha / palette (+tRNS) / 1-bit gray -- encoded here with
zlib from seeded pixels, plus a KITTI-like 8-bit RGB image written by Pillow (adaptive filters,
an independent encoder). expected.npz holds each file's pixels in cv::imread(IMREAD_UNCHANGED)
order (BGR / BGRA; palettes expanded; gray+alpha as BGRA; 1-bit gray as 0 / 255).

    python tests/golden/make_png.py      (rewrites tests/golden/png/)
"""
import os
import struct
import zlib

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "png")


def chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body))


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def filter_rows(rows, bpp, filters):
    """rows: list of bytes (unfiltered scanlines); filters: filter type per row."""
    out, prev = [], bytes(len(rows[0])) if rows else b""
    for r, f in zip(rows, filters):
        o = bytearray([f])
        for x in range(len(r)):
            a = r[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, paeth(a, b, c)][f]
            o.append((r[x] - pred) & 255)
        out.append(bytes(o))
        prev = r
    return b"".join(out)


def pack_bits(samples, depth):
    """One scanline of `depth`-bit samples, MSB first."""
    if depth == 8:
        return bytes(samples)
    out, acc, n = bytearray(), 0, 0
    for s in samples:
        acc = (acc << depth) | int(s)
        n += depth
        if n == 8:
            out.append(acc)
            acc, n = 0, 0
    if n:
        out.append(acc << (8 - n))
    return bytes(out)


def encode(samples, color, depth=8, interlace=False, plte=None, trns=None, seed=0):
    """samples: [h][w][spp] ints; filters chosen per row from a seeded cycle of all five."""
    h, w, spp = samples.shape
    rng = np.random.default_rng(seed)
    bpp = max(1, spp * depth // 8)

    def image_rows(img):
        return [pack_bits(img[y].reshape(-1), depth) for y in range(img.shape[0])]
    if interlace:
        data = b""
        for x0, y0, dx, dy in ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4),
                               (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)):
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                rows = image_rows(sub)
                data += filter_rows(rows, bpp, rng.integers(0, 5, len(rows)))
    else:
        rows = image_rows(samples)
        data = filter_rows(rows, bpp, [i % 5 for i in range(len(rows))])
    png = b"\x89PNG\r\n\x1a\n"
    png += chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, int(interlace)))
    if plte is not None:
        png += chunk(b"PLTE", bytes(np.asarray(plte, np.uint8).reshape(-1)))
    if trns is not None:
        png += chunk(b"tRNS", bytes(np.asarray(trns, np.uint8)))
    png += chunk(b"tEXt", b"Comment\x00slamgpu fixture")          # an ancillary chunk to skip
    z = zlib.compress(data, 9)
    png += chunk(b"IDAT", z[:len(z) // 2]) + chunk(b"IDAT", z[len(z) // 2:])  # split IDAT
    png += chunk(b"IEND", b"")
    return png


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(2024)
    exp = {}

    def smooth(h, w, c):  # gradients + noise: every filter type sees real predictions
        y, x = np.mgrid[0:h, 0:w]
        base = (3 * x + 5 * y)[..., None] + 40 * np.arange(c)
        return ((base + rng.integers(0, 40, (h, w, c))) % 256).astype(np.uint8)
    gray = smooth(23, 37, 1)
    exp["gray8"] = gray[..., 0]
    open(os.path.join(OUT, "gray8.png"), "wb").write(encode(gray, 0))
    rgb = smooth(17, 61, 3)
    exp["rgb8"] = rgb[..., ::-1]
    open(os.path.join(OUT, "rgb8.png"), "wb").write(encode(rgb, 2))
    exp["rgb8_adam7"] = rgb[..., ::-1]
    open(os.path.join(OUT, "rgb8_adam7.png"), "wb").write(encode(rgb, 2, interlace=True, seed=3))
    rgba = smooth(13, 29, 4)
    exp["rgba8"] = rgba[..., [2, 1, 0, 3]]
    open(os.path.join(OUT, "rgba8.png"), "wb").write(encode(rgba, 6))
    ga = smooth(11, 19, 2)
    exp["graya8"] = np.stack([ga[..., 0]] * 3 + [ga[..., 1]], -1)
    open(os.path.join(OUT, "graya8.png"), "wb").write(encode(ga, 4))
    plte = rng.integers(0, 256, (16, 3))
    trns = rng.integers(0, 256, 10)
    idx = rng.integers(0, 16, (9, 21, 1))
    bgra = np.concatenate([plte[idx[..., 0]][..., ::-1],
                           np.where(idx < 10, trns[np.minimum(idx, 9)], 255)], -1)
    exp["pal4_trns"] = bgra.astype(np.uint8)
    open(os.path.join(OUT, "pal4_trns.png"), "wb").write(
        encode(idx, 3, depth=4, plte=plte, trns=trns))
    bits = rng.integers(0, 2, (7, 27, 1))
    exp["gray1_adam7"] = (bits[..., 0] * 255).astype(np.uint8)
    open(os.path.join(OUT, "gray1_adam7.png"), "wb").write(
        encode(bits, 0, depth=1, interlace=True, seed=5))
    # a KITTI-like colour image from another encoder (Pillow, adaptive per-row filters)
    from PIL import Image
    kit = smooth(48, 124, 3)
    Image.fromarray(kit, "RGB").save(os.path.join(OUT, "pil_rgb8.png"), optimize=True)
    exp["pil_rgb8"] = kit[..., ::-1]
    np.savez_compressed(os.path.join(OUT, "expected.npz"), **exp)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
