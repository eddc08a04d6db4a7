"""Regenerates the committed golden fixtures from the oracle (CPU restatement).

These fixtures pin the oracle (and, through tests/test_golden.py's GPU leg, the HIP path)
against drift. They are NOT reference outputs: the reference cannot be built here and ships no
fixtures for this path ("parity unpinned"). Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_lib as O  # noqa: E402
from slam_framework_amd import synthetic as S  # noqa: E402

SMALL = dict(seed=5, cols=320, rows=240, nfeatures=500)
KITTI_SEEDS = [3000, 3001]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def small_case():
    t = O.tables(nfeatures=SMALL["nfeatures"])
    img = S.image(SMALL["seed"], SMALL["cols"], SMALL["rows"])
    k, d = O.extract(t, img)
    return img, k, d


def kitti_case(seed):
    t = O.tables()
    L, R = S.stereo_pair(seed)
    kl, dl, pl = O.extract(t, L, True)
    kr, dr, pr = O.extract(t, R, True)
    ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, S.KITTI_CAM[0], S.KITTI_CAM[4])
    return dict(n_left=len(kl), n_right=len(kr), n_stereo=int((depth > 0).sum()),
                image_left=sha(L), image_right=sha(R), kps_left=sha(kl), desc_left=sha(dl),
                kps_right=sha(kr), desc_right=sha(dr), u_right=sha(ur), depth=sha(depth))


def main():
    O.build()
    img, k, d = small_case()
    np.savez_compressed(os.path.join(HERE, "orb_small_320x240.npz"), image=img,
                        keypoints=k.view(np.uint8).reshape(len(k), 28), descriptors=d)
    js = {"params": {"nfeatures": 2000, "scale_factor": 1.2, "nlevels": 8, "ini_th": 20,
                     "min_th": 7, "camera": list(S.KITTI_CAM)},
          "cases": {str(s): kitti_case(s) for s in KITTI_SEEDS}}
    with open(os.path.join(HERE, "kitti_synthetic_hashes.json"), "w") as f:
        json.dump(js, f, indent=1)
    print("wrote fixtures:", len(k), "small keypoints")


if __name__ == "__main__":
    main()
