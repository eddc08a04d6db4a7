"""Bank-conflict model of orient_desc's sample reads (MI355X_MICROARCH.md, LDS table: a
ds_read_b32 is served in two groups of 32 lanes, bank = dword address mod 32, identical
addresses broadcast, each extra distinct address on a bank costs one cycle). Lane L reads sample
e of test 64 r + L at the keypoint's angle: 4 consecutive dwords from the column-major u16
row-sum table (stride = u16 rows per column). Prints the expected extra cycles per b32 access
for several column strides over random angles -- the gather is random at every stride.
Usage: python tools/lds_conflict_sim.py [n_angles]"""
import os
import re
import sys

import numpy as np


def main(n_angles=400):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = open(os.path.join(root, "slam_framework_amd/csrc/orb_pattern.inc")).read()
    s = re.sub(r"//.*", "", s)
    pat = np.array([int(x) for x in re.findall(r"-?\d+", s)][-1024:]).reshape(256, 2, 2)
    angles = np.random.default_rng(0).uniform(0, 2 * np.pi, n_angles)

    def extra(stride):
        tot = n = 0
        for th in angles:
            c, sn = np.cos(th), np.sin(th)
            for r in range(4):
                for e in range(2):
                    P = pat[64 * r:64 * r + 64, e]
                    x = np.rint(P[:, 0] * c - P[:, 1] * sn).astype(int) + 18
                    y = np.rint(P[:, 0] * sn + P[:, 1] * c).astype(int) + 18
                    base = (x * stride + y) * 2 // 4
                    for k in range(4):
                        for grp in (slice(0, 32), slice(32, 64)):
                            b = np.bincount(np.unique(base[grp] + k) % 32, minlength=32)
                            tot += b.max() - 1
                            n += 1
        return tot / n

    for stride in (42, 44, 46, 48, 50, 52):
        print(f"u16 rows per column {stride}: {extra(stride):.2f} extra cycles per 32-lane group "
              f"of a ds_read_b32")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400)
