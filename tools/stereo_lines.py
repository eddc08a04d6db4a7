"""Compulsory HBM bytes of stereo_match's SAD windows at cache-line granularity (analysis tool,
not the product). The kernel_bytes() model in bench.py counts 121 + 231 window bytes per left
keypoint; HBM moves whole lines, and the windows of different keypoints rarely share one, so the
line-granular figure is the floor the kernel's FETCH_SIZE traffic can reach. Keypoints, levels and
the stereo matches come from the oracle (oracle/, test infrastructure) on the bench's scene
(synthetic.layered_sequence); the right window is centred on the final u_right (the kernel
centres it on the best Hamming match, at most a pixel away), so keypoints whose SAD step was
rejected are not counted (an underestimate).
    python tools/stereo_lines.py
"""
import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import oracle_lib as O
from slam_framework_amd import synthetic as S
t = O.tables()
L, R = S.layered_sequence(1000, 4)
cam = S.KITTI_CAM
scale = [1.2 ** l for l in range(8)]
tot = {}
for f in range(4):
    kl, dl, pl = O.extract(t, L[f], True)
    kr, dr, pr = O.extract(t, R[f], True)
    ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, cam[0], cam[4])
    shapes = [pl.level(l).shape for l in range(8)]
    # level base addresses: level 0 = its own image (pitch 1280); levels >= 1 packed, pitch
    # round_up(w, 64), 256-aligned offsets
    bases, off = [0], 1 << 24
    pitches = [1280] + [((s[1] + 63) // 64) * 64 for s in shapes[1:]]
    for l in range(1, 8):
        bases.append(off); off += ((pitches[l] * shapes[l][0] + 255) // 256) * 256
    for LINE in (64, 128):
        lines = set(); nwin = 0; byte_model = 0
        for i, k in enumerate(kl):
            if ur[i] < 0:
                continue
            nwin += 1
            l = int(k["octave"]); s = 1.0 / scale[l]
            xcl = int(round(k["x"] * s)); yc = int(round(k["y"] * s)); xcr = int(round(ur[i] * s))
            for side, x0, x1 in ((0, xcl - 5, xcl + 5), (1 << 40, xcr - 10, xcr + 10)):
                for y in range(yc - 5, yc + 6):
                    a0 = side + bases[l] + y * pitches[l] + x0
                    a1 = side + bases[l] + y * pitches[l] + x1
                    for ln in range(a0 // LINE, a1 // LINE + 1):
                        lines.add(ln)
            byte_model += 121 + 231
        tot.setdefault(LINE, []).append((len(kl), nwin, len(lines) * LINE, byte_model))
for LINE, v in tot.items():
    a = np.array(v, float).mean(0)
    print(f"line {LINE}: kps {a[0]:.0f} windows {a[1]:.0f} window lines bytes/frame {a[2]/1e3:.1f} KB, byte model {a[3]/1e3:.1f} KB")
