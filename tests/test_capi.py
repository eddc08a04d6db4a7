"""The C-ABI library builds for gfx950, loads, and exports every function include/*.h declares
(no compute calls: no GPU here)."""
import os
import re

from slam_framework_amd import build, slamgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(slamgpu_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_header():
    build.build()
    lib = slamgpu.lib()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(slamgpu.EXPORTS)


def test_descriptor_distance_host():
    import numpy as np
    rng = np.random.default_rng(0)
    for _ in range(50):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert slamgpu.OrbMatcher.DescriptorDistance(a, b) == int(np.unpackbits(a ^ b).sum())
