"""Build libslamgpu.so (HIP kernels + C++ runtime) in-tree for gfx950.

`python -m slam_framework_amd.build` or `__graft_entry__.build()`. hipcc cross-compiles without a
GPU. -ffp-contract=off keeps float results bit-identical to the reference's expression-by-
expression semantics (explicit fmaf() only where the reference's Release build fuses).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libslamgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SLAMGPU_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc"))
    deps += glob.glob(os.path.join(os.path.dirname(PKG), "include", "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        build_capi_check()
        build_adapter_check()
        return LIB
    objdir = os.path.join(PKG, "build")
    os.makedirs(objdir, exist_ok=True)
    procs, objs = [], []
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for src, p in procs:
        out = p.communicate()[0].decode(errors="replace")
        if p.returncode != 0:
            failed.append(f"{src}:\n{out}")
        elif verbose and out.strip():
            print(out, file=sys.stderr)
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(failed))
    tmp = LIB + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-lz"],
                   check=True)
    os.replace(tmp, LIB)
    build_capi_check()
    build_adapter_check()
    return LIB


ROOT = os.path.dirname(PKG)
CAPI_SRC = os.path.join(ROOT, "tests", "capi_check.cpp")
CAPI_BIN = os.path.join(ROOT, "tests", "capi_check")
CAPI_KF_SRC = os.path.join(ROOT, "tests", "capi_kf_check.cpp")
CAPI_KF_BIN = os.path.join(ROOT, "tests", "capi_kf_check")


def build_capi_check() -> str:
    """g++ builds of tests/capi_check.cpp and tests/capi_kf_check.cpp against include/*.h*,
    linked to libslamgpu.so: the C++ caller side of the drop-in boundary, with no HIP or Python
    in between."""
    headers = glob.glob(os.path.join(ROOT, "include", "*.h*"))
    for src, exe in ((CAPI_SRC, CAPI_BIN), (CAPI_KF_SRC, CAPI_KF_BIN)):
        if os.path.exists(exe) and os.path.getmtime(exe) >= max(
                os.path.getmtime(d) for d in [src, LIB] + headers):
            continue
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"),
                        src, "-L", PKG, "-lslamgpu",
                        "-Wl,-rpath,$ORIGIN/../slam_framework_amd", "-o", exe], check=True)
    return CAPI_BIN


ADAPTER_SRC = os.path.join(ROOT, "tests", "adapter_check.cpp")
ADAPTER_BIN = os.path.join(ROOT, "tests", "adapter_check")


def build_adapter_check() -> str:
    """g++ build of tests/adapter_check.cpp: include/slamgpu_adapters.hpp (the OpenCV-free graph
    gathering of the reference-side adapters) compiled and driven on the CPU."""
    deps = [ADAPTER_SRC, LIB] + glob.glob(os.path.join(ROOT, "include", "*.h*"))
    if os.path.exists(ADAPTER_BIN) and os.path.getmtime(ADAPTER_BIN) >= max(
            os.path.getmtime(d) for d in deps):
        return ADAPTER_BIN
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-I",
                    os.path.join(ROOT, "include"), ADAPTER_SRC, "-L", PKG, "-lslamgpu",
                    "-Wl,-rpath,$ORIGIN/../slam_framework_amd", "-o", ADAPTER_BIN], check=True)
    return ADAPTER_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
