"""A/B timing of library builds: python tools/ab.py tools/abl/libslamgpu_a.so ... [-- bench args]
Runs bench.py once per build (SLAMGPU_LIB), each under its own time limit, and prints the step
time, throughput and per-kernel ms. Stops at the first failing run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
extra = ["--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-optimizer"]
if "--" in argv:
    i = argv.index("--")
    argv, extra = argv[:i], argv[i + 1:]
for lib in argv:
    env = dict(os.environ, SLAMGPU_LIB=os.path.abspath(lib))
    p = subprocess.run(["timeout", "-k", "10", "150", sys.executable, os.path.join(ROOT, "bench.py"),
                        *extra], env=env, capture_output=True, text=True)
    if p.returncode != 0:
        print(lib, "FAILED rc", p.returncode, p.stderr[-2000:], flush=True)
        sys.exit(1)
    d = json.loads(p.stdout.strip().splitlines()[-1])
    k = d.get("kernel_ms_per_step", {})
    ks = " ".join(f"{n}={v:.3f}" for n, v in k.items() if v > 0.02)
    print(f"{os.path.basename(lib):28s} {d['ms_per_step']:.3f} ms {d['value']:.0f} f/s | {ks}",
          flush=True)
