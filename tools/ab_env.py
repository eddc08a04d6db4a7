"""A/B timing of environment variants of one build:
    python tools/ab_env.py "SLAMGPU_FORK=0" "SLAMGPU_OCT_LVL=1" ... [-- bench args]
Each variant is a comma-separated list of NAME=VALUE settings ("-" for none). Runs bench.py once
per variant, each under its own time limit, and prints the step time, throughput and per-kernel
ms. Stops at the first failing run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
extra = ["--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-optimizer", "--no-bow"]
if "--" in argv:
    i = argv.index("--")
    argv, extra = argv[:i], argv[i + 1:]
for spec in argv:
    env = dict(os.environ)
    if spec != "-":
        for kv in spec.split(","):
            k, v = kv.split("=", 1)
            env[k] = v
    p = subprocess.run(["timeout", "-k", "10", "150", sys.executable, os.path.join(ROOT, "bench.py"),
                        *extra], env=env, capture_output=True, text=True)
    if p.returncode != 0:
        print(spec, "FAILED rc", p.returncode, p.stderr[-2000:], flush=True)
        sys.exit(1)
    d = json.loads(p.stdout.strip().splitlines()[-1])
    k = d.get("kernel_ms_per_step", {})
    ks = " ".join(f"{n}={v:.3f}" for n, v in k.items() if v > 0.02)
    lat = (d.get("drop_in") or {}).get("single_frame", {}).get("median_ms")
    ks_alone = {n: e.get("alone_ms_per_step") for n, e in d.get("kernels_standalone", {}).items()}
    al = " ".join(f"{n}={v:.3f}" for n, v in ks_alone.items() if v and v > 0.02)
    if al:
        ks += f" | alone {al}"
    print(f"{spec:36s} {d['ms_per_step']:.3f} ms {d['value']:.0f} f/s | {ks}"
          + (f" | drop-in {lat:.3f} ms" if lat else ""), flush=True)
