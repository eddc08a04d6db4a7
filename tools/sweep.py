"""Runs bench.py once per argument set and prints one summary line each (ms/step, frames/s,
in-step kernel split): python3 tools/sweep.py --inflight,2 --inflight,3,--streams,2 ...
(commas separate the arguments of one set: tools/gpu.sh py=tools/sweep.py:SET:SET ...;
KEY=VALUE tokens go to the environment, LIB=path picks a library build)
Every run adds the quick flags (--steps 10 --warmup 2 --no-cpu-baseline --no-optimizer)."""
import json
import os
import subprocess
import sys

QUICK = ["--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-optimizer"]


def main(argsets):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for a in argsets:
        toks = a.replace(",", " ").split()
        env = dict(os.environ)
        env.update(t.split("=", 1) for t in toks if "=" in t and not t.startswith("-"))
        lib = env.pop("LIB", None)  # LIB=path: that library build instead of the in-tree one
        if lib:
            env["SLAMGPU_LIB"] = os.path.abspath(os.path.join(root, lib))
        args = [t for t in toks if not ("=" in t and not t.startswith("-"))]
        cmd = [sys.executable, os.path.join(root, "bench.py")] + QUICK + args
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root, env=env)
        if r.returncode != 0:
            print(f"{a:32s} FAILED rc {r.returncode} {r.stderr[-400:]}", flush=True)
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        ks = " ".join(f"{k}={v:.3f}" for k, v in (d.get("kernel_ms_per_step") or {}).items() if v)
        sa = " ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in (d.get("kernels_standalone") or {}).items())
        print(f"{a:32s} {d['ms_per_step']:.3f} ms {d['value']:.0f} f/s | {ks}\n{'':32s} standalone: {sa}",
              flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
