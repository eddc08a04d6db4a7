"""Per-dispatch VALU wave-instruction counts from tools/pmc_valu.sh -> profiles/valu.json.

The VALU issue roofline of a kernel: SQ_INSTS_VALU per dispatch / dispatch time against the
chip's issue peak, 256 CUs x 4 SIMD-32 x one wave64 VALU instruction per 2 cycles x 2.4 GHz
(MI355X_MICROARCH.md, Execution model) = 1.2288e12 wave-instructions/s.
Usage: python tools/valu.py gpurun_out/valu [batch] > profiles/valu.json"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 128
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
grid = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("slamgpu::", "")
        k = k.replace("(anonymous namespace)::", "").split("(")[0]
        did = r.get("Dispatch_Id", "")
        acc[k][r["Counter_Name"]][did] += float(r["Counter_Value"])
        grid[(k, did)] = int(r.get("Grid_Size", 0) or 0)
# each kernel's batch dispatches only (grid >= 1/32 of its largest): the launches (the B=1 drop-in latency
# launches of the same kernels would drag a plain average down)
gmax = collections.defaultdict(int)
for (k, did), g in grid.items():
    gmax[k] = max(gmax[k], g)
out = {"batch": batch, "source": "tools/pmc_valu.sh + tools/valu.py (rocprofv3 --pmc, bench.py "
       "--steps 2 --warmup 1; each kernel's batch dispatches)", "valu_issue_peak_per_s": 1.2288e12, "kernels": {}}
for k, cs in acc.items():
    e = {}
    for c, disp in cs.items():
        v = [x for did, x in disp.items() if 32 * grid[(k, did)] >= gmax[k]]
        e[c.lower() + "_per_dispatch"] = sum(v) / len(v)
    out["kernels"][k] = e
print(json.dumps(out, indent=1, sort_keys=True))
