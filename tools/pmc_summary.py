"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(base, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("slamgpu::", "").replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "slamgpu" not in k and not any(x in k for x in ("kernel",)):
        continue
    out = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k[:40].ljust(40), " ".join(f"{c}={out[c]:.4g}" for c in sorted(out)))
