"""Per-dispatch HBM traffic from tools/pmc_traffic.sh output (FETCH_SIZE / WRITE_SIZE, KB).

Calibration (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts half the bytes of a
16-B-per-lane streaming read; other widths are uncalibrated, so the membench kernels copy16
(16 B/lane) and copy4 (4 B/lane, the width the ORB kernels use) are profiled beside the bench and
their known byte counts give the read factor per width. Writes are taken as reported.
Usage: python tools/traffic.py gpurun_out/traffic [kernel|-] [batch] > profiles/traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_key(name):
    """Short kernel name; anonymous-namespace kernels keep their own name."""
    n = name.replace("void ", "").replace("slamgpu::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def per_kernel(d, counter):
    """Mean counter value per dispatch of each kernel, over its batch dispatches only (grid at least
    1/32 of its largest): the launches the bench line describes (the same kernels also run at B=1 for the drop-in
    latency figures, and those would drag a plain average down)."""
    acc = collections.defaultdict(list)
    grid = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_key(r["Kernel_Name"])
            did = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
            acc[(k, did)].append(float(r["Counter_Value"]))
            grid[(k, did)] = int(r.get("Grid_Size", 0) or 0)
    gmax = collections.defaultdict(int)
    for (k, did), g in grid.items():
        gmax[k] = max(gmax[k], g)
    out = collections.defaultdict(list)
    for (k, did), v in acc.items():
        if 32 * grid[(k, did)] >= gmax[k]:
            out[k].append(sum(v))  # sum over dimensions of one dispatch
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
    want = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else None
    mb_f = per_kernel(os.path.join(base, "membench_fetch"), "FETCH_SIZE")
    mb_w = per_kernel(os.path.join(base, "membench_write"), "WRITE_SIZE")
    known = 512 << 20  # membench: each copy reads and writes 512 MiB
    cal = {}
    for k, v in mb_f.items():
        if k.startswith("copy16") or k.startswith("copy4") or k.startswith("copylds"):
            cal[k.split("(")[0]] = known / (v * 1024.0)
    f = per_kernel(os.path.join(base, "bench_fetch"), "FETCH_SIZE")
    w = per_kernel(os.path.join(base, "bench_write"), "WRITE_SIZE")
    read_factor = cal.get("copy4", 2.0)
    res = {"batch": batch,
           "command": "python3 bench.py " + os.environ.get("ARGS", "") + " (tools/pmc_traffic.sh)",
           "source": "tools/pmc_traffic.sh + tools/traffic.py",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, "
                     "kernel-trace only; each kernel's batch dispatches (grid >= 1/32 of its largest); FETCH_SIZE (KB) x read factor calibrated on membench "
                     "copy4/copy16 (known 512 MiB) + WRITE_SIZE (KB)",
           "calibration_read_factor": cal, "write_calibration": {k: known / (v * 1024.0) for k, v in mb_w.items()
                                                                if k.startswith("copy")},
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        if want and want not in k:
            continue
        fb = f.get(k, 0.0) * 1024.0 * read_factor
        wb = w.get(k, 0.0) * 1024.0
        res["kernels"][k] = {"fetch_kb_raw": f.get(k), "write_kb_raw": w.get(k),
                             "hbm_bytes_per_dispatch": fb + wb}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
