"""Kernel durations from a rocprofv3 --kernel-trace CSV, split by launch grid: the batch launches
the bench line times and the B=1 launches of its drop-in latency figures are different workloads,
and rocprofv3's own kernel_stats averages them together.
Usage: python tools/stats_by_grid.py <run_kernel_trace.csv> > profiles/<tag>_kernel_stats_by_grid.csv"""
import collections
import csv
import sys

acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").replace("slamgpu::", "")
    k = k.replace("(anonymous namespace)::", "").split("(")[0]
    g = "x".join(r[f"Grid_Size_{a}"] for a in "XYZ")
    acc[(k, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
w = csv.writer(sys.stdout)
w.writerow(["kernel", "grid", "calls", "avg_us", "median_us", "min_us", "max_us", "total_us"])
for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    s = sorted(v)
    w.writerow([k, g, len(v), round(sum(v) / len(v), 2), round(s[len(s) // 2], 2), round(s[0], 2),
                round(s[-1], 2), round(sum(v), 1)])
