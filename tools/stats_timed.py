"""Kernel durations inside bench.py's timed region, from a rocprofv3 --kernel-trace CSV of the same
command: bench launches `trace_marker_kernel` (slamgpu_trace_marker) with a 1 x 1 grid just
before and a 1 x 2 grid just after the timed steps, with the device drained on both sides, so the
launches that start after the first mark and end before the second are exactly the timed ones.
Their per-kernel average is what the bench line's roofline divides by (bench measures it live with
HIP events on context 0's launches; this counts every context's).
Usage: python tools/stats_timed.py <run_kernel_trace.csv> > profiles/<tag>_timed_kernel_stats.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marks = {}
    for r in rows:
        if "trace_marker_kernel" in r["Kernel_Name"]:
            marks[int(r["Grid_Size_Y"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if 1 not in marks or 2 not in marks:
        sys.exit("no trace_marker_kernel pair (ids 1 and 2) in the trace")
    lo, hi = marks[1][1], marks[2][0]
    acc = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > hi or "trace_marker_kernel" in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].replace("void ", "").replace("slamgpu::", "")
        k = k.replace("(anonymous namespace)::", "").split("(")[0]
        g = "x".join(r[f"Grid_Size_{a}"] for a in "XYZ")
        acc[(k, g)].append((e - s) / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "calls", "avg_us", "median_us", "min_us", "max_us", "total_us",
                "timed_region_us"])
    for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        sv = sorted(v)
        w.writerow([k, g, len(v), round(sum(v) / len(v), 2), round(sv[len(sv) // 2], 2),
                    round(sv[0], 2), round(sv[-1], 2), round(sum(v), 1), round((hi - lo) / 1e3, 1)])


if __name__ == "__main__":
    main()
