"""Timeline of bench.py's timed region from a rocprofv3 --kernel-trace CSV (the region between the
trace_marker_kernel launches, as tools/stats_timed.py): per hardware queue its busy fraction and
gaps, how much of the region has 0 / 1 / 2 / 3+ kernels running, and each kernel's time spent
running alone. With --steps N also prints the kernel sequence of the first N steps per queue.
Usage: python tools/timeline.py <run_kernel_trace.csv> [--steps N]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    nshow = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 0
    rows = list(csv.DictReader(open(path)))
    marks = {}
    for r in rows:
        if "trace_marker_kernel" in r["Kernel_Name"]:
            marks[int(r["Grid_Size_Y"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    lo, hi = marks[1][1], marks[2][0]
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > hi or "trace_marker_kernel" in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].replace("void ", "").replace("slamgpu::", "")
        k = k.replace("(anonymous namespace)::", "").split("(")[0]
        ks.append((s, e, k, r.get("Queue_Id", "?")))
    ks.sort()
    span = hi - lo
    print(f"timed region {span / 1e3:.1f} us, {len(ks)} kernels")
    byq = collections.defaultdict(list)
    for s, e, k, q in ks:
        byq[q].append((s, e, k))
    for q, v in sorted(byq.items()):
        busy = sum(e - s for s, e, _ in v)
        gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
        pos = [g for g in gaps if g > 0]
        print(f"queue {q}: {len(v)} kernels, busy {busy / span:.3f}, gaps > 0: {len(pos)}, "
              f"sum {sum(pos) / 1e3:.1f} us, median {sorted(pos)[len(pos) // 2] / 1e3 if pos else 0:.1f} us")
    # concurrency: sweep the start / end events
    ev = sorted([(s, 1, k) for s, e, k, _ in ks] + [(e, -1, k) for s, e, k, _ in ks])
    run = collections.Counter()
    hist = collections.Counter()
    alone = collections.Counter()
    t = lo
    for x, d, k in ev:
        n = sum(run.values())
        hist[min(n, 3)] += x - t
        if n == 1:
            alone[next(iter(+run))] += x - t
        t = x
        run[k] += d
    hist[0] += hi - t
    print("concurrency: " + ", ".join(f"{n}{'+' if n == 3 else ''}: {hist[n] / span:.3f}"
                                      for n in range(4)))
    print("running alone (us per region): " + ", ".join(
        f"{k}={v / 1e3:.0f}" for k, v in alone.most_common(12)))
    if nshow:
        for q, v in sorted(byq.items()):
            print(f"-- queue {q}")
            t0 = v[0][0]
            for s, e, k in v[:nshow]:
                print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {k}")


if __name__ == "__main__":
    main()
