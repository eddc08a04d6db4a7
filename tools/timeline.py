"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV: for the last bench step, each
kernel's start / end relative to the step's first kernel (us), to read the critical path."""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
key = "Kernel_Name"
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key].split("(")[0].replace("void ", "").replace("slamgpu::", ""))
      for r in rows]
ev.sort()
# steps start at pyr_down level 1 launch preceded by fast level 0 on the side stream: split at
# the first kernel of each step = the fast_cells launch that comes right before a pyr_down
marks = [i for i, e in enumerate(ev) if e[2].startswith("pyr_down") and (i == 0 or not ev[i - 1][2].startswith("pyr_down"))]
first = marks[-int(sys.argv[2]) if len(sys.argv) > 2 else -2]
nxt = [m for m in marks if m > first]
end = nxt[0] if nxt else len(ev)
t0 = min(e[0] for e in ev[max(0, first - 3):end])
for s, e, n in ev[max(0, first - 3):end]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n[:60]}")
