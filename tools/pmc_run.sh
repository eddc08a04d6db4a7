#!/bin/bash
# PMC passes over a command, one rocprofv3 run per counter group (kernel-trace only, never with
# sys/runtime traces; each pass under its own time limit, stop at the first failure).
#   GROUPS_FILE=tools/pmc_groups/orient_desc.txt KERNEL=orient_desc OUT=gpurun_out/r4a/pmc \
#     tools/pmc_run.sh python3 bench.py --steps 2 --warmup 1 --inflight 1 ...
set -e
export TMPDIR=/tmp
K=${KERNEL:-orient_desc}
OUT=${OUT:-gpurun_out/pmc/$K}
mkdir -p "$OUT"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  case "$grp" in \#*) continue ;; esac
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$K" --kernel-trace \
    --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1
  echo "pass $i ok: $grp"
done < "$GROUPS_FILE"
