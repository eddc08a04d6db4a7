#!/bin/bash
# Per-level pyr_down launch times (kernel trace of the short bench, split by launch grid) with the
# LDS-ring pyramid on (SLAMGPU_PYR_RING=1) and off: tools/pyr_levels.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for mode in 1 0; do
  export SLAMGPU_PYR_RING=$mode
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/ring$mode -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-optimizer > $O/ring$mode.json \
    2> $O/ring$mode.err || { echo "rocprof ring=$mode rc=$?"; exit 1; }
  f=$(ls $O/ring$mode/*/run_kernel_trace.csv $O/ring$mode/run_kernel_trace.csv 2>/dev/null | head -1)
  echo "ring=$mode $(tail -c 200 $O/ring$mode.json | grep -o '"ms_per_step": [0-9.]*')"
  python3 tools/stats_by_grid.py $f | grep -E "pyr_|kernel," | tee $O/ring${mode}_pyr.csv
done
