#!/bin/bash
# One rocprofv3 --pmc pass per library build (SLAMGPU_LIB) of the short bench command, with the
# counters given: tools/pmc_libs.sh OUTDIR "COUNTERS" lib1.so [lib2.so ...]
# then: python tools/pmc_summary.py OUTDIR/<lib name>   (one p<i> directory per pass)
set -o pipefail
export TMPDIR=/tmp
OUT=$1; CNT=$2; shift 2
mkdir -p $OUT
for lib in "$@"; do
  n=$(basename $lib .so)
  SLAMGPU_LIB=$(readlink -f $lib) timeout -s KILL 200 rocprofv3 --pmc $CNT --kernel-trace \
    --output-format csv -d $OUT/$n/p1 -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-optimizer > $OUT/$n.log 2>&1 || { echo "pmc $n rc=$?"; exit 1; }
  python3 tools/pmc_summary.py $OUT/$n | grep -E "orient_desc|fast_cells|pyr_down|stereo_match|octree_img|search_cand" | sed "s/^/$n /"
done
