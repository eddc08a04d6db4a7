#!/bin/bash
# HBM traffic per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass, kernel-trace
# only), for the bench command and for the membench calibration kernels (known byte counts).
#   tools/pmc_traffic.sh  -> gpurun_out/traffic/{bench,membench}_{fetch,write}/...
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/traffic}
ARGS=${ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --no-optimizer --no-alone"}  # recorded by traffic.py via ARGS
export ARGS
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/bench_$lc -o run -- python3 bench.py $ARGS > $OUT/bench_$lc.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/membench_$lc -o run -- ./tools/membench > $OUT/membench_$lc.log 2>&1
  echo "$c ok"
done
