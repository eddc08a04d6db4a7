#!/bin/bash
# One GPU call's worth of round evidence: bench line, rocprofv3 kernel stats of the same
# command, per-dispatch HBM traffic and VALU instruction counts.
#   TAG=r1g tools/round_profile.sh   -> gpurun_out/$TAG/...
set -e
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py > $OUT/stats.log 2>&1
OUT=$OUT/traffic timeout -k 10 700 tools/pmc_traffic.sh > $OUT/traffic.log 2>&1
OUT=$OUT/valu timeout -k 10 400 tools/pmc_valu.sh > $OUT/valu.log 2>&1
echo done
