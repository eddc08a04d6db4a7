#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES per dispatch of the bench's kernels (one rocprofv3
# --pmc pass, kernel-trace only) -> gpurun_out/valu/; tools/valu.py turns it into profiles/valu.json.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/valu}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --kernel-trace \
  --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --no-optimizer > $OUT/p1.log 2>&1
echo ok
