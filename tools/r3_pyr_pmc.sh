#!/bin/bash
# PMC passes (stall / issue breakdown) of the pyramid kernels: fused band kernel and, with
# SLAMGPU_PYR_FUSED=0, the per-level kernels. One rocprofv3 invocation per counter group.
#   TAG=r3w tools/r3_pyr_pmc.sh
export TMPDIR=/tmp
TAG=${TAG:-r3w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency --inflight 1"
i=0
for fused in 1 0; do
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    SLAMGPU_FORK=0 SLAMGPU_PYR_FUSED=$fused timeout -s KILL 120 rocprofv3 --pmc $grp \
      --kernel-include-regex "pyr_" --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
    echo "pass $i ok (fused=$fused): $grp"
  done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT
GROUPS
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
