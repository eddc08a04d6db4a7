#!/bin/bash
# Stall / issue breakdown PMC passes of the frontend kernels over a short bench run, one
# rocprofv3 invocation per counter group (kernel-trace only, never with sys/runtime traces).
#   OUT=gpurun_out/r2c/pmc tools/pmc_stalls.sh ; python3 tools/pmc_summary.py gpurun_out/r2c/pmc
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_stalls}
RE=${RE:-"fast_cells|orient_desc|pyr_down|octree|stereo_match"}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency --inflight 1"}
mkdir -p $OUT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RE" --kernel-trace \
    --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  echo "pass $i ok: $grp"
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE GRBM_COUNT
GROUPS
