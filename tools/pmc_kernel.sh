#!/bin/bash
# Per-kernel PMC passes over a short bench run: one rocprofv3 invocation per counter group,
# kernel-trace only (never combined with sys/runtime traces).
#   KERNEL=fast_cells tools/pmc_kernel.sh            -> gpurun_out/pmck/<kernel>/p<i>/...
#   CMD="python3 tools/pose_time.py 1024 2" KERNEL=pose_opt tools/pmc_kernel.sh
set -e
export TMPDIR=/tmp
K=${KERNEL:-fast_cells}
OUT=${OUT:-gpurun_out/pmck/$K}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
CMD=${CMD:-"python3 bench.py $ARGS"}
mkdir -p $OUT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$K" --kernel-trace \
    --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  echo "pass $i ok: $grp"
done <<GROUPS
MeanOccupancyPerCU
VALUBusy
SALUBusy
LdsUtil
VmemLatency
SmemLatency
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SPI_RA_VGPR_SIMD_FULL_CSN SPI_RA_LDS_CU_FULL_CSN SPI_RA_WAVE_SIMD_FULL_CSN SPI_RA_RES_STALL_CSN SPI_RA_TGLIM_CU_FULL_CSN SPI_RA_SGPR_SIMD_FULL_CSN
SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
GROUPS
