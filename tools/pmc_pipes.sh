#!/bin/bash
# Per-dispatch pipe counters of the bench's kernels, two rocprofv3 --pmc passes (kernel-trace
# only; per pass at most 8 SQ, 2 TA, 2 TD, 2 GRBM, 4 TCP counters) -> gpurun_out/pipes/p{1,2};
# tools/pipes.py turns them (with profiles/isa_mix.json) into profiles/pipes.json.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pipes}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency --no-alone"}
mkdir -p $OUT
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
i=1
for cnt in "$P1" "$P2"; do
  timeout -s KILL 240 rocprofv3 --pmc $cnt --kernel-trace --output-format csv -d $OUT/p$i -o run \
    -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pipes pass $i rc=$?"; exit 1; }
  echo "pipes pass $i ok"
  i=$((i + 1))
done
