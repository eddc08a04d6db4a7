#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter group; counters are
# collected with kernel-trace only, never with sys/runtime traces). Output: gpurun_out/pmc/<pass>/
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p $OUT
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  echo "pass $i ok"
done
