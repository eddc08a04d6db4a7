# orient_desc diagnosis per library build: texture path, issue / wait and LDS counters (three
# rocprofv3 --pmc passes): tools/pmc_od.sh OUT lib1.so [lib2.so ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
bash tools/pmc_libs.sh $OUT/ta "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "$@" && \
bash tools/pmc_libs.sh $OUT/sq "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES" "$@" && \
bash tools/pmc_libs.sh $OUT/lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" "$@"
