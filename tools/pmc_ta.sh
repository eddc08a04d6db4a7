# TA / TCP / TD pressure of the front-end kernels per library build (one rocprofv3 --pmc pass per
# build): tools/pmc_ta.sh OUT lib1.so [lib2.so ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
bash tools/pmc_libs.sh $OUT "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "$@"
