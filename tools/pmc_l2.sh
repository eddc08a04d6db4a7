# L1 -> L2 request pressure of the front-end kernels per library build (one --pmc pass each):
# tools/pmc_l2.sh OUT lib1.so [lib2.so ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
bash tools/pmc_libs.sh $OUT "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "$@"
