# Dynamic instruction mix per kernel (one rocprofv3 --pmc pass per build): tools/pmc_mix.sh OUT lib...
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
bash tools/pmc_libs.sh $OUT "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY" "$@"
