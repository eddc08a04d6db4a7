set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4pmc; mkdir -p $O
OUT=$O/traffic timeout -k 10 700 bash tools/pmc_traffic.sh > $O/traffic.log 2>&1 || exit 1
OUT=$O/valu timeout -k 10 400 bash tools/pmc_valu.sh > $O/valu.log 2>&1 || exit 1
exit 0
